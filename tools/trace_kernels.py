#!/usr/bin/env python3
"""Median / min duration per kernel of a rocprofv3 kernel trace (CSV dir):
    python tools/trace_kernels.py gpurun_out/xxx/prof [substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

import numpy as np

path = sys.argv[1]
subs = sys.argv[2:]
rows = defaultdict(list)
with open(glob.glob(os.path.join(path, "*kernel_trace.csv"))[0]) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        rows[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for name, d in sorted(rows.items(), key=lambda kv: -np.median(kv[1]) * len(kv[1])):
    if subs and not any(s in name for s in subs):
        continue
    d = np.array(d)
    print(f"{name[:48]:48s} calls {len(d):6d}  median {np.median(d):8.2f} us  min {d.min():8.2f}  p90 {np.percentile(d, 90):8.2f}")
