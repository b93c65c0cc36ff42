#!/usr/bin/env python3
"""Median duration per (kernel, grid, workgroup) of a rocprofv3 kernel trace:
    python tools/trace_by_grid.py gpurun_out/xxx/prof [substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

import numpy as np

path = sys.argv[1]
subs = sys.argv[2:]
rows = defaultdict(list)
with open(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if subs and not any(s in name for s in subs):
            continue
        key = (name[:40], r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Grid_Size_Y", ""),
               r.get("Grid_Size_Z", ""), r.get("Workgroup_Size_X", r.get("Workgroup_Size", "?")))
        rows[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for key, d in sorted(rows.items(), key=lambda kv: -np.median(kv[1]) * len(kv[1])):
    d = np.array(d)
    print(f"{key[0]:40s} grid {key[1]:>8s} {key[2]:>5s} {key[3]:>5s} wg {key[4]:>5s}  calls {len(d):5d}  "
          f"median {np.median(d):8.2f} us  total {d.sum() / 1e3:8.3f} ms")
