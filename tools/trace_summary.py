#!/usr/bin/env python3
"""Per-kernel duration distribution from a rocprofv3 --kernel-trace CSV dir.

    python tools/trace_summary.py gpurun_out/TAG/prof [--skip N]

--skip drops the first N dispatches of every kernel (warm-up).
--timeline [--step I] prints one step (from the I-th k_front, default the
second to last, to the next): start offset, duration and the gap before every kernel."""
import collections
import csv
import glob
import os
import re
import sys

import numpy as np


def main():
    d = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
    f = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    dur = collections.defaultdict(list)
    for r in rows:
        m = re.search(r"(k_\w+(?:<[^>]*>)?)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:40]
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    tot = 0.0
    print(f"{'kernel':34s} {'n':>5s} {'median us':>10s} {'p10':>8s} {'p90':>8s} {'sum us':>9s}")
    for k, v in sorted(dur.items(), key=lambda kv: -np.median(kv[1][skip:] or kv[1]) * len(kv[1])):
        v = np.array(v[skip:] or v)
        tot += v.sum()
        print(f"{k:34s} {len(v):5d} {np.median(v):10.1f} {np.percentile(v, 10):8.1f} {np.percentile(v, 90):8.1f} {v.sum():9.1f}")
    print(f"sum of kernel time {tot:.1f} us")


def timeline(d, anchor="k_front", which=-2, span=1):
    f = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    if len(idx) < span + 1:
        return
    a, b = idx[which], idx[min(which + span, len(idx) - 1)]
    t0 = int(rows[a]["Start_Timestamp"])
    prev_end = None
    q = "Queue_Id" if "Queue_Id" in rows[0] else None
    print(f"{'kernel':34s} {'start':>8s} {'dur':>7s} {'gap':>7s}" + ("  queue" if q else ""))
    for r in rows[a:b]:
        s_, e_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        m = re.search(r"(k_\w+(?:<[^>]*>)?)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:34]
        gap = "" if prev_end is None else f"{(s_ - prev_end) / 1000:7.1f}"
        print(f"{k:34s} {(s_ - t0) / 1000:8.1f} {(e_ - s_) / 1000:7.1f} {gap:>7s}" + (f"  {r[q]}" if q else ""))
        prev_end = e_ if prev_end is None else max(prev_end, e_)


if __name__ == "__main__":
    if "--timeline" in sys.argv:
        w = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else -2
        n = int(sys.argv[sys.argv.index("--span") + 1]) if "--span" in sys.argv else 1
        timeline(sys.argv[1], which=w, span=n)
        sys.exit(0)
    main()
