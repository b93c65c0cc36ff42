#!/usr/bin/env python3
"""Print the kernels of the last bench step from a rocprofv3 kernel trace
(CSV directory or .db): name, duration, grid, LDS, VGPRs.

    python tools/trace_step.py gpurun_out/prof_xxx [first-kernel-substring]
"""
import csv
import glob
import os
import sys


def rows_from(path):
    csvs = glob.glob(os.path.join(path, "*kernel_trace.csv"))
    if csvs:
        with open(csvs[0]) as f:
            for r in csv.DictReader(f):
                yield (r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Workgroup_Size_X", ""),
                       r.get("LDS_Block_Size", r.get("Lds_Size", "")), r.get("VGPR_Count", r.get("Arch_VGPR_Count", "")))
        return
    import sqlite3
    dbs = glob.glob(os.path.join(path, "*.db"))
    if not dbs:
        raise SystemExit(f"no kernel trace under {path}")
    db = sqlite3.connect(dbs[0])
    for r in db.execute("select name, start, end, grid_x, workgroup_x, lds_size, vgpr_count from kernels"):
        yield r


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_reset"
    rows = sorted(rows_from(path), key=lambda r: r[1])
    idx = [i for i, r in enumerate(rows) if first in r[0]]
    step = rows[idx[-1]:]
    t0 = step[0][1]
    total = 0.0
    for name, s, e, gx, wx, lds, vg in step:
        d = (e - s) / 1000
        total += d
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:58]
        print(f"{(s - t0) / 1000:9.2f} {d:9.2f} us  {short:58s} grid {gx} wg {wx} lds {lds} v{vg}")
    print(f"sum of kernel time {total:.1f} us, span {(step[-1][2] - t0) / 1000:.1f} us")


if __name__ == "__main__":
    main()
