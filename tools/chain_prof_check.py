#!/usr/bin/env python3
"""k_pn_chain durations from rocprofv3 kernel traces against bench.py's line.

    python tools/chain_prof_check.py PROF_ISO_DIR PROF_DEFAULT_DIR BENCH_LOG

For each trace: the stats-style average over every k_pn_chain launch, and the
per-chain average of the back-to-back section bench.py times for its roofline
(runs of 20 consecutive launches of one chain, chains A-D in order).  The
bench line's roofline.all_chains.ms is printed beside them."""
import csv
import glob
import json
import sys


def chain_runs(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    dur = [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in rows]
    chains = [t for n, t in dur if "k_pn_chain" in n]
    runs, cur = [], []
    for n, t in dur:
        if "k_pn_chain" in n:
            cur.append(t)
        else:
            if len(cur) >= 20:
                runs.append(cur)
            cur = []
    if len(cur) >= 20:
        runs.append(cur)
    return chains, runs


def main():
    iso, dflt, blog = sys.argv[1:4]
    line = json.loads(open(blog).read().strip().splitlines()[-1])
    ms = line["roofline"]["all_chains"]["ms"]
    print("bench line: chains A-D per launch (us, back-to-back events):", [round(v * 1e3, 1) for v in ms],
          "sum", round(sum(ms) * 1e3, 1), "| in forward:",
          [round(v * 1e3, 1) for v in line["roofline"]["all_chains"].get("in_forward_ms", [])])
    for name, d in (("isolated (--no-pipeline)", iso), ("default command", dflt)):
        chains, runs = chain_runs(d)
        avg = sum(chains) / len(chains) / 1e3
        print(f"{name}: {len(chains)} k_pn_chain launches, stats average {avg:.1f} us")
        b2b = [sum(r[-20:]) / 20 / 1e3 for r in runs[-4:]]
        if len(b2b) == 4:
            print(f"  back-to-back sections (A-D, us): {[round(v, 1) for v in b2b]} sum {sum(b2b):.1f}")


if __name__ == "__main__":
    main()
