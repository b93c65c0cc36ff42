#!/usr/bin/env python3
"""Per-kernel PMC summary from rocprofv3 --pmc passes (tools/gpu.sh pmc).

    python tools/pmc_summary.py gpurun_out/TAG [--json out.json]

Prints, per kernel (averaged over its dispatches): FETCH_SIZE / WRITE_SIZE
(KB, as rocprofv3 reports them) and the HBM bytes per launch derived per
MI355X_MICROARCH.md's HBM section (FETCH_SIZE doubled on gfx950 for wide
coalesced reads; WRITE_SIZE as is), plus the SQ/GRBM counters.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def kname(full):
    m = re.search(r"(k_\w+(?:<[^>]*>)?)\(", full)
    return m.group(1) if m else full.split("(")[0][-48:]


def load(d):
    """kernel -> counter -> per-dispatch values.  k_pn_chain dispatches are
    named A-D by their order within each forward (4 per forward)."""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        chain_seen = {}
        for r in rows:
            nm = r["Kernel_Name"]
            if "at::" in nm or "Cijk" in nm:
                continue
            key = kname(nm)
            if key.startswith("k_pn_chain"):
                did = r["Dispatch_Id"]
                if did not in chain_seen:
                    chain_seen[did] = len(chain_seen)
                key = "k_pn_chain " + "ABCD"[chain_seen[did] % 4]
            elif key.startswith("k_pn_fc"):
                key += f" grid={r['Grid_Size']}"
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    d = sys.argv[1]
    agg = load(d)
    out = {}
    for k, cs in agg.items():
        row = {c: sum(v) / len(v) for c, v in cs.items()}
        row["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in row and "WRITE_SIZE" in row:
            row["hbm_bytes"] = 2 * row["FETCH_SIZE"] * 1024 + row["WRITE_SIZE"] * 1024
        if "SQ_VALU_MFMA_BUSY_CYCLES" in row and row.get("GRBM_GUI_ACTIVE"):
            # MFMA cycles summed over all SIMDs / (GUI-active cycles summed over
            # the 8 XCDs x 128 SIMDs per XCD): the matrix pipes' busy fraction
            row["mfma_busy_frac"] = row["SQ_VALU_MFMA_BUSY_CYCLES"] / (row["GRBM_GUI_ACTIVE"] * 128.0)
        out[k] = row
    for k, row in sorted(out.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
        print(k)
        print("   " + ", ".join(f"{c}={v:.4g}" for c, v in row.items()))
    if "--json" in sys.argv:
        out["_source"] = d
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
