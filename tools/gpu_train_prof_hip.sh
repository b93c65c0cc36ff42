#!/bin/bash
# Kernel stats of the graphed training step on the HIP train kernels.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trprof -o trprof -- python3 tools/bench_train.py --steps 20 --warmup 5 --graph > gpurun_out/trprof.log 2>&1 || { tail -20 gpurun_out/trprof.log; exit 1; }
f=$(find gpurun_out/trprof -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/train_hip_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/train_hip_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot/1e6:.2f} ms over {len(rows)} kernels")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.3f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
