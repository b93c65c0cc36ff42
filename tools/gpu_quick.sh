#!/bin/bash
# Quick GPU pass: parity tests, k_front phases, bench (no CPU baseline).
# Usage (repo root, GPU box): bash tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-quick}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -u tools/front_phases.py > $OUT/front_U.txt 2>&1 || { echo "front_phases failed"; tail -20 $OUT/front_U.txt; exit 1; }
cat $OUT/front_U.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
