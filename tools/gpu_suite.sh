#!/bin/bash
# Round-record pass: the whole -m gpu suite (verbose, names kept), smoke and the
# default bench line. Usage (repo root, GPU box): bash tools/gpu_suite.sh TAG
set -o pipefail
TAG=${1:-suite}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
# multi-rank path rehearsal on one card (gloo collectives; the driver's 8-GPU run uses RCCL)
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline --no-other > $OUT/bench_2ranks.log 2>&1 || { echo "2-rank bench failed"; tail -30 $OUT/bench_2ranks.log; exit 1; }
tail -1 $OUT/bench_2ranks.log | cut -c1-300
