#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats of the
# pipelined bench and of an isolated (one graph per step, no overlap) run.
# Usage (from the repo root, on the GPU box): bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 10 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_iso -o run -- python3 $R/bench.py --steps 10 --no-pipeline --no-cpu-baseline > $OUT/prof_iso.log 2>&1 || { echo "rocprof iso failed"; tail -30 $OUT/prof_iso.log; exit 1; }
find $OUT/prof $OUT/prof_iso -name "*stats*" | head
