#!/bin/bash
# New labelled full-size tests + the default bench line (roofline by time per step).
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ndt_gpu.py -m gpu -k "labelled" -v --timeout 200 --timeout-method thread > $OUT/pytest_lab.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_lab.log; exit 1; }
tail -4 $OUT/pytest_lab.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
