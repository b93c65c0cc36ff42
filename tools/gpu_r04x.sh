#!/bin/bash
# round 4: graphed train step on resident input buffers (no per-step D2D copy)
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04x
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_training.py -m gpu > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
for rep in 1 2; do
  timeout -k 10 300 python -u tools/bench_train.py --graph --steps 30 --warmup 5 > $OUT/train_$rep.txt 2>&1 || exit 1
done
grep -o '"step_ms": [0-9.]*\|"eval_forward_after_step_ms": [0-9.]*' $OUT/train_*.txt
