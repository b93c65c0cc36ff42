#!/bin/bash
# round 4: x6 for the weight-gradient GEMMs only (default) vs none
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04s
mkdir -p $OUT
run() {
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_train_hip.py \
    tests/test_training.py tests/test_model.py -m gpu > $OUT/tests.txt 2>&1 || return 1
  for rep in 1 2; do
    timeout -k 10 300 python -u tools/bench_train.py --graph --steps 30 --warmup 5 > $OUT/train_dw_$rep.txt 2>&1 || return 1
    NDNET_TR_X6=0 timeout -k 10 300 python -u tools/bench_train.py --graph --steps 30 --warmup 5 > $OUT/train_none_$rep.txt 2>&1 || return 1
  done
}
run; rc=$?
tail -2 $OUT/tests.txt; grep -o '"step_ms": [0-9.]*\|"eval_forward_after_step_ms": [0-9.]*' $OUT/train_*.txt
exit $rc
