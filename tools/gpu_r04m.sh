#!/bin/bash
# round 4: train split-K parts for narrow layers; k_front point-ND batching only
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04m
mkdir -p $OUT
run() {
  timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_train_hip.py \
    tests/test_training.py tests/test_ndt_gpu.py -m gpu > $OUT/tests.txt 2>&1 || return 1
  timeout -k 10 300 python -u tools/bench_train.py --graph --steps 20 --warmup 5 > $OUT/train.txt 2>&1 || return 1
  timeout -k 10 300 python -u tools/bench_train.py --steps 20 --warmup 5 >> $OUT/train.txt 2>&1 || return 1
  for K in U L; do
    timeout -k 10 120 python -u tools/front_phases.py --kind $K > $OUT/front_$K.txt 2>&1 || return 1
  done
}
run; rc=$?
tail -3 $OUT/tests.txt; grep -v amdgpu $OUT/train.txt; grep -v amdgpu $OUT/front_*.txt
exit $rc
