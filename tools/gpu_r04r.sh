#!/bin/bash
# round 4: pooled BatchNorm forward with wave-level per-cloud maxima
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04r
mkdir -p $OUT
run() {
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_train_hip.py \
    tests/test_training.py -m gpu > $OUT/tests.txt 2>&1 || return 1
  NDNET_TR_X6=1 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_train_hip.py \
    tests/test_training.py -m gpu > $OUT/tests_x6.txt 2>&1
  [ $? -ge 2 ] && return 1  # 1 = some test failed (recorded), else an error
  for rep in 1 2; do
    timeout -k 10 300 python -u tools/bench_train.py --graph --steps 30 --warmup 5 > $OUT/train_$rep.txt 2>&1 || return 1
    NDNET_TR_X6=1 timeout -k 10 300 python -u tools/bench_train.py --graph --steps 30 --warmup 5 > $OUT/train_x6_$rep.txt 2>&1 || return 1
  done
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $R/tools/bench_train.py --graph --steps 10 --warmup 3 > $OUT/prof.log 2>&1) || return 1
  python3 tools/trace_by_grid.py $OUT/prof k_tr_bn > $OUT/by_grid.txt
  (cd /tmp && export TMPDIR=/tmp && NDNET_TR_X6=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof6 -o run -- python3 $R/tools/bench_train.py --graph --steps 10 --warmup 3 > $OUT/prof6.log 2>&1) || return 1
  python3 tools/trace_by_grid.py $OUT/prof6 k_tr_gemm > $OUT/by_grid_x6.txt
  python3 tools/trace_by_grid.py $OUT/prof k_tr_gemm > $OUT/by_grid_gemm.txt
}
run; rc=$?
tail -3 $OUT/tests.txt; grep -E 'passed|failed|FAILED|HIP vs|max' $OUT/tests_x6.txt | head -20; grep -o '"step_ms": [0-9.]*' $OUT/train_*.txt; cat $OUT/by_grid.txt $OUT/by_grid_gemm.txt $OUT/by_grid_x6.txt
rm -rf $OUT/prof $OUT/prof6
exit $rc
