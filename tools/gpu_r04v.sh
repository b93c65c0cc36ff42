#!/bin/bash
# round 4: train GEMM k-step 32 vs 16 (same sums), bit-identity check + step time
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04v
mkdir -p $OUT
run() {
  NDNET_TR_KT=32 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_train_hip.py \
    tests/test_training.py -m gpu > $OUT/tests_k32.txt 2>&1 || return 1
  for rep in 1 2; do
    timeout -k 10 300 python -u tools/bench_train.py --graph --steps 30 --warmup 5 > $OUT/train_k16_$rep.txt 2>&1 || return 1
    NDNET_TR_KT=32 timeout -k 10 300 python -u tools/bench_train.py --graph --steps 30 --warmup 5 > $OUT/train_k32_$rep.txt 2>&1 || return 1
  done
  (cd /tmp && export TMPDIR=/tmp && NDNET_TR_KT=32 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $R/tools/bench_train.py --graph --steps 10 --warmup 3 > $OUT/prof.log 2>&1) || return 1
  python3 tools/trace_by_grid.py $OUT/prof k_tr_gemm > $OUT/by_grid_k32.txt
}
run; rc=$?
tail -2 $OUT/tests_k32.txt; grep -o '"step_ms": [0-9.]*\|"loss": [0-9.]*' $OUT/train_*.txt; head -14 $OUT/by_grid_k32.txt
rm -rf $OUT/prof
exit $rc
