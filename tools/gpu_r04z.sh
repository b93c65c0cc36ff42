#!/bin/bash
# round 4: BatchNorm workgroups of 1024 threads for every layer (NDNET_TR_BN1024=2) vs C < 512 only
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04z
mkdir -p $OUT
run() {
  NDNET_TR_BN1024=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_train_hip.py -m gpu > $OUT/tests.txt 2>&1 || return 1
  for rep in 1 2; do
    timeout -k 10 300 python -u tools/bench_train.py --graph --steps 30 --warmup 5 > $OUT/train_b1_$rep.txt 2>&1 || return 1
    NDNET_TR_BN1024=2 timeout -k 10 300 python -u tools/bench_train.py --graph --steps 30 --warmup 5 > $OUT/train_b2_$rep.txt 2>&1 || return 1
  done
  (cd /tmp && export TMPDIR=/tmp && NDNET_TR_BN1024=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $R/tools/bench_train.py --graph --steps 10 --warmup 3 > $OUT/prof.log 2>&1) || return 1
  python3 tools/trace_by_grid.py $OUT/prof k_tr_bn > $OUT/by_grid.txt
}
run; rc=$?
tail -2 $OUT/tests.txt; grep -o '"step_ms": [0-9.]*' $OUT/train_*.txt; cat $OUT/by_grid.txt
rm -rf $OUT/prof
exit $rc
