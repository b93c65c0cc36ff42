#!/bin/bash
# round 4: 128 x 128 train-GEMM tiles from 256 / 128 workgroups up (default 512)
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04w
mkdir -p $OUT
for rep in 1 2; do
  for W in 512 256 128; do
    NDNET_TR_WIDE_MIN=$W timeout -k 10 300 python -u tools/bench_train.py --graph --steps 30 --warmup 5 > $OUT/train_w${W}_$rep.txt 2>&1 || exit 1
  done
done
grep -o '"step_ms": [0-9.]*' $OUT/train_*.txt
