#!/bin/bash
# Kernel statistics of the graphed training step (tools/bench_train.py --graph).
set -o pipefail
TAG=${1:-trainprof}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u $GRAFT_REPO_ROOT/tools/bench_train.py --graph --steps 20 --warmup 3 > $OUT/prof.log 2>&1 || { echo "prof failed"; tail -20 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cp $f $OUT/kernel_stats.csv
head -30 $OUT/kernel_stats.csv | cut -c1-220
