#!/bin/bash
# round 4: per-launch durations of the graphed training step's HIP train kernels by grid
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04q
mkdir -p $OUT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $R/tools/bench_train.py --graph --steps 10 --warmup 3 > $OUT/prof.log 2>&1) || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/trace_by_grid.py $OUT/prof k_tr_ > $OUT/by_grid.txt && cat $OUT/by_grid.txt
rm -rf $OUT/prof
