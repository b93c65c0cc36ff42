#!/bin/bash
# Isolated-step kernel traces (one graph per step) of U and L with the round-4 end state, plus memory copies.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04ai
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for K in U L; do
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof_$K -o run -- python3 $R/bench.py --kind $K --no-pipeline --no-cpu-baseline --no-other --steps 10 > $OUT/prof_$K.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$K.log; exit 1; }
python3 $R/tools/trace_step.py $OUT/prof_$K k_front > $OUT/step_$K.txt || exit 1
done
