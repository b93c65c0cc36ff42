#!/bin/bash
# Config C5 (16 x 100k -> 2000 -> 1000 -> 500, a forward per level): the bench
# line and one isolated step's kernel timeline.  Usage: bash tools/gpu_c5.sh TAG
set -o pipefail
TAG=${1:-c5}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --levels 2000,1000,500 --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --levels 2000,1000,500 --no-cpu-baseline --no-pipeline --steps 5 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
cd $R && python3 tools/trace_step.py $OUT/prof k_front | tee $OUT/step.txt
