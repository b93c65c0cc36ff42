#!/bin/bash
# Kernel trace of the default (pipelined: NDT || forward on two streams) bench.
# Usage (repo root, GPU box): bash tools/gpu_trace_pipe.sh TAG [bench args...]
set -o pipefail
TAG=${1:-trace_pipe}
shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-other "$@" > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
python3 $R/tools/trace_summary.py $OUT/prof --timeline --step 30
