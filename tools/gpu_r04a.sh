#!/bin/bash
# Round-4 start: FP64 issue/latency ubench, L bench line + isolated L kernel trace.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 60 ./tools/ubench/fp64_latency > $OUT/fp64.txt 2>&1 || { echo "ubench failed"; cat $OUT/fp64.txt; exit 1; }
cat $OUT/fp64.txt
timeout -k 10 300 python -u bench.py --kind L --no-cpu-baseline --no-other > $OUT/bench_L.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_L.log; exit 1; }
tail -1 $OUT/bench_L.log | cut -c1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_L -o run -- python3 $R/bench.py --kind L --no-pipeline --no-cpu-baseline --no-other --steps 10 > $OUT/prof_L.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_L.log; exit 1; }
python3 $R/tools/trace_step.py $OUT/prof_L > $OUT/step_L.txt && cat $OUT/step_L.txt
