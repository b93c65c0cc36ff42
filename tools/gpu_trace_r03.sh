#!/bin/bash
# Kernel traces of the pipelined bench: C2 (two steps) and C5 (two steps),
# plus per-kernel stats.  Usage: bash tools/gpu_trace_r03.sh TAG
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 $R/bench.py --no-cpu-baseline --no-other --steps 40 > $OUT/prof_c2.log 2>&1 || { echo "rocprof c2 failed"; tail -30 $OUT/prof_c2.log; exit 1; }
python3 $R/tools/trace_summary.py $OUT/prof_c2 --timeline --step 40 --span 2 > $OUT/timeline_c2.txt
python3 $R/tools/trace_summary.py $OUT/prof_c2 --skip 20 > $OUT/stats_c2.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 $R/bench.py --no-cpu-baseline --levels 2000,1000,500 --steps 30 > $OUT/prof_c5.log 2>&1 || { echo "rocprof c5 failed"; tail -30 $OUT/prof_c5.log; exit 1; }
python3 $R/tools/trace_summary.py $OUT/prof_c5 --timeline --step 30 --span 2 > $OUT/timeline_c5.txt
python3 $R/tools/trace_summary.py $OUT/prof_c5 --skip 20 > $OUT/stats_c5.txt
cat $OUT/timeline_c2.txt $OUT/timeline_c5.txt | head -150
