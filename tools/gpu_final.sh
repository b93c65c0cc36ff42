#!/bin/bash
# End-of-session check: the driver's bench command, C5 and L bench lines, and
# the rocprofv3 kernel stats of the default (pipelined) and isolated benches.
# Usage: bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 python -u bench.py --levels 2000,1000,500 --no-cpu-baseline > $OUT/c5.log 2>&1 || { echo "c5 failed"; tail -20 $OUT/c5.log; exit 1; }
tail -1 $OUT/c5.log | cut -c1-200
timeout -k 10 300 python -u bench.py --kind L --no-cpu-baseline --no-other > $OUT/l.log 2>&1 || { echo "L failed"; tail -20 $OUT/l.log; exit 1; }
tail -1 $OUT/l.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pipe -o run -- python3 $R/bench.py --no-cpu-baseline --steps 200 > $OUT/prof_pipe.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_pipe.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_iso -o run -- python3 $R/bench.py --no-cpu-baseline --no-pipeline --steps 200 > $OUT/prof_iso.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_iso.log; exit 1; }
echo done
