#!/bin/bash
# The bench line's chain timing against rocprofv3: the default bench line, then
# kernel traces + stats of the isolated (--no-pipeline) and the default command.
set -o pipefail
TAG=${1:-chainprof}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_iso -o run -- python3 $R/bench.py --no-pipeline --no-cpu-baseline --no-other > $OUT/prof_iso.log 2>&1 || { echo "rocprof iso failed"; tail -20 $OUT/prof_iso.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_def -o run -- python3 $R/bench.py > $OUT/prof_def.log 2>&1 || { echo "rocprof default failed"; tail -20 $OUT/prof_def.log; exit 1; }
tail -1 $OUT/prof_def.log | cut -c1-200
python3 $R/tools/chain_prof_check.py $OUT/prof_iso $OUT/prof_def $OUT/bench.log
