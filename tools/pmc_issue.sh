#!/bin/bash
# Issue-side PMC pass (instruction mix and per-unit active cycles) for the NDT kernels, U and L eager runs.
# Usage (repo root, GPU box): bash tools/pmc_issue.sh TAG
set -o pipefail
TAG=${1:-pmci}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
GRP="SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES"
for K in U L; do
  mkdir -p $OUT/$K
  timeout -s KILL 120 rocprofv3 --pmc $GRP --output-format csv -d $OUT/$K/pmc1 -o run -- python3 $R/bench.py --eager --kind $K --steps 3 --warmup 1 --no-cpu-baseline --no-other > $OUT/$K/pmc1.log 2>&1 || { echo "pmc $K failed"; tail -20 $OUT/$K/pmc1.log; exit 1; }
  python3 $R/tools/pmc_summary.py $OUT/$K > $OUT/summary_$K.txt 2>&1 || { echo "summary $K failed"; tail -5 $OUT/summary_$K.txt; exit 1; }
done
echo "pmc issue done"
