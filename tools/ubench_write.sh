#!/bin/bash
# WRITE_SIZE / FETCH_SIZE calibration of k_front's scatter store patterns
# (tools/ubench/write_width.hip), one counter per rocprofv3 pass.
# Usage (repo root, GPU box; the binary built in-tree beforehand):
#   bash tools/ubench_write.sh TAG
set -o pipefail
TAG=${1:-wwidth}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 60 $R/tools/ubench/write_width > $OUT/time.txt 2>&1 || { echo "write_width failed"; cat $OUT/time.txt; exit 1; }
cat $OUT/time.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc1 -o run -- $R/tools/ubench/write_width > $OUT/pmc1.log 2>&1 || { echo "pmc WRITE_SIZE failed"; tail -20 $OUT/pmc1.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc2 -o run -- $R/tools/ubench/write_width > $OUT/pmc2.log 2>&1 || { echo "pmc FETCH_SIZE failed"; tail -20 $OUT/pmc2.log; exit 1; }
cd $R && python3 tools/pmc_summary.py $OUT | tee $OUT/summary.txt
