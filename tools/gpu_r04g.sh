#!/bin/bash
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04g
mkdir -p $OUT
timeout -k 5 60 ./tools/ubench/lu_chain > $OUT/lu.txt 2>&1 || { echo "lu ubench failed"; cat $OUT/lu.txt; exit 1; }
cat $OUT/lu.txt
PYTEST_K="${PYTEST_K}" bash tools/gpu_r04b.sh
