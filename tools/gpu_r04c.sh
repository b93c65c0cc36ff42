#!/bin/bash
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04c
mkdir -p $OUT
for T in 256; do
timeout -k 10 120 python -u tools/wq_items.py --heavy $T > $OUT/wq_L_$T.txt 2>&1 || { echo "wq_items failed"; tail -30 $OUT/wq_L_$T.txt; exit 1; }
echo "== L heavy $T"; cat $OUT/wq_L_$T.txt
done
