#!/bin/bash
# Round 4: where k_welford_q's light quads spend their time (timing-only variants, wrong results).
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04h
mkdir -p $OUT
for V in base noload norecip both; do
  if [ $V = base ]; then unset NDNET_AMD_LIB; else export NDNET_AMD_LIB=$R/ndt-net_amd/lib/variants/libndnet_amd_$V.so; fi
  timeout -k 10 120 python -u tools/wq_items.py --kind U > $OUT/wq_U_$V.txt 2>&1 || { echo "wq_items $V failed"; tail -20 $OUT/wq_U_$V.txt; exit 1; }
  echo "== U $V"; grep "light items\|span" $OUT/wq_U_$V.txt
done
