#!/bin/bash
# C5 level-1 KL kernels of library variants: one isolated step's kernel times.
# Usage: bash tools/gpu_c5_trace_ab.sh TAG base NAME ...
set -o pipefail
TAG=$1
shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for V in "$@"; do
  if [ "$V" = base ]; then LIBV=""; else LIBV=$R/ndt-net_amd/lib/variants/libndnet_amd_$V.so; fi
  NDNET_AMD_LIB=$LIBV timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$V -o run -- python3 $R/bench.py --levels 2000,1000,500 --no-cpu-baseline --no-pipeline --steps 5 > $OUT/prof_$V.log 2>&1 || { echo "rocprof $V failed"; tail -20 $OUT/prof_$V.log; exit 1; }
  echo "== $V"
  (cd $R && python3 tools/trace_step.py $OUT/prof_$V k_front | grep -E "k_kl|k_welford|k_front")
done
