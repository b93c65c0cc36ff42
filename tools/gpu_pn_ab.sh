#!/bin/bash
# Chain stamps for A/B variants of the PointNet kernel (timing builds).
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for v in "$@"; do
  NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_$v.so timeout -k 10 120 python -u tools/pn_stamps.py > $OUT/stamps_$v.txt 2>&1 || { echo "stamps $v failed"; tail -20 $OUT/stamps_$v.txt; exit 1; }
  echo "=== $v"; grep -v amdgpu.ids $OUT/stamps_$v.txt
done
