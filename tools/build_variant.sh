#!/bin/bash
# Builds an A/B variant of lib/libndnet_amd.so with extra compile flags into
# lib/variants/libndnet_amd_NAME.so (select it with NDNET_AMD_LIB=...).
#   bash tools/build_variant.sh NAME "-DFLAG ..." ["pointnet-only flags"]
set -e
NAME=$1
FLAGS=$2
PNFLAGS=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/ndt-net_amd
mkdir -p $P/build/v_$NAME $P/lib/variants
C="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -Wno-unused-variable"
/opt/rocm/bin/hipcc $C -ffp-contract=off -fno-fast-math $FLAGS -c -o $P/build/v_$NAME/ndt_kernels.o $P/csrc/ndt_kernels.hip &
/opt/rocm/bin/hipcc $C $FLAGS $PNFLAGS -c -o $P/build/v_$NAME/pointnet_kernels.o $P/csrc/pointnet_kernels.hip &
/opt/rocm/bin/hipcc $C $FLAGS -c -o $P/build/v_$NAME/train_kernels.o $P/csrc/train_kernels.hip &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/lib/variants/libndnet_amd_$NAME.so \
  $P/build/v_$NAME/ndt_kernels.o $P/build/ndt_legacy_abi.o $P/build/v_$NAME/pointnet_kernels.o $P/build/pointnet_chain_t32.o $P/build/ply_ingest.o $P/build/v_$NAME/train_kernels.o -lpthread
echo "built $P/lib/variants/libndnet_amd_$NAME.so"
