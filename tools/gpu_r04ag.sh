#!/bin/bash
# Chain kernel with threadIdx laundered per layer (95 instead of 125 VGPRs): pointnet GPU parity + bench A/B vs the old build.
set -o pipefail
O=gpurun_out/r04ag
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_model.py tests/test_pipeline_gpu.py > $O/tests.txt 2>&1 && \
bash tools/ab_variants.sh r04ag_U base notid base notid > $O/ab_U.txt 2>&1 && \
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_stamps.so timeout -k 10 120 python tools/pn_stamps.py > $O/stamps.txt 2>&1
