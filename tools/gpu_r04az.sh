#!/bin/bash
# Chain kernel with layer functions force-inlined: weight prefetch two steps ahead (x6; d2) and three (fp32; d2d3) now
# compile without calls or scratch.  Model GPU parity of each variant, then bench A/B and chain stamps.
set -o pipefail
O=gpurun_out/r04az
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_model.py > $O/tests_base.txt 2>&1 && \
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_d2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_model.py > $O/tests_d2.txt 2>&1 && \
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_d2d3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_model.py > $O/tests_d2d3.txt 2>&1 && \
bash tools/ab_variants.sh r04az base d2 d2d3 base d2 d2d3 > $O/ab_U.txt 2>&1
