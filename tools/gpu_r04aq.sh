#!/bin/bash
# k_welford_q heavy loop: next group's LDS reads issued before this group's steps (asm ordering). Parity, items, bench A/B.
set -o pipefail
O=gpurun_out/r04aq
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ndt_gpu.py > $O/tests.txt 2>&1 && \
timeout -k 10 120 python tools/wq_items.py --kind L > $O/wq_L.txt 2>&1 && \
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_noorder.so timeout -k 10 120 python tools/wq_items.py --kind L > $O/wq_L_noorder.txt 2>&1 && \
AB_ARGS="--kind L" bash tools/ab_variants.sh r04aq_L base noorder base noorder > $O/ab_L.txt 2>&1 && \
bash tools/ab_variants.sh r04aq_U base noorder > $O/ab_U.txt 2>&1
