#!/bin/bash
# k_welford_q heavy loop with (rc, rl) from an LDS row: parity (NDT GPU tests), per-item timing, bench A/B vs the scalar-load loop.
set -o pipefail
O=gpurun_out/r04ae
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ndt_gpu.py > $O/tests.txt 2>&1 && \
timeout -k 10 120 python tools/wq_items.py --kind L > $O/wq_L.txt 2>&1 && \
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_srt.so timeout -k 10 120 python tools/wq_items.py --kind L > $O/wq_L_srt.txt 2>&1 && \
AB_ARGS="--kind L" bash tools/ab_variants.sh r04ae_L base srt base srt > $O/ab_L.txt 2>&1 && \
bash tools/ab_variants.sh r04ae_U base srt base srt > $O/ab_U.txt 2>&1
