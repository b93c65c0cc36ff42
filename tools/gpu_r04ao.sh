#!/bin/bash
# k_welford_q heavy loop with the light items skipped (timing only): does the CU's other work slow the heavy waves?
set -o pipefail
O=gpurun_out/r04ao
mkdir -p $O
timeout -k 10 120 python tools/wq_items.py --kind L > $O/wq_L.txt 2>&1 && \
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_heavyonly.so timeout -k 10 120 python tools/wq_items.py --kind L > $O/wq_L_heavyonly.txt 2>&1
