#!/bin/bash
# k_welford_q heavy loop: (rc, rl) scalar-load latency probe (timing-only variant with block 0's table rows).
set -o pipefail
mkdir -p gpurun_out/r04ad
timeout -k 10 120 python tools/wq_items.py --kind L > gpurun_out/r04ad/wq_L.txt 2>&1 && \
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_fixrt.so timeout -k 10 120 python tools/wq_items.py --kind L > gpurun_out/r04ad/wq_L_fixrt.txt 2>&1
