#!/bin/bash
# k_front: bisection grid loop on wave 0's lanes -- NDT parity, phases, A/B vs the serial loop.
set -o pipefail
O=gpurun_out/r04ak
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ndt_gpu.py > $O/tests.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind U > $O/front_U.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind L > $O/front_L.txt 2>&1 && \
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_serialgrid.so timeout -k 10 120 python tools/front_phases.py --kind L > $O/front_L_serial.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind U --share 2 > $O/front_U_s2.txt 2>&1 && \
bash tools/ab_variants.sh r04ak_U base serialgrid base serialgrid > $O/ab_U.txt 2>&1
