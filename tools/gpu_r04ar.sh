#!/bin/bash
# k_front pass keys: byte map marked with a plain store (no read-before-write round trip per point). Parity, phases, A/B.
set -o pipefail
O=gpurun_out/r04ar
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ndt_gpu.py > $O/tests.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind U > $O/front_U.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind L > $O/front_L.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind U --share 2 > $O/front_U_s2.txt 2>&1 && \
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_bmread.so timeout -k 10 120 python tools/front_phases.py --kind U --share 2 > $O/front_U_s2_bmread.txt 2>&1 && \
bash tools/ab_variants.sh r04ar_U base bmread base bmread > $O/ab_U.txt 2>&1
