#!/bin/bash
# Heavy NDs listed by descending count (a cloud's longest NDs share workgroups): parity, welford tail, L/U bench A/B.
set -o pipefail
O=gpurun_out/r04ax
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ndt_gpu.py > $O/tests.txt 2>&1 && \
timeout -k 10 120 python tools/wq_items.py --kind L > $O/wq_L.txt 2>&1 && \
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_nosort.so timeout -k 10 120 python tools/wq_items.py --kind L > $O/wq_L_nosort.txt 2>&1 && \
AB_ARGS="--kind L" bash tools/ab_variants.sh r04ax_L base nosort base nosort base nosort > $O/ab_L.txt 2>&1 && \
bash tools/ab_variants.sh r04ax_U base nosort > $O/ab_U.txt 2>&1
