#!/bin/bash
# k_welford_q reciprocal table sized by the heavy threshold (2 KB): parity + bench A/B vs the 32 KB table.
set -o pipefail
O=gpurun_out/r04au
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ndt_gpu.py > $O/tests.txt 2>&1 && \
bash tools/ab_variants.sh r04au_U base rt4096 base rt4096 base rt4096 > $O/ab_U.txt 2>&1 && \
AB_ARGS="--kind L" bash tools/ab_variants.sh r04au_L base rt4096 base rt4096 > $O/ab_L.txt 2>&1
