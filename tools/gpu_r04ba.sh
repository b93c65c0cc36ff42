#!/bin/bash
# k_welford_q heavy threshold (samples for a whole wave): 192 / 256 (default) / 384, L then U.
set -o pipefail
O=gpurun_out/r04ba
mkdir -p $O
AB_ARGS="--kind L" bash tools/ab_variants.sh r04ba_L base h192 h384 base h192 h384 > $O/ab_L.txt 2>&1 && \
bash tools/ab_variants.sh r04ba_U base h192 h384 > $O/ab_U.txt 2>&1
