#!/bin/bash
# Co-residency probe: k_welford_q with 2 KB of reciprocal LDS (RT 256) and/or 128 VGPRs (waves_per_eu 4), U and L pipelined bench.
set -o pipefail
O=gpurun_out/r04at
mkdir -p $O
bash tools/ab_variants.sh r04at_U base wqrt wq128 base wqrt wq128 > $O/ab_U.txt 2>&1 && \
AB_ARGS="--kind L" bash tools/ab_variants.sh r04at_L base wqrt wq128 > $O/ab_L.txt 2>&1
