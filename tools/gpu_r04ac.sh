#!/bin/bash
# k_welford_q per-item placement (HW_ID / XCC) on L and U.
set -o pipefail
mkdir -p gpurun_out/r04ac
timeout -k 10 120 python tools/wq_items.py --kind L > gpurun_out/r04ac/wq_L.txt 2>&1 && \
timeout -k 10 120 python tools/wq_items.py --kind U > gpurun_out/r04ac/wq_U.txt 2>&1
