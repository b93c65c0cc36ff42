#!/bin/bash
# k_front phase stamps at the pipeline's CU share 2 (G = 8 workgroups per cloud, 13 bins each).
set -o pipefail
O=gpurun_out/r04af
mkdir -p $O
timeout -k 10 120 python tools/front_phases.py --kind U --share 2 > $O/front_U_s2.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind L --share 2 > $O/front_L_s2.txt 2>&1
