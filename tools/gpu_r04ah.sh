#!/bin/bash
# k_front rank loop with LDS match slots: NDT parity, phase stamps (G = 16 and the pipeline's share 2), bench A/B.
set -o pipefail
O=gpurun_out/r04ah
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ndt_gpu.py tests/test_pipeline_gpu.py > $O/tests.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind U > $O/front_U.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind L > $O/front_L.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind U --share 2 > $O/front_U_s2.txt 2>&1 && \
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_nomatch.so timeout -k 10 120 python tools/front_phases.py --kind U --share 2 > $O/front_U_s2_nomatch.txt 2>&1 && \
bash tools/ab_variants.sh r04ah_U base nomatch base nomatch > $O/ab_U.txt 2>&1
