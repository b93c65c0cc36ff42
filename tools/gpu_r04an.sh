#!/bin/bash
# Pipeline: k_front share >= NDT streams (co-residency guard); pipeline GPU tests + the knob that failed before.
set -o pipefail
O=gpurun_out/r04an
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_pipeline_gpu.py > $O/tests.txt 2>&1 && \
AB_ARGS="--kind L" bash tools/ab_env.sh r04an_L n2:NDNET_PIPE_NDT_STREAMS=2 n2s1:NDNET_PIPE_NDT_STREAMS=2,NDNET_PIPE_CU_SHARE=1 n2s3:NDNET_PIPE_NDT_STREAMS=2,NDNET_PIPE_CU_SHARE=3 > $O/ab_L.txt 2>&1
