#!/bin/bash
# Pipeline knob re-check after the round-4 kernel changes (U, then L with 2 NDT streams).
set -o pipefail
O=gpurun_out/r04am
mkdir -p $O
bash tools/ab_env.sh r04am_U base wq2:NDNET_PIPE_WQ_SHARE=2 share1:NDNET_PIPE_CU_SHARE=1 share3:NDNET_PIPE_CU_SHARE=3 base > $O/ab_U.txt 2>&1 && \
AB_ARGS="--kind L" bash tools/ab_env.sh r04am_L n2:NDNET_PIPE_NDT_STREAMS=2 n2wq2:NDNET_PIPE_NDT_STREAMS=2,NDNET_PIPE_WQ_SHARE=2 n2s3:NDNET_PIPE_NDT_STREAMS=2,NDNET_PIPE_CU_SHARE=3 n2:NDNET_PIPE_NDT_STREAMS=2 > $O/ab_L.txt 2>&1
