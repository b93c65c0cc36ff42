#!/bin/bash
# round 4: NDT streams x forward streams x hardware queues (U and L)
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04p
mkdir -p $OUT
V="base f2n2:NDNET_PIPE_FWD_STREAMS=2,NDNET_PIPE_NDT_STREAMS=2 q8:GPU_MAX_HW_QUEUES=8 q8n2:GPU_MAX_HW_QUEUES=8,NDNET_PIPE_NDT_STREAMS=2 q8f4n2:GPU_MAX_HW_QUEUES=8,NDNET_PIPE_FWD_STREAMS=4,NDNET_PIPE_NDT_STREAMS=2 base2"
bash tools/ab_env.sh r04p_U $V > $OUT/U.txt 2>&1 && AB_ARGS="--kind L" bash tools/ab_env.sh r04p_L $V > $OUT/L.txt 2>&1
rc=$?
cat $OUT/U.txt; echo; cat $OUT/L.txt
exit $rc
