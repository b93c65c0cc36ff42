#!/bin/bash
# round 4: C5 multiscale with 1 / 2 NDT streams, 2 / 3 forward streams
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04u
mkdir -p $OUT
AB_ARGS="--levels 2000,1000,500" bash tools/ab_env.sh r04u base n2:NDNET_PIPE_NDT_STREAMS=2 f2n2:NDNET_PIPE_FWD_STREAMS=2,NDNET_PIPE_NDT_STREAMS=2 base2 > $OUT/c5.txt 2>&1
rc=$?
cat $OUT/c5.txt
exit $rc
