#!/bin/bash
# round 4: pipeline knobs after the welford / front changes (U and L)
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04o
mkdir -p $OUT
V="base share1:NDNET_PIPE_CU_SHARE=1 share4:NDNET_PIPE_CU_SHARE=4 wq2:NDNET_PIPE_WQ_SHARE=2 fwd2:NDNET_PIPE_FWD_STREAMS=2 ndt2:NDNET_PIPE_NDT_STREAMS=2 base2"
bash tools/ab_env.sh r04o_U $V > $OUT/U.txt 2>&1 && AB_ARGS="--kind L" bash tools/ab_env.sh r04o_L $V > $OUT/L.txt 2>&1
rc=$?
cat $OUT/U.txt; echo; cat $OUT/L.txt
exit $rc
