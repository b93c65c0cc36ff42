#!/bin/bash
# round 4: the in-place re-fold (ndnet_pn_fold_run) and the train forward vs
# the reference's out_train fixture, the training bench's re-fold stage,
# k_front phase stamps (U / L, plus the binning sub-marks build), then the
# multi-step capture probe (last: a crashing mode may take its child down)
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04k
mkdir -p $OUT
run() {
  timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_model.py tests/test_train_hip.py tests/test_pipeline_gpu.py tests/test_training.py \
    -m gpu -k "refold or mode_switch or fixture or keeps_captured or graphed or labelled or train_hip" > $OUT/tests.txt 2>&1 || return 1
  timeout -k 10 300 python -u tools/bench_train.py --steps 20 --warmup 5 > $OUT/train.txt 2>&1 || return 1
  timeout -k 10 300 python -u tools/bench_train.py --graph --steps 20 --warmup 5 >> $OUT/train.txt 2>&1 || return 1
  NDNET_TR_BN1024=1 timeout -k 10 300 python -u tools/bench_train.py --graph --steps 20 --warmup 5 > $OUT/train_bn1024.txt 2>&1 || return 1
  NDNET_TR_BN1024=1 timeout -k 10 300 python -u -m pytest -x -q \
    --timeout 120 --timeout-method thread tests/test_train_hip.py -m gpu > $OUT/tests_bn1024.txt 2>&1 || return 1
  bash tools/ab_env.sh r04k_prio base fwd:NDNET_PIPE_PRIORITY=fwd ndt:NDNET_PIPE_PRIORITY=ndt > $OUT/prio.txt 2>&1 || return 1
  for K in U L; do
    timeout -k 10 120 python -u tools/front_phases.py --kind $K > $OUT/front_$K.txt 2>&1 || return 1
    NDNET_FRONT_BINMARKS=1 NDNET_AMD_LIB=$R/ndt-net_amd/lib/variants/libndnet_amd_binmarks.so \
      timeout -k 10 120 python -u tools/front_phases.py --kind $K > $OUT/front_bin_$K.txt 2>&1 || return 1
  done
}
run; rc=$?
tail -25 $OUT/tests.txt; cat $OUT/train.txt $OUT/train_bn1024.txt; tail -3 $OUT/tests_bn1024.txt; cat $OUT/prio.txt; cat $OUT/front_*.txt 2>/dev/null
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/capture_probe.py > $OUT/probe.txt 2>&1; rc=$?
cat $OUT/probe.txt
exit $rc
