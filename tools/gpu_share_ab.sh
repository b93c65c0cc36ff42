#!/bin/bash
# Pipelined-step A/B of the NDT stage's CU shares (PipelinedSegmentation:
# NDNET_PIPE_CU_SHARE for k_front, NDNET_PIPE_WQ_SHARE for k_welford_q),
# interleaved on one box, + the CU-share parity test.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ndt_gpu.py tests/test_pipeline_gpu.py tests/test_model.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_share.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_share.log; exit 1; }
tail -2 $OUT/pytest_share.log
for v in 2:2 2:1 2:4 2:2 2:1 2:4; do
  f=${v%%:*}; w=${v#*:}
  NDNET_PIPE_CU_SHARE=$f NDNET_PIPE_WQ_SHARE=$w timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-other --steps 50 --warmup 5 > $OUT/bench_s${f}_${w}.log 2>&1 || { echo "bench share $v failed"; tail -20 $OUT/bench_s${f}_${w}.log; exit 1; }
  tail -1 $OUT/bench_s${f}_${w}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('share front $f welford $w', d['value'], d['ms_per_step'], 'ndt', d['config_lines']['C2_ndt_only']['ms_per_step'], 'fwd', d['config_lines']['C3_forward_only']['ms_per_step'])"
done
