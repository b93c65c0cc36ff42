#!/bin/bash
# Pipelined-step A/B of the NDT stage's CU share (PipelinedSegmentation,
# NDNET_PIPE_CU_SHARE), interleaved on one box, + the CU-share parity test.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ndt_gpu.py tests/test_pipeline_gpu.py -m gpu -k "cu_share or pipelined" -v --timeout 120 --timeout-method thread > $OUT/pytest_share.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_share.log; exit 1; }
tail -2 $OUT/pytest_share.log
for v in 1 2 1 2; do
  NDNET_PIPE_CU_SHARE=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-other --steps 50 --warmup 5 > $OUT/bench_s$v.log 2>&1 || { echo "bench share $v failed"; tail -20 $OUT/bench_s$v.log; exit 1; }
  tail -1 $OUT/bench_s$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('share $v', d['value'], d['ms_per_step'], 'ndt', d['config_lines']['C2_ndt_only']['ms_per_step'], 'fwd', d['config_lines']['C3_forward_only']['ms_per_step'])"
done
