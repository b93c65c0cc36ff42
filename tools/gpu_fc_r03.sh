#!/bin/bash
# FC-chain + forward-streams check: model / pipeline / training GPU tests,
# then interleaved bench lines: NDNET_PN_FC=chain (default) vs =mfma, and
# NDNET_PIPE_FWD_STREAMS=2.  Usage: bash tools/gpu_fc_r03.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_model.py tests/test_pipeline_gpu.py tests/test_training.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for v in "NDNET_PN_FC=chain" "NDNET_PN_FC=mfma" "NDNET_PIPE_FWD_STREAMS=2"; do
    n=${v//=/_}
    env $v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-other --steps 60 --warmup 6 > $OUT/bench_${n}_$r.log 2>&1 || { echo "bench $v failed"; tail -30 $OUT/bench_${n}_$r.log; exit 1; }
    tail -1 $OUT/bench_${n}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], 'fwd', d['config_lines']['C3_forward_only']['ms_per_step'], 'chains', d['roofline']['all_chains']['ms'], 'other', d['roofline']['all_chains']['forward_other_ms'])"
  done
done
