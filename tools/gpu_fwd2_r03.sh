#!/bin/bash
# Forward streams 1 vs 2 (NDNET_PIPE_FWD_STREAMS): pipeline + model tests,
# then interleaved bench lines (C2 U with L, and C5).  Usage: bash tools/gpu_fwd2_r03.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py tests/test_model.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for f in 1 2; do
    NDNET_PIPE_FWD_STREAMS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 60 --warmup 6 > $OUT/bench_f${f}_$r.log 2>&1 || { echo "bench f$f failed"; tail -30 $OUT/bench_f${f}_$r.log; exit 1; }
    tail -1 $OUT/bench_f${f}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('F=$f', d['value'], d['ms_per_step'], 'L', d['other_distribution']['value'])"
  done
done
for f in 1 2; do
  NDNET_PIPE_FWD_STREAMS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --levels 2000,1000,500 > $OUT/bench_c5_f$f.log 2>&1 || { echo "bench c5 f$f failed"; tail -30 $OUT/bench_c5_f$f.log; exit 1; }
  tail -1 $OUT/bench_c5_f$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 F=$f', d['value'], d['ms_per_step'])"
done
