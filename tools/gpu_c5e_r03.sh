#!/bin/bash
# C5 eager vs lazy retained lists (NDNET_PIPE_EAGER_LEVELS), pipeline tests,
# and the training-step timing (tools/bench_train.py).  Usage: bash tools/gpu_c5e_r03.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for e in 1 0; do
    NDNET_PIPE_EAGER_LEVELS=$e timeout -k 10 300 python -u bench.py --no-cpu-baseline --levels 2000,1000,500 > $OUT/bench_c5_e${e}_$r.log 2>&1 || { echo "bench c5 e$e failed"; tail -30 $OUT/bench_c5_e${e}_$r.log; exit 1; }
    tail -1 $OUT/bench_c5_e${e}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 eager=$e', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 python -u tools/bench_train.py > $OUT/train.log 2>&1 || { echo "bench_train failed"; tail -30 $OUT/train.log; exit 1; }
tail -1 $OUT/train.log
