#!/bin/bash
# NDT streams 1 vs 2 (NDNET_PIPE_NDT_STREAMS): pipeline tests, then C2 (U + L line) and C5, interleaved.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for n in 1 2; do
    NDNET_PIPE_NDT_STREAMS=$n timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 60 --warmup 6 > $OUT/b_${n}_$r.log 2>&1 || { echo "bench n$n failed"; tail -20 $OUT/b_${n}_$r.log; exit 1; }
    tail -1 $OUT/b_${n}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2 ndt streams $n', d['value'], d['ms_per_step'], 'L', d['other_distribution']['value'], d['other_distribution']['ms_per_step'])"
    NDNET_PIPE_NDT_STREAMS=$n timeout -k 10 200 python -u bench.py --no-cpu-baseline --levels 2000,1000,500 > $OUT/c5_${n}_$r.log 2>&1 || { echo "c5 n$n failed"; tail -20 $OUT/c5_${n}_$r.log; exit 1; }
    tail -1 $OUT/c5_${n}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 ndt streams $n', d['value'], d['ms_per_step'])"
  done
done
