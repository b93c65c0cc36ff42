#!/bin/bash
# u16 rank-bin histograms in k_front: NDT + pipeline GPU tests, then C2 / C5 bench lines.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ndt_gpu.py tests/test_pipeline_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 60 --warmup 6 > $OUT/b_$r.log 2>&1 || { echo "bench failed"; tail -20 $OUT/b_$r.log; exit 1; }
  tail -1 $OUT/b_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['value'], d['ms_per_step'], 'L', d['other_distribution']['value'], d['stages_ms'])"
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --levels 2000,1000,500 > $OUT/c5_$r.log 2>&1 || { echo "c5 failed"; tail -20 $OUT/c5_$r.log; exit 1; }
  tail -1 $OUT/c5_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', d['value'], d['ms_per_step'], d['stages_ms'])"
done
