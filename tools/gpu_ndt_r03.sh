#!/bin/bash
# NDT-side iteration: the NDT GPU tests, then the default bench line (U, with
# the L line) and a C5 line.  Usage: bash tools/gpu_ndt_r03.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ndt_gpu.py tests/test_pipeline_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_ndt.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest_ndt.log; exit 1; }
tail -2 $OUT/pytest_ndt.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 60 --warmup 6 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('run', d['value'], d['ms_per_step'], 'L', d['other_distribution']['value'], 'fwd', d['config_lines']['C3_forward_only']['ms_per_step'], 'ndt', d['config_lines']['C2_ndt_only']['ms_per_step'], d['stages_ms'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --levels 2000,1000,500 > $OUT/bench_c5.log 2>&1 || { echo "bench c5 failed"; tail -30 $OUT/bench_c5.log; exit 1; }
tail -1 $OUT/bench_c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', d['value'], d['ms_per_step'], d['stages_ms'])"
