#!/bin/bash
# Pipeline tests first, then the rest of the GPU suite, smoke, two default
# bench lines, chain stamps and a C5 line.  Usage: bash tools/gpu_pipe_r03.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_pipe.log 2>&1 || { echo "pipeline tests failed rc=$?"; tail -40 $OUT/pytest_pipe.log; exit 1; }
tail -2 $OUT/pytest_pipe.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --deselect tests/test_pipeline_gpu.py > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for u in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 60 --warmup 6 > $OUT/bench_$u.log 2>&1 || { echo "bench $u failed"; tail -30 $OUT/bench_$u.log; exit 1; }
  tail -1 $OUT/bench_$u.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('run', d['value'], d['ms_per_step'], 'L', d['other_distribution']['value'], 'fwd', d['config_lines']['C3_forward_only']['ms_per_step'], 'ndt', d['config_lines']['C2_ndt_only']['ms_per_step'])"
done
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_stamps.so timeout -k 10 120 python -u tools/pn_stamps.py > $OUT/stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/stamps.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --levels 2000,1000,500 > $OUT/bench_c5.log 2>&1 || { echo "bench c5 failed"; tail -30 $OUT/bench_c5.log; exit 1; }
tail -1 $OUT/bench_c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', d['value'], d['ms_per_step'])"
