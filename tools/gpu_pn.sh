#!/bin/bash
# PointNet kernel iteration: model + pipeline GPU tests, chain stamps, bench.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_model.py tests/test_pipeline_gpu.py tests/test_training.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_pn.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_pn.log; exit 1; }
tail -2 $OUT/pytest_pn.log
NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_stamps.so timeout -k 10 120 python -u tools/pn_stamps.py > $OUT/stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'fwd', d['config_lines']['C3_forward_only']['ms_per_step'], 'ndt', d['config_lines']['C2_ndt_only']['ms_per_step'], 'chains', r['all_chains']['ms'], 'frac', r['frac'], 'other', r['all_chains']['forward_other_ms'])"
