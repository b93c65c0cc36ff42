#!/bin/bash
# 32-point chain tiles everywhere (NDNET_PN_TILE32=force: 8-wave workgroups, two per CU) vs auto, C2 and C5.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 env NDNET_PN_TILE32=force python -u -m pytest tests/test_model.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for t in 1 force; do
    NDNET_PN_TILE32=$t timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-other --steps 60 --warmup 6 > $OUT/b_${t}_$r.log 2>&1 || { echo "bench $t failed"; tail -20 $OUT/b_${t}_$r.log; exit 1; }
    tail -1 $OUT/b_${t}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2 t32=$t', d['value'], d['ms_per_step'], 'fwd', d['config_lines']['C3_forward_only']['ms_per_step'], 'chains', d['roofline']['all_chains']['ms'])"
  done
done
for t in 1 force; do
  NDNET_PN_TILE32=$t timeout -k 10 200 python -u bench.py --no-cpu-baseline --levels 2000,1000,500 > $OUT/c5_$t.log 2>&1 || { echo "c5 $t failed"; tail -20 $OUT/c5_$t.log; exit 1; }
  tail -1 $OUT/c5_$t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 t32=$t', d['value'], d['ms_per_step'])"
done
