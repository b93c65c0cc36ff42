#!/bin/bash
# round 4: heavy-item wave priority in k_welford_q (s_setprio 3 vs 0) and the
# train split-K A/B (NDNET_TR_DW_PARTS 256 vs 32), alternated in one run
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04n
mkdir -p $OUT
V0=$R/ndt-net_amd/lib/variants/libndnet_amd_prio0.so
run() {
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ndt_gpu.py -m gpu \
    > $OUT/tests.txt 2>&1 || return 1
  for K in L U; do
    timeout -k 10 120 python -u tools/wq_items.py --kind $K > $OUT/items_${K}_prio3.txt 2>&1 || return 1
    NDNET_AMD_LIB=$V0 timeout -k 10 120 python -u tools/wq_items.py --kind $K > $OUT/items_${K}_prio0.txt 2>&1 || return 1
  done
  for rep in 1 2; do
    for K in L U; do
      timeout -k 10 200 python bench.py --kind $K --no-cpu-baseline --no-other --steps 50 > $OUT/bench_${K}_prio3_$rep.log 2>&1 || return 1
      NDNET_AMD_LIB=$V0 timeout -k 10 200 python bench.py --kind $K --no-cpu-baseline --no-other --steps 50 > $OUT/bench_${K}_prio0_$rep.log 2>&1 || return 1
    done
  done
  for rep in 1 2; do
    for P in 256 32; do
      NDNET_TR_DW_PARTS=$P timeout -k 10 300 python -u tools/bench_train.py --graph --steps 30 --warmup 5 > $OUT/train_parts${P}_$rep.txt 2>&1 || return 1
    done
  done
}
run; rc=$?
tail -2 $OUT/tests.txt
for f in $OUT/items_*; do echo "== $f"; head -1 $f; grep "cycles per sample" $f; done
for f in $OUT/bench_*.log; do tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $f)', d['value'], d['ms_per_step'], d.get('stages_ms',{}).get('welford + LU chains'))" 2>/dev/null; done
for f in $OUT/train_*.txt; do echo "$(basename $f) $(grep -o '"step_ms": [0-9.]*' $f)"; done
exit $rc
