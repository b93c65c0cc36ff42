#!/bin/bash
# Pipelined-step A/B of NDT CU shares (variant libs), interleaved in one box:
# base (k_front on every CU) vs share2 (k_front G = CUs / 2B, k_welford_q on half the CUs).
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for v in base share2 base share2; do
  NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-other --steps 50 --warmup 5 > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 $OUT/bench_$v.log; exit 1; }
  tail -1 $OUT/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], 'ndt', d['config_lines']['C2_ndt_only']['ms_per_step'], 'fwd', d['config_lines']['C3_forward_only']['ms_per_step'], d['stages_ms'])"
done
