#!/bin/bash
# A/B of library variants: model tests on the main build, chain stamps of
# stamps_<v> variants, interleaved bench lines of the main build and <v>.
# Usage: bash tools/gpu_ab_r03.sh TAG VARIANT
set -o pipefail
OUT=gpurun_out/$1; V=$2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_model.py tests/test_pipeline_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for s in stamps stamps_$V; do
  NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_$s.so timeout -k 10 120 python -u tools/pn_stamps.py > $OUT/$s.txt 2>&1 || { echo "stamps $s failed"; tail -20 $OUT/$s.txt; exit 1; }
  echo "=== $s"; grep "launch span\|layer\|input tile" $OUT/$s.txt
done
for r in 1 2; do
  for lib in main $V; do
    if [ $lib = main ]; then L=""; else L="NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_$lib.so"; fi
    env $L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-other --steps 60 --warmup 6 > $OUT/bench_${lib}_$r.log 2>&1 || { echo "bench $lib failed"; tail -30 $OUT/bench_${lib}_$r.log; exit 1; }
    tail -1 $OUT/bench_${lib}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], 'fwd', d['config_lines']['C3_forward_only']['ms_per_step'], 'chains', d['roofline']['all_chains']['ms'])"
  done
done
