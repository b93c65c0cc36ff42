#!/bin/bash
# round 4: k_front phase cuts (byte-map reads batched, rank-loop LDS reads
# ahead, both ND blocks' counts in one round trip, point-ND lookups batched):
# the bit-exact NDT suite, phase stamps, isolated kernel traces, bench lines
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04l
mkdir -p $OUT
run() {
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ndt_gpu.py \
    tests/test_pipeline_gpu.py -m gpu > $OUT/tests.txt 2>&1 || return 1
  for K in U L; do
    timeout -k 10 120 python -u tools/front_phases.py --kind $K > $OUT/front_$K.txt 2>&1 || return 1
    NDNET_FRONT_BINMARKS=1 NDNET_AMD_LIB=$R/ndt-net_amd/lib/variants/libndnet_amd_binmarks.so \
      timeout -k 10 120 python -u tools/front_phases.py --kind $K > $OUT/front_bin_$K.txt 2>&1 || return 1
  done
  (cd /tmp && export TMPDIR=/tmp && for K in U L; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$K -o run -- python3 $R/bench.py --kind $K --no-pipeline --no-cpu-baseline --no-other --steps 10 > $OUT/prof_$K.log 2>&1 || exit 1
    python3 $R/tools/trace_kernels.py $OUT/prof_$K > $OUT/kernels_$K.txt || exit 1
  done) || return 1
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_train -o run -- python3 $R/tools/bench_train.py --graph --steps 20 --warmup 5 > $OUT/prof_train.log 2>&1) || return 1
  cp $OUT/prof_train/run_kernel_stats.csv $OUT/train_kernel_stats.csv 2>/dev/null || cp $(ls $OUT/prof_train/*kernel_stats.csv | head -1) $OUT/train_kernel_stats.csv
  for K in U L; do
    timeout -k 10 200 python bench.py --kind $K --no-cpu-baseline --no-other --steps 50 > $OUT/bench_$K.log 2>&1 || return 1
  done
}
run; rc=$?
tail -3 $OUT/tests.txt; cat $OUT/front_*.txt $OUT/kernels_*.txt 2>/dev/null
for K in U L; do tail -1 $OUT/bench_$K.log 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$K', d['value'], d['ms_per_step'], d.get('stages_ms'))" 2>/dev/null; done
rm -rf $OUT/prof_U $OUT/prof_L $OUT/prof_train
exit $rc
