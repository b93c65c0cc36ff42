#!/bin/bash
# round 4: k_front staged scatter re-enabled at CU share 1 (LDS reserved for its records)
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04aa
mkdir -p $OUT
run() {
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ndt_gpu.py tests/test_pipeline_gpu.py -m gpu > $OUT/tests.txt 2>&1 || return 1
  for K in U L; do
    timeout -k 10 120 python -u tools/front_phases.py --kind $K > $OUT/front_$K.txt 2>&1 || return 1
  done
  (cd /tmp && export TMPDIR=/tmp && for K in U L; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$K -o run -- python3 $R/bench.py --kind $K --no-pipeline --no-cpu-baseline --no-other --steps 10 > $OUT/prof_$K.log 2>&1 || exit 1
    python3 $R/tools/trace_by_grid.py $OUT/prof_$K k_front k_welford > $OUT/kernels_$K.txt || exit 1
  done) || return 1
  timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || return 1
}
run; rc=$?
tail -2 $OUT/tests.txt; grep -v amdgpu $OUT/front_*.txt | grep -E "last end|scattered|offsets  "; cat $OUT/kernels_*.txt
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['stages_ms'], d['config_lines']['C2_ndt_only'], d['other_distribution']['value'])"
rm -rf $OUT/prof_U $OUT/prof_L
exit $rc
