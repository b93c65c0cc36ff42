#!/bin/bash
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04e
mkdir -p $OUT
for T in 1 256 100000; do
timeout -k 10 120 python -u tools/wq_items.py --heavy $T > $OUT/wq_L_$T.txt 2>&1 || { echo "wq_items failed"; tail -30 $OUT/wq_L_$T.txt; exit 1; }
echo "== L heavy $T"; grep -v amdgpu.ids $OUT/wq_L_$T.txt | tail -6
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_U -o run -- python3 $R/bench.py --kind U --no-pipeline --no-cpu-baseline --no-other --steps 10 > $OUT/prof_U.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_U.log; exit 1; }
python3 $R/tools/trace_kernels.py $OUT/prof_U k_welford k_lu
