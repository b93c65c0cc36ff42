#!/bin/bash
# round 4: bench line with the L other-distribution on two NDT streams + settle
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04t
mkdir -p $OUT
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py > $OUT/bench_$rep.log 2>&1 || { tail -20 $OUT/bench_$rep.log; exit 1; }
  tail -1 $OUT/bench_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['other_distribution'])"
done
