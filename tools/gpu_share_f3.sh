#!/bin/bash
# NDT CU shares (front, welford) under 3 forward streams, C2 and C5, interleaved.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for r in 1 2; do
  for v in 2:1 1:1 2:2; do
    f=${v%%:*}; w=${v#*:}
    NDNET_PIPE_CU_SHARE=$f NDNET_PIPE_WQ_SHARE=$w timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-other --steps 60 --warmup 6 > $OUT/b_${f}_${w}_$r.log 2>&1 || { echo "bench $v failed"; tail -20 $OUT/b_${f}_${w}_$r.log; exit 1; }
    tail -1 $OUT/b_${f}_${w}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2 front $f welford $w', d['value'], d['ms_per_step'])"
    NDNET_PIPE_CU_SHARE=$f NDNET_PIPE_WQ_SHARE=$w timeout -k 10 200 python -u bench.py --no-cpu-baseline --levels 2000,1000,500 > $OUT/c5_${f}_${w}_$r.log 2>&1 || { echo "c5 $v failed"; tail -20 $OUT/c5_${f}_${w}_$r.log; exit 1; }
    tail -1 $OUT/c5_${f}_${w}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 front $f welford $w', d['value'], d['ms_per_step'])"
  done
done
