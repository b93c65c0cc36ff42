#!/bin/bash
# (forward streams, NDT streams) = (3, 1) vs (2, 2): C2 U + L line, interleaved.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for r in 1 2; do
  for v in 3:1 2:2; do
    f=${v%%:*}; n=${v#*:}
    NDNET_PIPE_FWD_STREAMS=$f NDNET_PIPE_NDT_STREAMS=$n timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 60 --warmup 6 > $OUT/b_${f}_${n}_$r.log 2>&1 || { echo "bench $v failed"; tail -20 $OUT/b_${f}_${n}_$r.log; exit 1; }
    tail -1 $OUT/b_${f}_${n}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fwd $f ndt $n', d['value'], d['ms_per_step'], 'L', d['other_distribution']['value'])"
  done
done
