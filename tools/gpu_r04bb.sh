#!/bin/bash
# C5 (three ND levels) pipeline with 1 vs 2 NDT streams.
set -o pipefail
O=gpurun_out/r04bb
mkdir -p $O
for V in n1:NDNET_PIPE_NDT_STREAMS=1 n2:NDNET_PIPE_NDT_STREAMS=2 n1:NDNET_PIPE_NDT_STREAMS=1 n2:NDNET_PIPE_NDT_STREAMS=2; do
  N=${V%%:*}; E=${V#*:}
  env $E timeout -k 10 200 python bench.py --levels 2000,1000,500 --no-cpu-baseline --steps 30 > $O/$N.log 2>&1 || { echo "$N failed"; tail -5 $O/$N.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/$N.log').read().strip().splitlines()[-1]); print('$N', d['value'], d['ms_per_step'])"
done
