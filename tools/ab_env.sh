#!/bin/bash
# A/B of environment settings on the default bench (clouds/s, ms per step,
# the four chain kernels' ms).  Each argument is NAME or NAME:VAR=VAL,VAR=VAL.
# Usage (repo root, GPU box): bash tools/ab_env.sh TAG base x6n:NDNET_PN_X6_NARROW=1 ...
set -o pipefail
TAG=$1
shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
for A in "$@"; do
  V=${A%%:*}
  ENVS=""
  [ "$V" != "$A" ] && ENVS=${A#*:}
  env ${ENVS//,/ } timeout -k 10 150 python bench.py --no-cpu-baseline --no-other --steps 50 ${AB_ARGS} > $OUT/$V.log 2>&1 || { echo "$V failed"; tail -5 $OUT/$V.log; exit 1; }
  python3 - "$V" "$OUT/$V.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:10s} {d['value']:10.1f} clouds/s {d['ms_per_step']:.4f} ms  chains {r['all_chains']['ms']}  fwd {d['stages_ms'].get('pointnet_fwd')}")
PY
done
