#!/bin/bash
# A/B of library variants on the NDT stage: C2 U (+ the L line) and C5 --
# clouds/s and the per-stage ms of each.  Usage: bash tools/ab_ndt.sh TAG base NAME ...
set -o pipefail
TAG=$1
shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
for V in "$@"; do
  if [ "$V" = base ]; then LIBV=""; else LIBV=$R/ndt-net_amd/lib/variants/libndnet_amd_$V.so; fi
  for CFG in c2 c5; do
    ARGS="--no-cpu-baseline --steps 30"
    [ $CFG = c5 ] && ARGS="$ARGS --levels 2000,1000,500"
    NDNET_AMD_LIB=$LIBV timeout -k 10 200 python bench.py $ARGS > $OUT/${V}_$CFG.log 2>&1 || { echo "$V $CFG failed"; tail -5 $OUT/${V}_$CFG.log; exit 1; }
    python3 - "$V $CFG" "$OUT/${V}_$CFG.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
o = d.get("other_distribution") or {}
st = {k.split(" ")[0]: v for k, v in d["stages_ms"].items()}
print(f"{sys.argv[1]:12s} {d['value']:9.1f} clouds/s {d['ms_per_step']:.4f} ms  L {o.get('value', '-')}  stages {st}")
PY
  done
done
