#!/bin/bash
# A/B of library variants (tools/build_variant.sh) on the default bench:
# clouds/s, ms per step and the four chain kernels' ms for each.
# Usage (repo root, GPU box): bash tools/ab_variants.sh TAG base NAME1 NAME2 ...
set -o pipefail
TAG=$1
shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
for V in "$@"; do
  if [ "$V" = base ]; then LIBV=""; else LIBV=$R/ndt-net_amd/lib/variants/libndnet_amd_$V.so; fi
  NDNET_AMD_LIB=$LIBV timeout -k 10 150 python bench.py --no-cpu-baseline --no-other --steps 50 ${AB_ARGS} > $OUT/$V.log 2>&1 || { echo "$V failed"; tail -5 $OUT/$V.log; exit 1; }
  python3 - "$V" "$OUT/$V.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:10s} {d['value']:10.1f} clouds/s {d['ms_per_step']:.4f} ms  chains {r['all_chains']['ms']}  fwd {d['stages_ms'].get('pointnet_fwd')}")
PY
done
