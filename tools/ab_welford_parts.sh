set -o pipefail
R=$(pwd)
for V in ${VARIANTS:-base noload nochain nolc}; do
  if [ "$V" = base ]; then LIBV=""; else LIBV=$R/ndt-net_amd/lib/variants/libndnet_amd_$V.so; fi
  for CFG in ${CFGS:-c2 c5}; do
    ARGS="--no-cpu-baseline --steps 10 --no-other --no-pipeline"
    [ $CFG = c5 ] && ARGS="$ARGS --levels 2000,1000,500"
    [ $CFG = l ] && ARGS="$ARGS --kind L"
    NDNET_AMD_LIB=$LIBV timeout -k 10 200 python bench.py $ARGS > gpurun_out/wq_$V$CFG.log 2>&1 || { echo "$V failed"; tail -5 gpurun_out/wq_$V$CFG.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/wq_$V$CFG.log').read().strip().splitlines()[-1]); print('$V $CFG', {k.split(' ')[0]: v for k, v in d['stages_ms'].items()})"
  done
done
