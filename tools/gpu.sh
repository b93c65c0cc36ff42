#!/bin/bash
# The one GPU-box runner (replaces round 1-4's per-experiment gpu_*.sh /
# pmc*.sh / ab_*.sh recipes).  Every GPU step runs under its own time limit,
# steps are chained so the first failure (or time-out) ends the call, and all
# output goes under gpurun_out/TAG.  Run from the repo root on the GPU box:
#
#   bash tools/gpu.sh suite   TAG                 whole -m gpu suite + smoke + default bench
#                                                 + the 2-rank (gloo, one card) bench rehearsal
#   bash tools/gpu.sh tests   TAG [pytest args]   selected GPU tests (e.g. tests/test_model.py -k fp32)
#   bash tools/gpu.sh bench   TAG [bench args]    bench lines (args passed to bench.py)
#   bash tools/gpu.sh final   TAG                 driver command + C5 + L lines + pipelined / isolated stats
#   bash tools/gpu.sh ab      TAG NAME[:VAR=VAL,VAR=VAL] ...   env A/B on the bench (AB_ARGS: bench args)
#   bash tools/gpu.sh abfull  TAG NAME[:VAR=VAL,...] ...      the same with the L (other distribution) line
#   bash tools/gpu.sh variants TAG base NAME ...  library-variant A/B (tools/build_variant.sh NAME)
#   bash tools/gpu.sh trace   TAG [bench args]    isolated-step kernel trace (one graph per step) + summary
#   bash tools/gpu.sh pmc     TAG ndt|pn|chain|cache|issue|lds  PMC passes, one counter group per run
#                                                 (NDNET_AMD_LIB=<variant .so> runs a library variant)
#   bash tools/gpu.sh train   TAG                 train-path tests + the eager / graphed train step
#   bash tools/gpu.sh stamps  TAG                 per-layer chain stamps (variant "stamps")
#   bash tools/gpu.sh py      TAG tool.py [args]  a python tool under a time limit (output kept)
set -o pipefail
CMD=${1:?command}
TAG=${2:?tag}
shift 2
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"

step() {  # step NAME SECONDS LOG cmd...: runs cmd under a time limit, stops the call on failure
  local name=$1 secs=$2 log=$3
  shift 3
  timeout -k 10 $secs "$@" > $log 2>&1 || { echo "$name failed rc=$?"; tail -30 $log; exit 1; }
}

line() {  # the bench line's headline fields
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
st = {k.split(" ")[0]: v for k, v in (d.get("stages_ms") or {}).items()}
cl = {k: v.get("value") for k, v in (d.get("config_lines") or {}).items()}
o = d.get("other_distribution") or {}
ol = f"  L {o.get('value', 0):.1f} stages {o.get('stages_ms')}" if o else ""
print(f"{sys.argv[1]:12s} {d['value']:10.1f} {d['unit']}  {d['ms_per_step']:.4f} ms/step  "
      f"frac {r.get('frac')}  chains {r.get('all_chains', {}).get('ms')}  stages {st}  {cl}{ol}")
PY
}

pmc_passes() {  # pmc_passes DIR "cmd" group...
  local dir=$1 cmd=$2 i=0
  shift 2
  cd /tmp && export TMPDIR=/tmp
  for grp in "$@"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $dir/pmc$i -o run -- $cmd > $dir/pmc$i.log 2>&1 \
      || { echo "pmc pass $i ($grp) failed"; tail -20 $dir/pmc$i.log; exit 1; }
  done
  cd $R && python3 tools/pmc_summary.py $dir > $dir/summary.txt 2>&1 && cat $dir/summary.txt
}

SQ_BUSY="SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS"
SQ_MIX="SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INST_CYCLES_VMEM,SQ_ACTIVE_INST_VALU"
GRBM="GRBM_GUI_ACTIVE,GRBM_COUNT"

case $CMD in
suite)
  step pytest 700 $OUT/pytest_gpu.log $PYT tests -m gpu
  tail -2 $OUT/pytest_gpu.log
  step smoke 200 $OUT/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
  tail -1 $OUT/smoke.log
  step bench 300 $OUT/bench.log python -u bench.py
  line bench $OUT/bench.log
  step bench2 400 $OUT/bench_2ranks.log python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 \
    --no-cpu-baseline
  tail -1 $OUT/bench_2ranks.log | cut -c1-300
  ;;
tests)
  step pytest 900 $OUT/pytest.log $PYT -m gpu "$@"
  tail -3 $OUT/pytest.log
  ;;
bench)
  step bench 400 $OUT/bench.log python -u bench.py "$@"
  tail -1 $OUT/bench.log | cut -c1-600
  ;;
final)
  step bench 400 $OUT/bench.log python -u bench.py --gpus 1 --steps 20 --warmup 5
  line driver $OUT/bench.log
  step c5 300 $OUT/c5.log python -u bench.py --levels 2000,1000,500 --no-cpu-baseline
  line C5 $OUT/c5.log
  step L 300 $OUT/l.log python -u bench.py --kind L --no-cpu-baseline --no-other
  line L $OUT/l.log
  cd /tmp && export TMPDIR=/tmp
  step prof_pipe 300 $OUT/prof_pipe.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pipe -o run \
    -- python3 $R/bench.py --no-cpu-baseline --steps 200
  step prof_iso 300 $OUT/prof_iso.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_iso -o run \
    -- python3 $R/bench.py --no-cpu-baseline --no-pipeline --steps 200
  ;;
ab)
  for A in "$@"; do
    V=${A%%:*}
    ENVS=""
    [ "$V" != "$A" ] && ENVS=${A#*:}
    step $V 200 $OUT/$V.log env ${ENVS//,/ } python bench.py --no-cpu-baseline --no-other --steps 50 ${AB_ARGS}
    line $V $OUT/$V.log
  done
  ;;
abfull)  # as ab, with the other distribution's line (the two-NDT-stream L pipeline) in the run
  for A in "$@"; do
    V=${A%%:*}
    ENVS=""
    [ "$V" != "$A" ] && ENVS=${A#*:}
    step $V 300 $OUT/$V.log env ${ENVS//,/ } python bench.py --no-cpu-baseline --steps 100 ${AB_ARGS}
    line $V $OUT/$V.log
  done
  ;;
variants)
  for V in "$@"; do
    LIBV=""
    [ "$V" != base ] && LIBV=$R/ndt-net_amd/lib/variants/libndnet_amd_$V.so
    step $V 200 $OUT/$V.log env NDNET_AMD_LIB=$LIBV python bench.py --no-cpu-baseline --no-other --steps 50 ${AB_ARGS}
    line $V $OUT/$V.log
  done
  ;;
trace)
  cd /tmp && export TMPDIR=/tmp
  step trace 300 $OUT/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python3 $R/bench.py --no-pipeline --no-cpu-baseline --no-other "$@"
  tail -1 $OUT/prof.log | cut -c1-300
  python3 $R/tools/trace_summary.py $OUT/prof --skip 3 | head -30
  ;;
pmc)
  KIND=${1:?ndt|pn|chain|cache|issue}
  case $KIND in
  ndt)  # U dispatches only (the L split would mix L clouds in)
    pmc_passes $OUT "python3 $R/bench.py --eager --steps 3 --warmup 1 --no-cpu-baseline --no-other" \
      FETCH_SIZE WRITE_SIZE $SQ_BUSY $GRBM ;;
  pn)
    pmc_passes $OUT "python3 $R/tools/pn_forward.py --reps 3" $SQ_BUSY $SQ_MIX FETCH_SIZE WRITE_SIZE $GRBM ;;
  chain)
    pmc_passes $OUT "python3 $R/tools/pn_forward.py --reps 3" $SQ_MIX $SQ_BUSY \
      "SQ_INSTS_MFMA,SQ_ACTIVE_INST_MISC,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_INSTS_SMEM,SQ_ACTIVE_INST_SCA,SQ_INST_LEVEL_LDS,SQ_INSTS_BRANCH" $GRBM ;;
  cache)
    pmc_passes $OUT "python3 $R/tools/pn_forward.py --reps 3" "TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_DRAM_sum" \
      "TCP_TCC_READ_REQ_sum,TCP_TCC_READ_REQ_LATENCY_sum,TCP_PENDING_STALL_CYCLES_sum,TCP_TOTAL_CACHE_ACCESSES_sum" $GRBM ;;
  issue)
    for K in U L; do
      mkdir -p $OUT/$K
      pmc_passes $OUT/$K "python3 $R/bench.py --eager --kind $K --steps 3 --warmup 1 --no-cpu-baseline --no-other" \
        "SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES"
    done ;;
  kl)  # the KL stage's kernels on L clouds (k_kl_rank_chunks, k_kl_sort / k_kl_merge): issue mix, LDS, waits
    pmc_passes $OUT "python3 $R/tools/sort_marks.py --kind L" $SQ_MIX \
      "SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES" \
      $SQ_BUSY $GRBM ;;
  lds)  # the chains' LDS instruction mix and bank conflicts only (one pass)
    pmc_passes $OUT "python3 $R/tools/pn_forward.py --reps 3" $SQ_MIX ;;
  *) echo "unknown pmc kind $KIND"; exit 2 ;;
  esac
  ;;
train)
  step pytest 400 $OUT/pytest.log $PYT tests/test_train_hip.py tests/test_training.py -m gpu
  tail -3 $OUT/pytest.log
  step eager 200 $OUT/train_eager.log python -u tools/bench_train.py --steps 20 --warmup 5
  tail -1 $OUT/train_eager.log
  step graph 200 $OUT/train_graph.log python -u tools/bench_train.py --steps 20 --warmup 5 --graph
  tail -1 $OUT/train_graph.log
  ;;
trtrace)  # kernel trace of the graphed train step + per-kernel summary
  cd /tmp && export TMPDIR=/tmp
  step trtrace 300 $OUT/trprof.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trprof -o run \
    -- python3 $R/tools/bench_train.py --steps 10 --warmup 3 --graph
  tail -1 $OUT/trprof.log | cut -c1-300
  cd $R && python3 tools/trace_summary.py $OUT/trprof > $OUT/trprof_summary.txt && head -60 $OUT/trprof_summary.txt
  ;;
py)  # a python tool (e.g. tools/wq_items.py --kind L), output to gpurun_out/TAG/<tool>.txt
  NAME=$(basename ${1%.py})
  step $NAME 300 $OUT/$NAME.txt python -u "$@"
  cat $OUT/$NAME.txt
  ;;
stamps)
  export NDNET_AMD_LIB=$R/ndt-net_amd/lib/variants/libndnet_amd_stamps.so
  step warm 120 $OUT/stamps_warm.txt python -u tools/pn_stamps.py
  cat $OUT/stamps_warm.txt
  step cold 120 $OUT/stamps_cold.txt python -u tools/pn_stamps.py --cold
  cat $OUT/stamps_cold.txt
  ;;
*)
  echo "unknown command $CMD"
  exit 2
  ;;
esac
