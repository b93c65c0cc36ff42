#!/bin/bash
# Round 4: heavy-loop ubench + k_welford_q PMC (where wave time goes) on L.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04f
mkdir -p $OUT
timeout -k 5 60 ./tools/ubench/fp64_latency > $OUT/fp64.txt 2>&1 || { echo "ubench failed"; tail $OUT/fp64.txt; exit 1; }
grep "hv_block\|phase1g" $OUT/fp64.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "counter list failed (ignored)"
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQ_INSTS_[A-Z_]*\|SQ_ACTIVE_INST_[A-Z_]*\|SQ_WAIT_INST_[A-Z_]*" $OUT/counters.txt | sort -u | tr '\n' ' '
echo
RUN="python3 $R/tools/wq_items.py --reps 2"
i=0
for grp in "SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_SCA" "SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_VMEM_RD,SQ_INSTS_BRANCH,SQ_WAVES,SQ_INSTS_VALU_FP64" "SQC_ICACHE_MISSES,SQC_ICACHE_HITS,GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- $RUN > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/pmc$i.log; }
done
echo "pmc done"
