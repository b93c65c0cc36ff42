#!/bin/bash
# MFMA ceiling microbenchmark + PMC passes over the PointNet forward only
# (tools/pn_forward.py).  Usage (repo root, GPU box): bash tools/pmc_pn.sh TAG
set -o pipefail
TAG=${1:-pmc_pn}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 60 ./tools/ubench/mfma_peak > $OUT/mfma_peak.txt 2>&1 || { echo "mfma_peak failed"; cat $OUT/mfma_peak.txt; exit 1; }
cat $OUT/mfma_peak.txt
cd /tmp && export TMPDIR=/tmp
PN="python3 $R/tools/pn_forward.py --reps 3"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $PN > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
i=0
for grp in "SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS" "SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INST_CYCLES_VMEM,SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "GRBM_GUI_ACTIVE,GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- $PN > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -20 $OUT/pmc$i.log; exit 1; }
done
echo "pmc done"
