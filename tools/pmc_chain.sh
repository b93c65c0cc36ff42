#!/bin/bash
# Instruction-mix and LDS-conflict counters of the PointNet forward's kernels
# (tools/pn_forward.py), one rocprofv3 --pmc pass per group.
# Usage (repo root, GPU box): bash tools/pmc_chain.sh TAG
set -o pipefail
TAG=${1:-pmc_chain}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PN="python3 $R/tools/pn_forward.py --reps 3"
i=0
for grp in "SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INST_CYCLES_VMEM,SQ_ACTIVE_INST_VALU" "SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS" "SQ_INSTS_MFMA,SQ_ACTIVE_INST_MISC,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_INSTS_SMEM,SQ_ACTIVE_INST_SCA,SQ_INST_LEVEL_LDS,SQ_INSTS_BRANCH" "GRBM_GUI_ACTIVE,GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- $PN > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -20 $OUT/pmc$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
echo "pmc done"
