#!/bin/bash
# Cache / latency PMC passes over the PointNet forward (tools/pn_forward.py):
# L2 hit/miss, memory-side reads, L1->L2 read latency, instruction-cache
# misses and the instruction mix.  Usage (repo root, GPU box): bash tools/pmc_cache.sh TAG
set -o pipefail
TAG=${1:-pmc_cache}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PN="python3 $R/tools/pn_forward.py --reps 3"
i=0
for grp in "TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_DRAM_sum" "TCP_TCC_READ_REQ_sum,TCP_TCC_READ_REQ_LATENCY_sum,TCP_PENDING_STALL_CYCLES_sum,TCP_TOTAL_CACHE_ACCESSES_sum" "SQC_ICACHE_MISSES,SQC_ICACHE_HITS,SQC_DCACHE_MISSES,SQC_DCACHE_HITS" "SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_MFMA,SQ_INSTS_SALU,SQ_INSTS_VALU,SQ_WAIT_INST_LDS,SQ_INSTS_SMEM,SQ_WAVES" "GRBM_GUI_ACTIVE,GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- $PN > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -20 $OUT/pmc$i.log; exit 1; }
done
cd $R && python3 tools/pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
