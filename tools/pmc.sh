#!/bin/bash
# PMC passes over a short eager bench run (one counter group per run, as
# MI355X_MICROARCH.md's rocprofv3 section prescribes), plus k_front's phase
# stamps.  Usage (repo root, on the GPU box): bash tools/pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 python -u tools/front_phases.py > $OUT/front_U.txt 2>&1 || { echo "front_phases U failed"; tail -20 $OUT/front_U.txt; exit 1; }
timeout -k 10 120 python -u tools/front_phases.py --kind L > $OUT/front_L.txt 2>&1 || { echo "front_phases L failed"; tail -20 $OUT/front_L.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --eager --steps 3 --warmup 1 --no-cpu-baseline --no-other"  # U dispatches only (the L split would mix L clouds in)
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "counter list failed (ignored)"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS" "GRBM_GUI_ACTIVE,GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- $BENCH > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -20 $OUT/pmc$i.log; exit 1; }
done
echo "pmc done"
