#!/bin/bash
# Per-layer chain stamps (warm and L2-cold) from the -DNDNET_PN_STAMPS build.
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
export NDNET_AMD_LIB=$PWD/ndt-net_amd/lib/variants/libndnet_amd_stamps.so
timeout -k 10 120 python -u tools/pn_stamps.py > $OUT/stamps_warm.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/stamps_warm.txt; exit 1; }
cat $OUT/stamps_warm.txt
timeout -k 10 120 python -u tools/pn_stamps.py --cold > $OUT/stamps_cold.txt 2>&1 || { echo "stamps cold failed"; tail -20 $OUT/stamps_cold.txt; exit 1; }
cat $OUT/stamps_cold.txt
unset NDNET_AMD_LIB
timeout -k 10 200 python -u -m pytest tests/test_pipeline_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_pipe.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_pipe.log; exit 1; }
tail -3 $OUT/pytest_pipe.log
