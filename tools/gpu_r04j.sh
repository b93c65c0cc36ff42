#!/bin/bash
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04j
mkdir -p $OUT
timeout -k 10 600 python -u tools/capture_probe.py > $OUT/probe.txt 2>&1; rc=$?
cat $OUT/probe.txt
exit $rc
