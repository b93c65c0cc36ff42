#!/bin/bash
# k_front: the search's debug guesses / counts kept in LDS until the end (no global store before each barrier).
# Baseline "serialgrid": the previous build (global stores per iteration).
set -o pipefail
O=gpurun_out/r04al
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ndt_gpu.py > $O/tests.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind U > $O/front_U.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind L > $O/front_L.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind U --share 2 > $O/front_U_s2.txt 2>&1 && \
bash tools/ab_variants.sh r04al_U base serialgrid base serialgrid > $O/ab_U.txt 2>&1
