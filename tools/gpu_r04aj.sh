#!/bin/bash
# k_front: where the first counted pass's set-up goes (mark 19 after thread 0's grid loop).
set -o pipefail
O=gpurun_out/r04aj
mkdir -p $O
timeout -k 10 120 python tools/front_phases.py --kind U > $O/front_U.txt 2>&1 && \
timeout -k 10 120 python tools/front_phases.py --kind L > $O/front_L.txt 2>&1
