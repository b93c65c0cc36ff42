#!/bin/bash
# Labelled NDT path: parity tests, then the training-step timings.
set -o pipefail
TAG=${1:-lbl}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ndt_gpu.py tests/test_training.py -m gpu -x -v --timeout 200 --timeout-method thread -k "labelled or golden or fixture or adam or graphed" > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u tools/bench_train.py > $OUT/train_eager.log 2>&1 || { echo "eager train bench failed"; tail -20 $OUT/train_eager.log; exit 1; }
tail -1 $OUT/train_eager.log
timeout -k 10 200 python -u tools/bench_train.py --graph > $OUT/train_graph.log 2>&1 || { echo "graphed train bench failed"; tail -20 $OUT/train_graph.log; exit 1; }
tail -1 $OUT/train_graph.log
