#!/bin/bash
# Train-mode HIP kernels: parity tests, then the training step timed on the
# HIP blocks and on the torch composition (A/B), eager and graphed.
set -o pipefail
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_hip.py tests/test_training.py -m gpu > gpurun_out/train_hip_tests.log 2>&1 || { tail -40 gpurun_out/train_hip_tests.log; exit 1; }
tail -3 gpurun_out/train_hip_tests.log
timeout -k 10 120 python -u tools/bench_train.py --steps 20 --warmup 5 > gpurun_out/train_hip_bench.log 2>&1 || { tail -30 gpurun_out/train_hip_bench.log; exit 1; }
timeout -k 10 120 python -u tools/bench_train.py --steps 20 --warmup 5 --graph >> gpurun_out/train_hip_bench.log 2>&1 || { tail -30 gpurun_out/train_hip_bench.log; exit 1; }
NDNET_TRAIN_PATH=torch timeout -k 10 120 python -u tools/bench_train.py --steps 20 --warmup 5 >> gpurun_out/train_hip_bench.log 2>&1 || exit 1
NDNET_TRAIN_PATH=torch timeout -k 10 120 python -u tools/bench_train.py --steps 20 --warmup 5 --graph >> gpurun_out/train_hip_bench.log 2>&1 || exit 1
cat gpurun_out/train_hip_bench.log
