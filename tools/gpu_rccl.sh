#!/bin/bash
# Training-path checks on one card: test_training's GPU tests (the one-rank
# nccl DDP step, the graphed train step), the eager and graphed train-step
# timings, then (last, allowed to fail) the bench's two-rank path over nccl.
set -o pipefail
TAG=${1:-rccl}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_training.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python -u tools/bench_train.py > $OUT/train_eager.log 2>&1 || { echo "eager train bench failed"; tail -20 $OUT/train_eager.log; exit 1; }
tail -1 $OUT/train_eager.log
timeout -k 10 200 python -u tools/bench_train.py --graph > $OUT/train_graph.log 2>&1 || { echo "graphed train bench failed"; tail -20 $OUT/train_graph.log; exit 1; }
tail -1 $OUT/train_graph.log
timeout -k 10 180 python -u bench.py --gpus 2 --dist-backend nccl --steps 20 --warmup 5 --no-cpu-baseline --no-other > $OUT/bench_2ranks_nccl.log 2>&1
echo "2-rank nccl rc=$?"
tail -5 $OUT/bench_2ranks_nccl.log | cut -c1-400
