#!/bin/bash
# The multi-rank bench path on one card: 2 ranks (torchrun, gloo collectives, both on cuda:0).
set -o pipefail
O=gpurun_out/r04av
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --no-cpu-baseline > $O/bench2.log 2>&1
rc=$?
tail -3 $O/bench2.log | cut -c1-400
exit $rc
