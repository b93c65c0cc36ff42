#!/bin/bash
# Forward streams 2 vs 3, C2 and C5, plus the driver's bench command.  Usage: bash tools/gpu_f3_r03.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for r in 1 2; do
  for f in 2 3; do
    NDNET_PIPE_FWD_STREAMS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-other --steps 60 --warmup 6 > $OUT/bench_f${f}_$r.log 2>&1 || { echo "bench f$f failed"; tail -30 $OUT/bench_f${f}_$r.log; exit 1; }
    tail -1 $OUT/bench_f${f}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('F=$f', d['value'], d['ms_per_step'])"
    NDNET_PIPE_FWD_STREAMS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --levels 2000,1000,500 > $OUT/bench_c5_f${f}_$r.log 2>&1 || { echo "bench c5 f$f failed"; tail -30 $OUT/bench_c5_f${f}_$r.log; exit 1; }
    tail -1 $OUT/bench_c5_f${f}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 F=$f', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { echo "driver bench failed"; tail -30 $OUT/bench_driver.log; exit 1; }
tail -1 $OUT/bench_driver.log | cut -c1-400
