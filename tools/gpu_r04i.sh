#!/bin/bash
# Round 4: the driver's default bench command (with C5 line, L split, CPU baseline).
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04i
mkdir -p $OUT
timeout -k 10 500 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['config_lines'])[:600]); print(d['other_distribution'])"
