#!/bin/bash
# Round 4: NDT parity + per-item welford timing + L/U bench lines with the stage split.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ndt_gpu.py -x -q --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -u tools/wq_items.py > $OUT/wq_L.txt 2>&1 || { echo "wq_items failed"; tail -30 $OUT/wq_L.txt; exit 1; }
grep -v amdgpu.ids $OUT/wq_L.txt | tail -7
timeout -k 10 120 python -u tools/wq_items.py --kind U > $OUT/wq_U.txt 2>&1 || { echo "wq_items failed"; tail -30 $OUT/wq_U.txt; exit 1; }
grep -v amdgpu.ids $OUT/wq_U.txt | tail -5
timeout -k 10 300 python -u bench.py --kind L --no-cpu-baseline --no-other > $OUT/bench_L.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_L.log; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench_L.log').read().strip().splitlines()[-1]);print('L', d['value'], d['ms_per_step'], d['stages_ms'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-other > $OUT/bench_U.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_U.log; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench_U.log').read().strip().splitlines()[-1]);print('U', d['value'], d['ms_per_step'], d['stages_ms'])"
