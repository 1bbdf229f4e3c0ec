#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "in_cell_order or uniform_tile" > gpurun_out/pytest_t5.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_t5.log; exit 1; }
tail -1 gpurun_out/pytest_t5.log
timeout -k 10 400 python scripts/sweep_tiles.py 900000 16 2.5,3.1,3.5 4x4x4,4x4x5,4x4x3,5x4x4,5x5x4,4x5x5,5x5x5,3x4x4,8x4x4,4x8x4 > gpurun_out/sweep2.log 2>&1 || { echo SWEEP_FAIL; tail gpurun_out/sweep2.log; exit 1; }
sort -t: -k8 gpurun_out/sweep2.log | grep -v BEST | python -c "
import sys, json
rows=[json.loads(l) for l in sys.stdin if l.startswith('{')]
rows.sort(key=lambda r: r['ms'])
for r in rows[:12]: print(r)"
for d in "" "--deterministic"; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 $d > gpurun_out/_b.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/_b.json').read().strip().splitlines()[-1]); print('det' if d['in_cell_sort'] else 'nondet', d['ms_per_step'], d['ms_build'], d['ms_solve'], d['check'])"
done
