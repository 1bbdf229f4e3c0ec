#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
: > gpurun_out/adapt2.jsonl
for g in clustered surface uniform; do
  timeout -k 10 300 python bench.py --gen $g --n 900000 --k 16 --steps 10 --warmup 2 > gpurun_out/_a.json 2> gpurun_out/adapt.err || { echo BENCH_FAIL $g; tail -5 gpurun_out/adapt.err; exit 1; }
  tail -1 gpurun_out/_a.json >> gpurun_out/adapt2.jsonl
done
timeout -k 10 300 python bench.py --gen clustered --n 900000 --k 16 --steps 5 --warmup 1 --fixed-grid > gpurun_out/_a.json 2> gpurun_out/adapt.err || { echo BENCH_FAIL fixed; tail -5 gpurun_out/adapt.err; exit 1; }
tail -1 gpurun_out/_a.json >> gpurun_out/adapt2.jsonl
python -c "
import json
for l in open('gpurun_out/adapt2.jsonl'):
    d=json.loads(l); print(d['data'][:20], round(d['ms_per_step'],3), d['ms_build'], d['ms_solve'], d.get('grid'), d.get('exact_path_queries'), d['check'])"
