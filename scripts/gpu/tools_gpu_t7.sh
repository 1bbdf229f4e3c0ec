#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash scripts/bench_suite.sh > gpurun_out/suite.out 2>&1 || { echo SUITE_FAIL; tail -20 gpurun_out/suite.out; exit 1; }
python -c "
import json
for l in open('gpurun_out/bench_suite.jsonl'):
    d=json.loads(l); print(d['suite_label'][:48].ljust(48), round(d['ms_per_step'],4), '%.3g'%d['value'], d.get('ms_build'), d.get('ms_solve'), d.get('exact_path_queries'), d.get('check'))"
