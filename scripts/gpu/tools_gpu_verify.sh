#!/bin/bash
# GPU tests + headline and K=50/K=64 benches (after a plan/kernel default change)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/verify_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/verify_tests.log; exit 1; }
tail -1 gpurun_out/verify_tests.log
: > gpurun_out/verify_bench.jsonl
for k in 16 50 64; do
  timeout -k 10 200 python bench.py --n 900000 --k $k --steps 30 --warmup 5 > gpurun_out/_v.json 2> gpurun_out/verify_bench.err || { echo BENCH_FAIL $k; tail gpurun_out/verify_bench.err; exit 1; }
  tail -1 gpurun_out/_v.json >> gpurun_out/verify_bench.jsonl
done
python -c "
import json
for l in open('gpurun_out/verify_bench.jsonl'):
    d=json.loads(l); print(d['config']['model'], round(d['ms_per_step'],4), '%.3g'%d['value'], d['ms_build'], d['ms_solve'], d['exact_path_queries'], d['check'])"
