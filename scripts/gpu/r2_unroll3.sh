#!/bin/bash
# K=50 bucket with unroll 1: GPU suite + benches.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/unroll3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for a in "--k 16" "--k 8" "--k 32" "--k 16" "--k 50"; do
  f=$O/b_$(echo $a | tr -d ' -').json
  timeout -k 10 180 python bench.py $a > $f 2> $f.err || { echo BENCH_FAIL $a; tail $f.err; exit 1; }
  python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$a', round(d['ms_per_step'],4), d['exact_path_queries'], d['check'])"
done
