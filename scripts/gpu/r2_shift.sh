#!/bin/bash
# A/B: shifted staging window at domain faces for the whole-block lane walk (K > 40).
set -o pipefail
R=$PWD
export PYTHONPATH=$R
mkdir -p gpurun_out/shift
for a in "--k 50" "--k 64" "--k 41" "--k 16" "--k 50 --gen clustered" "--k 50 --n 3000000"; do
  f=gpurun_out/shift/bench_$(echo $a | tr -d ' -').json
  timeout -k 10 180 python bench.py $a > $f 2> $f.err || { echo BENCH_FAIL $a; tail $f.err; exit 1; }
  python -c "import json; d=json.load(open('$f')); print('$a', round(d['ms_per_step'],4), d.get('ms_solve'), d.get('exact_path_queries'), d.get('check'))"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/shift/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/shift/pytest.log; exit 1; }
tail -2 gpurun_out/shift/pytest.log
