#!/bin/bash
# Round 2, session 4 re-entry check: GPU tests, headline bench, K=50/64, clustered, dist world 1.
set -o pipefail
R=$PWD
export PYTHONPATH=$R
mkdir -p gpurun_out/s4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/s4/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/s4/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/s4/pytest_gpu.log
for a in "--k 16" "--k 50" "--k 64" "--gen clustered" "--dist" "--dist --k 50"; do
  f=gpurun_out/s4/bench_$(echo $a | tr -d ' -').json
  timeout -k 10 180 python bench.py $a > $f 2> $f.err || { echo BENCH_FAIL $a; tail $f.err; exit 1; }
  cut -c1-300 $f
done
