#!/bin/bash
# Round 3 final tree: the driver's round-end commands (GPU tests, smoke, default bench).
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
tail -c 500 $O/bench.json
echo done
