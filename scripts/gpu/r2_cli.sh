#!/bin/bash
# GPU suite (query ranges, lazy outputs) + smoke + headline bench.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/cli
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 120 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
cut -c1-250 $O/bench.json
