#!/bin/bash
# Full GPU suite + smoke + the driver's bench (round-5 state).
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-r5full}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 200 python bench.py --dist --steps 20 --warmup 5 > $O/bench_dist.json 2> $O/bench_dist.err || { echo DIST_BENCH_FAIL; tail $O/bench_dist.err; exit 1; }
cat $O/bench_dist.json
