#!/bin/bash
# Round-3 end rehearsal on the final tree: the driver's commands (GPU tests, smoke, default bench),
# kernel stats of the default (pipelined) bench, the distributed path at world 1 for comparison.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/${END_DIR:-end3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 200 python bench.py --dist --steps 30 --warmup 5 > $O/bench_dist1.json 2> $O/bench_dist1.err || { echo DIST_FAIL; tail $O/bench_dist1.err; exit 1; }
timeout -k 10 300 python bench.py --dist --n 12500000 --steps 10 --warmup 3 > $O/bench_dist12m.json 2> $O/bench_dist12m.err || { echo DIST12_FAIL; tail $O/bench_dist12m.err; exit 1; }
tail -c 400 $O/bench_dist12m.json
tail -c 600 $O/bench_dist1.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --steps 30 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || { echo PROF_FAIL; exit 1; }
echo done
