#!/bin/bash
# Round-4 end rehearsal on the final tree: the driver's commands (GPU tests, smoke, the bench at
# the driver's 20 / 5 steps), every BASELINE configuration (scripts/bench_suite.sh), kernel stats
# of the headline and of the distributed step at world 1.
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${END_DIR:-end4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 2400 bash scripts/bench_suite.sh > $O/suite.log 2>&1 || { echo SUITE_FAIL; tail -20 $O/suite.log; exit 1; }
cp gpurun_out/bench_suite.jsonl $O/bench_suite.jsonl
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || { echo PROF_FAIL; exit 1; }
(cd /tmp && MASTER_PORT=$((29500 + RANDOM % 300)) timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_dist -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof_dist.log 2>&1) || { echo PROF_DIST_FAIL; exit 1; }
echo done
