#!/bin/bash
# GPU suite + steady-step A/B (route_steady / fused global ids / counters) + bin-thread A/B with
# solve times + kernel trace of the distributed step.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/steady
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for t in 256 1024 256 1024; do
  KN_BIN_THREADS=$t timeout -k 10 120 python bench.py --no-check > $O/b_$t.json 2> $O/b_$t.err || { echo FAIL $t; tail $O/b_$t.err; exit 1; }
  echo "threads $t $(python -c "import json;d=json.load(open('$O/b_$t.json'));print(d['ms_per_step'], d['ms_build'], d['ms_solve'])")"
done
for i in 1 2; do
  timeout -k 10 180 python bench.py --dist > $O/dist_$i.json 2> $O/dist_$i.err || { echo DIST_FAIL; tail $O/dist_$i.err; exit 1; }
  cut -c1-200 $O/dist_$i.json; grep -o '"check": {[^}]*}' $O/dist_$i.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_dist -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 20 > $GRAFT_REPO_ROOT/$O/prof_dist.log 2>&1 || { echo PROF_FAIL; tail $GRAFT_REPO_ROOT/$O/prof_dist.log; exit 1; }
echo done
