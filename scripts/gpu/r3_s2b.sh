#!/bin/bash
# Round 3 (session 2): new defaults (x sub-cells for K <= 16, row order for K > 40, u16 cell
# boundaries): GPU tests, bounds-checked run, smoke, default bench, bench suite, kernel stats.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u scripts/diag_checked_r3.py > $O/checked.log 2>&1 || { echo CHECKED_FAIL; tail -20 $O/checked.log; exit 1; }
tail -2 $O/checked.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 900 bash scripts/bench_suite.sh > $O/suite.log 2>&1 || { echo SUITE_FAIL; tail -20 $O/suite.log; exit 1; }
cp gpurun_out/bench_suite.jsonl $O/
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --steps 30 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || { echo PROF_FAIL; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof50 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --k 50 --steps 20 > $GRAFT_REPO_ROOT/$O/prof50.log 2>&1) || { echo PROF50_FAIL; exit 1; }
echo done
timeout -k 10 300 python scripts/ab_multi.py ring 900000 8,16,32 uniform 12 > $O/ab_ring.jsonl 2>> $O/err.log || { echo ABR_FAIL; tail -20 $O/err.log; exit 1; }
cat $O/ab_ring.jsonl
for st in 0 1; do
  KN_HOST_STAGE=$st KN_ARENA_CACHE=$st timeout -k 10 200 ./bin/knn_cli --uniform 900000 --k 16 --api-bench 5 > $O/api16_stage$st.json 2>> $O/err.log || { echo API_FAIL; tail $O/err.log; exit 1; }
  echo "stage=$st $(cat $O/api16_stage$st.json)"
done
KN_LOG=DEBUG timeout -k 10 100 ./bin/knn_cli --uniform 900000 --k 16 --api-bench 2 > /dev/null 2> $O/api_phases.log || true
grep "host phases" $O/api_phases.log | tail -3
timeout -k 10 400 python scripts/ab_tree.py tfilt 900000 16,50 clustered,surface,uniform 6 > $O/ab_tfilt.jsonl 2>> $O/err.log || { echo ABT_FAIL; tail -20 $O/err.log; cat $O/ab_tfilt.jsonl; exit 1; }
cat $O/ab_tfilt.jsonl
