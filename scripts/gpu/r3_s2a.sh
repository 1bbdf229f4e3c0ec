#!/bin/bash
# Round 3 (session 2): rehearsal of the round-end commands on the restored tree, then the
# lane-walk row-order A/B (_C vs _C_rowo, interleaved in process).
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python scripts/ab_multi.py rowo 900000 8,16,32,50 uniform 12 > $O/ab_rowo.jsonl 2>> $O/err.log || { echo AB_FAIL; tail -20 $O/err.log; exit 1; }
cat $O/ab_rowo.jsonl
timeout -k 10 200 python scripts/ab_multi.py rowo 900000 16 blue,clustered 8 >> $O/ab_rowo.jsonl 2>> $O/err.log || { echo AB2_FAIL; tail -20 $O/err.log; exit 1; }
tail -2 $O/ab_rowo.jsonl
(cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --steps 30 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 ) || { echo PROF_FAIL; exit 1; }
echo done
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/ab_xsub.py 900000 8,16,32,50 uniform 10 1 2 > $O/ab_xsub.jsonl 2>> $O/err.log || { echo ABX_FAIL; tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python scripts/ab_xsub.py 900000 16,50 uniform 10 1 4 >> $O/ab_xsub.jsonl 2>> $O/err.log || { echo ABX4_FAIL; tail -20 $O/err.log; exit 1; }
cat $O/ab_xsub.jsonl
