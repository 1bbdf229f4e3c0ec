#!/bin/bash
# host API + kernel trace of the world-1 distributed pipeline, two query streams vs one (eager)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5disthip
S=/tmp/r5disthip
mkdir -p $O $S
(cd /tmp && KN_DIST_CAPTURE=0 KN_DIST_QSTREAMS=2 KN_DIST_SETS=2 KN_DIST_DEFER=0 MASTER_PORT=29671 timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace -d $S/q2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/q2.log 2>&1) || { echo PROF_FAIL; tail $O/q2.log; exit 1; }
timeout 300 python scripts/prof_hostgaps.py $S/q2/run_results.db 12 > $O/q2_gaps.txt 2>&1 || { echo ANALYSIS_FAIL; tail $O/q2_gaps.txt; exit 1; }
(cd /tmp && KN_DIST_CAPTURE=0 KN_DIST_QSTREAMS=1 MASTER_PORT=29672 timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace -d $S/q1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/q1.log 2>&1) || { echo PROF_FAIL; tail $O/q1.log; exit 1; }
timeout 300 python scripts/prof_hostgaps.py $S/q1/run_results.db 12 > $O/q1_gaps.txt 2>&1 || { echo ANALYSIS_FAIL; tail $O/q1_gaps.txt; exit 1; }
head -30 $O/q2_gaps.txt
