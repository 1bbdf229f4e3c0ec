#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5prof
mkdir -p $O
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/p20 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/p20.log 2>&1) || { echo PROF_FAIL; exit 1; }
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/p200 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --steps 200 --warmup 50 > $GRAFT_REPO_ROOT/$O/p200.log 2>&1) || { echo PROF_FAIL; exit 1; }
python scripts/prof_steps.py $(ls $O/p20/*/run_results.db 2>/dev/null || ls $O/p20/run_results.db) 28
python scripts/prof_steps.py $(ls $O/p200/*/run_results.db 2>/dev/null || ls $O/p200/run_results.db) 12
python scripts/prof_db.py $(ls $O/p20/*/run_results.db 2>/dev/null || ls $O/p20/run_results.db) | head -14
