#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5distprof
mkdir -p $O
for q in 1 2; do
(cd /tmp && KN_DIST_QSTREAMS=$q KN_DIST_CAPTURE=0 MASTER_PORT=2965$q timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/q$q -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/q$q.log 2>&1) || { echo PROF_FAIL; tail $O/q$q.log; exit 1; }
python scripts/prof_steps.py $O/q$q/run_results.db 14
python scripts/prof_db.py $O/q$q/run_results.db --timeline 40 | tail -42 | cut -c1-120
done
