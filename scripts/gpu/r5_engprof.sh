#!/bin/bash
# rocprof step periods of the engine pipeline: one vs two query streams (900K K=16, 60 / 10)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5engprof
mkdir -p $O
for q in 1 2; do
(cd /tmp && KN_PIPE_QSTREAMS=$q timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/q$q -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --steps 60 --warmup 10 > $GRAFT_REPO_ROOT/$O/q$q.log 2>&1) || { echo PROF_FAIL; tail $O/q$q.log; exit 1; }
echo "== qstreams $q"
python scripts/prof_steps.py $O/q$q/run_results.db 20 | tail -3
python - $O/q$q/run_results.db <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
q = [i for i,(n,s,e,_) in enumerate(rows) if 'knn_tile_kernel' in n]
i0 = q[-8]
t0 = rows[i0][1]
for n,s,e,qid in rows[i0:i0+24]:
    print(f"{(s-t0)/1e3:9.1f} {(e-t0)/1e3:9.1f} {(e-s)/1e3:7.1f} q{qid} {n[:60]}")
PY
done
