#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5distprof3
mkdir -p $O
for q in 2; do export KN_DIST_SETS=2 KN_DIST_DEFER=0;
(cd /tmp && KN_DIST_QSTREAMS=$q KN_DIST_CAPTURE=0 MASTER_PORT=2965$q timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/q$q -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/q$q.log 2>&1) || { echo PROF_FAIL; tail $O/q$q.log; exit 1; }
python scripts/prof_steps.py $O/q$q/run_results.db 12
python - $O/q$q/run_results.db <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall() if 'queue_id' in [r[1] for r in c.execute("pragma table_info(kernels)")] else [(n,s,e,0) for n,s,e in c.execute("select name, start, end from kernels order by start")]
q = [i for i,(n,s,e,_) in enumerate(rows) if 'knn_tile_kernel' in n]
i0 = q[-12]
t0 = rows[i0][1]
for n,s,e,qid in rows[i0:i0+50]:
    print(f"{(s-t0)/1e3:9.1f} {(e-t0)/1e3:9.1f} {(e-s)/1e3:7.1f} q{qid} {n[:70]}")
PY
done
