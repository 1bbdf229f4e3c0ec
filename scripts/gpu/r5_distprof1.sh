#!/bin/bash
# rocprof timelines of the world-1 distributed pipeline, one query stream, eager vs graph stages
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5distprof1
mkdir -p $O
for cap in 0 1; do
(cd /tmp && KN_DIST_CAPTURE=$cap MASTER_PORT=2966$cap timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c$cap -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 60 --warmup 10 > $GRAFT_REPO_ROOT/$O/c$cap.log 2>&1) || { echo PROF_FAIL; tail $O/c$cap.log; exit 1; }
echo "== capture $cap"; tail -1 $O/c$cap.log | cut -c1-200
python scripts/prof_steps.py $O/c$cap/run_results.db 20
python - $O/c$cap/run_results.db <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
q = [i for i,(n,s,e,_) in enumerate(rows) if 'knn_tile_kernel' in n]
i0 = q[-8]
t0 = rows[i0][1]
for n,s,e,qid in rows[i0:i0+36]:
    print(f"{(s-t0)/1e3:9.1f} {(e-t0)/1e3:9.1f} {(e-s)/1e3:7.1f} q{qid} {n[:60]}")
PY
done
