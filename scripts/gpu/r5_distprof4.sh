#!/bin/bash
# world-1 distributed pipeline timeline, final defaults (coverage of query kernels, side-stream load)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5distprof4
mkdir -p $O
(cd /tmp && MASTER_PORT=29671 timeout -k 10 240 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/t -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 80 --warmup 10 > $GRAFT_REPO_ROOT/$O/t.log 2>&1) || { echo PROF_FAIL; tail $O/t.log; exit 1; }
python - $O/t/run_results.db <<'PY'
import sqlite3, sys
import numpy as np
from collections import defaultdict
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
tiles = [r for r in rows if 'knn_tile' in r[0]]
tiles = tiles[-60:-2]
t0, t1 = tiles[0][1], tiles[-1][1]
ev = []
for n, s, e, q in rows:
    if 'knn_tile' in n and s < t1 and e > t0:
        ev.append((max(s, t0), 1)); ev.append((min(e, t1), -1))
ev.sort()
cur = 0; last = t0; cov = {0: 0, 1: 0, 2: 0}
for t, d in ev:
    cov[min(cur, 2)] += t - last
    cur += d; last = t
tot = t1 - t0
print(f"window {tot/1e3:.1f} us over {len(tiles)-1} steps: {tot/1e3/(len(tiles)-1):.1f} us/step")
for k in (0, 1, 2):
    print(f"  {k} tile kernels running: {100*cov[k]/tot:.1f} %")
agg = defaultdict(list)
for n, s, e, q in rows:
    if t0 <= s < t1: agg[n[:45]].append((e - s) / 1e3)
for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    print(f"   {n:45s} n={len(v):3d} med={np.median(v):6.1f} per step={sum(v)/(len(tiles)-1):6.1f}")
i0 = rows.index(tiles[20])
for n, s, e, q in rows[i0:i0+34]:
    print(f"{(s-rows[i0][1])/1e3:9.1f} {(e-rows[i0][1])/1e3:9.1f} {(e-s)/1e3:7.1f} q{q} {n[:50]}")
PY
