#!/bin/bash
# engine pipeline timeline (two query streams at equal priority), 900K K=16, 80 / 10
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${OUT:-r5engprof2}
mkdir -p $O
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/t -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --steps 80 --warmup 10 > $GRAFT_REPO_ROOT/$O/t.log 2>&1) || { echo PROF_FAIL; tail $O/t.log; exit 1; }
python - $O/t/run_results.db <<'PY'
import sqlite3, sys
import numpy as np
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
tiles = [r for r in rows if 'knn_tile' in r[0]]
tiles = tiles[-60:-2]
t0, t1 = tiles[0][1], tiles[-1][1]
# coverage: time with >=1 tile running, with 2 running
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
dur = np.array([(e - s) / 1e3 for n, s, e, q in tiles])
print(f"tile duration median {np.median(dur):.1f} us")
b = [r for r in rows if ('bucket' in r[0] or 'bbox' in r[0] or 'scan_blocks' in r[0]) and t0 <= r[1] < t1]
print(f"build kernels in window: {sum((e-s) for n,s,e,q in b)/1e3/(len(tiles)-1):.1f} us/step of kernel time")
i0 = rows.index(tiles[20])
for n, s, e, q in rows[i0:i0+30]:
    print(f"{(s-rows[i0][1])/1e3:9.1f} {(e-rows[i0][1])/1e3:9.1f} {(e-s)/1e3:7.1f} q{q} {n[:50]}")
PY
