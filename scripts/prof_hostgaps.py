"""Host enqueue vs device start of the query kernels in a rocprofv3 --hip-trace --kernel-trace
database: per step, when the host issued the tile kernel's launch (or graph launch) and when the
kernel started on the GPU. usage: python scripts/prof_hostgaps.py run_results.db [steps]"""
import sqlite3
import sys

db = sys.argv[1]
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
print("tables:", ", ".join(t for t in tabs if not t.startswith("rocpd_info")))
cols = {t: [r[1] for r in c.execute(f"pragma table_info('{t}')")] for t in tabs}
api = next((t for t in ("regions", "regions_and_samples") if t in cols), None)
print("api table:", api, cols.get(api))
k = c.execute("select name, start, end, corr_id, queue_id from kernels order by start").fetchall()
tiles = [r for r in k if "knn_tile_kernel" in r[0]]
tiles = tiles[-nsteps - 2:-2]
if api:
    # API calls by correlation id
    q = f"select name, start, end, corr_id from {api} where corr_id in ({','.join(str(t[3]) for t in tiles)})"
    calls = {r[3]: r for r in c.execute(q).fetchall()}
    t0 = tiles[0][1]
    for t in tiles:
        a = calls.get(t[3])
        if a:
            print(f"tile q{t[4]} host call {(a[1]-t0)/1e3:9.1f}..{(a[2]-t0)/1e3:9.1f}  gpu {(t[1]-t0)/1e3:9.1f}..{(t[2]-t0)/1e3:9.1f}  lag {(t[1]-a[2])/1e3:7.1f} us  ({a[0][:30]})")
        else:
            print(f"tile q{t[4]} no api row, gpu {(t[1]-t0)/1e3:9.1f}")
    # host API timeline during the window
    lo, hi = tiles[2][1], tiles[6][1]
    rows = c.execute(f"select name, start, end from {api} where start >= ? and start <= ? order by start", (lo - 400000, hi)).fetchall()
    print(f"{len(rows)} api calls in the window")
    for n, s, e in rows[:200]:
        print(f"  {(s-t0)/1e3:9.1f} {(e-s)/1e3:7.1f} {n[:60]}")
