"""Summarise a rocprofv3 SQLite trace (run_results.db): per-kernel stats and, with --timeline,
the dispatches of the last N-kernel window (start offset, duration, gap to the previous end)."""
import argparse
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--timeline", type=int, default=0, help="print the last N dispatches")
ap.add_argument("--skip-first", type=int, default=0)
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
rows = rows[a.skip_first:]
agg = defaultdict(lambda: [0, 0.0])
for name, s, e in rows:
    agg[name][0] += 1
    agg[name][1] += (e - s) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"{'calls':>6} {'total_us':>10} {'mean_us':>9} {'share':>6}  kernel")
for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{n:6d} {t:10.1f} {t / n:9.2f} {100 * t / tot:5.1f}%  {name[:100]}")
if a.timeline:
    tl = rows[-a.timeline:]
    t0 = tl[0][1]
    prev = None
    print("\n  start_us   dur_us   gap_us  kernel")
    for name, s, e in tl:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} {gap:8.1f}  {name[:90]}")
        prev = e
