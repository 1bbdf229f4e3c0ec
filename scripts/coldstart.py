"""Cold-start table from a rocprofv3 kernel trace of the driver's bench command: per step (one
query-kernel dispatch), the query kernel's duration and the start-to-start period, plus the
idle gap on the query stream before it (previous query end -> this query start)."""
import sqlite3
import sys

db = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "knn_tile_kernel"
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
q = [(s, e) for n, s, e in rows if pat in n]
print(f"{len(rows)} dispatches, {len(q)} query dispatches ({pat})")
print(f"{'step':>4} {'query_us':>9} {'period_us':>9} {'gap_us':>7}")
for i, (s, e) in enumerate(q):
    per = (s - q[i - 1][0]) / 1e3 if i else 0.0
    gap = (s - q[i - 1][1]) / 1e3 if i else 0.0
    print(f"{i:4d} {(e - s) / 1e3:9.1f} {per:9.1f} {gap:7.1f}")
last = q[-20:]
if len(last) > 1:
    d = sum((e - s) for s, e in last) / len(last) / 1e3
    per = (last[-1][0] - last[0][0]) / (len(last) - 1) / 1e3
    print(f"last {len(last)}: mean query {d:.1f} us, mean period {per:.1f} us")
