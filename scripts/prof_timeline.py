"""Per-step timeline of a rocprofv3 kernel trace (rocpd sqlite): kernel, start offset, duration and
the idle gap before it -- shows host-sync bubbles between launches.
usage: python scripts/prof_timeline.py run_results.db [first_kernel_substring] [n_rows]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name}, start, end from kernels order by start").fetchall()
anchor = sys.argv[2] if len(sys.argv) > 2 else None
nrows = int(sys.argv[3]) if len(sys.argv) > 3 else 60
if anchor:
    hits = [i for i, r in enumerate(rows) if anchor in r[0]]
    i0 = hits[len(hits) // 2] if hits else 0  # a step from the middle of the run
else:
    i0 = max(0, len(rows) - nrows)
t0 = rows[i0][1]
prev_end = rows[i0 - 1][2] if i0 else t0
busy = 0
print(f"{'t_us':>9s} {'dur_us':>8s} {'gap_us':>8s}  kernel")
for n, s, e in rows[i0:i0 + nrows]:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {(s - prev_end) / 1e3:8.1f}  {n[:90]}")
    busy += e - s
    prev_end = max(prev_end, e)
span = prev_end - t0
print(f"span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({100 * busy / max(span, 1):.0f}%)")
