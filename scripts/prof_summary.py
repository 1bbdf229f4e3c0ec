"""Summarise a rocprofv3 (ROCm 7.x rocpd sqlite) kernel trace: per-kernel calls / total / avg us.
usage: python scripts/prof_summary.py gpurun_out/prof/run_results.db [> profiles/x.txt]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                 f"from kernels group by {name} order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"{'kernel':70s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'%':>6s}")
for n, cnt, s, a, mn, mx in rows:
    print(f"{n[:70]:70s} {cnt:6d} {s / 1e3:10.1f} {a / 1e3:9.2f} {mn / 1e3:9.2f} {mx / 1e3:9.2f} {100 * s / tot:6.1f}")
