"""Per-kernel totals of a rocprofv3 kernel trace (rocpd sqlite): calls, total / mean / share.
usage: python scripts/kernel_stats.py run_results.db [n_rows]"""
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
agg = defaultdict(lambda: [0, 0])
for n, s, e in c.execute(f"select {name}, start, end from kernels"):
    a = agg[n.replace("(anonymous namespace)::", "").split("(")[0][:80]]
    a[0] += 1
    a[1] += e - s
tot = sum(v[1] for v in agg.values()) or 1
nrows = int(sys.argv[2]) if len(sys.argv) > 2 else 20
print(f"{'calls':>6s} {'total_us':>10s} {'mean_us':>9s} {'share':>6s}  kernel")
for k, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:nrows]:
    print(f"{cnt:6d} {t / 1e3:10.1f} {t / cnt / 1e3:9.2f} {100 * t / tot:5.1f}%  {k}")
