"""Per-step view of a rocprofv3 kernel trace of the pipelined engine: for every query-kernel
dispatch (knn_tile_kernel / knn_tree_kernel) its duration, the period since the previous one's
start, the overlap with it, and the build kernels' time inside that period.
usage: python scripts/prof_steps.py run_results.db [last_n_steps]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = c.execute("select name, start, end from kernels order by start").fetchall()
q = [(s, e) for n, s, e in rows if "knn_tile_kernel" in n or "knn_tree_kernel" in n]
b = [(s, e) for n, s, e in rows if "bucket_" in n or "bbox" in n or "scan_blocks" in n]
print(f"{len(rows)} dispatches, {len(q)} query dispatches")
print(" step  query_us  period_us  overlap_prev_us  build_us_in_period")
sel = q[-last:]
for i, (s, e) in enumerate(sel):
    if i == 0:
        print(f"{i:5d} {(e - s) / 1e3:9.1f}")
        continue
    ps, pe = sel[i - 1]
    bt = sum(min(be, s) - max(bs, ps) for bs, be in b if be > ps and bs < s) / 1e3
    print(f"{i:5d} {(e - s) / 1e3:9.1f} {(s - ps) / 1e3:10.1f} {max(0, pe - s) / 1e3:16.1f} {bt:18.1f}")
if len(sel) > 2:
    per = [(sel[i][0] - sel[i - 1][0]) / 1e3 for i in range(1, len(sel))]
    print(f"mean query {sum((e - s) for s, e in sel) / len(sel) / 1e3:.1f} us, mean period {sum(per) / len(per):.1f} us")
