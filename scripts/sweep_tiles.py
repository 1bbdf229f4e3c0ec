"""Sweep grid density / tile shape / halo for the tile kernel (solve time, device events).
KN_QUERY_ALGO=lane|tile selects the kernel variant.
usage: python scripts/sweep_tiles.py [n] [k] [ppc,..] [TXxTYxTZ,..] [halo,..]"""
import itertools, json, sys
import torch
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
res = []
PPC = [float(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1.5, 2.0, 2.5, 3.1, 4.0, 5.0]
TILES = ([tuple(int(v) for v in t.split("x")) for t in sys.argv[4].split(",")] if len(sys.argv) > 4 else
         [(4, 4, 4), (8, 4, 4), (4, 4, 2), (8, 8, 2), (6, 6, 6), (8, 4, 2)])
HALOS = [int(h) for h in sys.argv[5].split(",")] if len(sys.argv) > 5 else [0]  # 0 = plan default
for ppc, tile, halo in itertools.product(PPC, TILES, HALOS):
    plan = ops.Plan.auto(n, k, ppc, tile, halo)
    if plan.lds_bytes > 160 * 1024:
        continue
    g = ops.build_grid(pts, k, plan=plan)
    ops.query(g, k)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        a.record(); idx, d2, info = ops.query(g, k, return_info=True); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    c = info["counters"].tolist()
    r = {"ppc": ppc, "tile": tile, "halo": plan.halo, "cap": plan.lds_capacity, "lds": plan.lds_bytes, "ms": round(ts[2], 4), "exact": c[0], "dense": c[2]}
    res.append(r)
    print(json.dumps(r), flush=True)
best = min(res, key=lambda r: r["ms"])
print("BEST", json.dumps(best))
