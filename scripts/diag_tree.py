"""Grid vs tree path: device time of query (hipEvent), tree build, counters, on one cloud.
usage: python scripts/diag_tree.py gen n k"""
import json
import sys

import torch

import cuda_knearests_amd as kn
from cuda_knearests_amd.utils import blue_cloud, clustered_cloud, surface_cloud, uniform_cloud

gen, n, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
p = {"uniform": uniform_cloud, "clustered": clustered_cloud, "surface": surface_cloud, "blue": blue_cloud}[gen](n, seed=0).cuda()
g = kn.build_grid(p, k, adaptive=True)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        out = fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps, out


tb, _ = timed(lambda: kn.ops.knn_ops.load().tree_build(g.sorted, g.cell_start, g.geom, list(g.plan.dims), False))
tr = kn.ops.knn_ops.load().tree_build(g.sorted, g.cell_start, g.geom, list(g.plan.dims), True)
tg, (ig, dg, infog) = timed(lambda: kn.query(g, k, return_info=True))
tt, (it, dt, infot) = timed(lambda: kn.query(g, k, algo="tree", return_info=True))
same = bool(torch.equal(dg, dt))
C = kn.ops.knn_ops.load()
w = int(C.occupancy(g.cell_start).item()) / n
tgb, _ = timed(lambda: kn.build_grid(p, k, adaptive=True), reps=3)
print(json.dumps({"gen": gen, "n": n, "k": k, "dims": g.plan.dims, "w_final": round(w, 2), "grid_build_ms": round(tgb, 3), "grid_query_ms": round(tg, 4),
                  "tree_build_ms": round(tb, 4), "leaves": int(tr[2]), "tree_query_ms": round(tt, 4),
                  "grid_counters": infog["counters"].tolist(), "tree_counters": infot["counters"].tolist(),
                  "dist_equal": same}), flush=True)
