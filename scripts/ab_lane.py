"""In-process A/B of the two LDS-staged tile kernels on one grid: wave-uniform union stream
(flags=4) vs per-lane walk (flags=8). Checks bit-identical results, then interleaved timing.
usage: python scripts/ab_lane.py [n] [k] [rounds] [module] [gen]   (module: _C or _C_checked)"""
import importlib
import json
import sys

import torch

from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud, clustered_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 10
mod = sys.argv[4] if len(sys.argv) > 4 else "_C"
gen = sys.argv[5] if len(sys.argv) > 5 else "uniform"
C = importlib.import_module(f"cuda_knearests_amd.{mod}")
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev) if gen == "uniform" else clustered_cloud(n, seed=0, device=dev)
plan = ops.Plan.auto(n, k)
s, cs, perm, geom = C.build(pts, plan.dims, True, None)
inf = float("inf")


def run(flags):
    return C.query(s, cs, geom, plan.dims, k, n, None, [-inf, -inf, -inf, inf, inf, inf], plan.tile, plan.halo,
                   plan.lds_capacity, True, True, flags)


A = run(4)
B = run(8)
torch.cuda.synchronize()
same = torch.equal(A[0], B[0]) and torch.equal(A[1], B[1])
res = {"n": n, "k": k, "gen": gen, "module": mod, "identical": same,
       "tile_counters": A[2].tolist(), "lane_counters": B[2].tolist()}
if mod.startswith("_C_checked"):
    res["debug_words"] = C.debug_words(True)
ta, tb = [], []
for _ in range(rounds):
    for flags, acc in ((4, ta), (8, tb)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(flags)
        e1.record()
        e1.synchronize()
        acc.append(e0.elapsed_time(e1))
ta.sort()
tb.sort()
res["tile_ms"] = round(ta[len(ta) // 2], 4)
res["lane_ms"] = round(tb[len(tb) // 2], 4)
print(json.dumps(res), flush=True)
