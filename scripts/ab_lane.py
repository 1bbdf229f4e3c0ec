"""In-process A/B of the lane-walk region: union-stream tile kernel (flags=4), lane walk over the
whole staged block (flags=8, _C) and lane walk over the lane's own cell +- H (flags=8,
_C_lanehb, built with -DKN_LANE_FULL=0). Checks bit-identical results; counters[0] is the
number of queries sent to the exact fallback kernel.
usage: python scripts/ab_lane.py [n] [k] [rounds] [gen]"""
import importlib
import json
import sys

import torch

from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud, clustered_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 10
gen = sys.argv[4] if len(sys.argv) > 4 else "uniform"
A = importlib.import_module("cuda_knearests_amd._C")
B = importlib.import_module("cuda_knearests_amd._C_lanehb")
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev) if gen == "uniform" else clustered_cloud(n, seed=0, device=dev)
plan = ops.Plan.auto(n, k)
s, cs, perm, geom = A.build(pts, plan.dims, True, None)
inf = float("inf")
cases = {"tile": (A, 4), "lane_full": (A, 8), "lane_own_h": (B, 8)}


def run(name):
    mod, flags = cases[name]
    return mod.query(s, cs, geom, plan.dims, k, n, None, [-inf, -inf, -inf, inf, inf, inf], plan.tile, plan.halo,
                     plan.lds_capacity, True, True, flags)


outs = {c: run(c) for c in cases}
torch.cuda.synchronize()
ref = outs["tile"]
res = {"n": n, "k": k, "gen": gen,
       "identical": all(torch.equal(ref[0], o[0]) and torch.equal(ref[1], o[1]) for o in outs.values()),
       "exact_queries": {c: int(o[2][0]) for c, o in outs.items()}}
ts = {c: [] for c in cases}
for _ in range(rounds):
    for c in cases:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(c)
        e1.record()
        e1.synchronize()
        ts[c].append(e0.elapsed_time(e1))
res["ms"] = {c: round(sorted(v)[len(v) // 2], 4) for c, v in ts.items()}
print(json.dumps(res), flush=True)
