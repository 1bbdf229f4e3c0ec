"""Wave-uniform work of the lane walk (variant _C_wstats: KN_CHECKED=1 KN_WALK_STATS=1): row
iterations, lockstep candidate steps and med3 networks per wave, plus per-lane candidates from the
checked build (_C_checked). usage: python scripts/walk_stats.py [n] [k ...]"""
import importlib, json, sys, torch
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
ks = [int(v) for v in sys.argv[2:]] or [16]
W = importlib.import_module("cuda_knearests_amd._C_wstats")
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
inf = float("inf")
for k in ks:
    plan = ops.Plan.auto(n, k)
    s, cs, perm, geom = W.build(pts, plan.dims, True, None)
    args = (s, cs, geom, plan.dims, k, n, None, [-inf, -inf, -inf, inf, inf, inf], plan.tile, plan.halo,
            plan.lds_capacity, True, True, 0)
    out = W.query(*args, xsub=plan.xsub)
    torch.cuda.synchronize()
    c = [int(v) for v in out[2].tolist()] if len(out) > 2 else None
    print(json.dumps({"n": n, "k": k, "counters": c,
                      "rows_per_wave": c[4] / c[7], "steps_per_wave": c[5] / c[7], "networks_per_wave": c[6] / c[7]}))
