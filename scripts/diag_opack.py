"""Oracle check of the grid path on a clustered cloud (grid forced, dense tiles -> exact path)
for _C and _C_opack: mismatching rows against the kd-tree oracle per module.
usage: python scripts/diag_opack.py [k] [modules, comma-separated]"""
import importlib, sys, torch
import cuda_knearests_amd as kn
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import clustered_cloud

dev = torch.device("cuda", 0)
inf = float("inf")
k = int(sys.argv[1]) if len(sys.argv) > 1 else 16
mods = sys.argv[2].split(",") if len(sys.argv) > 2 else ["_C", "_C_opack"]
for n in (100000, 300000):
    p = clustered_cloud(n, seed=0)
    oi, od = kn.knn_cpu(p, k, "kdtree")
    for name in mods:
        M = importlib.import_module(f"cuda_knearests_amd.{name}")
        plan = ops.Plan.auto(n, k)
        s, cs, perm, geom = M.build(p.to(dev), plan.dims, True, None)
        r = M.query(s, cs, geom, plan.dims, k, n, None, [-inf, -inf, -inf, inf, inf, inf], plan.tile, plan.halo,
                    plan.lds_capacity, True, True, 0, None, 0, None, 0, plan.xsub)
        d2 = r[1].cpu()
        bad = (d2 != od).any(1)
        print(n, name, "exact-path", int(r[2][0]), "rows differing from oracle", int(bad.sum()),
              "first", int(bad.nonzero()[0, 0]) if bad.any() else -1, flush=True)
