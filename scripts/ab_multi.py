"""In-process interleaved A/B of the query kernel over several K and clouds: _C vs _C_<variant>.
usage: python scripts/ab_multi.py <variant> [n] [k,k,...] [gen,gen,...] [rounds]
Prints one JSON line per (cloud, K): identical rows?, exact-path counters, median/min ms."""
import importlib, json, sys, torch
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd import utils

var = sys.argv[1]
n0 = int(sys.argv[2]) if len(sys.argv) > 2 else 900000
ks = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "16,50").split(",")]
gens = (sys.argv[4] if len(sys.argv) > 4 else "uniform").split(",")
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 10
A = importlib.import_module("cuda_knearests_amd._C")
B = importlib.import_module(f"cuda_knearests_amd._C_{var}")
dev = torch.device("cuda", 0)
inf = float("inf")
for gen in gens:
    if gen.startswith("xyz:"):  # a reference-format point file (normalised), e.g. xyz:data/pts20K.xyz
        from cuda_knearests_amd import read_xyz
        pts = read_xyz(gen[4:], normalize=True).float().to(dev)
    else:
        pts = getattr(utils, f"{gen}_cloud")(n0, seed=0, device=dev)
    n = pts.size(0)
    for k in ks:
        plan = ops.Plan.auto(n, k)
        s, cs, perm, geom = A.build(pts, plan.dims, True, None)
        args = lambda: (s, cs, geom, plan.dims, k, n, None, [-inf, -inf, -inf, inf, inf, inf], plan.tile, plan.halo,
                        plan.lds_capacity, True, True, 0, None, 0, None, 0, plan.xsub)
        ra = A.query(*args())
        rb = B.query(*args())
        torch.cuda.synchronize()
        same = torch.equal(ra[0], rb[0]) and torch.equal(ra[1], rb[1])
        ta, tb = [], []
        ev = lambda: torch.cuda.Event(enable_timing=True)
        for r in range(rounds):
            for mod, acc in ((A, ta), (B, tb)):
                e0, e1 = ev(), ev()
                e0.record(); mod.query(*args()); e1.record(); e1.synchronize()
                acc.append(e0.elapsed_time(e1))
        ta.sort(); tb.sort()
        print(json.dumps({"gen": gen, "n": n, "k": k, "identical": same,
                          "counters_C": [int(v) for v in ra[2][:4].tolist()],
                          f"counters_{var}": [int(v) for v in rb[2][:4].tolist()],
                          "C_ms": [round(ta[len(ta) // 2], 4), round(ta[0], 4)],
                          f"{var}_ms": [round(tb[len(tb) // 2], 4), round(tb[0], 4)]}), flush=True)
