"""In-process interleaved A/B of the tree query: _C vs _C_<variant> on adaptive grids.
usage: python scripts/ab_tree.py <variant> [n] [k,k] [gen,gen] [rounds] -> one JSON line per case"""
import importlib, json, sys, torch
import cuda_knearests_amd as kn
from cuda_knearests_amd import utils

var = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 900000
ks = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "16").split(",")]
gens = (sys.argv[4] if len(sys.argv) > 4 else "clustered,surface,uniform").split(",")
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 8
A = importlib.import_module("cuda_knearests_amd._C")
B = importlib.import_module(f"cuda_knearests_amd._C_{var}")
dev = torch.device("cuda", 0)
for gen in gens:
    pts = getattr(utils, f"{gen}_cloud")(n, seed=0, device=dev)
    for k in ks:
        g = kn.build_grid(pts, k, adaptive=True)
        dims = list(g.plan.dims)
        # each module builds its own tree (variants may change the leaves)
        trees = {id(M): M.tree_build(g.sorted, g.cell_start, g.geom, dims, True) for M in (A, B)}
        L = trees[id(A)][2]
        run = lambda M: M.tree_query(trees[id(M)][0], trees[id(M)][1], dims, g.n, k, g.n, None, True, 0)
        ra, rb = run(A), run(B)
        torch.cuda.synchronize()
        same = torch.equal(ra[0], rb[0]) and torch.equal(ra[1], rb[1])
        ta, tb = [], []
        ev = lambda: torch.cuda.Event(enable_timing=True)
        for r in range(rounds):
            for M, acc in ((A, ta), (B, tb)):
                e0, e1 = ev(), ev()
                e0.record(); run(M); e1.record(); e1.synchronize()
                acc.append(e0.elapsed_time(e1))
        ta.sort(); tb.sort()
        print(json.dumps({"gen": gen, "n": n, "k": k, "leaves": int(L), "identical": same,
                          "counters_C": [int(v) for v in ra[2].tolist()], f"counters_{var}": [int(v) for v in rb[2].tolist()],
                          "C_ms": [round(ta[len(ta) // 2], 4), round(ta[0], 4)],
                          f"{var}_ms": [round(tb[len(tb) // 2], 4), round(tb[0], 4)]}), flush=True)
