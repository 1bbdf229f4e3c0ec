"""In-process interleaved A/B of the grid's x subdivision (AutoParams::xsub): plan xsub=A vs xsub=B,
same extension, build + query timed separately, rows compared.
usage: python scripts/ab_xsub.py [n] [k,k,...] [gen,gen,...] [rounds] [xa] [xb]"""
import json, sys, torch
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd import utils
from cuda_knearests_amd._ext import load

n0 = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
ks = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "16").split(",")]
gens = (sys.argv[3] if len(sys.argv) > 3 else "uniform").split(",")
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 10
xa = int(sys.argv[5]) if len(sys.argv) > 5 else 1
xb = int(sys.argv[6]) if len(sys.argv) > 6 else 2
C = load()
dev = torch.device("cuda", 0)
inf = float("inf")
ev = lambda: torch.cuda.Event(enable_timing=True)
for gen in gens:
    if gen.startswith("xyz:"):
        from cuda_knearests_amd import read_xyz
        pts = read_xyz(gen[4:], normalize=True).float().to(dev)
    else:
        pts = getattr(utils, f"{gen}_cloud")(n0, seed=0, device=dev)
    n = pts.size(0)
    for k in ks:
        plans = {x: ops.Plan.auto(n, k, xsub=x) for x in (xa, xb)}
        def build(p):
            return C.build(pts, p.dims, True, None)
        def query(p, g):
            s, cs, perm, geom = g
            return C.query(s, cs, geom, p.dims, k, n, None, [-inf, -inf, -inf, inf, inf, inf], p.tile, p.halo,
                           p.lds_capacity, True, True, 0, None, 0, None, 0, p.xsub)
        grids = {x: build(p) for x, p in plans.items()}
        res = {x: query(p, grids[x]) for x, p in plans.items()}
        torch.cuda.synchronize()
        same = torch.equal(res[xa][0], res[xb][0]) and torch.equal(res[xa][1], res[xb][1])
        tb = {xa: [], xb: []}
        tq = {xa: [], xb: []}
        for r in range(rounds):
            for x, p in plans.items():
                e0, e1, e2 = ev(), ev(), ev()
                e0.record(); g = build(p); e1.record(); query(p, g); e2.record(); e2.synchronize()
                tb[x].append(e0.elapsed_time(e1)); tq[x].append(e1.elapsed_time(e2))
        med = lambda v: round(sorted(v)[len(v) // 2], 4)
        out = {"gen": gen, "n": n, "k": k, "identical": same}
        for x, p in plans.items():
            out[f"x{x}"] = {"dims": p.dims, "tile": p.tile, "halo": p.halo, "cap": p.lds_capacity, "lds": p.lds_bytes,
                            "exact_path": int(res[x][2][0].item()), "build_ms": med(tb[x]), "query_ms": med(tq[x]),
                            "query_min": round(min(tq[x]), 4)}
        print(json.dumps(out), flush=True)
