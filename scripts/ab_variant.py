"""In-process interleaved A/B of the tile kernel: _C (baseline) vs _C_<variant> (guide §5.4 rule 24).
usage: python scripts/ab_variant.py <variant> [n] [k] [rounds]"""
import importlib, sys, torch
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

var = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 900000
k = int(sys.argv[3]) if len(sys.argv) > 3 else 16
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 10
A = importlib.import_module("cuda_knearests_amd._C")
B = importlib.import_module(f"cuda_knearests_amd._C_{var}")
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
plan = ops.Plan.auto(n, k)
s, cs, perm, geom = A.build(pts, plan.dims, True, None)
inf = float("inf")
args = lambda: (s, cs, geom, plan.dims, k, n, None, [-inf, -inf, -inf, inf, inf, inf], plan.tile, plan.halo, plan.lds_capacity, True, True, 0)
kw = {"xsub": plan.xsub}  # the plan's x sub-cells (dims[0] and tile[0] count sub-cells)
ref = A.query(*args(), **kw)
out = B.query(*args(), **kw)
torch.cuda.synchronize()
print("identical:", torch.equal(ref[0], out[0]) and torch.equal(ref[1], out[1]), flush=True)
if "chk" in var:
    print("debug_words:", B.debug_words(False), flush=True)
ta, tb = [], []
ev = lambda: torch.cuda.Event(enable_timing=True)
for r in range(rounds):
    # alternate which variant runs first in a round (no position bias)
    order = ((A, ta), (B, tb)) if r % 2 == 0 else ((B, tb), (A, ta))
    for mod, acc in order:
        e0, e1 = ev(), ev()
        e0.record(); mod.query(*args(), **kw); e1.record(); e1.synchronize()
        acc.append(e0.elapsed_time(e1))
ta.sort(); tb.sort()
print(f"baseline median {ta[len(ta)//2]:.4f} min {ta[0]:.4f} | {var} median {tb[len(tb)//2]:.4f} min {tb[0]:.4f} ms", flush=True)
