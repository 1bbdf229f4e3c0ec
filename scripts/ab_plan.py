"""In-process interleaved A/B of two builds of the query kernels on one grid, with an optional
plan override (halo / tile / LDS capacity), reporting time and the exact-path count.
usage: python scripts/ab_plan.py <variant> <n> <k> [halo] [rounds] [gen]
  variant: suffix of cuda_knearests_amd._C_<variant> (built by _build.build_variant), or 'base'"""
import importlib
import sys

import torch

from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import clustered_cloud, uniform_cloud

var = sys.argv[1]
n = int(sys.argv[2])
k = int(sys.argv[3])
halo = int(sys.argv[4]) if len(sys.argv) > 4 else 0
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 10
gen = sys.argv[6] if len(sys.argv) > 6 else "uniform"
A = importlib.import_module("cuda_knearests_amd._C")
B = A if var == "base" else importlib.import_module(f"cuda_knearests_amd._C_{var}")
dev = torch.device("cuda", 0)
pts = (uniform_cloud if gen == "uniform" else clustered_cloud)(n, seed=0).to(dev)
plan = ops.Plan.auto(n, k, halo=halo)
s, cs, perm, geom = A.build(pts, plan.dims, True, None)
inf = float("inf")


def args(flags=0):
    return (s, cs, geom, plan.dims, k, n, None, [-inf, -inf, -inf, inf, inf, inf], plan.tile, plan.halo,
            plan.lds_capacity, True, True, flags)


ra, rb = A.query(*args()), B.query(*args())
torch.cuda.synchronize()
print(f"plan dims {plan.dims} tile {plan.tile} halo {plan.halo} cap {plan.lds_capacity} lds {plan.lds_bytes}",
      flush=True)
print("identical:", torch.equal(ra[0], rb[0]) and torch.equal(ra[1], rb[1]),
      "counters A", ra[2].tolist(), "B", rb[2].tolist(), flush=True)
ta, tb = [], []


def ev():
    return torch.cuda.Event(enable_timing=True)


for r in range(rounds):
    for mod, acc in ((A, ta), (B, tb)):
        e0, e1 = ev(), ev()
        e0.record()
        mod.query(*args())
        e1.record()
        e1.synchronize()
        acc.append(e0.elapsed_time(e1))
ta.sort()
tb.sort()
print(f"A(_C) median {ta[len(ta) // 2]:.4f} min {ta[0]:.4f} | B({var}) median {tb[len(tb) // 2]:.4f} "
      f"min {tb[0]:.4f} ms", flush=True)
