"""Sweep of the query kernel's LDS plan for occupancy: grid density (points per cell) x LDS slot
capacity slack (standard deviations of the staged count). Reports LDS bytes per workgroup,
workgroups per CU (160 KB LDS), exact-path queries, median query time, and whether the rows
equal the default plan's (distances bit for bit).
usage: python scripts/sweep_occ.py <n> <k> <ppc,...> <sd,...> [rounds]"""
import math
import sys

import torch

from cuda_knearests_amd._ext import load
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

C = load()
n, k = int(sys.argv[1]), int(sys.argv[2])
ppcs = [float(x) for x in sys.argv[3].split(",")]
sds = [float(x) for x in sys.argv[4].split(",")]
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 15
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
inf = float("inf")
ref = None


def ev():
    return torch.cuda.Event(enable_timing=True)


for ppc in ppcs:
    plan = ops.Plan.auto(n, k, ppc)
    s, cs, perm, geom = C.build(pts, plan.dims, False, None)
    actual = n / (plan.dims[0] * plan.dims[1] * plan.dims[2])
    staged = (plan.tile[0] + 2 * plan.halo) * (plan.tile[1] + 2 * plan.halo) * (plan.tile[2] + 2 * plan.halo) * actual
    for sd in sds:
        cap = int(math.ceil((staged + sd * math.sqrt(staged) + 64) / 64.0)) * 64
        lds = C.query_lds_bytes(plan.tile, plan.halo, cap) if hasattr(C, "query_lds_bytes") else -1
        args = (s, cs, geom, plan.dims, k, n, None, [-inf, -inf, -inf, inf, inf, inf], plan.tile, plan.halo, cap,
                True, True, 0)
        out = C.query(*args)
        torch.cuda.synchronize()
        if ref is None:
            ref = out
        same = torch.equal(out[1], ref[1])
        ts = []
        for _ in range(rounds):
            e0, e1 = ev(), ev()
            e0.record()
            C.query(*args)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        print(f"ppc {ppc} actual {actual:.3f} dims {plan.dims} sd {sd} cap {cap} lds {lds} "
              f"wg/cu {160 * 1024 // lds if lds > 0 else '?'} exact {int(out[2][0])} "
              f"median {ts[len(ts) // 2]:.4f} min {ts[0]:.4f} ms same_d2 {same}", flush=True)
