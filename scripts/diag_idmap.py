"""Query-kernel cost of the multi-GPU id_map gather (local slot -> global id) and of the
point order, lane walk (flags=8) vs union stream (flags=4), on one grid.
usage: python scripts/diag_idmap.py [n] [k]"""
import json, sys
import torch
from cuda_knearests_amd import _C as C
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12500000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
plan = ops.Plan.auto(n, k)
inf = float("inf")
ident = torch.arange(n, device=dev, dtype=torch.int32)
rnd = torch.randperm(n, device=dev).to(torch.int32)


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize(); ts.append(a.elapsed_time(b))
    return round(sorted(ts)[reps // 2], 4)


for order in ("random", "cell-sorted input"):
    p = pts
    if order != "random":  # feed the build its own cell-sorted output (as a routed rank might)
        s0, _, _, _ = C.build(pts, plan.dims, False, None)
        p = s0[:, :3].contiguous()
    s, cs, perm, geom = C.build(p, plan.dims, False, None)
    for name, idm in (("none", None), ("identity", ident), ("random", rnd)):
        for flags in (4, 8):
            q = lambda: C.query(s, cs, geom, plan.dims, k, n, idm, [-inf, -inf, -inf, inf, inf, inf], plan.tile,
                                plan.halo, plan.lds_capacity, True, True, flags)
            q()
            print(json.dumps({"n": n, "k": k, "input_order": order, "id_map": name, "flags": flags, "ms": timed(q)}),
                  flush=True)
