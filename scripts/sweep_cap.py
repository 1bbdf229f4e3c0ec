"""LDS capacity (staged points per workgroup) sweep of the default query kernel: smaller caps
raise occupancy (5 instead of 4 workgroups/CU below 32 KB) but overflowing tiles go to the
exact path. usage: python scripts/sweep_cap.py [n] [k] [cap,..]"""
import dataclasses
import json
import sys

import torch

from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
caps = [int(c) for c in sys.argv[3].split(",")] if len(sys.argv) > 3 else [2048, 1920, 1880, 1856, 1792]
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
base = ops.Plan.auto(n, k)
g = ops.build_grid(pts, k, plan=base)
ref = ops.query(g, k)
for cap in caps:
    plan = ops.Plan(list(base.dims), list(base.tile), base.halo, cap, 0)
    gg = dataclasses.replace(g, plan=plan)
    idx, d2, info = ops.query(gg, k, return_info=True)
    torch.cuda.synchronize()
    same = torch.equal(idx, ref[0]) and torch.equal(d2, ref[1])
    ts = []
    for _ in range(9):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); ops.query(gg, k); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    print(json.dumps({"n": n, "k": k, "cap": cap, "identical": same, "ms": round(ts[len(ts) // 2], 4),
                      "exact": int(info["counters"][0])}), flush=True)
