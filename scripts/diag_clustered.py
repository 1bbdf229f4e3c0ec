"""Clustered-cloud breakdown: grid plan, LDS-overflow tiles, exact-path queries by cause, and
per-kernel device times (hipEvent) of the tile pass vs the exact pass.
usage: python scripts/diag_clustered.py [n] [k]"""
import sys

import torch

import cuda_knearests_amd as kn
from cuda_knearests_amd.utils import clustered_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dev = torch.device("cuda", 0)
p = clustered_cloud(n, seed=0).to(dev)
g = kn.build_grid(p, k, adaptive=True)
C = kn.ops.knn_ops.load() if hasattr(kn, "ops") else None
cs = g.cell_start
counts = (cs[1:] - cs[:-1]).float()
print("plan", g.plan, "cells", counts.numel(), "max/cell", int(counts.max()), "mean occupied",
      float(counts[counts > 0].mean()), flush=True)
for rep in range(2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    idx, d2, info = kn.query(g, k, return_info=True)
    e1.record()
    e1.synchronize()
    c = info["counters"].tolist()
    print(f"query {e0.elapsed_time(e1):.3f} ms counters {c}", flush=True)
# exact path alone for the same fallback set: tiles disabled on the fallback queries only is not
# exposed; time the all-exact path for scale
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
kn.query(g, k, use_tiles=False)
e1.record()
e1.synchronize()
print(f"all-exact query {e0.elapsed_time(e1):.3f} ms", flush=True)
