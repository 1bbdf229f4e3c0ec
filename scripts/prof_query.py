"""Minimal driver for rocprofv3 PMC passes: one build + a few queries (900K, k=16 by default).
usage: python scripts/prof_query.py [n] [k] [reps]"""
import sys

import torch

import cuda_knearests_amd as kn
from cuda_knearests_amd.utils import uniform_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
g = kn.build_grid(pts, k)
for _ in range(reps):
    idx, d2 = kn.query(g, k)
torch.cuda.synchronize()
print("ok", idx.shape, flush=True)
