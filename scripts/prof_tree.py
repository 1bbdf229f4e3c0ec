"""Minimal driver for rocprofv3 PMC passes on the tree path: a clustered (or surface) cloud through
the native engine (auto-selected tree path), a few solves.
usage: python scripts/prof_tree.py [n] [k] [gen] [reps]"""
import sys

import torch

from cuda_knearests_amd._ext import load
from cuda_knearests_amd.utils import clustered_cloud, surface_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
gen = sys.argv[3] if len(sys.argv) > 3 else "clustered"
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
dev = torch.device("cuda", 0)
pts = (clustered_cloud if gen == "clustered" else surface_cloud)(n, seed=0, device=dev)
C = load()
e = C.Engine(k)
e.prepare(pts)
for _ in range(reps):
    e.solve()
torch.cuda.synchronize()
print("ok", e.info(), e.counters(), flush=True)
