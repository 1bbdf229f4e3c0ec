"""Bounds-checked run (KN_CHECKED=1 loads _C_checked) of the tree path after the round-3 exact
kernel change (breadth-first sweep of bounded listed queries, stacked node distances on the
depth-first walk, K > 64 every query): clustered and surface clouds through algo="tree",
squared distances against the kd-tree oracle, then the violation words (all 0 = no out-of-range
index)."""
import os

os.environ["KN_CHECKED"] = "1"
import torch

import cuda_knearests_amd as kn
from cuda_knearests_amd._ext import load
from cuda_knearests_amd.utils import clustered_cloud, surface_cloud

C = load()
assert "checked" in C.__name__, C.__name__
dev = torch.device("cuda", 0)
C.debug_words(True)
clouds = {"clustered": clustered_cloud(60000, seed=16), "surface": surface_cloud(60000, seed=17)}
bad = 0
for name, cloud in clouds.items():
    p = cloud.to(dev)
    for k in (16, 50, 80):
        g = kn.build_grid(p, k, adaptive=True)
        oi, od = kn.knn_cpu(cloud, k, method="kdtree")
        # flags 1: no query certifies in the tree kernel, every one takes the exact kernel with
        # its bound (the breadth-first sweep for all of them)
        for flags in (0, 1):
            idx, d2 = kn.query(g, k, algo="tree", flags=flags)
            torch.cuda.synchronize()
            ok = torch.equal(d2.cpu(), od)
            bad += 0 if ok else 1
            print(f"{name} k={k} tree flags={flags} exact={ok}", flush=True)
print("debug_words:", C.debug_words(False), flush=True)
print("CHECKED_OK" if bad == 0 else f"CHECKED_BAD {bad}")
