"""Bounds-checked run (KN_CHECKED=1 loads _C_checked) over the round-3 session-2 paths: x sub-cell
grids (K <= 16), u16 row-relative cell boundaries, the distance-sorted row order (K > 40),
small tiles (pts20K), a dense clustered cloud on the grid path, then the per-file violation
words (all 0xFFFFFFFF = no out-of-range index) and an oracle check of every result."""
import os

os.environ["KN_CHECKED"] = "1"
import torch

import cuda_knearests_amd as kn
from cuda_knearests_amd._ext import load
from cuda_knearests_amd.utils import clustered_cloud, uniform_cloud

C = load()
assert "checked" in C.__name__, C.__name__
dev = torch.device("cuda", 0)
C.debug_words(True)
clouds = {"uniform": uniform_cloud(150000, seed=5), "clustered": clustered_cloud(60000, seed=6),
          "pts20K": kn.read_xyz("data/pts20K.xyz", normalize=True).float()}
bad = 0
for name, cloud in clouds.items():
    p = cloud.to(dev)
    for k in (8, 16, 50):
        for algo in ("grid", "auto"):
            g = kn.build_grid(p, k, adaptive=algo == "auto")
            idx, d2 = kn.query(g, k, algo=algo)
            torch.cuda.synchronize()
            oi, od = kn.knn_cpu(cloud, k, method="kdtree")
            ok = torch.equal(d2.cpu(), od)
            bad += 0 if ok else 1
            print(f"{name} k={k} {algo} plan={g.plan.dims}/{g.plan.tile}/x{g.plan.xsub} exact={ok}", flush=True)
print("debug_words:", C.debug_words(False), flush=True)
print("CHECKED_OK" if bad == 0 else f"CHECKED_BAD {bad}")
