"""Why do K=50/64 queries take the exact path on a uniform cloud? Counters, position of the
fallback queries (distance to the domain faces in cells, position in the tile) and their true
K-th distance vs the scanned block."""
import sys

import torch

from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
for k in (50, 64):
    pts = uniform_cloud(n, seed=0, device=dev)
    g = ops.build_grid(pts, k)
    idx, d2, info = ops.query(g, k, return_info=True)
    c = info["counters"].tolist()
    sl = info["exact_path"][: c[0]].long()
    orig = g.perm[sl].long()
    geom = g.geom.view(torch.float32)[:9].tolist()
    org, cell = geom[:3], geom[3:6]
    dims = torch.tensor(g.plan.dims, device=dev)
    q = pts[orig]
    cc = ((q - torch.tensor(org, device=dev)) / torch.tensor(cell, device=dev)).floor().int()
    edge = torch.minimum(cc, dims - 1 - cc)  # cells to the nearest domain face, per axis
    nface = (edge == 0).sum(1)
    print(f"n={n} k={k} plan={g.plan} counters={c[:6]}", flush=True)
    print("  faces touched (0..3) histogram:", torch.bincount(nface, minlength=4).tolist(), flush=True)
    print("  min edge distance histogram:", torch.bincount(edge.min(1).values.clamp(max=9), minlength=10).tolist())
    print("  cell mod 4 histogram x:", torch.bincount((cc[:, 0] % 4), minlength=4).tolist())
    dk = d2[orig, k - 1].sqrt()
    print("  K-th distance / cell: min %.2f mean %.2f max %.2f" % (
        float((dk / cell[0]).min()), float((dk / cell[0]).mean()), float((dk / cell[0]).max())))
    alld = d2[:, k - 1].sqrt() / cell[0]
    print("  all queries K-th / cell: mean %.2f p99 %.2f max %.2f" % (
        float(alld.mean()), float(alld.quantile(0.99)) if alld.numel() < 16_000_000 else -1, float(alld.max())))
