"""Where are the exact-path (fallback) queries of the tile kernel?"""
import torch
import cuda_knearests_amd as kn
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

dev = torch.device("cuda", 0)
for n in (100000, 900000):
    pts = uniform_cloud(n, seed=0, device=dev)
    g = ops.build_grid(pts, 16)
    idx, d2, info = ops.query(g, 16, return_info=True)
    c = info["counters"].tolist()
    sl = info["exact_path"][: c[0]].long()
    orig = g.perm[sl].long()
    geom = g.geom.view(torch.float32)[:9].tolist()
    org, cell = geom[:3], geom[3:6]
    q = pts[orig]
    cc = ((q - torch.tensor(org, device=dev)) / torch.tensor(cell, device=dev)).floor().int()
    print(n, g.plan, "counters", c, flush=True)
    tile = (cc // 4)
    print(" cells:", cc[:20].tolist(), flush=True)
    print(" cell mod tile:", (cc % 4)[:20].tolist(), flush=True)
    # true K-th distance vs cell size
    for o in orig.tolist()[:5]:
        dd = ((pts - pts[o]) ** 2).sum(1); dd[o] = float("inf")
        v = torch.topk(dd, 16, largest=False).values
        print("  dK", float(v[-1].sqrt()), "cell", cell[0], flush=True)
