"""Why do some queries miss certification in the tile kernel? Dump their distance profiles."""
import torch
import cuda_knearests_amd as kn
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

dev = torch.device("cuda", 0)
pts = uniform_cloud(900000, seed=0, device=dev)
g = ops.build_grid(pts, 16)
print(g.plan, flush=True)
idx, d2, info = ops.query(g, 16, return_info=True)
c = info["counters"].tolist()
print("counters", c, flush=True)
sl = info["exact_path"][: c[0]].long()
orig = g.perm[sl].long()
sb = (g.plan.lds_capacity - 1).bit_length()
for o in orig.tolist()[:12]:
    q = pts[o]
    dd = ((pts - q) ** 2).sum(1)
    dd[o] = float("inf")
    v, i = torch.topk(dd, 22, largest=False)
    bits = v.view(torch.int32)
    trunc = (bits >> sb).tolist()
    print(o, "d2:", [f"{x:.6g}" for x in v.tolist()[:20]], flush=True)
    print("   buckets:", trunc[:20], flush=True)
    print("   cell:", ((q - torch.tensor([0., 0, 0], device=dev)) / 1000 * 66).floor().tolist(), flush=True)
