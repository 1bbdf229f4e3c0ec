"""Graph replay of the steady distributed step (world 1, RCCL), on the build selected by
KN_CHECKED (1: bounds-checked, out-of-range indices are reported instead of faulting):
back-to-back replays without host synchronisation, then every step's validity, the rows
against the eager steady step, and (checked build) the violation words.
usage: KN_CHECKED=1 python scripts/diag_dist_graph.py [steps] [n]"""
import os
import sys

import torch
import torch.distributed as dist

from cuda_knearests_amd._ext import load
from cuda_knearests_amd.parallel import DistributedKNearests
from cuda_knearests_amd.utils import uniform_cloud

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
n = int(sys.argv[2]) if len(sys.argv) > 2 else 900000
for k_, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29541"), ("RANK", "0"), ("WORLD_SIZE", "1")):
    os.environ.setdefault(k_, v)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
C = load()
print("module", C.__name__, flush=True)
pts = uniform_cloud(n, seed=3, device=dev)
ref = DistributedKNearests(k=16, deterministic=False)
ref.solve(pts)
r_eager = ref.solve(pts)  # steady, eager
assert r_eager.valid()
dk = DistributedKNearests(k=16, deterministic=False)
dk.graph_steady = True
dk.solve(pts)  # validating step
res = [dk.solve(pts, async_=True) for _ in range(steps)]  # capture once, then replays
torch.cuda.synchronize()
ok = all(r.valid() for r in res)
last = res[-1]
same = torch.equal(last.neighbors, r_eager.neighbors) and torch.equal(last.d2, r_eager.d2) and \
    torch.equal(last.ids, r_eager.ids)
print("graph", bool(last.stats.get("graph")), "valid", ok, "same rows as eager", same, flush=True)
if "checked" in C.__name__:
    w = C.debug_words(False)
    print("debug words (build, query, route, tree):", w, flush=True)
    sys.exit(0 if ok and same and all(v == 0 for v in w[0::4]) else 1)
sys.exit(0 if ok and same else 1)
