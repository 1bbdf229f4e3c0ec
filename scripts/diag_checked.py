"""Bounds-checked run (KN_CHECKED=1 loads _C_checked): today's new indexing paths -- steady
distributed steps with the own segment placed directly (loopback 4 ranks), global ids fused
into the bucket sort, the seeded exact kernel (K=64), query ranges, the adaptive local grid on a
clustered share -- then the per-file violation words (all zero = no out-of-range index)."""
import os
import sys

os.environ["KN_CHECKED"] = "1"
import torch

import cuda_knearests_amd as kn
from cuda_knearests_amd._ext import load
from cuda_knearests_amd.parallel import DistributedKNearests, run_loopback
from cuda_knearests_amd.utils import clustered_cloud, uniform_cloud

C = load()
assert "checked" in C.__name__, C.__name__
dev = torch.device("cuda", 0)
C.debug_words(True)
for gen in (uniform_cloud, clustered_cloud):
    cloud = gen(120000, seed=4)
    owner = torch.arange(cloud.size(0)) % 4

    def body(t):
        m = owner == t.rank
        ids = torch.nonzero(m).flatten().to(torch.int32).to(dev)
        dk = DistributedKNearests(k=16, transport=t, deterministic=False)
        for i in range(3):
            r = dk.solve(cloud[m].contiguous().to(dev), ids, async_=i > 0)
            r.valid()
        return r.stats

    print(gen.__name__, run_loopback(4, body)[0], flush=True)
p = uniform_cloud(300000, seed=5, device=dev)
m = kn.KNearests(k=64, device=dev).prepare(p).solve()
print("k64", m.info, flush=True)
ri, rd = m.solve_range(1000, 50000)
torch.cuda.synchronize()
w = C.debug_words(False)
print("debug words (build, query, route, tree):", w, flush=True)
sys.exit(0 if all(v == 0 for v in w[0::4]) else 1)
