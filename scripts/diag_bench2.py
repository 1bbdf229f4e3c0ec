"""bench.run_single flow; argv: n, setdev(0/1), sync_each_warmup(0/1)."""
import sys, time
import torch
from cuda_knearests_amd import KNearests
from cuda_knearests_amd.utils import uniform_cloud

n = int(sys.argv[1]); setdev = sys.argv[2] == "1"; sync_each = sys.argv[3] == "1"
dev = torch.device("cuda", 0)
if setdev:
    torch.cuda.set_device(dev)
pts = uniform_cloud(n, seed=0, device=dev)
kn = KNearests(k=16, device=dev)
kn.prepare(pts); kn.solve()
torch.cuda.synchronize()
print("eager", kn.info, flush=True)
for i in range(2):
    kn.step(pts, capture=True)
    if sync_each:
        torch.cuda.synchronize()
torch.cuda.synchronize()
print("warmup", flush=True)
for i in range(5):
    kn.step(pts, capture=True)
    torch.cuda.synchronize()
    print("step", i, flush=True)
print("done", flush=True)
