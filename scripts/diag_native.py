"""Native Engine (own arena, own stream, hipGraph) replay diagnostic."""
import sys, time
import torch
from cuda_knearests_amd._ext import load
from cuda_knearests_amd.utils import uniform_cloud
import cuda_knearests_amd as kn

C = load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
dev = torch.device("cuda", 0)
if len(sys.argv) > 2 and sys.argv[2] == "setdev":
    torch.cuda.set_device(dev)
pts = uniform_cloud(n, seed=0, device=dev)
e = C.Engine(16)
e.prepare(pts)
e.solve()
i0, d0 = e.results(dev)
print("eager", e.info(), e.counters(), flush=True)
e.launch_graph(2)
e.sync()
print("warmup ok", flush=True)
for it in range(5):
    t = time.perf_counter()
    e.launch_graph(10)
    e.sync()
    print(it, f"{(time.perf_counter() - t) * 100:.4f} ms/iter", flush=True)
i1, d1 = e.results(dev)
print("same as eager:", torch.equal(i0, i1), torch.equal(d0, d1), flush=True)
ri, rd = kn.knn(pts, 16)
print("same as torch ops:", torch.equal(ri, i1), torch.equal(rd, d1), flush=True)
