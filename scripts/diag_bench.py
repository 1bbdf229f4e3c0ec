"""Replicates bench.run_single step by step with syncs + checked-build OOB reports."""
import os, sys, time
import torch
from cuda_knearests_amd import KNearests
from cuda_knearests_amd._ext import load
from cuda_knearests_amd.utils import uniform_cloud

C = load()
print("module", C.__name__, "checked", C.CHECKED, flush=True)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
pts = uniform_cloud(n, seed=0, device=dev)
kn = KNearests(k=16, device=dev)
kn.prepare(pts); kn.solve()
torch.cuda.synchronize()
print("eager", kn.info, C.debug_words(True), flush=True)
for i in range(2):
    kn.step(pts, capture=True)
torch.cuda.synchronize()
print("warmup", C.debug_words(True), flush=True)
for i in range(8):
    kn.step(pts, capture=True)
    torch.cuda.synchronize()
    print("step", i, C.debug_words(True), flush=True)
print("done", flush=True)
