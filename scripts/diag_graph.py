"""Diagnostic: eager vs graph-replayed build+query, one sync per step with timing."""
import sys, time
import torch
import cuda_knearests_amd as kn
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

mode = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
plan = ops.Plan.auto(n, 16)
print(plan, flush=True)
if mode == "eager":
    for i in range(10):
        t = time.perf_counter()
        g = ops.build_grid(pts, 16, plan=plan)
        idx, d2, info = ops.query(g, 16, return_info=True)
        torch.cuda.synchronize()
        print(i, f"{(time.perf_counter()-t)*1e3:.3f} ms", info["counters"].tolist(), flush=True)
elif mode == "graph":
    static = pts.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = ops.build_grid(static, 16, plan=plan)
        ops.query(g, 16)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        g = ops.build_grid(static, 16, plan=plan)
        idx, d2, info = ops.query(g, 16, return_info=True)
    print("captured", flush=True)
    for i in range(10):
        t = time.perf_counter()
        graph.replay()
        torch.cuda.synchronize()
        print(i, f"{(time.perf_counter()-t)*1e3:.3f} ms", info["counters"].tolist(), flush=True)

if mode == "engine":
    e = kn.KNearests(k=16, device=dev)
    e.prepare(pts)
    e.solve()
    print("eager ok", e.info, flush=True)
    for i in range(12):
        t = time.perf_counter()
        e.step(pts, capture=True)
        if len(sys.argv) > 3:
            torch.cuda.synchronize()
        print(i, f"{(time.perf_counter()-t)*1e3:.3f} ms", flush=True)
    torch.cuda.synchronize()
    print("engine done", flush=True)
