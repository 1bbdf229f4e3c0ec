"""Query-kernel time vs cloud size and plan (small-cloud diagnosis).
usage: python scripts/diag_small.py  -> one JSON line per (cloud, k, tile)"""
import json, os, sys, torch
import cuda_knearests_amd as kn
from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import dataset, uniform_cloud
from cuda_knearests_amd import read_xyz

dev = torch.device("cuda", 0)
C = ops.load()
clouds = {"pts20K": read_xyz(str(dataset("pts20K.xyz")), normalize=True).float().to(dev)}
for n in (20000, 100000, 300000, 900000):
    clouds[f"u{n}"] = uniform_cloud(n, seed=0, device=dev)
inf = float("inf")
for name, pts in clouds.items():
    n = pts.size(0)
    for k in (8, 16, 50):
        base = ops.Plan.auto(n, k)
        tiles = [None] if os.environ.get("KN_DIAG_TILES") is None else [None, [1, 1, 1], [2, 2, 2], [4, 4, 4]]
        for t in tiles:
            plan = base if t is None else ops.Plan.auto(n, k, tile=t)
            g = kn.build_grid(pts, k, plan=plan)
            for _ in range(3):
                idx, d2, info = kn.query(g, k, return_info=True)
            if n <= 100000:  # exact against the kd-tree oracle
                _, od = kn.knn_cpu(pts.cpu(), k, "kdtree")
                assert torch.equal(d2.cpu(), od), (name, k)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                kn.query(g, k)
            e1.record()
            e1.synchronize()
            print(json.dumps({"qgroup": os.environ.get("KN_QGROUP", "auto"), "cloud": name, "n": n, "k": k, "dims": plan.dims, "tile": plan.tile, "halo": plan.halo,
                              "lds_capacity": plan.lds_capacity, "ms_query": e0.elapsed_time(e1) / 20,
                              "counters": info["counters"].cpu().tolist()}), flush=True)
