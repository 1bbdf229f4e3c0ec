"""In-process interleaved A/B of tree-path kernel variants on the native engine (900K clustered /
surface, K=16; AB_K=k for another K): configs = extension suffixes built by
cuda_knearests_amd._build.build_variant. Rows must equal the baseline's.
usage: python scripts/ab_tree.py suffix[,suffix...] [rounds] [steps]"""
import os
import importlib
import sys
import time

import torch

from cuda_knearests_amd.utils import clustered_cloud, surface_cloud

sufs = [""] + [s for s in (sys.argv[1].split(",") if len(sys.argv) > 1 else []) if s]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
dev = torch.device("cuda", 0)
for gen, fn in (("clustered", clustered_cloud), ("surface", surface_cloud)):
    pts = fn(900000, seed=0, device=dev)
    engines, ref = [], None
    for suf in sufs:
        C = importlib.import_module("cuda_knearests_amd._C" + suf)
        e = C.Engine(int(os.environ.get("AB_K", "16")))
        e.prepare(pts)
        e.solve()
        i, d = e.results(dev)
        same = True if ref is None else (torch.equal(i, ref[0]) and torch.equal(d, ref[1]))
        if ref is None:
            ref = (i.clone(), d.clone())
        e.launch_pipelined(20, -1)
        e.sync()
        engines.append((suf or "base", e, same, [], e.counters()))
    for _ in range(rounds):
        for name, e, same, acc, _c in engines:
            e.sync()
            t0 = time.perf_counter()
            e.launch_pipelined(steps, -1)
            e.sync()
            acc.append((time.perf_counter() - t0) * 1e3 / steps)
    for name, e, same, acc, cnt in engines:
        acc.sort()
        print(f"{gen} {name}: median {acc[len(acc) // 2]:.4f} min {acc[0]:.4f} ms/step identical {same} "
              f"counters {cnt}", flush=True)
