"""Pipelined-step sweep of the query tile shape and grid density under the round-5 pipeline
(two query streams, three grid sets): C.Engine(k, points_per_cell, tile) on a 900K uniform cloud,
W untimed + K timed launch_pipelined steps, two interleaved passes. Rows are checked against the
default plan's rows. usage: python scripts/tile_sweep.py K [N [small]] (N points, default 900000)"""
import sys
import time

import torch

from cuda_knearests_amd._ext import load
from cuda_knearests_amd.utils import uniform_cloud

C = load()
k = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda", 0)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 900000
pts = uniform_cloud(n, seed=0, device=dev)
configs = [(0.0, []), (0.0, [8, 4, 4]), (0.0, [4, 8, 4]), (0.0, [4, 4, 8]), (0.0, [8, 8, 4]), (0.0, [2, 4, 4]),
           (2.9, []), (4.0, [])]
if len(sys.argv) > 3 and sys.argv[3] == "small":  # tile shapes for clouds of < ~1 launch round of 4^3 tiles
    configs = [(0.0, []), (0.0, [2, 4, 4]), (0.0, [4, 2, 4]), (0.0, [2, 2, 4]), (0.0, [2, 2, 2])]
ref = None
res = {}
for rnd in range(2):
    for ppc, tile in configs:
        e = C.Engine(k, ppc, tile)
        e.prepare(pts)
        e.launch_pipelined(60, -1)
        e.sync()
        t0 = time.perf_counter()
        e.launch_pipelined(200, -1)
        e.sync()
        ms = (time.perf_counter() - t0) * 1e3 / 200
        idx, d2 = e.results(dev)
        if ref is None:
            ref = (idx.clone(), d2.clone())
        same = bool(torch.equal(d2, ref[1]))
        res.setdefault((ppc, tuple(tile)), []).append(ms)
        info = e.info()
        print(f"n={n} k={k} ppc={ppc} tile={tile} grid={info.get('dims')} plan_tile={info.get('tile')} "
              f"lds={info.get('lds_bytes')} ms={ms:.4f} d2_equal={same}", flush=True)
        del e
for key, v in res.items():
    print(f"n={n} K={k} summary", key, " ".join(f"{x:.4f}" for x in v))
