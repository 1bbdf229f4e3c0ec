"""In-process interleaved A/B of the tile query where the variant changes the PLAN (x halo, LDS
capacity): each module computes its own plan (auto_params) and queries with it. Rows must be
identical; counters[0] = exact-path queries.
usage: python scripts/ab_plan.py <variant> [n] [k] [rounds]"""
import importlib
import sys

import torch

from cuda_knearests_amd.utils import uniform_cloud

var = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 900000
k = int(sys.argv[3]) if len(sys.argv) > 3 else 16
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 10
mods = [importlib.import_module("cuda_knearests_amd._C"), importlib.import_module(f"cuda_knearests_amd._C_{var}")]
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
inf = float("inf")
runs = []
for M in mods:
    d = M.auto_params(n, k, 0.0, [], 0, None, 0)
    s, cs, perm, geom = M.build(pts, list(d["dims"]), True, None)
    args = (s, cs, geom, list(d["dims"]), k, n, None, [-inf, -inf, -inf, inf, inf, inf], list(d["tile"]), int(d["halo"]),
            int(d["lds_capacity"]), True, True, 0)
    out = M.query(*args, xsub=int(d["xsub"]))
    runs.append((M, args, int(d["xsub"]), out, d))
torch.cuda.synchronize()
a, b = runs[0][3], runs[1][3]
print("identical:", bool(torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])),
      "exact-path", int(a[2][0]), int(b[2][0]), "lds", runs[0][4]["lds_bytes"], runs[1][4]["lds_bytes"],
      "cap", runs[0][4]["lds_capacity"], runs[1][4]["lds_capacity"], flush=True)
ts = [[], []]
ev = lambda: torch.cuda.Event(enable_timing=True)
for r in range(rounds):
    order = (0, 1) if r % 2 == 0 else (1, 0)
    for i in order:
        M, args, xs, _, _ = runs[i]
        e0, e1 = ev(), ev()
        e0.record(); M.query(*args, xsub=xs); e1.record(); e1.synchronize()
        ts[i].append(e0.elapsed_time(e1))
for t in ts:
    t.sort()
print(f"baseline median {ts[0][len(ts[0]) // 2]:.4f} min {ts[0][0]:.4f} | {var} median {ts[1][len(ts[1]) // 2]:.4f} "
      f"min {ts[1][0]:.4f} ms", flush=True)
