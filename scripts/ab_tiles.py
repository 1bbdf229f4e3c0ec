"""In-process interleaved A/B of tile plans on the pipelined engine step (900K uniform): configs =
(extension suffix, tile hint in cells). Variant extensions come from
cuda_knearests_amd._build.build_variant(name, flags) (round 4: -DKN_TILE_WG=512, since removed,
and -DKN_TOPK_MARGIN=1; profiles/ab_r4_tiles_margin.txt). Rows must equal the baseline's.
usage: python scripts/ab_tiles.py [n] [k] [rounds] [steps] [variants]
variants: comma-separated extension suffixes ("base" = _C), optionally with a tile hint
("base@4x4x8"; none = the auto plan), replacing the built-in configs (e.g. "base,_op3")."""
import importlib
import sys
import time

import torch

from cuda_knearests_amd.utils import uniform_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 100
configs = [("", [0, 0, 0]), ("_wg512", [4, 4, 8]), ("_wg512", [4, 8, 4]), ("_wg512", [0, 0, 0]), ("", [4, 4, 8]),
           ("_wg512", [8, 4, 4]), ("_m1", [0, 0, 0]), ("_wg512m1", [4, 4, 8])]
if len(sys.argv) > 5:
    # "<suffix>[@TXxTYxTZ]": e.g. "base,base@4x4x8,_op3"
    def _cfg(v):
        suf, _, t = v.partition("@")
        return ("" if suf == "base" else suf, [int(x) for x in t.split("x")] if t else [0, 0, 0])
    configs = [_cfg(v) for v in sys.argv[5].split(",")]
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
engines = []
ref = None
for suf, tile in configs:
    try:
        C = importlib.import_module("cuda_knearests_amd._C" + suf)
    except ImportError as e:
        print("skip", suf, e, flush=True)
        continue
    e = C.Engine(k, 0.0, tile, 0, False, True, True, 0, True, 0)
    e.prepare(pts)
    e.solve()
    i, d = e.results(dev)
    same = True if ref is None else (torch.equal(i, ref[0]) and torch.equal(d, ref[1]))
    if ref is None:
        ref = (i, d)
    e.launch_pipelined(20, -1)
    e.sync()
    engines.append((f"{suf or 'base'} tile {tile} dims {e.info()['dims']}", e, same, []))
    print(engines[-1][0], "identical", same, "counters", e.counters(), flush=True)
for r in range(rounds):
    for name, e, same, acc in engines:
        e.sync()
        t0 = time.perf_counter()
        e.launch_pipelined(steps, -1)
        e.sync()
        acc.append((time.perf_counter() - t0) * 1e3 / steps)
for name, e, same, acc in engines:
    acc.sort()
    print(f"{name}: median {acc[len(acc) // 2]:.4f} min {acc[0]:.4f} ms/step identical {same}", flush=True)
