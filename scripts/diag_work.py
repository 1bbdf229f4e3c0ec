"""Work statistics of the tile kernel from the checked build (_C_checked: per-chunk counters).
usage: python scripts/diag_work.py [n] [k]"""
import importlib
import json
import sys

import torch

from cuda_knearests_amd.ops import knn_ops as ops
from cuda_knearests_amd.utils import uniform_cloud

n = int(sys.argv[1]) if len(sys.argv) > 1 else 900000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
C = importlib.import_module("cuda_knearests_amd._C_checked")
dev = torch.device("cuda", 0)
pts = uniform_cloud(n, seed=0, device=dev)
plan = ops.Plan.auto(n, k)
s, cs, perm, geom = C.build(pts, plan.dims, True, None)
inf = float("inf")
out = C.query(s, cs, geom, plan.dims, k, n, None, [-inf, -inf, -inf, inf, inf, inf], plan.tile, plan.halo,
              plan.lds_capacity, True, True, 0)
torch.cuda.synchronize()
c = out[2].tolist()
res = {"n": n, "k": k, "plan": {"dims": plan.dims, "tile": plan.tile, "halo": plan.halo, "cap": plan.lds_capacity},
       "exact_path": c[0], "uncertified": c[1], "dense_tiles": c[2], "rescans": c[3], "rows": c[4],
       "cand": c[5], "ins": c[6], "chunks": c[7], "debug_words": C.debug_words(True)}
res["chunks_ideal"] = (n + 63) // 64
res["cand_per_chunk"] = c[5] / max(1, c[7])
res["rows_per_chunk"] = c[4] / max(1, c[7])
res["ins_per_cand"] = c[6] / max(1, c[5])
res["cand_per_query_lane"] = c[5] * 64 / n
print(json.dumps(res), flush=True)
