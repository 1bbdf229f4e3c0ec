"""Diagnostics of kn::DistPipeline in loopback mode (one GPU): W virtual ranks, partitioned
uniform or clustered shares; prints each rank's local flag and whether its rows equal the torch
path's steady step. usage: python scripts/diag_loopback_pipe.py W uniform|clustered FIELD_G
(run with KN_ROUTE_FUSED=0/1 to compare the steady routers)."""
import sys

import torch

from cuda_knearests_amd._ext import load
from cuda_knearests_amd.parallel import DistributedKNearests, SpatialDecomposition, run_loopback
from cuda_knearests_amd.utils import clustered_cloud, uniform_cloud

world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
gen = sys.argv[2] if len(sys.argv) > 2 else "uniform"
fg = int(sys.argv[3]) if len(sys.argv) > 3 else 64
C = load()
cuda = torch.device("cuda", 0)
n = 60000
if gen == "uniform":
    shares = []
    for r in range(world):
        blo, bhi = SpatialDecomposition(world, (0.0,) * 3, (1000.0,) * 3).rank_box(r)
        u = uniform_cloud(n, seed=400 + r, device=cuda, lo=0.0, hi=1.0)
        shares.append((u * torch.tensor([bhi[a] - blo[a] for a in range(3)], device=cuda)
                       + torch.tensor(blo, device=cuda)).contiguous())
else:
    shares = [c.contiguous() for c in clustered_cloud(n * world, seed=77).to(cuda).chunk(world)]


def body(t):
    dk = DistributedKNearests(k=16, transport=t, halo_field=fg)
    r1 = dk.solve(shares[t.rank])
    for _ in range(6):
        r1 = dk.solve(shares[t.rank])
        if r1.stats.get("steady"):
            break
    # the torch steady path by hand (distributed.py _steady_body, world > 1): its query counters
    st = dk._steady
    pts_in = shares[t.rank]
    totals, send, partials, lpts, lgids = C.route_steady(pts_in, None, st["plan"], world, st["cap"], t.rank,
                                                         st["place"])
    recv = dk._a2a(send[:st["x"]], st["cross_send"], st["cross_recv"])
    _, _, _, _, counters, *_ = C.dist_local(recv, send[:0], st["recv_own"], st["recv_halo"], t.rank,
                                            list(st["grid"]), st["hdr"], dk.k, dk.points_per_cell, dk.deterministic,
                                            st["exact_grid"], False, st["dims"], lpts, lgids, st["use_tree"],
                                            field_cert=st.get("field_cert"))
    stats = dict(r1.stats)
    stats["torch_counters"] = counters[:8].tolist()
    stats["valid"] = r1.valid()
    return dk._steady, r1.ids.clone(), r1.neighbors.clone(), r1.d2.clone(), stats


out = run_loopback(world, body)
pipes = []
for r, (st, _, _, _, _) in enumerate(out):
    pipes.append(C.DistPipe(None, shares[r], None, st["plan"], st["metas"], [int(v) for v in st["tot"].tolist()],
                            [float(v) for v in st["hdr"]], list(st["grid"]), list(st["dims"]), list(st["recv_own"]),
                            list(st["recv_halo"]), list(st["cross_send"]), list(st["cross_recv"]), list(st["place"]),
                            int(st["cap"]), 16, 0.0, True, int(st["exact_grid"]), int(st["use_tree"]), False,
                            [world, r], st.get("field"), st.get("field_cert")))
for p in pipes:
    p.loopback_stage(0)
for r in range(world):
    for d in range(world):
        m = out[r][0]["cross_send"][d]
        if d != r and m:
            pipes[d].recv_view(r, m).copy_(pipes[r].send_view(d, m))
torch.cuda.synchronize()
for p in pipes:
    p.loopback_stage(1)
for r, (st, ids, nb, d2, stats) in enumerate(out):
    g, i, d = pipes[r].outputs(0)
    print(f"rank {r}: flag {pipes[r].flag_local()} field {st.get('field') is not None} tot {st['tot'].tolist()} "
          f"rows equal {torch.equal(g, ids) and torch.equal(i, nb) and torch.equal(d, d2)} "
          f"halo {stats.get('n_halo')} width {stats.get('halo_width'):.3f} words {pipes[r].debug_words()} torch {stats['torch_counters']} valid {stats['valid']}", flush=True)
