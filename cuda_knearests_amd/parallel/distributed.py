"""Multi-GPU k-nearest neighbours: spatial split + halo exchange over RCCL (NEW component).

One process per GPU, ``torch.distributed`` with backend ``"nccl"`` (= RCCL over xGMI on
ROCm) or ``"gloo"`` (CPU ranks, used by the tests). Per solve:

1. global domain: one all-reduce of the local bounding boxes (min/max packed in 6 floats);
2. redistribution: every point goes to the rank whose box contains it -- ONE
   ``all_to_all_single`` of packed float4 {x, y, z, bits(global id)} rows (counts first);
3. halo: each owned point within ``h`` of another rank's box is sent to that rank -- ONE
   more ``all_to_all_single``. ``h`` starts at ``halo_factor`` x the expected K-th neighbour
   radius of the cloud;
4. local solve on owned + halo points (GPU: the LDS-tiled HIP kernel; CPU: native grid
   solver), queries = owned points, ids remapped to global ids on the device, certification
   against the rank's *complete box* (own box grown by h, unbounded at the domain boundary);
5. if any rank has an uncertified query (its K-th distance leaves the complete box) the halo
   is doubled and steps 3-4 are repeated (an all-reduce decides; rare).

Messages are few and large (two all-to-alls per solve): xGMI is point-to-point, so one
all-to-all-v of the whole payload keeps all 7 links of a 2x2x2 decomposition busy at once.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import knn_ops as ops
from .decomposition import SpatialDecomposition

INF = math.inf


def _pack(points: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    return torch.cat([points, ids.to(torch.int32).view(torch.float32).unsqueeze(1)], 1)


def _unpack(rows: torch.Tensor):
    return rows[:, :3].contiguous(), rows[:, 3].contiguous().view(torch.int32)


@dataclass
class DistResult:
    ids: torch.Tensor        # (n_owned,) global ids of this rank's query points
    neighbors: torch.Tensor  # (n_owned, k) global ids (-1 = empty)
    d2: torch.Tensor         # (n_owned, k) squared distances
    stats: dict


class DistributedKNearests:
    def __init__(self, k: int = 16, group=None, halo_factor: float = 1.6, points_per_cell: float = 0.0,
                 deterministic: bool = True, max_rounds: int = 8):
        self.k = int(k)
        self.group = group
        self.halo_factor = float(halo_factor)
        self.points_per_cell = float(points_per_cell)
        self.deterministic = deterministic
        self.max_rounds = max_rounds
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    # ------------------------------------------------------------------ helpers ------
    def _a2a(self, send: torch.Tensor, send_counts: list, recv_counts: list) -> torch.Tensor:
        out = send.new_empty((sum(recv_counts),) + tuple(send.shape[1:]))
        dist.all_to_all_single(out, send, recv_counts, send_counts, group=self.group)
        return out

    def _counts(self, send_counts: torch.Tensor) -> list:
        recv = torch.empty_like(send_counts)
        dist.all_to_all_single(recv, send_counts, group=self.group)
        return recv.tolist()

    def domain(self, points: torch.Tensor):
        if points.numel():
            lo, hi = points.min(0).values, points.max(0).values
        else:
            lo = torch.full((3,), INF, device=points.device)
            hi = torch.full((3,), -INF, device=points.device)
        v = torch.cat([-lo, hi]).float()
        dist.all_reduce(v, op=dist.ReduceOp.MAX, group=self.group)
        v = v.tolist()
        lo = tuple(-x for x in v[:3])
        hi = tuple(v[3:])
        return lo, hi

    # ------------------------------------------------------------------- phases ------
    def redistribute(self, dec: SpatialDecomposition, points: torch.Tensor, ids: torch.Tensor):
        owner = dec.owner(points)
        order = torch.argsort(owner, stable=True)
        counts = torch.bincount(owner, minlength=self.world)
        rows = _pack(points, ids)[order]
        recv = self._counts(counts)
        got = self._a2a(rows, counts.tolist(), recv)
        return _unpack(got)

    def halo(self, dec: SpatialDecomposition, points: torch.Tensor, ids: torch.Tensor, h: float):
        sel, counts = [], []
        h2 = h * h
        for r in range(self.world):
            if r == self.rank:
                counts.append(0)
                continue
            m = torch.nonzero(dec.box_dist2(points, r) <= h2).squeeze(1)
            sel.append(m)
            counts.append(int(m.numel()))
        idx = torch.cat(sel) if sel else torch.empty(0, dtype=torch.long, device=points.device)
        rows = _pack(points, ids)[idx]
        recv = self._counts(torch.tensor(counts, dtype=torch.long, device=points.device))
        got = self._a2a(rows, counts, recv)
        return _unpack(got)

    def local_solve(self, pts: torch.Tensor, gids: torch.Tensor, n_owned: int, complete: list):
        if pts.is_cuda:
            g = ops.build_grid(pts, self.k, points_per_cell=self.points_per_cell,
                               deterministic=self.deterministic)
            idx, d2, info = ops.query(g, self.k, n_queries=n_owned, id_map=gids, complete=complete,
                                      return_info=True)
            n_unc = int(info["counters"][1].item())
            return idx, d2, n_unc
        idx, d2, unc = ops.knn_cpu(pts, self.k, "grid", n_queries=n_owned, complete=complete,
                                   points_per_cell=self.points_per_cell)
        gl = gids.long()
        mapped = torch.where(idx >= 0, gl[idx.clamp(min=0).long()], torch.full_like(gl[:1], -1)).to(torch.int32)
        return mapped, d2, int(unc.numel())

    # -------------------------------------------------------------------- solve ------
    def solve(self, points: torch.Tensor, ids: Optional[torch.Tensor] = None,
              partitioned: bool = False, domain=None) -> DistResult:
        """kNN of the distributed cloud. ``points``: this rank's (N_r, 3) float32 share (any
        distribution; ``partitioned=True`` promises they already lie in this rank's box).
        ``ids``: their global ids (int32); default = rank offset + arange."""
        points = points.contiguous().float()
        dev = points.device
        if ids is None:
            n_all = torch.tensor([points.size(0)], dtype=torch.long, device=dev)
            sizes = [torch.zeros_like(n_all) for _ in range(self.world)]
            dist.all_gather(sizes, n_all, group=self.group)
            off = int(sum(int(s.item()) for s in sizes[: self.rank]))
            ids = torch.arange(off, off + points.size(0), dtype=torch.int32, device=dev)
        lo, hi = domain if domain is not None else self.domain(points)
        dec = SpatialDecomposition(self.world, lo, hi)
        if partitioned:
            own_pts, own_ids = points, ids.to(torch.int32)
        else:
            own_pts, own_ids = self.redistribute(dec, points, ids)
        n_owned = own_pts.size(0)
        n_tot = torch.tensor([n_owned], dtype=torch.long, device=dev)
        dist.all_reduce(n_tot, group=self.group)
        vol = max(1e-30, (hi[0] - lo[0]) * (hi[1] - lo[1]) * (hi[2] - lo[2]))
        h = self.halo_factor * ops.expected_kth_radius(int(n_tot.item()), self.k, vol)
        diag = math.sqrt(sum((hi[a] - lo[a]) ** 2 for a in range(3)))
        rounds = 0
        while True:
            rounds += 1
            hp, hid = self.halo(dec, own_pts, own_ids, h)
            pts = torch.cat([own_pts, hp])
            gids = torch.cat([own_ids, hid])
            complete = dec.complete_box(self.rank, h) if h < diag else [-INF] * 3 + [INF] * 3
            idx, d2, n_unc = self.local_solve(pts, gids, n_owned, complete)
            flag = torch.tensor([n_unc], dtype=torch.long, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
            if int(flag.item()) == 0 or h >= diag or rounds >= self.max_rounds:
                break
            h *= 2.0
        stats = {"n_owned": n_owned, "n_halo": int(hp.size(0)), "halo_width": h, "rounds": rounds,
                 "grid": dec.grid}
        return DistResult(own_ids, idx, d2, stats)
