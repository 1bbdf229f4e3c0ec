"""Multi-GPU k-nearest neighbours: spatial split + ONE routing all-to-all over RCCL (NEW component).

The reference is single-GPU (knearests.cu has no streams, devices or collectives).
Here: one process per GPU, ``torch.distributed`` with backend ``"nccl"`` (= RCCL over xGMI on
ROCm) or ``"gloo"`` (CPU ranks, used by the tests). DESIGN.md §5 has the full picture.

Full (validating) step, GPU ranks:
1. **meta + plan** -- the local bbox/count is all-gathered (speculatively: the previous step's
   metas plan the routing and this step's metas travel with the counts in one all-gather);
   ``route_begin`` computes on the device the global domain, the halo width ``h`` (halo_factor x
   the expected K-th neighbour radius), the rank boxes (count-balanced kd splits by default) and
   routes every point to its OWNER and, as HALO copies, to every rank whose box is within ``h``.
   One host sync reads the split sizes.
2. **route** -- one ``all_to_all_single`` of float4 rows {x, y, z, bits(global id)} (self-last
   layout: the rank's own rows never enter the collective).
3. **local solve** (``dist_local``) -- occupancy-adaptive local grid over the rank's box + halo,
   owned points are the queries, global ids written by the build; the grid kernels, or the tree
   path when the local grid had to be refined; every query certified against the rank's
   *complete box* (own box grown by h, unbounded on domain faces).
4. **forwarding round** (rare) -- uncertified queries go to the ranks within their K-th distance
   and are answered there (exact in one round).

Steady state (after a validated single-round step): no host synchronisation at all -- cached
plan, the own segment placed straight into the local rows, an on-device check of the step's
assumptions all-reduced into a flag that is read asynchronously (``DistResult.valid``).
xGMI is point-to-point: with 2x2x2 ranks every rank neighbours all 7 others, so the single
all-to-all keeps all 7 links busy at once.
"""
from __future__ import annotations

import collections
import math
import time
from dataclasses import dataclass
from typing import Optional

import torch

from ..ops import knn_ops as ops
from .decomposition import SpatialDecomposition, balanced_splits, factor3
from ..utils import get_logger
from .transport import CollectiveError, HostStagedTransport, TorchDistTransport

_log = get_logger("knearests.dist")

INF = math.inf
HDR = 24  # doubles in the device plan header (kn::kPlanHdr, csrc/include/kn/route.h)
META_I32 = 16  # one rank's meta (8 float64) as int32 words


def _pack(points: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    return torch.cat([points, ids.to(torch.int32).view(torch.float32).unsqueeze(1)], 1)


def _unpack(rows: torch.Tensor):
    return rows[:, :3].contiguous(), rows[:, 3].contiguous().view(torch.int32)


def halo_send_width(h: float, lo, hi) -> float:
    """Halo width used for SENDING: h plus a slack far above fp32 rounding of the box / distance
    arithmetic, so every point the receiver's certification (which uses h) relies on is sent."""
    scale = max(max(abs(v) for v in lo), max(abs(v) for v in hi), max(hi[a] - lo[a] for a in range(3)))
    return h * (1.0 + 1e-5) + 1e-5 * scale


def route_rows_torch(dec: SpatialDecomposition, points: torch.Tensor, ids: torch.Tensor, h_send: float,
                     h_inner: Optional[float] = None, wz: float = INF):
    """Reference router (any device): send rows [owned | halo] per destination + (world, 2) counts.
    Same decisions and same stable order as the native router (route.hip). Position-dependent
    halo: points farther than ``wz`` from every domain face use the interior width ``h_inner``."""
    owner = dec.owner(points)
    rows = _pack(points, ids)
    dev = points.device
    hf = torch.tensor(h_send, dtype=torch.float32, device=dev)
    h2 = hf * hf  # fp32 square, as the native router computes it
    if h_inner is not None and h_inner != h_send:
        hif = torch.tensor(h_inner, dtype=torch.float32, device=dev)
        lo_t = torch.tensor(dec.lo, dtype=torch.float32, device=dev)
        hi_t = torch.tensor(dec.hi, dtype=torch.float32, device=dev)
        zp = torch.minimum((points - lo_t).min(1).values, (hi_t - points).min(1).values)
        h2 = torch.where(zp <= torch.tensor(wz, dtype=torch.float32, device=dev), h2, hif * hif)
    parts, counts = [], []
    for d in range(dec.world):
        own_m = owner == d
        halo_m = (~own_m) & (dec.box_dist2(points, d) <= h2)
        parts += [rows[own_m], rows[halo_m]]
        counts.append([int(own_m.sum()), int(halo_m.sum())])
    send = torch.cat(parts) if parts else rows[:0]
    return send, torch.tensor(counts, dtype=torch.int32, device=points.device)


@dataclass
class DistResult:
    ids: torch.Tensor        # (n_owned,) global ids of this rank's query points
    neighbors: torch.Tensor  # (n_owned, k) global ids (-1 = empty)
    d2: torch.Tensor         # (n_owned, k) squared distances
    stats: dict
    # steady-state (sync-free) steps: a device flag, copied to pinned host memory at the end of
    # the step. Non-zero: the step's routing assumption (previous step's metas and counts) did not
    # hold on some rank, or some query was not certified -- the rows must not be used.
    flag: Optional[torch.Tensor] = None
    event: Optional[object] = None
    # native pipelined steps (kn::DistPipeline): waits for the step (polling RCCL's async error
    # under a deadline) and returns True when its sticky flag is clear; keeps the pipeline (whose
    # buffers the rows view) alive
    waiter: Optional[object] = None

    def valid(self) -> bool:
        """True when the rows are final (waits for the step's flag; no-op for synchronous steps).
        Reading it never changes the solver's state: which path the next step takes is decided
        inside solve() from the flags of earlier steps, identically on every rank."""
        if self.waiter is not None:
            return bool(self.waiter())
        if self.flag is None:
            return True
        if self.event is not None:
            self.event.synchronize()
        return int(self.flag.item()) == 0


class DistributedKNearests:
    # halo_factor: h = halo_factor x the cloud's mean K-th neighbour radius. Queries on an edge of
    # the global domain see a quarter ball (radius x 4^(1/3) ~ 1.59); at 1.6 a 100M / 8-rank run
    # needed a growth round (profiles/bench_suite_r1.jsonl). 2.5 keeps even those at a Poisson
    # tail ~1e-13 per query for +4 % halo points per rank.
    def __init__(self, k: int = 16, group=None, halo_factor: float = 2.5, points_per_cell: float = 0.0,
                 deterministic: bool = True, max_rounds: int = 8, native_route: Optional[bool] = None,
                 transport=None, device_plan: bool = True, timeout_s: Optional[float] = None,
                 balance: str = "count", adaptive: bool = True, native_pipeline: Optional[bool] = None,
                 force_collectives: Optional[bool] = None, inner_halo: Optional[float] = None,
                 halo_field: Optional[int] = None):
        self.k = int(k)
        # occupancy-adaptive local grids (GPU): a rank whose share is clustered re-bins finer, as
        # the 1-GPU engine does; steady steps reuse the validated step's grid (no extra sync)
        self.adaptive = bool(adaptive)
        if balance not in ("count", "volume"):
            raise ValueError("balance must be 'count' or 'volume'")
        # rank boxes: "count" = kd splits at global quantiles (every rank ~N/world points, also
        # for clustered clouds), "volume" = equal-volume slices of the domain
        self.balance = balance
        self.group = group
        self.halo_factor = float(halo_factor)
        # Position-dependent halo (round 4): points farther than w = h_e + h_i from every face of
        # the global domain are routed with the interior width h_i = min(h_e, inner x radius) --
        # an interior query's K-th ball is whole, while a query near a domain face sees a truncated
        # one (radius x 4^(1/3) at an edge), which the edge width h_e = halo_factor x radius covers.
        # None: the K-dependent Poisson-tail factor (C.inner_halo_factor: K=16 -> 1.55); 0: one width.
        self.inner_halo = inner_halo
        self.points_per_cell = float(points_per_cell)
        self.deterministic = deterministic
        self.max_rounds = max_rounds
        self.native_route = native_route  # None: native router on GPU tensors, torch router on CPU
        # timeout_s: failure detection -- a collective that fails or does not complete in time
        # raises CollectiveError on this rank instead of hanging (transport.py)
        self.comm = transport if transport is not None else TorchDistTransport(group, timeout_s=timeout_s)
        self.rank = self.comm.rank
        self.world = self.comm.world
        self.device_plan = device_plan  # GPU: plan the routing on the device (1 host sync, not 2)
        self._grid = None
        self._send_cap = 0  # send-buffer rows of the native path (grows to the largest step seen)
        self.send_headroom = 0.25  # first-step send buffer: (1 + headroom) x local points
        self.host_marks = None  # list -> (stage, perf_counter) marks of the native step (profiling)
        # Speculative routing (world > 1): plan with the previous step's gathered metas and
        # exchange {this step's meta, counts} in ONE all-gather instead of an all-gather of the
        # metas followed by an all-to-all of the counts. Checked exactly on the host: if any
        # rank's meta changed, the step re-plans with the new metas (one extra round trip).
        self.speculative = True
        self._spec = None  # (metas on device, metas on host (world, 8) f64, grid, kd splits or None)
        # Steady state (no host synchronisation at all): once a full step has been validated, the
        # next steps assume the same metas and counts, enqueue everything with the known split
        # sizes, and verify the assumption ON THE DEVICE (own meta and send counts unchanged, no
        # uncertified query); the per-step flag is all-reduced and copied back asynchronously
        # (DistResult.valid). A failed assumption costs one re-run of that step the full way.
        self.steady = True
        self._steady = None
        # uncertified queries: forward just those queries to the ranks within their K-th distance
        # (one targeted round) instead of re-routing everything with a doubled halo
        self.forward = True
        # Steady steps forward on the device (fixed slots per rank pair, two equal-split
        # all-to-alls, no host sync) once the validated step needed forwarding; with a halo wide
        # enough that no query is uncertified (uniform clouds at the default factor) they skip the
        # two extra collectives, and a rare uncertified query fails the step's flag instead.
        # Slots per rank pair: twice the validated step's forwarded total (all ranks; a bound on
        # every pair's count), a power of two in [256, fwd_slots_max]; more than that and the
        # steady state is not entered. An overflowing steady step fails its flag.
        self.fwd_slots_max = 65536
        # Adaptive halo: a validated step that needed forwarding widens the halo for the next
        # full step (x1.6, up to halo_boost_max) instead of entering the steady state with device
        # forwarding -- a forwarded query costs one wave of the exact kernel on the destination's
        # grid every step (8x900K clustered loopback: 72 ms/step forwarding ~600 queries at halo
        # 2.5 vs 17.6 ms with a 4.0 halo and none; uniform at 1.3: 10.1 vs 4.8 ms at 2.5). The
        # boost is collective (n_fwd is all-reduced), kept across steps.
        self.halo_boost = 1.0
        self.halo_boost_max = 4.0
        self.boost_decay_after = 2  # clean validated full steps in a row before the boost decays
        self._boost_clean = 0
        # hipGraph replay of the steady step (torch.cuda.CUDAGraph): the default at world 1 (round
        # 3; no collective inside the captured step), opt-in above (KN_DIST_GRAPH=1 or
        # graph_steady = True: capturing RCCL collectives cannot be exercised on a one-GPU box);
        # KN_DIST_GRAPH=0 / graph_steady = False turn it off. Replayed rows live in the graph's
        # static buffers until the next solve (read-only: at world 1 `ids` of an async replayed
        # step is the caller's id tensor or the cached 0..n-1 table; synchronous calls return
        # copies). At world 1 200 back-to-back replays are valid and
        # bit-identical to the eager steady step on the release and the bounds-checked builds, host
        # enqueue 0.14 -> 0.06 ms per step (profiles/ab_r2_dist_graph.txt). The world-1 steady
        # step skips the routing passes (the share is the local set), reads the caller's input in
        # place and copies its flag out inside the graph (one graph launch per step, no stream op
        # between replays; profiles/bench_r3_dist_world1.txt).
        self.graph_steady = None
        self._graph = None
        # Native pipelined steady steps (round 4, csrc/runtime/dist.hpp): the rank's own RCCL
        # communicator, route + exchange + build of step i+1 on a second stream while step i
        # queries, the flag's all-reduce after it -- all hipGraph-replayed (the 1-GPU pipelined
        # step plus the communication). Default on GPU ranks over torch.distributed "nccl" whenever
        # the steady plan needs no device forwarding; KN_DIST_PIPE=0 / native_pipeline=False: the
        # torch path above. force_collectives (KN_DIST_FORCE_COLLECTIVES=1): at world 1 the rank's
        # own rows also travel through RCCL (self send / recv + unpack), exercising the exchange
        # of world > 1 on one GPU.
        import os

        self.native_pipeline = native_pipeline
        if force_collectives is None:
            force_collectives = os.environ.get("KN_DIST_FORCE_COLLECTIVES") == "1"
        self.force_collectives = bool(force_collectives)
        self.pipe_unroll = int(os.environ.get("KN_DIST_UNROLL", "10"))  # steps per graph in run_steps
        # Density-adaptive halo field (round 4, GPU ranks on the native router, world > 1): after a
        # full step routed with the global widths, every owned query whose K-th ball leaves its own
        # box raises the send width of the field cells within a few cells of it to its K-th
        # distance (C.field_splat; the ranks' fields are MAX-all-reduced). The next full step routes
        # each point with its cell's width and certifies a query when its K-th distance is within
        # the radius the field guarantees at its cell (C.field_cert) or its ball stays in its own
        # box; that step becomes the steady plan. Widths follow the measured distances, so dense
        # clusters cut by a rank boundary ship a thin halo and sparse regions a wide one (CPU study
        # of 8 x 900K, scripts/halo_study.py: clustered 30 % -> 8.8 %, uniform 12.8 % -> 6.2 %
        # halo rows at G = 64). A field step that still forwards queries splats again (max-merged);
        # after three such steps the field is dropped for the global widths, and so is a field whose
        # halo is not smaller than the global widths' (sparse outliers force coarse cells: small
        # clustered clouds). The steady state thus starts after the second full step. halo_field_g: cells per axis (halo_field, else
        # KN_HALO_FIELD_G, default 64; 0 disables).
        self.halo_field_g = int(os.environ.get("KN_HALO_FIELD_G", "64")) if halo_field is None else int(halo_field)
        self._field = None  # the width field (G^3 float32 on the device) of the next full step
        self._field_retries = 0
        self._field_ref_halo = 0  # halo rows (all ranks) of the last full step with the global widths
        self.wait_timeout_s = float(timeout_s) if timeout_s else 300.0
        self._rcomm = None
        self._pipe = None
        self.pipe_mode = None  # "graph" / "eager": how the native pipeline runs (set when built)
        # asynchronous steady results not yet checked by the solver. Before the next steady step
        # all but the newest are checked (their steps are long done, so this rarely waits, and it
        # bounds the host's lead to ~2 steps): an invalid one drops the steady plan. The flags
        # are all-reduced and every rank checks the same steps at the same call, so all ranks
        # take the same path (a caller's own valid() calls decide nothing).
        self._pending = collections.deque()

    # ------------------------------------------------------------------ helpers ------
    def _inner_factor(self) -> float:
        """Interior halo factor of the current step (x the adaptive boost), 0 = one width."""
        if self.inner_halo is not None:
            return float(self.inner_halo) * self.halo_boost
        return float(ops.load().inner_halo_factor(self.k)) * self.halo_boost

    def _a2a(self, send: torch.Tensor, send_counts: list, recv_counts: list) -> torch.Tensor:
        out = send.new_empty((sum(recv_counts),) + tuple(send.shape[1:]))
        self.comm.all_to_all_single(out, send, recv_counts, send_counts)
        return out

    def meta(self, points: torch.Tensor):
        """One all-gather: global domain (lo, hi) and every rank's point count."""
        if points.is_cuda:
            v = ops.load().local_meta(points)  # native bbox pass, stays on the device
        else:
            v = torch.empty(8, dtype=torch.float64)
            if points.numel():
                mn, mx = torch.aminmax(points, dim=0)
                v[0:3] = mn.double()
                v[3:6] = mx.double()
            else:
                v[0:3] = INF
                v[3:6] = -INF
            v[6] = points.size(0)
            v[7] = 0.0
        m = torch.stack(self.comm.all_gather(v)).cpu()  # host sync 1
        lo = tuple(float(x) for x in m[:, 0:3].min(0).values)
        hi = tuple(float(x) for x in m[:, 3:6].max(0).values)
        if not all(math.isfinite(x) for x in lo + hi):
            lo, hi = (0.0, 0.0, 0.0), (1.0, 1.0, 1.0)  # empty global cloud
        counts = [int(x) for x in m[:, 6]]
        return lo, hi, counts

    def domain(self, points: torch.Tensor):
        lo, hi, _ = self.meta(points)
        return lo, hi

    def _splits(self, points: torch.Tensor, metas: torch.Tensor, grid) -> Optional[torch.Tensor]:
        """Count-balanced kd splits for ``grid`` from this step's points (collective; on the
        points' device, no host sync), or None for equal-volume boxes / one rank."""
        if self.balance != "count" or self.world == 1:
            return None
        m = metas.view(-1, 8)
        lo, hi = m[:, 0:3].min(0).values, m[:, 3:6].max(0).values
        bad = ~(torch.isfinite(lo) & torch.isfinite(hi))
        lo = torch.where(bad, torch.zeros_like(lo), lo)  # empty global cloud: the unit box
        hi = torch.where(bad, torch.ones_like(hi), hi)
        return balanced_splits(points, lo, hi, grid, self.comm.all_gather_cat)

    def _use_native(self, points: torch.Tensor) -> bool:
        return points.is_cuda if self.native_route is None else bool(self.native_route)

    def exchange(self, dec: SpatialDecomposition, points: torch.Tensor, ids: torch.Tensor, h_send: float,
                 h_inner: Optional[float] = None, wz: float = INF):
        """Route points to owner + halo ranks in one all-to-all (points farther than ``wz`` from
        the domain faces with the interior send width ``h_inner``).
        Returns (points (n,3) owned-first, global ids (n,), n_owned)."""
        ids = ids.to(torch.int32).contiguous()
        hin = float(h_send if h_inner is None else h_inner)
        if self._use_native(points):
            C = ops.load()
            lo, hi = list(dec.lo), list(dec.hi)
            boxes = dec.boxes()
            bc, totals = C.route_count(points, lo, hi, list(dec.grid), boxes, float(h_send), dec.splits, hin, float(wz))
            recv_tot = torch.empty_like(totals)
            self.comm.all_to_all_single(recv_tot, totals)
            both = torch.cat([totals, recv_tot]).cpu()  # host sync 2 (send + receive splits)
            send_counts = [int(a + b) for a, b in both[: self.world].tolist()]
            recv_own = [int(a) for a, _ in both[self.world:].tolist()]
            recv_halo = [int(b) for _, b in both[self.world:].tolist()]
            send = C.route_scatter(points, ids, lo, hi, list(dec.grid), boxes, float(h_send), bc, totals,
                                   sum(send_counts), dec.splits, hin, float(wz))
            recv = self._a2a(send, send_counts, [a + b for a, b in zip(recv_own, recv_halo)])
            pts, gids = C.route_unpack(recv, recv_own, recv_halo)
            return pts, gids, sum(recv_own)
        send, totals = route_rows_torch(dec, points, ids, h_send, hin, wz)
        recv_tot = torch.empty_like(totals)
        self.comm.all_to_all_single(recv_tot, totals)
        st, rt = totals.tolist(), recv_tot.tolist()
        recv = self._a2a(send, [a + b for a, b in st], [a + b for a, b in rt])
        own_parts, halo_parts, off = [], [], 0
        for a, b in rt:
            own_parts.append(recv[off:off + a])
            halo_parts.append(recv[off + a:off + a + b])
            off += a + b
        rows = torch.cat(own_parts + halo_parts) if rt else recv
        pts, gids = _unpack(rows)
        return pts, gids, sum(a for a, _ in rt)

    def local_solve(self, pts: torch.Tensor, gids: torch.Tensor, n_owned: int, complete: list, box: list):
        if pts.is_cuda:
            ext = [box[3] - box[0], box[4] - box[1], box[5] - box[2]]
            plan = ops.Plan.auto(pts.size(0), self.k, self.points_per_cell, extent=ext)
            g = ops.build_grid(pts, self.k, plan=plan, deterministic=self.deterministic, box=box)
            idx, d2, info = ops.query(g, self.k, n_queries=n_owned, id_map=gids, complete=complete,
                                      return_info=True)
            return idx, d2, info["counters"][1:2].long()
        idx, d2, unc = ops.knn_cpu(pts, self.k, "grid", n_queries=n_owned, complete=complete,
                                   points_per_cell=self.points_per_cell)
        gl = gids.long()
        mapped = torch.where(idx >= 0, gl[idx.clamp(min=0).long()], torch.full_like(gl[:1], -1)).to(torch.int32)
        return mapped, d2, torch.tensor([unc.numel()], dtype=torch.long)

    # ------------------------------------------------------- native (GPU) fast path ------
    def _solve_native(self, points: torch.Tensor, ids: Optional[torch.Tensor]) -> DistResult:
        """Device-planned solve. Everything before the one routing sync is enqueued back to back:
        local meta -> all-gather -> ``route_begin`` (route plan, per-destination counts, and the
        scatter into a send buffer sized from earlier steps) -> counts all-to-all. The host then
        reads the plan header and both count tables in ONE copy. The rank's own segment sits at
        the end of the send buffer ("self-last") and never enters the collective: the payload
        all-to-all carries only rows that change rank, and ``route_unpack_split`` reads the own
        segment in place. The certification flag is the second sync. The decomposition grid is
        cached across calls and re-planned if the domain's shape asks for another one."""
        C = ops.load()
        world, rank = self.world, self.rank
        marks = self.host_marks
        mark = marks.append if marks is not None else (lambda _: None)
        mark(("start", time.perf_counter()))
        local = C.local_meta(points)
        spec = self._spec if (world > 1 and self.speculative) else None
        if spec is not None:
            metas, grid, splits = spec[0], spec[2], spec[3]
        else:
            metas = self.comm.all_gather_cat(local) if world > 1 else local  # (world*8,) f64, on device
            grid = self._grid or factor3(world, (1.0, 1.0, 1.0))
            splits = self._splits(points, metas, grid)
        hf = self.halo_factor * self.halo_boost
        nh = 2 * HDR
        src_pts, src_ids = points, (ids.to(torch.int32).contiguous() if ids is not None else None)
        rounds = 0
        growth = 0  # halo-doubling re-routes (the steady state needs a step without any)
        own_pts = own_ids = None
        n_fwd = 0
        while True:
            rounds += 1
            while True:
                cap = max(self._send_cap, int(src_pts.size(0) * (1.0 + self.send_headroom)) + 1024)
                inner = self._inner_factor() * hf / (self.halo_factor * self.halo_boost)
                # the halo field routes the first round (growth rounds widen the global widths)
                fld = self._field if rounds == 1 else None
                plan, sync, bc, send = C.route_begin(src_pts, src_ids, metas, rank, list(grid), self.k, hf, cap,
                                                     splits, inner, fld)
                totals = sync[nh:nh + 2 * world]
                if spec is not None:
                    # one all-gather of {meta, counts}; the rows this rank receives are column
                    # `rank` of every source's counts
                    row = META_I32 + 2 * world  # int32 per rank: 8 f64 meta + 2*world counts
                    gathered = self.comm.all_gather_cat(torch.cat([local.view(torch.int32), totals]))
                    mark(("enqueued", time.perf_counter()))
                    host = torch.cat([sync[:nh], gathered]).cpu()
                    mark(("synced", time.perf_counter()))
                    g = host[nh:].view(world, row)
                    new_metas = g[:, :META_I32].contiguous().view(torch.float64)
                    if not torch.equal(new_metas, spec[1]):
                        # a rank's cloud changed: re-plan with this step's metas (on device)
                        _log.info("rank %d: speculative routing plan stale (a rank's meta changed), re-planning", rank)
                        metas = gathered.view(world, row)[:, :META_I32].contiguous().view(torch.float64).flatten()
                        splits = self._splits(points, metas, grid)
                        spec = self._spec = None
                        continue
                    gl = g.tolist()
                    rt = [v for d in range(world) for v in gl[d][META_I32 + 2 * rank:META_I32 + 2 + 2 * rank]]
                    hv = host[:nh].view(torch.float64).tolist() + gl[rank][META_I32:] + rt
                    meta_host = spec[1]
                else:
                    if world > 1:  # rows to receive land in the tail of the same sync buffer
                        self.comm.all_to_all_single(sync[nh + 2 * world:], totals)
                    # sync 1: plan header (f64 viewed as int32 pairs) + both count tables (+ the
                    # gathered metas, kept for the next step's speculative routing), one copy
                    mark(("enqueued", time.perf_counter()))
                    host = torch.cat([sync, metas.view(torch.int32)]).cpu() if world > 1 else sync.cpu()
                    mark(("synced", time.perf_counter()))
                    meta_host = host[sync.numel():].view(torch.float64).view(world, 8) if world > 1 else None
                    host = host[:sync.numel()]
                    hv = host[:nh].view(torch.float64).tolist() + host[nh:].tolist()
                lo, hi = tuple(hv[0:3]), tuple(hv[3:6])
                want = factor3(world, tuple(max(hi[a] - lo[a], 1e-30) for a in range(3)))
                if want == tuple(grid):
                    break
                _log.info("rank %d: domain shape asks for rank grid %s (was %s), re-planning", rank, want, tuple(grid))
                grid = want  # domain shape changed: re-plan with the matching decomposition
                splits = self._splits(points, metas, grid)
            self._grid = tuple(grid)
            if world > 1 and rounds == 1:
                self._spec = (metas, meta_host, tuple(grid), splits)
            spec = None  # growth rounds re-route with the normal exchange
            h, hs, full = hv[6], hv[7], hv[10] != 0.0
            # a field plan: the certified radius of every field cell, for this plan's domain
            used_field = hv[22] != 0.0 and fld is not None
            cert = C.field_cert(fld, hv[:HDR]) if used_field else None
            tot = [int(x) for x in hv[HDR:HDR + 2 * world]]
            rtot = [int(x) for x in hv[HDR + 2 * world:HDR + 4 * world]] if world > 1 else tot
            send_counts = [tot[2 * d] + tot[2 * d + 1] for d in range(world)]
            recv_own = [rtot[2 * d] for d in range(world)]
            recv_halo = [rtot[2 * d + 1] for d in range(world)]
            need = sum(send_counts)
            self._send_cap = max(self._send_cap, need + need // 8 + 1024)
            if need > send.size(0):  # did not fit: route_begin wrote nothing, scatter again
                _log.debug("rank %d: send buffer %d < %d rows, re-scattering", rank, send.size(0), need)
                send = C.route_scatter_dev(src_pts, src_ids, plan, world, bc, totals, need, rank)
            cross_send = [0 if d == rank else send_counts[d] for d in range(world)]
            cross_recv = [0 if d == rank else recv_own[d] + recv_halo[d] for d in range(world)]
            x = sum(cross_send)
            if world > 1:
                recv = self._a2a(send[:x], cross_send, cross_recv)
            else:
                recv = send[:0]
            # unpack + local build + owned-point queries: one native call (same arithmetic as
            # local_solve with SpatialDecomposition's boxes)
            pts, gids, idx, d2, counters, *local_grid = C.dist_local(
                recv, send[x:x + send_counts[rank]], recv_own, recv_halo, rank, list(grid), hv[:HDR], self.k,
                self.points_per_cell, self.deterministic, 0, self.adaptive, field_cert=cert)
            mark(("local_enqueued", time.perf_counter()))
            n_owned = sum(recv_own)
            if rounds == 1:
                own_pts, own_ids = pts[:n_owned], gids[:n_owned]
            flag = counters[1:2].clone()  # uncertified queries (int32)
            if world > 1:
                self.comm.all_reduce_max(flag)
            done = int(flag.item()) == 0 or full or rounds >= self.max_rounds  # sync 2
            mark(("flag_synced", time.perf_counter()))
            n_fwd = 0
            if not done and self.forward:
                # targeted second round: only the uncertified queries travel (query forwarding)
                n_fwd = self._forward_round(hv, grid, pts, gids, idx, d2, counters, local_grid, splits)
                _log.info("rank %d: %d uncertified queries (all ranks) answered by query forwarding", rank, n_fwd)
                rounds += 1
                done = True
            if done:
                break
            hf *= 2.0
            growth += 1
            _log.info("rank %d: uncertified queries, growth round %d with halo factor %.3g", rank, rounds + 1, hf)
            src_pts, src_ids = own_pts, own_ids
        field_next = self._update_field(points, pts, n_owned, d2, hv, grid, used_field, n_fwd, growth, full)
        stats = {"n_owned": n_owned, "n_halo": int(pts.size(0) - n_owned),
                 "halo_width": hv[23] if used_field else h, "halo_field": bool(used_field), "rounds": rounds,
                 "grid": tuple(grid), "forwarded": n_fwd, "exact_path": int(counters[0].item()),
                 "local_dims": tuple(int(v) for v in local_grid[5].tolist()),
                 "local_tree": bool(local_grid[6].item())}
        _log.debug("rank %d: step %s", rank, stats)
        widen = n_fwd > 0 and self.halo_boost * 1.6 <= self.halo_boost_max + 1e-9
        if widen:
            self.halo_boost *= 1.6
            self._boost_clean = 0
            _log.info("rank %d: %d queries forwarded; halo factor for the next steps %.3g", rank, n_fwd,
                      self.halo_factor * self.halo_boost)
        elif n_fwd == 0 and growth == 0 and self.halo_boost > 1.0:
            # the boost decays once the cloud no longer needs it: after boost_decay_after validated
            # full steps in a row that forwarded nothing (n_fwd is all-reduced and growth follows the
            # all-reduced flag, so every rank decays together), one x1.6 step back toward 1
            self._boost_clean += 1
            if self._boost_clean >= self.boost_decay_after:
                self.halo_boost = max(1.0, self.halo_boost / 1.6)
                self._boost_clean = 0
                _log.info("rank %d: halo boost decays to %.3g", rank, self.halo_boost)
        else:
            self._boost_clean = 0
        if growth == 0 and not full and self.steady and not widen and not field_next and \
                2 * n_fwd <= self.fwd_slots_max:
            # validated single-round step: the steady-state assumption for the next ones
            self._steady = {
                "fwd": n_fwd > 0,  # device forwarding in the steady steps
                "F": max(256, 1 << max(0, 2 * n_fwd - 1).bit_length()),  # slots per rank pair
                "metas": metas, "grid": tuple(grid), "hdr": hv[:HDR], "cap": int(send.size(0)), "splits": splits,
                "plan": plan,  # the validated route plan (steady steps do not re-plan)
                "dims": [int(v) for v in local_grid[5].tolist()],  # the local grid (maybe refined)
                "use_tree": int(local_grid[6].item()),  # the local solve ran the tree path
                "tot": torch.tensor(tot, dtype=torch.int32, device=points.device),
                "send_counts": send_counts, "recv_own": recv_own, "recv_halo": recv_halo,
                "cross_send": cross_send, "cross_recv": cross_recv, "x": x,
                # direct placement of the own segment in steady steps: [own_base, halo_base, rows,
                # planned own count, planned halo count] (a different self count writes nothing)
                "place": [sum(recv_own[:rank]), n_owned + sum(recv_halo[:rank]), n_owned + sum(recv_halo),
                          tot[2 * rank], tot[2 * rank + 1]],
                "n": int(points.size(0)), "ids": ids is not None, "stats": dict(stats),
                # fallback launch sized from the validated step's list (short list: 256 WGs)
                "exact_grid": 256 if int(counters[0].item()) < 4096 else 0,
                # halo field plan: the width field (the route plan points at it) and its radii
                "field": fld if used_field else None, "field_cert": cert,
            }
            if world == 1:  # ids of the world-1 steady step (no routing) when the caller gives none
                self._steady["gids1"] = torch.arange(points.size(0), dtype=torch.int32, device=points.device)
        else:
            self._steady = None
        return DistResult(own_ids, idx, d2, stats)

    def _update_field(self, points, pts, n_owned, d2, hv, grid, used_field, n_fwd, growth, full) -> bool:
        """Halo field after a full step (collective: every rank takes the same branch). Returns
        True when a new field was made for the next full step (this step is then not the steady
        plan)."""
        G = self.halo_field_g
        if G <= 0 or self.world == 1 or not points.is_cuda or full or growth:
            return False
        # the step's halo rows over all ranks (the field must beat the global widths' halo)
        nh = torch.tensor([int(pts.size(0) - n_owned)], dtype=torch.int64, device=pts.device)
        halo_all = sum(int(x.item()) for x in self.comm.all_gather(nh))
        if used_field and n_fwd == 0:
            self._field_retries = 0
            if halo_all >= self._field_ref_halo:
                # sparse outliers forced cells so coarse that the field ships more than the global
                # widths (small clustered clouds): back to the global widths for good
                _log.info("rank %d: halo field %d rows >= global %d: global widths", self.rank, halo_all,
                          self._field_ref_halo)
                self.halo_field_g = 0
                self._field = None
                return True  # one more full step with the global widths, then steady
            return False  # the field plan certified every query: it becomes the steady plan
        if not used_field:
            self._field_ref_halo = halo_all
        if used_field:
            self._field_retries += 1
            if self._field_retries > 3:  # a changing cloud outruns the field: global widths
                self._field = None
                self._field_retries = 0
                return False
        C = ops.load()
        # cells per axis: the largest K-th distance must fit in the field's reach (3 rings of
        # cells: 3 x 0.998 x the smallest cell edge), else such queries could never be certified
        dk = d2[:n_owned, self.k - 1] if n_owned else d2.new_zeros(1)
        rmax = torch.where(torch.isfinite(dk), dk, torch.zeros_like(dk)).max().sqrt().reshape(1).float()
        self.comm.all_reduce_max(rmax)
        ext_min = min(hv[3 + a] - hv[a] for a in range(3))
        r = float(rmax.item())
        G = min(G, int(math.floor(3 * 0.998 * ext_min / (r * 1.02))) if r > 0.0 else G)
        if G < 4:  # cells wider than a quarter of the domain: the global widths do as well
            self._field = None
            return False
        F = self._field.clone() if (used_field and self._field is not None and self._field.numel() == G ** 3) \
            else torch.zeros(G * G * G, dtype=torch.float32, device=pts.device)
        stat = C.field_splat(pts, n_owned, d2, self.k, hv[:HDR], self.rank, list(grid), F)
        self.comm.all_reduce_max(F)
        self.comm.all_reduce_max(stat)
        if int(stat[0].item()) > 0:  # a query with fewer than K neighbours in the whole cloud
            self._field = None
            return False
        self._field = F
        return True

    def _forward_round(self, hv, grid, pts, gids, idx, d2, counters, local_grid, splits=None) -> int:
        """Query forwarding for the uncertified queries of a round (targeted second round,
        replaces re-routing every owned point with a doubled halo). Each uncertified query q
        with local K-th distance r (an upper bound of the true one: the local set is a subset)
        goes to every other rank whose box lies within r; that rank answers with the exact K
        nearest among ITS local points (owned + halo, global-id grid); the origin merges its own
        K with the answers (deduplicated by global id). Every true neighbour lies within r, so it
        is owned by a consulted rank and ranks in that rank's own local top K: the merge is
        exact in one round. Returns the number of forwarded queries (all ranks)."""
        C = ops.load()
        world, rank, k = self.world, self.rank, self.k
        dev = pts.device
        sorted_, cell_start, geom, perm, uncert, dims_t = local_grid[:6]
        n_unc = int(counters[1].item())
        U = uncert[:n_unc].long()
        q = pts[U]
        qg = gids[U]
        r2 = d2[U, k - 1] if n_unc else d2.new_empty(0)
        lo, hi = tuple(hv[0:3]), tuple(hv[3:6])
        dec = SpatialDecomposition(world, lo, hi, tuple(grid), splits.tolist() if splits is not None else None)
        # conservative box test: the float32 box arithmetic may not miss a rank
        r2c = torch.where(torch.isfinite(r2), r2 * (1.0 + 1e-5) + 1e-6, torch.full_like(r2, INF))
        masks = []
        for d in range(world):
            if d == rank:
                masks.append(torch.zeros(n_unc, dtype=torch.bool, device=dev))
            else:
                masks.append(dec.box_dist2(q, d) <= r2c)
        rows = torch.cat([q, qg.to(torch.int32).view(torch.float32).unsqueeze(1)], 1)
        send = torch.cat([rows[m] for m in masks]) if n_unc else rows[:0]
        scount = torch.tensor([int(m.sum()) for m in masks], dtype=torch.int64)
        rcount = torch.empty_like(scount)
        cdev = torch.device("cpu") if isinstance(self.comm, HostStagedTransport) or not pts.is_cuda else dev
        sc_d = scount.to(cdev)
        rc_d = torch.empty_like(sc_d)
        self.comm.all_to_all_single(rc_d, sc_d, [1] * world, [1] * world)
        rcount = rc_d.cpu()
        recv = self._a2a(send.contiguous(), scount.tolist(), rcount.tolist())
        # answer the received queries from the local grid
        if recv.size(0):
            ridx, rd2 = C.query_external(sorted_, cell_start, geom, dims_t.tolist(), k, recv.contiguous(), perm)
        else:
            ridx, rd2 = idx.new_empty((0, k)), d2.new_empty((0, k))
        back = torch.cat([ridx.view(torch.float32), rd2], 1).contiguous()  # (M, 2k)
        ans = self._a2a(back, rcount.tolist(), scount.tolist())
        if n_unc:
            M = k * world
            cand_d = torch.full((n_unc, M), INF, device=dev)
            cand_i = torch.full((n_unc, M), -1, dtype=torch.int32, device=dev)
            cand_d[:, :k] = d2[U]
            cand_i[:, :k] = idx[U]
            off = 0
            for d in range(world):
                m = masks[d]
                c = int(scount[d])
                if c:
                    blk = ans[off:off + c]
                    sel = torch.nonzero(m).flatten()
                    cand_i[sel, (d + 1 if d < rank else d) * k:(d + 1 if d < rank else d) * k + k] = \
                        blk[:, :k].contiguous().view(torch.int32)
                    cand_d[sel, (d + 1 if d < rank else d) * k:(d + 1 if d < rank else d) * k + k] = blk[:, k:]
                off += c
            # (d2, id) order; duplicates (a halo copy answered by two ranks) are adjacent
            key = (cand_d.view(torch.int32).to(torch.int64) << 32) | (cand_i.to(torch.int64) & 0xFFFFFFFF)
            key = torch.where(cand_i >= 0, key, torch.full_like(key, torch.iinfo(torch.int64).max))
            key = torch.sort(key, dim=1).values
            dup = torch.zeros_like(key, dtype=torch.bool)
            dup[:, 1:] = key[:, 1:] == key[:, :-1]
            key = torch.where(dup, torch.full_like(key, torch.iinfo(torch.int64).max), key)
            key = torch.sort(key, dim=1).values[:, :k]
            empty = key == torch.iinfo(torch.int64).max
            new_i = torch.where(empty, torch.full_like(key, -1), key & 0xFFFFFFFF).to(torch.int32)
            new_d = torch.where(empty, torch.full_like(key, 0x7F800000), key >> 32).to(torch.int32).view(torch.float32)
            idx[U] = new_i
            d2[U] = new_d
        tot = torch.tensor([n_unc], dtype=torch.int64, device=cdev)
        if world > 1:
            # the sum is only a statistic: max-reduce the per-rank counts' sum through a MAX of one
            parts = self.comm.all_gather(tot)
            return int(sum(int(x.item()) for x in parts))
        return n_unc

    def _steady_body(self, points: torch.Tensor, ids: Optional[torch.Tensor], sink=None):
        """Device work of one steady step (no host synchronisation): -> (owned gids, idx, d2,
        flag); the flag is already all-reduced. sink (world 1, graph capture): (sticky (1,) int32
        GPU, host (1,) int32 pinned) that the flag kernel max-accumulates / stores into."""
        st = self._steady
        C = ops.load()
        world, rank = self.world, self.rank
        src_ids = ids.to(torch.int32).contiguous() if ids is not None else None
        if world == 1:
            # a world of one routes every point to itself, in order, with no halo: the share IS the
            # local point set (ids: the caller's or 0..n-1). Skip the routing passes; the flag
            # checks this share's {lo, hi, n} against the validated step's meta (one bbox pass)
            # and the uncertified count, as steady_flag_partials does. Rows are bit-identical.
            gin = src_ids if src_ids is not None else st["gids1"]
            if gin.numel() != points.size(0):  # a share of another size: the flag fails below
                gin = torch.zeros(points.size(0), dtype=torch.int32, device=points.device)
            n = points.size(0)
            pts, gids, idx, d2, counters, *lg = C.dist_local(
                points.new_empty((0, 4)), points.new_empty((0, 4)), [n], [0], 0, [1, 1, 1], st["hdr"], self.k,
                self.points_per_cell, self.deterministic, st["exact_grid"], False, st["dims"], points, gin,
                st["use_tree"])
            sticky, host = sink if sink is not None else (None, None)
            flag = C.steady_flag_local(points, st["metas"], 0, counters, sticky, host)
            return gids, idx, d2, flag
        # counts + scatter with the validated plan; the share's bbox comes from the counting pass,
        # and the rank's own segment goes straight to its local rows (no send-buffer copy, no
        # unpack of it): only rows received from other ranks are unpacked
        totals, send, partials, lpts, lgids = C.route_steady(points, src_ids, st["plan"], world, st["cap"], rank,
                                                             st["place"])
        x = st["x"]
        if world > 1:
            recv = self._a2a(send[:x], st["cross_send"], st["cross_recv"])
        else:
            recv = send[:0]
        pts, gids, idx, d2, counters, *lg = C.dist_local(recv, send[:0], st["recv_own"], st["recv_halo"],
                                                         rank, list(st["grid"]), st["hdr"], self.k,
                                                         self.points_per_cell, self.deterministic, st["exact_grid"],
                                                         False, st["dims"], lpts, lgids, st["use_tree"],
                                                         field_cert=st.get("field_cert"))
        check = counters  # the flag's word [1]: uncertified queries (no forwarding) or slot overflow
        if world > 1 and st.get("fwd"):
            # uncertified queries answered inside the step: fixed-capacity forwarding slots and
            # equal-split all-to-alls, so nothing waits for the host (kn/route.h launch_fwd_pack)
            F = st["F"]
            umax = world * F
            sorted_, cell_start, geom, perm, uncert = lg[:5]
            fsend, slot_of, check = C.fwd_pack(st["plan"], world, rank, F, self.k, uncert, counters, umax, pts,
                                               gids, d2)
            frecv = torch.empty_like(fsend)
            self.comm.all_to_all_single(frecv, fsend)
            aidx, ad2 = C.fwd_answer(sorted_, cell_start, geom, list(st["dims"]), self.k, frecv, perm)
            ans = torch.cat([aidx.view(torch.float32), ad2], 1)  # one collective for both halves
            back = torch.empty_like(ans)
            self.comm.all_to_all_single(back, ans)
            C.fwd_merge(world, F, self.k, uncert, counters, umax, slot_of,
                        back[:, :self.k].contiguous().view(torch.int32), back[:, self.k:].contiguous(), idx, d2)
        flag = C.steady_flag_partials(partials, points.size(0), st["metas"], rank, totals, st["tot"], check)
        if world > 1:
            self.comm.all_reduce_max(flag)
        return gids[:sum(st["recv_own"])], idx, d2, flag

    def _use_graph(self, points: torch.Tensor) -> bool:
        if not points.is_cuda:
            return False
        if self.graph_steady is not None:
            return bool(self.graph_steady)
        import os

        # default at world 1 (no collective inside the captured step); KN_DIST_GRAPH=1 also for
        # world > 1 (RCCL capture), =0 never
        env = os.environ.get("KN_DIST_GRAPH")
        on = env == "1" or (env != "0" and self.world == 1)
        return on and isinstance(self.comm, TorchDistTransport)

    def _use_pipe(self, points: torch.Tensor) -> bool:
        st = self._steady
        if st is None or st.get("fwd") or not points.is_cuda:
            return False
        if not isinstance(self.comm, TorchDistTransport) or isinstance(self.comm, HostStagedTransport):
            return False
        if not getattr(self.comm, "stream_ordered", False):  # RCCL ("nccl") groups only
            return False
        if self.native_pipeline is not None:
            return bool(self.native_pipeline)
        import os

        return os.environ.get("KN_DIST_PIPE", "1") != "0" and hasattr(ops.load(), "DistPipe")

    def _rank_comm(self, dev: torch.device):
        """This rank's own RCCL communicator (collective: every rank calls it at the same step;
        the unique id travels over the process group)."""
        if self._rcomm is None:
            C = ops.load()
            uid = C.rccl_unique_id() if self.rank == 0 else bytes(128)
            t = torch.tensor(list(uid), dtype=torch.uint8, device=dev)
            parts = self.comm.all_gather(t)
            uid0 = bytes(parts[0].cpu().tolist())
            self._rcomm = C.RankComm(uid0, self.world, self.rank, dev.index if dev.index is not None else 0)
        return self._rcomm

    def _agree(self, ok: bool, dev: torch.device) -> bool:
        """True when ``ok`` holds on EVERY rank (a MAX all-reduce of the failure bit): decisions
        that change which collectives a rank issues are taken by all ranks together."""
        bad = torch.tensor([0 if ok else 1], dtype=torch.int32, device=dev)
        self.comm.all_reduce_max(bad)
        return int(bad.item()) == 0

    def _capture_mode(self) -> bool:
        """Graph capture of the native pipeline's stages (RCCL calls included): KN_DIST_CAPTURE=1
        captures, default eager at every world size: the stages are enqueued per step on the two
        streams (same order and overlap, one enqueue per kernel). Eager measured FASTER than the
        captured per-stage graphs at world 1 (900K K=16, 200 / 50, two passes: 0.3191 / 0.3210 vs
        0.3280 / 0.3271 ms, profiles/r5_dist.txt), and at world > 1 an eager RCCL step is the
        library's ordinary use (captured multi-peer point-to-point has never run on more than one
        rank here), so every world size now times the same mode."""
        import os

        return os.environ.get("KN_DIST_CAPTURE") == "1"

    def _pipe_for(self, points: torch.Tensor, ids: Optional[torch.Tensor]):
        """The native pipeline of the current steady plan over these input tensors (read in
        place; other storage builds a new one). Collective when it builds: construction is local,
        then every rank learns whether all ranks constructed theirs before any enters the eager
        warm-up step (so one rank's local failure -- an allocation, a plan check -- sends all ranks
        to the torch path together instead of leaving its peers blocked in a collective), and the
        graph capture's outcome is agreed on the same way (any failure: every rank runs eagerly).
        Returns None when the native pipeline is unavailable on some rank."""
        st = self._steady
        ids32 = ids.to(torch.int32).contiguous() if ids is not None else None
        p = self._pipe
        same = (p is not None and p["st"] is st and p["pts"].data_ptr() == points.data_ptr()
                and p["n"] == points.size(0) and (p["ids"] is None) == (ids32 is None)
                and (ids32 is None or p["ids"].data_ptr() == ids32.data_ptr()))
        if same:
            return p
        if p is not None and p["st"] is st:
            # other input tensors under the same steady plan (a caller passing a fresh tensor every
            # step, or a share whose size changed): the pipeline reads them from now on -- local,
            # no rebuild, so no rank ever enters a collective its peers do not (a changed size
            # fails the step's flag on every rank; the next step then takes the full path together)
            p["pipe"].rebind(points, ids32)
            p["pts"], p["ids"], p["n"] = points, ids32, points.size(0)
            self.pipe_mode = p["pipe"].mode()
            return p
        self._pipe = None  # release the old pipeline's buffers first
        C = ops.load()
        world1_force = self.world == 1 and self.force_collectives
        pipe, err = None, ""
        try:
            rc = self._rank_comm(points.device)
            pipe = C.DistPipe(rc, points, ids32, st["plan"], st["metas"],
                              [int(v) for v in st["tot"].tolist()], [float(v) for v in st["hdr"]], list(st["grid"]),
                              list(st["dims"]), list(st["recv_own"]), list(st["recv_halo"]), list(st["cross_send"]),
                              list(st["cross_recv"]), list(st["place"]), int(st["cap"]), self.k, self.points_per_cell,
                              bool(self.deterministic), int(st["exact_grid"]), int(st["use_tree"]), world1_force, None,
                              st.get("field"), st.get("field_cert"))
        except RuntimeError as e:
            err = str(e)
        if not self._agree(pipe is not None, points.device):
            _log.warning("rank %d: native pipeline unavailable on some rank (%s); torch steady path", self.rank,
                         err or "a peer failed")
            return None
        try:
            pipe.warmup(self.wait_timeout_s)  # collective eager step under the deadline
        except RuntimeError as e:
            raise CollectiveError(f"rank {self.rank}: native pipeline warm-up step failed: {e}") from e
        mode = "eager"
        if self._capture_mode():
            ok = pipe.prepare_graphs(self.pipe_unroll)
            if not ok:
                _log.warning("rank %d: graph capture of the native pipeline failed (%s)", self.rank, pipe.error())
            if self._agree(ok, points.device):
                mode = "graph"
            else:
                pipe.set_eager(True)
        self.pipe_mode = mode
        p = self._pipe = {"pipe": pipe, "st": st, "pts": points, "ids": ids32, "n": points.size(0),
                          "outs": [pipe.outputs(i) for i in range(pipe.sets())], "primed": False}
        return p

    def _solve_pipe(self, points: torch.Tensor, ids: Optional[torch.Tensor], iters: int = 1,
                    resident: bool = False) -> DistResult:
        """``iters`` steady steps through the native pipeline (one call; unrolled graphs when
        iters > 1). resident: keep the next step's build enqueued after the call (the caller
        promises the points do not change before the next call)."""
        st = self._steady
        p = self._pipe_for(points, ids)
        if p is None:
            # the native pipeline could not be built on every rank: the torch steady path, for good
            # (decided collectively in _pipe_for, so every rank takes it)
            self.native_pipeline = False
            self._pipe = None
            res = None
            for _ in range(iters):
                res = self._solve_steady(points, ids)
            return res
        pipe = p["pipe"]
        try:
            last = pipe.launch(iters, self.pipe_unroll if iters > 1 else 0, bool(resident))
        except RuntimeError as e:
            # an enqueue failed after the peers may have issued this step's collectives: the group
            # cannot continue (wait() would time out); fail loudly on this rank
            raise CollectiveError(f"rank {self.rank}: pipelined launch failed: {e}") from e
        gids, idx, d2 = p["outs"][pipe.last_set()]
        stats = dict(st["stats"])
        stats["steady"] = True
        stats["graph"] = pipe.mode() == "graph"
        stats["pipelined"] = True
        stats["pipe_mode"] = pipe.mode()
        stats["capture_fallbacks"] = int(pipe.capture_fallbacks())
        timeout = self.wait_timeout_s
        rank = self.rank

        def waiter() -> bool:
            try:
                return pipe.wait(last, timeout) == 0
            except RuntimeError as e:
                raise CollectiveError(f"rank {rank}: pipelined step failed: {e}") from e

        return DistResult(gids, idx, d2, stats, waiter=waiter)

    def run_steps(self, points: torch.Tensor, iters: int, ids: Optional[torch.Tensor] = None,
                  resident: bool = False) -> DistResult:
        """``iters`` steps of the same share in one call (benchmarks, repeated solves of a
        resident cloud): in the steady state all of them are enqueued at once into the native
        pipeline (U steps per graph launch, no host round trip); otherwise asynchronous
        ``solve`` calls until the steady state is reached (e.g. the halo-field step after the
        first full step), then the rest through the pipeline. Returns the last step's result;
        its ``valid()`` covers every pipelined step."""
        points = points.contiguous().float()
        if iters <= 0:
            raise ValueError("iters must be positive")
        self._maybe_inject_failure()
        res = None
        left = iters
        while left > 0:
            if self.steady and self._steady is not None and self._use_native(points) and self.device_plan:
                self._check_pending(keep=0)
                if self._steady is not None and self._use_pipe(points):
                    res = self._solve_pipe(points, ids, left, resident)
                    self._pending.append(res)
                    return res
            res = self.solve(points, ids, async_=True)
            left -= 1
        return res

    def _maybe_inject_failure(self) -> None:
        """Test hook (bench supervisor, tests/test_gpu_distributed.py): KN_DIST_INJECT_FAIL=r makes
        rank r raise in its first run_steps() call -- the pipelined launch of the bench's timed path
        -- while the native pipeline is enabled (KN_DIST_PIPE != 0), so a fallback attempt with
        KN_DIST_PIPE=0 runs clean. Its peers are then blocked in the step's collectives, as after a
        real failure."""
        import os

        inj = os.environ.get("KN_DIST_INJECT_FAIL", "")
        if (inj.strip() and int(inj) == self.rank and os.environ.get("KN_DIST_PIPE", "1") != "0"
                and not getattr(self, "_injected", False)):
            self._injected = True
            raise CollectiveError(f"rank {self.rank}: injected failure (KN_DIST_INJECT_FAIL) at its first pipelined "
                                  "launch (stage: launch)")

    def profile_step(self, points: torch.Tensor, ids: Optional[torch.Tensor] = None) -> dict:
        """Per-phase device times (ms) of one serial steady step of the native pipeline
        (collective: every rank calls it): ms_route, ms_exchange, ms_build, ms_query,
        ms_finish. {} when the steady native pipeline is not in use."""
        points = points.contiguous().float()
        if self._steady is None or not self._use_pipe(points):
            return {}
        self._check_pending(keep=0)
        if self._steady is None:
            return {}
        p = self._pipe_for(points, ids)
        if p is None:
            self.native_pipeline = False
            return {}
        return dict(p["pipe"].profile())

    def _solve_steady(self, points: torch.Tensor, ids: Optional[torch.Tensor]) -> DistResult:
        """One step with no host synchronisation (see ``self.steady``): the native pipeline
        (``_use_pipe``), else replayed from a torch hipGraph when ``_use_graph``."""
        st = self._steady
        if self._use_pipe(points):
            return self._solve_pipe(points, ids)
        if self._use_graph(points):
            g = self._graph
            ids32 = ids.to(torch.int32).contiguous() if ids is not None else None
            # Direct input: the graph reads the caller's tensors in place while every call passes
            # the same storage (a training / serving loop refilling one buffer); it keeps them
            # alive, so an equal address is that storage. The first call with other tensors
            # recaptures once on graph-owned input buffers filled by a copy per step.
            same = (g is not None and g["direct"] and points.data_ptr() == g["pts"].data_ptr()
                    and (ids32 is None or ids32.data_ptr() == g["idsb"].data_ptr()))
            if (g is None or g["st"] is not st or g["n"] != points.size(0) or g["ids"] != (ids is not None)
                    or (g["direct"] and not same)):
                direct = g is None or g["st"] is not st
                sp = points if direct else points.clone()
                si = (ids32 if direct else ids32.clone()) if ids32 is not None else None
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    for _ in range(2):  # warm-up: allocator pools, kernel attributes
                        self._steady_body(sp, si)
                torch.cuda.current_stream().wait_stream(side)
                # the step's flag leaves the device inside the graph (no stream op between
                # replays): a sticky max over the replays of this graph into one pinned word, so a
                # step reads its own flag or a later one's -- never valid after an invalid step (an
                # invalid step drops the graph). World 1: the flag kernel itself stores it.
                sticky = torch.zeros(1, dtype=torch.int32, device=points.device)
                host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    out = self._steady_body(sp, si, sink=(sticky, host) if self.world == 1 else None)
                    if self.world > 1:
                        torch.maximum(sticky, out[3], out=sticky)
                        host.copy_(sticky, non_blocking=True)
                g = self._graph = {"graph": graph, "pts": sp, "ids": si is not None, "idsb": si, "out": out,
                                   "st": st, "n": points.size(0), "direct": direct, "host": host}
            if not g["direct"]:
                g["pts"].copy_(points)
                if ids32 is not None:
                    g["idsb"].copy_(ids32)
            g["graph"].replay()
            gid, idx, d2, _ = g["out"]
            ev = torch.cuda.Event()
            ev.record()
            stats = dict(st["stats"])
            stats["steady"] = True
            stats["graph"] = True
            return DistResult(gid, idx, d2, stats, flag=g["host"], event=ev)
        gid, idx, d2, flag = self._steady_body(points, ids)
        if st.get("gids1") is not None and gid.data_ptr() == st["gids1"].data_ptr():
            gid = gid.clone()  # world 1: never hand out the cached id table itself
        host = torch.empty(1, dtype=torch.int32, pin_memory=points.is_cuda)
        host.copy_(flag, non_blocking=True)
        ev = torch.cuda.Event() if points.is_cuda else None
        if ev is not None:
            ev.record()
        stats = dict(st["stats"])
        stats["steady"] = True
        stats["graph"] = False
        return DistResult(gid, idx, d2, stats, flag=host, event=ev)

    def _drop_steady(self) -> None:
        _log.info("rank %d: steady-state step invalid (routing changed or uncertified query), "
                  "the next step takes the full path", self.rank)
        self._steady = None
        self._graph = None
        if self._pipe is not None:
            self._pipe["pipe"].sync()
        self._pipe = None
        self._pending.clear()

    def _check_pending(self, keep: int) -> None:
        while len(self._pending) > keep:
            if not self._pending.popleft().valid():
                self._drop_steady()

    # -------------------------------------------------------------------- solve ------
    def solve(self, points: torch.Tensor, ids: Optional[torch.Tensor] = None,
              partitioned: bool = False, domain=None, async_: bool = False) -> DistResult:
        """kNN of the distributed cloud. ``points``: this rank's (N_r, 3) float32 share (any
        distribution; ``partitioned`` is accepted for API compatibility -- points already in
        this rank's box simply route to itself). ``ids``: their global ids (int32); default =
        rank offset + arange.

        ``async_``: in the steady state (same share sizes and layout as the last validated
        step) return without any host synchronisation; the caller checks ``result.valid()``
        before using the rows and re-solves synchronously if it is False. Synchronous calls
        (the default) do that check themselves."""
        points = points.contiguous().float()
        if domain is None and self._use_native(points) and self.device_plan:
            # every rank takes the same path: _steady is set and cleared only on collective
            # outcomes (the all-reduced flags), so it is never decided from local data alone -- a
            # rank whose share changed still runs the steady step and its on-device check fails
            if self.steady and self._steady is not None:
                self._check_pending(keep=1 if async_ else 0)
            if self.steady and self._steady is not None:
                res = self._solve_steady(points, ids)
                if async_:
                    self._pending.append(res)
                    return res
                if res.valid():
                    if res.stats.get("graph"):  # graph buffers are reused by the next replay
                        res = DistResult(res.ids.clone(), res.neighbors.clone(), res.d2.clone(), res.stats)
                    return res
                self._drop_steady()  # assumption failed or a query is uncertified: the full way
            self._pending.clear()  # a full step replaces the plan the pending steps ran with
            return self._solve_native(points, ids)
        dev = points.device
        lo, hi, counts = self.meta(points)
        if domain is not None:
            lo, hi = tuple(domain[0]), tuple(domain[1])
        if ids is None:
            off = sum(counts[: self.rank])
            ids = torch.arange(off, off + points.size(0), dtype=torch.int32, device=dev)
        dec = SpatialDecomposition(self.world, lo, hi)
        if self.balance == "count" and self.world > 1:
            sp = balanced_splits(points, torch.tensor(lo, dtype=torch.float64), torch.tensor(hi, dtype=torch.float64),
                                 dec.grid, self.comm.all_gather_cat)
            dec = SpatialDecomposition(self.world, lo, hi, dec.grid, sp.tolist())
        n_total = sum(counts)
        vol = max(1e-30, (hi[0] - lo[0]) * (hi[1] - lo[1]) * (hi[2] - lo[2]))
        rk = ops.expected_kth_radius(n_total, self.k, vol)
        h = self.halo_factor * rk
        # position-dependent halo: interior width h_i <= h (route.hip route_plan_kernel's rule)
        inner = self._inner_factor() / self.halo_boost
        h_in = min(h, inner * rk) if inner > 0.0 else h
        scale = max(max(abs(v) for v in lo), max(abs(v) for v in hi), max(hi[a] - lo[a] for a in range(3)))
        diag = math.sqrt(sum((hi[a] - lo[a]) ** 2 for a in range(3)))
        blo, bhi = dec.rank_box(self.rank)
        rounds = 0
        src_pts, src_ids = points, ids
        while True:
            rounds += 1
            full = h >= diag
            hs = halo_send_width(h, lo, hi) if not full else 2.0 * diag + 1.0
            his = halo_send_width(h_in, lo, hi) if not full else hs
            wz = h + h_in
            pts, gids, n_owned = self.exchange(dec, src_pts, src_ids, hs, his, wz)
            if rounds == 1:
                own_pts, own_ids = pts[:n_owned], gids[:n_owned]
            if full:
                complete = [-INF] * 3 + [INF] * 3
            else:
                complete = (dec.complete_box(self.rank, h_in) + [h - h_in, wz - 1e-5 * scale] + list(lo) + list(hi))
            box = [max(lo[a], blo[a] - hs) for a in range(3)] + [min(hi[a], bhi[a] + hs) for a in range(3)]
            idx, d2, n_unc = self.local_solve(pts, gids, n_owned, complete, box)
            flag = n_unc.to(dev) if dev.type != "cpu" else n_unc
            self.comm.all_reduce_max(flag)
            if int(flag.item()) == 0 or full or rounds >= self.max_rounds:  # host sync 3
                break
            h *= 2.0
            h_in *= 2.0
            # owned points are in place: re-route them (owner = this rank) for the wider halo
            src_pts, src_ids = own_pts, own_ids
        stats = {"n_owned": n_owned, "n_halo": int(pts.size(0) - n_owned), "halo_width": h, "rounds": rounds,
                 "grid": dec.grid}
        return DistResult(own_ids, idx, d2, stats)
