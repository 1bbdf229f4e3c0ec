"""Functional ops: grid build, kNN query, CPU oracles.

GPU ops call the hand-written gfx950 HIP kernels in ``csrc/kernels`` through the ``_C``
extension, on the current PyTorch stream (graph-capturable: no host synchronisation and no
allocation outside the caching allocator). CPU ops call the native host library
(``csrc/host``): the kd-tree oracle, brute force and the CPU grid solver.

Index conventions (reference knearests.h / test_knearests.cu:158):
* ``knn(points, k)`` returns ``(idx, d2)`` in ORIGINAL order: ``idx[i, j]`` is the j-th
  nearest neighbour of input point ``i`` (self excluded, ascending squared distance ``d2``,
  ties broken by index, ``-1`` for slots that cannot be filled when N <= k).
* ``Grid.perm[s]`` is the original index of stored point ``s``; ``to_stored_space`` gives the
  reference's stored-space view.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import torch

from .._ext import load

INF = float("inf")
# query flags (kn/kernels.h kQueryFlag*): the wide exact re-rank window, for clouds with many
# exactly equal distances (KNearests sets it from the previous solve's cooperative re-ranks)
QUERY_FLAG_WIDE = 16


@dataclass
class Plan:
    """Grid + tile plan (``kn::AutoParams``)."""

    dims: list
    tile: list
    halo: int
    lds_capacity: int
    lds_bytes: int = 0
    # x sub-cells per y/z cell width: dims[0] and tile[0] count sub-cells, the x halo is halo * xsub
    xsub: int = 1

    @staticmethod
    def auto(n: int, k: int, points_per_cell: float = 0.0, tile: Sequence[int] = (),
             halo: int = 0, extent: Optional[Sequence[float]] = None, xsub: int = 0) -> "Plan":
        d = load().auto_params(int(n), int(k), float(points_per_cell), list(tile), int(halo),
                               list(extent) if extent is not None else None, int(xsub))
        return Plan(list(d["dims"]), list(d["tile"]), int(d["halo"]), int(d["lds_capacity"]),
                    int(d["lds_bytes"]), int(d["xsub"]))


@dataclass
class Grid:
    """A built uniform grid on the GPU (result of :func:`build_grid`)."""

    sorted: torch.Tensor      # (N, 4) float32 {x, y, z, bits(original index)}
    cell_start: torch.Tensor  # (C + 1,) int32
    perm: torch.Tensor        # (N,) int32, stored -> original
    geom: torch.Tensor        # (16,) int32 packed kn::GridGeom
    plan: Plan
    n: int = 0
    extra: dict = field(default_factory=dict)


def _check_gpu_points(points: torch.Tensor) -> torch.Tensor:
    if points.dim() != 2 or points.size(1) != 3:
        raise ValueError("points must be (N, 3)")
    if not points.is_cuda:
        raise ValueError("GPU op called with a CPU tensor (use knn_cpu for the host path)")
    return points.contiguous().float()


def build_grid(points: torch.Tensor, k: int = 16, plan: Optional[Plan] = None,
               points_per_cell: float = 0.0, deterministic: bool = True,
               box: Optional[Sequence[float]] = None, adaptive: bool = False) -> Grid:
    """Bin ``points`` (N,3 float32, GPU) into a uniform grid (bbox, count, scan, scatter).

    ``adaptive``: measure the mean occupancy of a point's cell (one small reduction + one host
    sync) and re-bin with finer cells while it is far above a Poisson grid's (clustered clouds,
    points on surfaces); tile / halo / LDS plan stay those of the target density. Not for use
    inside graph capture (it synchronises)."""
    points = _check_gpu_points(points)
    n = points.size(0)
    if plan is None:
        extent = None
        if box is not None:
            extent = [box[3] - box[0], box[4] - box[1], box[5] - box[2]]
        plan = Plan.auto(n, k, points_per_cell, extent=extent)
    C = load()
    bx = list(map(float, box)) if box is not None else None
    probe = adaptive and n > 0
    # probe grids skip the in-cell order (a clustered cloud's first grid has cells of thousands
    # of points); the final grid is ordered once
    s, cs, perm, geom = C.build(points, list(plan.dims), bool(deterministic) and not probe, bx)
    refined = False
    for _ in range(3 if probe else 0):
        w = int(C.occupancy(cs).item()) / n
        dims = C.refine_dims(list(plan.dims), w, int(k), float(points_per_cell), n, plan.xsub)
        if dims is None:
            break
        # refined grids are isotropic (xsub 1)
        tile = [max(1, plan.tile[0] // plan.xsub), plan.tile[1], plan.tile[2]]
        plan = Plan(list(dims), tile, plan.halo, plan.lds_capacity,
                    int(C.query_lds_bytes(tile, plan.halo, plan.lds_capacity, 1)), 1)
        s, cs, perm, geom = C.build(points, list(plan.dims), False, bx)
        refined = True
    if probe and deterministic:
        C.cell_sort(s, cs, perm, geom)
    # a grid that had to be refined serves a density one cell size cannot: query("auto") takes
    # the Morton-leaf tree (same rule as kn::Engine, csrc/runtime/engine.cpp)
    return Grid(s, cs, perm, geom, plan, n, {"algo": "tree" if refined else "grid"})


def build_tree(grid: Grid, count_leaves: bool = False) -> tuple:
    """Morton-leaf box tree over the grid's points (``kn/tree.h``), cached on the grid: the
    density-adaptive query structure for clouds one cell size cannot serve (clusters, scans).
    Returns ``(workspace, nodes, leaves)``. Stream-ordered: the leaf count stays on the device
    (``leaves`` is -1 unless ``count_leaves``, which costs one host sync)."""
    t = grid.extra.get("tree")
    if t is None or (count_leaves and t[2] < 0):
        t = tuple(load().tree_build(grid.sorted, grid.cell_start, grid.geom, list(grid.plan.dims), count_leaves))
        grid.extra["tree"] = t
    return t


def query(grid: Grid, k: int, n_queries: Optional[int] = None, id_map: Optional[torch.Tensor] = None,
          complete: Optional[Sequence[float]] = None, use_tiles: bool = True, with_dist: bool = True,
          return_info: bool = False, flags: int = 0, algo: str = "grid", first: int = 0):
    """kNN of the grid's points (original index in [first, n_queries)) against all grid points.

    ``first`` > 0 solves a query range (grid kernels; row r = original index first + r): batched
    solves of clouds whose whole N x K result does not fit next to the grid.

    ``algo``: ``"grid"`` (LDS-tiled grid kernels + exact fallback), ``"tree"`` (Morton-leaf tree,
    :func:`build_tree`; not with ``complete``) or ``"auto"`` (the grid's ``plan`` choice, see
    :func:`build_grid`). Returns ``(idx, d2)`` (+ ``info`` dict with the device counters and the
    uncertified query list when ``return_info``). ``idx`` values are original indices, or
    ``id_map[...]``.
    """
    if not 1 <= k <= 128:
        raise ValueError("k must be in [1, 128]")
    if algo == "auto":
        algo = grid.extra.get("algo", "grid")
    nq = grid.n if n_queries is None else int(n_queries)
    if first:
        algo = "grid"  # query ranges run on the grid kernels
    if algo == "tree":
        if complete is not None:
            raise ValueError("the tree path serves complete (single-GPU) point sets only")
        ws, nodes, _ = build_tree(grid)
        idx, d2, counters = load().tree_query(ws, nodes, list(grid.plan.dims), grid.n, int(k), nq, id_map,
                                              bool(with_dist), int(flags) & 1)
        if return_info:
            return idx, (d2 if with_dist else None), {"counters": counters,
                                                      "uncertified": counters.new_zeros(0),
                                                      "exact_path": None}
        return idx, (d2 if with_dist else None)
    if algo != "grid":
        raise ValueError(f"unknown algo {algo!r}")
    comp = list(complete) if complete is not None else [-INF, -INF, -INF, INF, INF, INF]
    p = grid.plan
    halo, cap = p.halo, p.lds_capacity
    idx, d2, counters, uncert, fallback = load().query(grid.sorted, grid.cell_start, grid.geom, list(p.dims), int(k), nq,
                                             id_map, comp, list(p.tile), int(halo), int(cap), bool(use_tiles),
                                             bool(with_dist), int(flags), None, 0, None, int(first),
                                             int(p.xsub))
    if return_info:
        return idx, (d2 if with_dist else None), {"counters": counters, "uncertified": uncert,
                                                  "exact_path": fallback}
    return idx, (d2 if with_dist else None)


def knn(points: torch.Tensor, k: int = 16, points_per_cell: float = 0.0, deterministic: bool = True,
        use_tiles: bool = True, with_dist: bool = True, adaptive: bool = True, algo: str = "auto"):
    """All-points k-nearest neighbours on the GPU. Returns ``(idx int32 (N,k), d2 float32 (N,k))``.
    ``algo``: "auto" (grid, or the tree when the adaptive grid had to be refined), "grid", "tree"."""
    g = build_grid(points, k, points_per_cell=points_per_cell, deterministic=deterministic, adaptive=adaptive)
    if not use_tiles:
        algo = "grid"
    return query(g, k, use_tiles=use_tiles, with_dist=with_dist, algo=algo)


def to_stored_space(idx: torch.Tensor, perm: torch.Tensor) -> torch.Tensor:
    """Original-space result -> reference stored-space view (knearests.cu:129,145)."""
    return load().to_stored_space(idx.contiguous(), perm.contiguous())


# ---------------------------------------------------------------------------- CPU ops ---
def knn_cpu(points: torch.Tensor, k: int = 16, method: str = "grid", threads: int = 0,
            n_queries: Optional[int] = None, complete: Optional[Sequence[float]] = None,
            points_per_cell: float = 0.0):
    """Host kNN. ``method``: 'grid' (engine algorithm), 'kdtree' (oracle) or 'brute'."""
    pts = points.detach().to("cpu", torch.float32).contiguous()
    C = load()
    if method == "kdtree":
        return tuple(C.kdtree_knn(pts, int(k), int(threads)))
    if method == "brute":
        return tuple(C.brute_knn(pts, int(k), int(threads)))
    if method != "grid":
        raise ValueError(f"unknown method {method!r}")
    nq = pts.size(0) if n_queries is None else int(n_queries)
    comp = list(complete) if complete is not None else [-INF, -INF, -INF, INF, INF, INF]
    idx, d2, unc = C.grid_knn_cpu(pts, nq, int(k), float(points_per_cell), comp, int(threads))
    return idx, d2, unc


def check_knn(points: torch.Tensor, idx: torch.Tensor, oracle_idx: torch.Tensor,
              oracle_d2: torch.Tensor) -> dict:
    """Distance-aware comparison (see csrc/host/host.hpp ``check_knn``), vectorised in torch.

    Rows must hold valid, distinct, non-self ids in ascending distance whose fp32 squared
    distances equal the oracle's bit for bit; ids may differ only among equal distances.
    """
    pts = points.detach().cpu().float()
    idx = idx.detach().cpu().long()
    oi = oracle_idx.detach().cpu().long()
    od = oracle_d2.detach().cpu().float()
    n, k = idx.shape
    empty = idx < 0
    bad = (empty != (oi < 0)).any(1)
    safe = idx.clamp(min=0)
    bad |= (safe >= pts.size(0)).any(1)
    safe = safe.clamp(max=pts.size(0) - 1)
    rows = torch.arange(n).unsqueeze(1)
    bad |= ((safe == rows) & ~empty).any(1)
    srt = torch.sort(torch.where(empty, torch.full_like(safe, -1 - torch.arange(k).unsqueeze(0)).expand_as(safe), safe), 1).values
    bad |= (srt[:, 1:] == srt[:, :-1]).any(1)
    q = pts[:n].unsqueeze(1)
    c = pts[safe]
    dx, dy, dz = (c - q).unbind(-1)
    d2 = torch.addcmul(torch.addcmul(dx * dx, dy, dy), dz, dz)  # rounding may differ from fma; compare loosely
    d2 = torch.where(empty, torch.full_like(d2, INF), d2)
    bad |= (d2[:, 1:] < d2[:, :-1] * (1 - 1e-6)).any(1)
    rel = (d2 - od).abs() / od.abs().clamp(min=1e-30)
    bad |= ((rel > 1e-5) & ~empty).any(1)
    nb = int(bad.sum())
    return {"rows": n, "bad_rows": nb, "first_bad": int(bad.nonzero()[0, 0]) if nb else -1}


def read_xyz(path: str, normalize: bool = False) -> torch.Tensor:
    """Read a reference-format .xyz file (first line = count); optional [0,1000]^3 normalisation."""
    return load().read_xyz(str(path), bool(normalize))


def write_xyz(path: str, points: torch.Tensor) -> None:
    load().write_xyz(str(path), points.detach().cpu().float().contiguous())


def normalize_1000(points: torch.Tensor) -> torch.Tensor:
    return load().normalize_1000(points.detach().cpu().float().contiguous())


def expected_kth_radius(n: int, k: int, volume: float) -> float:
    """K-th neighbour radius of a uniform cloud of n points in ``volume``."""
    return (3.0 * (k + 1) * volume / (4.0 * math.pi * max(1, n))) ** (1.0 / 3.0)
