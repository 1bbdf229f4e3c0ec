"""``KNearests`` -- the flagship engine object (Python mirror of the knearests.h C API).

Reference API (knearests.h:21-29): ``kn_prepare / kn_solve / kn_free / kn_get_points /
kn_get_knearests / kn_get_permutation / kn_print_stats``. Here:

    kn = KNearests(k=50)              # default K = 50 (reference params.h:4)
    kn.prepare(points)                # (N,3) tensor / ndarray; uploaded if on the host
    kn.solve()
    kn.get_knearests()                # (N,K) stored-space ids (reference semantics)
    kn.get_permutation()              # perm[stored] = original id
    kn.get_points()                   # stored-order points
    kn.neighbors, kn.distances        # original-order results (extension)
    kn.print_stats()

``device='cpu'`` runs the same algorithm with the native host solver (no GPU needed).
``capture=True`` records build+solve into a CUDA(HIP) graph on the first ``step`` and
replays it afterwards (the bench path).
"""
from __future__ import annotations

import logging
import sys
import time
from typing import Optional

import numpy as np
import torch

from ..ops import knn_ops as ops
from ..ops.knn_ops import QUERY_FLAG_WIDE
from .._ext import load
from ..utils import get_logger

_log = get_logger()


class KNearests:
    def __init__(self, k: int = 50, device: str | torch.device = "cuda", points_per_cell: float = 0.0,
                 tile=(), halo: int = 0, deterministic: bool = True, use_tiles: bool = True,
                 with_distances: bool = True, verbose: bool = False, algo: str = "auto"):
        if not 1 <= int(k) <= 128:
            raise ValueError("k must be in [1, 128]")
        if algo not in ("auto", "grid", "tree"):
            raise ValueError("algo must be 'auto', 'grid' or 'tree'")
        # query structure: the uniform grid, the Morton-leaf tree, or auto (the tree when the
        # occupancy-adaptive grid had to be refined: clusters, surfaces)
        self.algo = algo if use_tiles else "grid"
        self.k = int(k)
        self.device = torch.device(device)
        self.points_per_cell = float(points_per_cell)
        self.tile = tuple(tile)
        self.halo = int(halo)
        self.deterministic = bool(deterministic)
        self.use_tiles = bool(use_tiles)
        self.with_distances = bool(with_distances)
        # verbose=True logs the reference's timing lines at WARNING (always shown); otherwise
        # they are INFO records of the "knearests" logger (env KN_LOG=INFO shows them)
        self.verbose = verbose
        self._qflags = 0  # query flags learned from the last eager solve (wide re-rank window)
        self._lvl = logging.WARNING if verbose else logging.INFO
        self.grid: Optional[ops.Grid] = None
        self.points: Optional[torch.Tensor] = None
        self.neighbors: Optional[torch.Tensor] = None
        self.distances: Optional[torch.Tensor] = None
        self.info: dict = {}
        self.timings = {"ms_build": 0.0, "ms_solve": 0.0}
        self._graph = None  # native engine (hipGraph) used by step(capture=True)
        self._graph_n = -1
        self._static = None

    # ------------------------------------------------------------------ lifecycle ----
    def _as_tensor(self, points) -> torch.Tensor:
        if isinstance(points, np.ndarray):
            points = torch.from_numpy(np.ascontiguousarray(points, dtype=np.float32))
        t = torch.as_tensor(points, dtype=torch.float32)
        if t.dim() != 2 or t.size(1) != 3:
            raise ValueError("points must be (N, 3)")
        return t.to(self.device).contiguous()

    def plan(self, n: int, xsub: int = 0) -> ops.Plan:
        return ops.Plan.auto(n, self.k, self.points_per_cell, self.tile, self.halo, xsub=xsub)

    def prepare(self, points) -> "KNearests":
        """Upload (if needed) and bin the points (reference kn_prepare, knearests.cu:235-344)."""
        self.points = self._as_tensor(points)
        self.neighbors = self.distances = None
        self._graph = None
        if self.device.type == "cpu":
            return self
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        self.grid = ops.build_grid(self.points, self.k, plan=self.plan(self.points.size(0)),
                                   deterministic=self.deterministic, adaptive=True)
        t1.record()
        t1.synchronize()
        self.timings["ms_build"] = t0.elapsed_time(t1)
        _log.log(self._lvl, "kn_firstbuild: %.3f msec (grid %s, algo %s)", self.timings["ms_build"],
                 self.grid.plan.dims, self.grid.extra.get("algo", "grid"))
        return self

    def solve(self) -> "KNearests":
        """All-points kNN (reference kn_solve, knearests.cu:348-392)."""
        if self.points is None:
            raise RuntimeError("solve() before prepare()")
        if self.device.type == "cpu":
            t = time.perf_counter()
            idx, d2, unc = ops.knn_cpu(self.points, self.k, "grid", points_per_cell=self.points_per_cell)
            self.timings["ms_solve"] = (time.perf_counter() - t) * 1e3
            self.neighbors, self.distances = idx, d2
            self.info = {"uncertified": int(unc.numel()), "exact_path": 0}
            _log.log(self._lvl, "kn_solve (cpu): %.3f msec (%s)", self.timings["ms_solve"], self.info)
            return self
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        idx, d2, info = ops.query(self.grid, self.k, use_tiles=self.use_tiles,
                                  with_dist=self.with_distances, return_info=True, algo=self.algo,
                                  flags=self._qflags)
        t1.record()
        t1.synchronize()
        self.timings["ms_solve"] = t0.elapsed_time(t1)
        c = info["counters"].cpu()
        # many cooperative re-rank finishes (exactly equal distances: lattice-like clouds): the
        # next solves take the wide re-rank window (kn/kernels.h kQueryFlagWide), as kn::Engine
        self._qflags = QUERY_FLAG_WIDE if int(c[3]) * 64 > self.grid.n else 0
        algo = self.grid.extra.get("algo", "grid") if self.algo == "auto" else self.algo
        self.info = {"exact_path": int(c[0]), "uncertified": int(c[1]), "dense_tiles": int(c[2]), "algo": algo}
        self.neighbors, self.distances = idx, d2
        _log.log(self._lvl, "kn_solve: %.3f msec (%s)", self.timings["ms_solve"], self.info)
        if self.info["exact_path"] > max(1024, self.grid.n // 100):
            _log.warning("kn_solve: %d of %d queries took the exact path (strongly non-uniform cloud?)",
                         self.info["exact_path"], self.grid.n)
        return self

    def solve_range(self, first: int, count: int):
        """Neighbours of the points with original index in [first, first + count) only: ``(ids,
        d2)`` of shape (count, K), row r = point first + r (extension; the C API's
        kn_solve_range). The whole-cloud N x K result is never allocated, so a cloud whose result
        does not fit next to its grid is solved in batches."""
        if self.grid is None:
            raise RuntimeError("solve_range() before prepare() (GPU)")
        first, count = int(first), int(count)
        if first < 0 or count < 0 or first + count > self.grid.n:
            raise ValueError("query range outside [0, N)")
        return ops.query(self.grid, self.k, n_queries=first + count, use_tiles=self.use_tiles,
                         with_dist=self.with_distances, algo="grid", first=first)

    def set_k(self, k: int) -> "KNearests":
        """Re-solve with another K without rebuilding the grid (extension)."""
        if not 1 <= int(k) <= 128:
            raise ValueError("k must be in [1, 128]")
        self.k = int(k)
        if self.grid is not None:
            p = self.plan(self.grid.n, xsub=self.grid.plan.xsub)  # the x subdivision stays with the grid
            self.grid.plan.halo, self.grid.plan.tile = p.halo, p.tile
            self.grid.plan.lds_capacity = p.lds_capacity
        self.neighbors = self.distances = None
        self._graph = None
        return self

    # ------------------------------------------------------------- bench fast path ---
    def step(self, points: Optional[torch.Tensor] = None, capture: bool = True):
        """build + solve of the whole cloud.

        ``capture=False``: eager torch ops on the current stream. ``capture=True``: the native
        C++ runtime (``kn::Engine``: own device arena and stream); build + solve are captured
        into one hipGraph on first use and replayed on every later call, so a step costs one
        graph launch instead of ~10 kernel launches. Results land in ``neighbors``/``distances``.
        """
        if self.device.type == "cpu":
            if points is not None:
                self.prepare(points)
            return self.solve()
        pts = self.points if points is None else points
        if not capture:
            g = ops.build_grid(pts, self.k, plan=self.plan(pts.size(0)), deterministic=self.deterministic)
            self.neighbors, self.distances = ops.query(g, self.k, use_tiles=self.use_tiles,
                                                       with_dist=self.with_distances, algo=self.algo,
                                                       flags=self._qflags)
            self.grid = g
            return self
        if self._graph is None or self._graph_n != pts.size(0):
            self._graph = load().Engine(self.k, self.points_per_cell, list(self.tile), self.halo,
                                        self.deterministic, self.use_tiles, True, self.device.index or 0,
                                        True, {"auto": 0, "grid": 1, "tree": 2}[self.algo])
            self._graph_n = pts.size(0)
            self._graph.prepare(pts)  # eager first build: decides the (occupancy-adaptive) grid
            self._graph.solve()  # eager first solve: its counters pick the captured query variant
        # the engine keeps its own copy of the input, so every step re-uploads (D2D) + replays
        self._graph.prepare_async(pts)
        self._graph.launch_graph(1)
        self._graph.sync()
        self.neighbors, self.distances = self._graph.results(self.device)
        return self

    # ------------------------------------------------------------------ getters ------
    def get_points(self) -> torch.Tensor:
        """Points in stored (cell-bucketed) order (reference kn_get_points)."""
        if self.device.type == "cpu":
            raise RuntimeError("stored order is a GPU-engine concept; use .points")
        return self.grid.sorted[:, :3].contiguous()

    def get_permutation(self) -> torch.Tensor:
        """perm[stored] = original index (reference kn_get_permutation)."""
        return self.grid.perm

    def get_knearests(self) -> torch.Tensor:
        """(N,K) neighbours in stored space (reference kn_get_knearests semantics)."""
        if self.neighbors is None:
            raise RuntimeError("not solved")
        return ops.to_stored_space(self.neighbors, self.grid.perm)

    def get_distances(self) -> torch.Tensor:
        return self.distances

    def stats(self) -> dict:
        s = dict(self.timings)
        s.update(self.info)
        s["k"] = self.k
        if self.grid is not None:
            cs = self.grid.cell_start
            cnt = (cs[1:] - cs[:-1]).cpu()
            s.update({"n": self.grid.n, "dims": list(self.grid.plan.dims), "num_cells": int(cnt.numel()),
                      "min_cell": int(cnt.min()) if cnt.numel() else 0,
                      "max_cell": int(cnt.max()) if cnt.numel() else 0,
                      "avg_cell": float(cnt.float().mean()) if cnt.numel() else 0.0,
                      "empty_cells": int((cnt == 0).sum()),
                      "histogram": torch.bincount(cnt.long()).tolist()})
        return s

    def print_stats(self, file=sys.stderr) -> None:
        """Reference kn_print_stats (knearests.cu:440-466)."""
        s = self.stats()
        for key in ("n", "k", "dims", "num_cells", "min_cell", "max_cell", "avg_cell", "empty_cells",
                    "exact_path", "uncertified", "ms_build", "ms_solve"):
            if key in s:
                print(f"{key}: {s[key]}", file=file)
        for i, c in enumerate(s.get("histogram", [])):
            if c:
                print(f"  [{i:2d}] {c}", file=file)

    # ---------------------------------------------------------------- persistence ----
    def save(self, path: str) -> None:
        """Save the binned structure (extension: reference rebuilds on every kn_prepare)."""
        g = self.grid
        torch.save({"k": self.k, "sorted": g.sorted.cpu(), "cell_start": g.cell_start.cpu(),
                    "perm": g.perm.cpu(), "geom": g.geom.cpu(), "dims": list(g.plan.dims),
                    "xsub": int(g.plan.xsub), "points": self.points.cpu()}, path)

    @classmethod
    def load(cls, path: str, device="cuda", **kw) -> "KNearests":
        d = torch.load(path, map_location="cpu", weights_only=True)
        kn = cls(k=kw.pop("k", d["k"]), device=device, **kw)
        kn.points = d["points"].to(kn.device)
        plan = kn.plan(d["sorted"].size(0), xsub=int(d.get("xsub", 1)))
        plan.dims = list(d["dims"])
        kn.grid = ops.Grid(d["sorted"].to(kn.device), d["cell_start"].to(kn.device), d["perm"].to(kn.device),
                           d["geom"].to(kn.device), plan, d["sorted"].size(0))
        return kn

    def free(self) -> None:
        """Release device buffers (reference kn_free)."""
        self.grid = self.points = self.neighbors = self.distances = None
        self._graph = self._static = None


def native_loaded() -> bool:
    try:
        load()
        return True
    except Exception:
        return False
