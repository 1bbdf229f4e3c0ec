"""Spatial domain decomposition of the point grid across ranks (NEW: the reference is single-GPU).

World sizes factor into a px x py x pz box grid (2 -> 2x1x1, 4 -> 2x2x1, 8 -> 2x2x2, any N by
balanced factorisation, largest factor on the longest axis). Each rank owns one box; a point
belongs to the box containing it. With 2x2x2 every rank neighbours all 7 others, so the halo
all-to-all uses every point-to-point xGMI link of an MI355X node.

Boxes are either equal-volume slices of the domain, or COUNT-BALANCED (``splits``): a kd
decomposition with x splits at global quantiles, then y splits per x slab, then z splits per
(x, y) column, so a clustered cloud gives every rank about N / world points
(:func:`balanced_splits`; the native router reads the same kd layout, ``kn::RouteParams``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Optional, Sequence

import torch

SPLIT_BINS = 4096  # histogram bins per axis for the quantile splits


def factor3(world: int, extent: Sequence[float] = (1.0, 1.0, 1.0), tol: float = 1e-2) -> tuple:
    """Balanced 3-factorisation of ``world`` (minimises the surface of the rank boxes).

    Factorisations within ``tol`` (relative) of the best surface count as ties and the first one
    in a fixed order wins. A nearly cubic cloud (random data: extents 999.98 / 999.99 / 999.97)
    therefore always gets the same grid as the exact cube. Otherwise the split axis would
    follow noise, and data laid out by one grid would be re-routed by another."""
    cands = []
    for a in range(1, world + 1):
        if world % a:
            continue
        for b in range(1, world // a + 1):
            if (world // a) % b:
                continue
            c = world // a // b
            f = (a, b, c)
            # surface of one box for the given domain extent
            bx, by, bz = (extent[i] / f[i] for i in range(3))
            cands.append((f, bx * by + by * bz + bx * bz))
    best_cost = min(c for _, c in cands)
    return next(f for f, c in cands if c <= best_cost * (1.0 + tol))


def split_count(grid: Sequence[int]) -> int:
    """Floats in a kd splits array for decomposition ``grid`` (kn::route_split_count)."""
    px, py, pz = grid
    return (px + 1) + px * (py + 1) + px * py * (pz + 1)


def _edges(hist: torch.Tensor, parts: int, lo: torch.Tensor, hi: torch.Tensor) -> torch.Tensor:
    """Quantile edges of each row of ``hist`` (rows x SPLIT_BINS counts): (rows, parts + 1) float32,
    first = lo, last = hi, inner edges at the upper edge of the bin holding the j/parts quantile."""
    cs = hist.cumsum(-1)
    tot = cs[:, -1:]
    j = torch.arange(1, parts, device=hist.device, dtype=torch.int64)
    t = (tot * j + parts - 1) // parts
    b = torch.searchsorted(cs, t)
    ext = hi - lo
    inner = lo + (b.double() + 1.0) * ext / SPLIT_BINS
    inner = torch.minimum(torch.maximum(inner, lo), hi).float()
    rows = hist.size(0)
    return torch.cat([lo.float().expand(rows, 1), inner, hi.float().expand(rows, 1)], 1)


def balanced_splits(points: torch.Tensor, lo: torch.Tensor, hi: torch.Tensor, grid: Sequence[int],
                    gather: Callable[[torch.Tensor], torch.Tensor]) -> torch.Tensor:
    """Count-balanced kd splits (float32, on ``points.device``, layout of kn::RouteParams): three
    histogram passes (x; y per x slab; z per column) of SPLIT_BINS bins, each summed over the
    ranks through ``gather`` (an all-gather-cat). ``lo``/``hi``: the global domain as 3-element
    tensors (may stay on the device: no host synchronisation). Collective: every rank calls it."""
    px, py, pz = grid
    dev = points.device
    world_sum = lambda h: gather(h.contiguous()).view(-1, h.numel()).sum(0)  # noqa: E731
    lo = lo.to(dev, torch.float64).flatten()
    hi = hi.to(dev, torch.float64).flatten()
    lo32, ext32 = lo.float(), (hi - lo).float().clamp(min=1e-30)
    B = SPLIT_BINS

    def bins(a: int) -> torch.Tensor:
        f = (points[:, a] - lo32[a]) / ext32[a] * B
        return torch.floor(f).clamp(0, B - 1).long()

    one = torch.ones(points.size(0), dtype=torch.int64, device=dev)
    hx = world_sum(torch.zeros(B, dtype=torch.int64, device=dev).index_add_(0, bins(0), one))
    ex = _edges(hx.view(1, B), px, lo[0:1].view(1, 1), hi[0:1].view(1, 1))[0]  # (px + 1,)
    ix = (points[:, 0:1] >= ex[1:px].view(1, -1)).sum(1) if px > 1 else torch.zeros_like(one)
    hy = world_sum(torch.zeros(px * B, dtype=torch.int64, device=dev).index_add_(0, ix * B + bins(1), one))
    ey = _edges(hy.view(px, B), py, lo[1:2].view(1, 1), hi[1:2].view(1, 1))  # (px, py + 1)
    iy = (points[:, 1:2] >= ey[ix, 1:py]).sum(1) if py > 1 else torch.zeros_like(one)
    col = ix + px * iy
    hz = world_sum(torch.zeros(px * py * B, dtype=torch.int64, device=dev).index_add_(0, col * B + bins(2), one))
    ez = _edges(hz.view(px * py, B), pz, lo[2:3].view(1, 1), hi[2:3].view(1, 1))  # (px * py, pz + 1)
    return torch.cat([ex, ey.flatten(), ez.flatten()]).contiguous()


@dataclass
class SpatialDecomposition:
    world: int
    lo: tuple  # global domain
    hi: tuple
    grid: tuple = None  # (px, py, pz)
    splits: Optional[list] = None  # count-balanced kd splits (host floats), see balanced_splits

    def __post_init__(self):
        ext = tuple(max(self.hi[a] - self.lo[a], 1e-30) for a in range(3))
        if self.grid is None:
            self.grid = factor3(self.world, ext)
        assert self.grid[0] * self.grid[1] * self.grid[2] == self.world
        if self.splits is not None:
            self.splits = [float(v) for v in self.splits]
            assert len(self.splits) == split_count(self.grid)

    def coords(self, rank: int) -> tuple:
        px, py, _ = self.grid
        return rank % px, (rank // px) % py, rank // (px * py)

    def _kd(self):
        px, py, pz = self.grid
        s = self.splits
        xs = s[:px + 1]
        ys = s[px + 1:px + 1 + px * (py + 1)]
        zs = s[px + 1 + px * (py + 1):]
        return xs, ys, zs

    def rank_box(self, rank: int) -> tuple:
        c = self.coords(rank)
        if self.splits is not None:
            px, py, pz = self.grid
            xs, ys, zs = self._kd()
            col = c[0] + px * c[1]
            lo = (xs[c[0]], ys[c[0] * (py + 1) + c[1]], zs[col * (pz + 1) + c[2]])
            hi = (xs[c[0] + 1], ys[c[0] * (py + 1) + c[1] + 1], zs[col * (pz + 1) + c[2] + 1])
            return lo, hi
        lo, hi = [], []
        for a in range(3):
            w = (self.hi[a] - self.lo[a]) / self.grid[a]
            lo.append(self.lo[a] + c[a] * w)
            hi.append(self.hi[a] if c[a] == self.grid[a] - 1 else self.lo[a] + (c[a] + 1) * w)
        return tuple(lo), tuple(hi)

    def owner(self, points: torch.Tensor) -> torch.Tensor:
        """Owning rank of each point (int64). Points outside the domain clamp to edge boxes."""
        dev = points.device
        if self.splits is not None:
            # kd splits: inner splits <= the coordinate (a point on a split belongs to the upper
            # box), compared in float32 as the native router does
            px, py, pz = self.grid
            xs, ys, zs = (torch.tensor(v, dtype=torch.float32, device=dev) for v in self._kd())
            ix = (points[:, 0:1] >= xs[1:px].view(1, -1)).sum(1)
            iy = (points[:, 1:2] >= ys.view(px, py + 1)[ix, 1:py]).sum(1)
            col = ix + px * iy
            iz = (points[:, 2:3] >= zs.view(px * py, pz + 1)[col, 1:pz]).sum(1)
            return ix + px * (iy + py * iz)
        lo = torch.tensor(self.lo, dtype=torch.float32, device=dev)
        hi = torch.tensor(self.hi, dtype=torch.float32, device=dev)
        g = torch.tensor(self.grid, dtype=torch.float32, device=dev)
        f = (points - lo) / (hi - lo).clamp(min=1e-30) * g
        c = torch.floor(f).clamp(min=0)
        c = torch.minimum(c, g - 1).long()
        return c[:, 0] + self.grid[0] * (c[:, 1] + self.grid[1] * c[:, 2])

    def complete_box(self, rank: int, h: float) -> list:
        """Box in which a rank holding its points + an h-halo has the complete cloud: its own box
        grown by h, unbounded on the faces that lie on the global domain boundary."""
        lo, hi = self.rank_box(rank)
        c = self.coords(rank)
        out_lo, out_hi = [], []
        for a in range(3):
            out_lo.append(-math.inf if c[a] == 0 else lo[a] - h)
            out_hi.append(math.inf if c[a] == self.grid[a] - 1 else hi[a] + h)
        return out_lo + out_hi

    def box_dist2(self, points: torch.Tensor, rank: int) -> torch.Tensor:
        """Squared distance from each point to rank's box (0 inside)."""
        lo, hi = self.rank_box(rank)
        dev = points.device
        lo_t = torch.tensor(lo, dtype=torch.float32, device=dev)
        hi_t = torch.tensor(hi, dtype=torch.float32, device=dev)
        d = torch.clamp(lo_t - points, min=0) + torch.clamp(points - hi_t, min=0)
        dd = d * d
        # fixed summation order ((x + y) + z): the native router (route.hip) uses the same
        return (dd[:, 0] + dd[:, 1]) + dd[:, 2]

    def boxes(self) -> list:
        """All rank boxes flattened [lo0, lo1, lo2, hi0, hi1, hi2] * world (router input)."""
        out = []
        for r in range(self.world):
            lo, hi = self.rank_box(r)
            out += list(lo) + list(hi)
        return out
