"""CPU study of halo rules for the spatial split (no GPU): how many halo rows each rank receives
under (a) the global width h = f x the mean-density K-th radius (the plan's rule), (b) the exact
need (every point that is among the K nearest of a query owned by another rank), and (c) a
width field H on a coarse cell grid, splatted from the previous step's measured K-th distances
of the queries whose ball leaves their box (H[c] = max R over the queries within m cells, m =
ceil(R / s)), with the matching certification (R <= min H over the m-neighbourhood).

usage: python scripts/halo_study.py [clustered|uniform|surface] [n_total] [world] [k]"""
import math
import sys
import time

import numpy as np
import torch
from scipy.spatial import cKDTree

from cuda_knearests_amd.parallel.decomposition import SpatialDecomposition, balanced_splits, factor3
from cuda_knearests_amd.utils import clustered_cloud, surface_cloud, uniform_cloud

gen = sys.argv[1] if len(sys.argv) > 1 else "clustered"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 7_200_000
world = int(sys.argv[3]) if len(sys.argv) > 3 else 8
k = int(sys.argv[4]) if len(sys.argv) > 4 else 16
pts = {"clustered": clustered_cloud, "uniform": uniform_cloud, "surface": surface_cloud}[gen](n, seed=0)
t0 = time.time()
lo, hi = pts.min(0).values.double(), pts.max(0).values.double()
grid = factor3(world, tuple((hi - lo).tolist()))
splits = balanced_splits(pts, lo, hi, grid, lambda h: h)
dec = SpatialDecomposition(world, tuple(lo.tolist()), tuple(hi.tolist()), grid, splits.tolist())
own = dec.owner(pts)
boxes = torch.tensor([list(a) + list(b) for a, b in (dec.rank_box(r) for r in range(world))], dtype=torch.float64)
tree = cKDTree(pts.numpy())
d, idx = tree.query(pts.numpy(), k=k + 1, workers=8)
R = torch.from_numpy(d[:, -1]).float()  # K-th distance (self is the 0-th)
nb = torch.from_numpy(idx[:, 1:].astype(np.int64))
print(f"# {gen} n={n} world={world} grid={grid} k={k}: kNN {time.time() - t0:.1f}s", flush=True)
cnt = torch.bincount(own, minlength=world).double()


def box_d(p, r):  # distance to rank r's box
    b = boxes[r]
    dd = torch.clamp(b[:3].float() - p, min=0) + torch.clamp(p - b[3:].float(), min=0)
    return dd.norm(dim=1)


def margin(p, r):  # distance to the nearest face of r's box that is not a domain face
    b = boxes[r]
    m = torch.full((p.size(0),), math.inf)
    for a in range(3):
        if b[a] > lo[a]:
            m = torch.minimum(m, p[:, a] - float(b[a]))
        if b[3 + a] < hi[a]:
            m = torch.minimum(m, float(b[3 + a]) - p[:, a])
    return m


def report(name, sent):  # sent: (world,) halo rows received per rank
    frac = sent / cnt
    print(f"{name:42s} halo_frac max {frac.max():.4f} mean {frac.mean():.4f}", flush=True)


# (b) exact need
need = torch.zeros(world)
for r in range(world):
    q = own == r
    x = nb[q].flatten()
    x = x[own[x] != r].unique()
    need[r] = x.numel()
report("exact need (reverse kNN across boxes)", need)

# (a) global width
vol = float(torch.prod(hi - lo))
rk = (3.0 * (k + 1) * vol / (4.0 * math.pi * n)) ** (1.0 / 3.0)
for f in (2.5, 4.0):
    h = f * rk
    s = torch.zeros(world)
    for r in range(world):
        o = own != r
        s[r] = int((box_d(pts[o], r) <= h).sum())
    report(f"global width f={f} h={h:.1f}", s)

# (c) width field on cells of size s (from the measured R of boundary queries)
bq = torch.zeros(n, dtype=torch.bool)
for r in range(world):
    q = (own == r).nonzero().flatten()
    bq[q] = R[q] > margin(pts[q], r)
print(f"boundary queries: {int(bq.sum())} ({bq.float().mean():.4f}); R max {R.max():.1f}, "
      f"p99.9 {R.quantile(0.999):.1f}", flush=True)
for G in (16, 32, 64, 128):
    ext = (hi - lo).float()
    cs = ext / G
    cell = lambda p: torch.minimum(((p - lo.float()) / cs).floor().long().clamp(min=0), torch.tensor(G - 1))  # noqa
    H = torch.zeros(G ** 3)
    qi = bq.nonzero().flatten()
    m = torch.ceil(R[qi] / cs.min()).long()
    c = cell(pts[qi])
    lost = int((m > 3).sum())
    for mm in (1, 2, 3):
        sel = m == mm
        if not sel.any():
            continue
        cc, rr = c[sel], R[qi][sel]
        r1 = torch.arange(-mm, mm + 1)
        off = torch.stack(torch.meshgrid(r1, r1, r1, indexing="ij"), -1).view(-1, 3)
        for i0 in range(0, cc.size(0), 20000):
            ci = cc[i0:i0 + 20000, None, :] + off[None]
            ok = ((ci >= 0) & (ci < G)).all(-1)
            flat = (ci[..., 0] + G * (ci[..., 1] + G * ci[..., 2]))[ok]
            val = rr[i0:i0 + 20000, None].expand(-1, off.size(0))[ok]
            H.scatter_reduce_(0, flat, val, "amax")
    cp = cell(pts)
    hp = H[cp[:, 0] + G * (cp[:, 1] + G * cp[:, 2])] * 1.0001
    s = torch.zeros(world)
    for r in range(world):
        o = own != r
        s[r] = int((box_d(pts[o], r) <= hp[o]).sum())
    report(f"field G={G} (cell {float(cs.min()):.1f}; {lost} queries R > 3 cells)", s)
