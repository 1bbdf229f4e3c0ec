"""CPU model of the density-adaptive halo field (csrc/kernels/route.hip field_splat_kernel /
field_cert_kernel, kn::field_geom / field_cell, route_halo's field branch, complete_margin3): the
certification rule is sound for ANY field -- a query certified by the field has every point of
its K-th ball in its rank's local set -- and for the field splatted from the measured K-th
distances of a static cloud every query is certified. Runs without a GPU (float32 numpy
arithmetic mirrors the kernels')."""
import numpy as np
import pytest
from scipy.spatial import cKDTree

LEVELS = 3  # kn::kFieldLevels


def geom(lo, hi, g):
    ext = np.maximum((hi - lo).astype(np.float32), np.float32(1e-30))
    inv = (np.float32(g) / ext).astype(np.float32)
    return lo.astype(np.float32), inv, g, np.float32(0.998) / inv.max()


def cells(fg, p):
    lo, inv, g, _ = fg
    c = np.floor((p.astype(np.float32) - lo) * inv).astype(np.int64)
    return np.clip(c, 0, g - 1)


def flat(g, c):
    return c[..., 0] + g * (c[..., 1] + g * c[..., 2])


def splat(fg, q, R, boundary):
    _, _, g, rstep = fg
    F = np.zeros(g ** 3, np.float32)
    cq = cells(fg, q)
    for i in np.nonzero(boundary)[0]:
        m = 1
        while m < LEVELS and R[i] > m * rstep:
            m += 1
        r = np.arange(-m, m + 1)
        off = np.stack(np.meshgrid(r, r, r, indexing="ij"), -1).reshape(-1, 3)
        cc = np.clip(cq[i] + off, 0, g - 1)
        np.maximum.at(F, flat(g, cc), R[i])
    return F


def cert(fg, F):
    _, _, g, rstep = fg
    F3 = F.reshape(g, g, g)  # [z, y, x]
    out = np.zeros_like(F3)
    best = np.zeros_like(F3)
    for m in range(1, LEVELS + 1):
        mn = np.full_like(F3, np.inf)
        for dz in range(-m, m + 1):
            for dy in range(-m, m + 1):
                for dx in range(-m, m + 1):
                    sh = np.full_like(F3, np.inf)
                    zs = slice(max(0, dz), g + min(0, dz)); zd = slice(max(0, -dz), g + min(0, -dz))
                    ys = slice(max(0, dy), g + min(0, dy)); yd = slice(max(0, -dy), g + min(0, -dy))
                    xs = slice(max(0, dx), g + min(0, dx)); xd = slice(max(0, -dx), g + min(0, -dx))
                    sh[zd, yd, xd] = F3[zs, ys, xs]
                    mn = np.minimum(mn, sh)
        best = np.maximum(best, np.minimum(mn, m * rstep))
    out[...] = best
    return out.reshape(-1)


def box_dist(p, lo, hi):
    d = np.maximum(lo - p, 0) + np.maximum(p - hi, 0)
    return np.sqrt((d * d).sum(1))


@pytest.mark.parametrize("seed,field", [(0, "measured"), (1, "measured"), (2, "random"), (3, "random")])
def test_field_certification_is_sound(seed, field):
    rng = np.random.default_rng(seed)
    n, k, g = 6000, 8, 12
    pts = np.concatenate([rng.random((n // 2, 3)) * 100,
                          50 + 6 * rng.standard_normal((n // 2, 3))]).clip(0, 100).astype(np.float32)
    lo, hi = pts.min(0), pts.max(0)
    fg = geom(lo, hi, g)
    split = np.float32(np.median(pts[:, 0]))  # two ranks split at x = median
    own = (pts[:, 0] >= split).astype(int)
    boxes = [(np.array([lo[0], lo[1], lo[2]]), np.array([split, hi[1], hi[2]])),
             (np.array([split, lo[1], lo[2]]), np.array([hi[0], hi[1], hi[2]]))]
    d, _ = cKDTree(pts).query(pts, k=k + 1)
    R = d[:, -1].astype(np.float32)
    # own-box margin: distance to the split plane (the other faces are domain faces)
    margin = np.where(own == 0, split - pts[:, 0], pts[:, 0] - split)
    if field == "measured":
        F = splat(fg, pts, R * np.float32(1.000001), R > margin)
    else:
        # arbitrary widths around the measured scale, some cells empty
        F = ((0.3 + rng.random(g ** 3)) * R.max() * (rng.random(g ** 3) > 0.1)).astype(np.float32)
    C = cert(fg, F)
    width = F[flat(g, cells(fg, pts))]
    tree = cKDTree(pts)
    certified_by_field = 0
    for r in (0, 1):
        local = (own == r) | (box_dist(pts, *boxes[r]) <= width)  # route_halo's field rule
        q = np.nonzero(own == r)[0]
        cq = C[flat(g, cells(fg, pts[q]))]
        ok = (R[q] <= margin[q]) | (R[q] <= cq)  # complete_margin3 with the field
        certified_by_field += int(((R[q] > margin[q]) & ok).sum())
        for i in q[ok]:
            ball = tree.query_ball_point(pts[i], R[i] * 0.9999)
            assert local[ball].all(), (r, i)
        if field == "measured":
            assert ok.all(), int((~ok).sum())  # a static cloud: every query certified
    assert certified_by_field > 0
