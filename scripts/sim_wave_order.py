"""numpy replay of the lane walk's wave cost under different assignments of a tile's queries to
waves (re-bucket queries so a wave stops paying its slowest lane's rows).

Models knn_tile_kernel<K, M, LANE=true> as built for K <= 40 (csrc/kernels/query.hip):
  * inner 3x3 rows (z then y centre-out 0, +1, -1) row-synchronous: a row iteration costs the
    wave 3 * max(span // 3) + max(span % 3) candidate steps (unroll-3 loop + remainder);
  * outer rows (Chebyshev ring 2 of the 5x5 block) PACKED: each lane marks the rows its bound
    reaches (distance-sorted table, mirrored to the lane's half of its cell), iteration i visits
    every lane's i-th marked row;
  * the K+M+1 bound (self included, as in the kernel).
Orders: row (shipped: tile row (z, y) then x), quad (quadrant of the query inside its (y, z)
cell, then row order), oct (+ x half), morton4 (2-bit Morton of (fy, fz)), sorted by predicted
span (sum of inner-row chord lengths at the expected bound), ...
usage: python scripts/sim_wave_order.py K xsub [ntiles]
"""
import os
import sys

import numpy as np

rng = np.random.default_rng(2)
G = 28
rho = 3.4
N = int(G ** 3 * rho)
P = rng.random((N, 3)) * G
K = int(sys.argv[1]) if len(sys.argv) > 1 else 16
xs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
NT = int(sys.argv[3]) if len(sys.argv) > 3 else 6
M = 2 if K <= 32 else 1
KM = K + M + 1
H = 2
cx = np.floor(P[:, 0] * xs).astype(int)
cy = np.floor(P[:, 1]).astype(int)
cz = np.floor(P[:, 2]).astype(int)
key = (cz * G + cy) * (G * xs) + cx
o = np.lexsort((np.arange(N), key))
ks = key[o]
Ps = P[o]
start = np.searchsorted(ks, np.arange(G * G * G * xs + 1))


def gap(m):
    return m - 0.75 if m > 0 else (-m - 0.25 if m < 0 else 0.0)


def co(m):
    return 2 * m - 1 if m > 0 else -2 * m


ent = [(oy, oz) for oz in range(-H, H + 1) for oy in range(-H, H + 1)]
ent.sort(key=lambda e: (gap(e[0]) ** 2 + gap(e[1]) ** 2, abs(e[1]), abs(e[0]), -e[1], -e[0]))
outer = [e for e in ent if max(abs(e[0]), abs(e[1])) >= 2]
inner = [(dy, dz) for dz in (0, 1, -1) for dy in (0, 1, -1)]


def slab(q, c):
    return max(0.0, c - q, q - (c + 1))


def walk(q):
    """Per-lane spans: inner rows (9 entries, 0 = skipped) and the packed outer rows in visit
    order (list of spans of the rows that were marked)."""
    qcx = int(q[0] * xs)
    qcy = int(q[1])
    qcz = int(q[2])
    Hx = H * xs
    best = np.full(KM, np.inf)

    def span(y, z):
        dyz2 = slab(q[1], y) ** 2 + slab(q[2], z) ** 2
        tau = best[-1]
        if dyz2 > tau:
            return 0
        if np.isinf(tau):
            x0, x1 = qcx - Hx, qcx + Hx
        else:
            rr = np.sqrt(tau - dyz2)
            x0 = max(qcx - Hx, int(np.floor((q[0] - rr) * xs)))
            x1 = min(qcx + Hx, int(np.floor((q[0] + rr) * xs)))
        if x0 > x1:
            return 0
        base = (z * G + y) * (G * xs)
        s0 = start[base + x0]
        s1 = start[base + x1 + 1]
        if s1 > s0:
            d = ((Ps[s0:s1] - q) ** 2).sum(1)
            for v in d:
                if v < best[-1]:
                    best[-1] = v
                    best.sort()
        return s1 - s0

    si = [span(qcy + dy, qcz + dz) for (dy, dz) in inner]
    fy = q[1] - qcy
    fz = q[2] - qcz
    sgy = -1 if fy < 0.5 else 1
    sgz = -1 if fz < 0.5 else 1
    tau0 = best[-1]
    marked = [(oy, oz) for (oy, oz) in outer
              if slab(q[1], qcy + sgy * oy) ** 2 + slab(q[2], qcz + sgz * oz) ** 2 <= tau0]
    so = [span(qcy + sgy * oy, qcz + sgz * oz) for (oy, oz) in marked]
    return si, so, int(sum(si) + sum(so))


def wave_cost(lanes):
    si = np.array([l[0] for l in lanes])
    c = 0
    rows = 0
    for t in range(si.shape[1]):
        s = si[:, t]
        if (s > 0).any():
            c += 3 * (s // 3).max() + (s % 3).max()
            rows += 1
    n = max(len(l[1]) for l in lanes)
    for i in range(n):
        s = np.array([l[1][i] if i < len(l[1]) else 0 for l in lanes])
        if (s > 0).any():
            c += 3 * (s // 3).max() + (s % 3).max()
        rows += 1
    return c, rows


tiles = []
trng = np.random.default_rng(7)
while len(tiles) < NT:
    t = tuple(int(v) for v in trng.integers(3, G - 7, 3))
    tiles.append(t)

ORDERS = os.environ.get("ORDERS", "row,quad,oct,morton4,pred,exact").split(",")
res = {k: [0, 0, 0] for k in ORDERS}
cand = 0.0
nq = 0
for (tx, ty, tz) in tiles:
    sel = np.where((P[:, 0] >= tx) & (P[:, 0] < tx + 4) & (P[:, 1] >= ty) & (P[:, 1] < ty + 4) &
                   (P[:, 2] >= tz) & (P[:, 2] < tz + 4))[0]
    Q = P[sel]
    k2 = (np.floor(Q[:, 2]) * G + np.floor(Q[:, 1])) * G * xs + np.floor(Q[:, 0] * xs)
    ordr = np.lexsort((sel, k2))
    Q = Q[ordr]
    L = [walk(q) for q in Q]
    cand += sum(l[2] for l in L)
    nq += len(L)
    fy = Q[:, 1] - np.floor(Q[:, 1])
    fz = Q[:, 2] - np.floor(Q[:, 2])
    fx = Q[:, 0] * xs - np.floor(Q[:, 0] * xs)
    base = np.arange(len(Q))
    for name in ORDERS:
        if name == "row":
            perm = base
        elif name == "quad":
            perm = np.lexsort((base, (fy >= 0.5) + 2 * (fz >= 0.5)))
        elif name == "oct":
            perm = np.lexsort((base, (fx >= 0.5) + 2 * (fy >= 0.5) + 4 * (fz >= 0.5)))
        elif name == "morton4":
            iy = np.minimum(3, (fy * 4).astype(int))
            iz = np.minimum(3, (fz * 4).astype(int))
            m = sum((((iy >> b) & 1) << (2 * b)) | (((iz >> b) & 1) << (2 * b + 1)) for b in range(2))
            perm = np.lexsort((base, m))
        elif name == "pred":
            # predicted cost: distance of the query to its cell's y/z faces (near faces need
            # the neighbour rows): sort by the max-face-distance class, then quadrant
            dy = np.minimum(fy, 1 - fy)
            dz = np.minimum(fz, 1 - fz)
            perm = np.lexsort((base, (fy >= 0.5) + 2 * (fz >= 0.5), np.minimum(dy, dz) < 0.2))
        elif name == "exact":
            # oracle: sorted by each lane's true total (upper bound of what any cheap key can do)
            perm = np.argsort([l[2] for l in L], kind="stable")
        else:
            raise SystemExit(name)
        for c0 in range(0, len(Q), 64):
            w = [L[i] for i in perm[c0:c0 + 64]]
            cst, rows = wave_cost(w)
            res[name][0] += cst
            res[name][1] += rows
            res[name][2] += 1
print(f"K={K} xsub={xs} KM={KM} tiles={NT} mean candidates/query {cand / nq:.1f}")
for name in ORDERS:
    c, r, nw = res[name]
    print(f"  {name:8s} candidate steps/wave {c / nw:6.1f}   row iterations/wave {r / nw:5.1f}")
