"""Lockstep replay of the K <= 40 lane walk (knn_tile_kernel<K, M, LANE=true>, csrc/kernels/query.hip)
under different top-K insertion policies (decouple a lane's insertion cost from
the wave's).

Walk model (as shipped): the 3x3 inner rows (z then y, centre-out 0, +1, -1) row-synchronous, then
the outer ring of the 5x5 block packed (each lane marks the rows its bound reaches; iteration i
visits every lane's i-th marked row). A row iteration runs the unroll-3 loop: steps = 3 *
max(span // 3) + max(span % 3) over the lanes; a lane's candidate at a step is its next point.

Policies:
  now      the shipped ballot-gated network: a step runs the KM-slot med3 network when ANY lane's
           key is below its current bound (the bound updates at once).
  q<B>[r]  deferred: a key below the lane's bound AS OF ITS LAST FLUSH goes into a per-lane queue
           (LDS); when some lane's queue holds B keys the wave flushes (networks = the largest
           queue, every queue drained); 'r': also flush at the end of every row iteration (the
           row cuts of the next row then use a fresh bound). Bounds and row cuts see only
           flushed keys.

Cost (issue cycles per wave, calibrated classes): candidate step 25 (+6 queue
write and +3 capacity check in the deferred policies), network KM * 4 (+8 drain overhead per
deferred network), row iteration 150.
usage: python scripts/sim_deferred_topk.py K [xsub] [ntiles] [policies]"""
import re
import sys

import numpy as np

rng = np.random.default_rng(2)
G = 28
rho = 3.4
N = int(G ** 3 * rho)
P = rng.random((N, 3)) * G
K = int(sys.argv[1]) if len(sys.argv) > 1 else 16
xs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
NT = int(sys.argv[3]) if len(sys.argv) > 3 else 4
POL = (sys.argv[4] if len(sys.argv) > 4 else "now,q4,q4r,q8,q8r,q16r").split(",")
M = 2
KM = K + M + 1
H = 2
cxa = np.floor(P[:, 0] * xs).astype(int)
cya = np.floor(P[:, 1]).astype(int)
cza = np.floor(P[:, 2]).astype(int)
key = (cza * G + cya) * (G * xs) + cxa
o = np.lexsort((np.arange(N), key))
Ps = P[o]
start = np.searchsorted(key[o], np.arange(G * G * G * xs + 1))


def gap(m):
    return m - 0.75 if m > 0 else (-m - 0.25 if m < 0 else 0.0)


ent = [(oy, oz) for oz in range(-H, H + 1) for oy in range(-H, H + 1)]
ent.sort(key=lambda e: (gap(e[0]) ** 2 + gap(e[1]) ** 2, abs(e[1]), abs(e[0]), -e[1], -e[0]))
outer = [e for e in ent if max(abs(e[0]), abs(e[1])) >= 2]
inner = [(dy, dz) for dz in (0, 1, -1) for dy in (0, 1, -1)]


def slab(q, c):
    return max(0.0, c - q, q - (c + 1))


class Lane:
    def __init__(self, q):
        self.q = q
        self.c = (int(q[0] * xs), int(q[1]), int(q[2]))
        self.keys = np.full(KM, np.inf)  # sorted top-(K+M+1), self included (as in the kernel)
        self.queue = []
        self.ins = 0

    def bound(self):
        return self.keys[-1]

    def span(self, y, z):
        q = self.q
        dyz2 = slab(q[1], y) ** 2 + slab(q[2], z) ** 2
        tau = self.bound()
        if dyz2 > tau:
            return np.zeros(0)
        Hx = H * xs
        if np.isinf(tau):
            x0, x1 = self.c[0] - Hx, self.c[0] + Hx
        else:
            rr = np.sqrt(tau - dyz2)
            x0 = max(self.c[0] - Hx, int(np.floor((q[0] - rr) * xs)))
            x1 = min(self.c[0] + Hx, int(np.floor((q[0] + rr) * xs)))
        if x0 > x1:
            return np.zeros(0)
        base = (z * G + y) * (G * xs)
        s0, s1 = start[base + x0], start[base + x1 + 1]
        return ((Ps[s0:s1] - q) ** 2).sum(1)

    def insert(self, v):
        if v < self.keys[-1]:
            self.keys[-1] = v
            self.keys.sort()
            self.ins += 1


def run_wave(qs, pol):
    lanes = [Lane(q) for q in qs]
    st = {"steps": 0, "nets": 0, "rows": 0, "flushes": 0}
    # h<R>q<B>: the first R row iterations insert at once (fill), later ones defer (row-end flush)
    # a<B>: a row iteration defers only when every lane's list is full at its start
    auto = re.match(r"a(\d+)$", pol)
    if auto:
        pol = "h99q" + auto.group(1)
    hyb = re.match(r"h(\d+)q(\d+)$", pol)
    R = int(hyb.group(1)) if hyb else 0
    B = int(hyb.group(2)) if hyb else (int(pol[1:].rstrip("r")) if pol != "now" else 0)
    row_flush = pol.endswith("r") or bool(hyb)
    st["ri"] = 0

    def flush():
        n = max(len(l.queue) for l in lanes)
        if n:
            st["nets"] += n
            st["flushes"] += 1
            for l in lanes:
                for v in l.queue:
                    l.insert(v)
                l.queue = []

    def row_iter(spans):
        # spans: per-lane distance arrays for this row iteration (lockstep unroll-3 loop)
        L = np.array([len(s) for s in spans])
        if not (L > 0).any():
            st["ri"] += 1
            return
        st["rows"] += 1
        nsteps = 3 * (L // 3).max() + (L % 3).max()
        # lane position per step: the unroll-3 body covers positions 3i..3i+2 in lockstep, the
        # remainder loop runs max(L % 3) more steps; model a lane's j-th candidate at step j
        # (same count; the order of positions inside a step group does not change the policies)
        now = pol == "now" or st["ri"] < R
        if auto:
            now = any(np.isinf(l.bound()) for l, s in zip(lanes, spans) if len(s))
        st["ri"] += 1
        for j in range(nsteps):
            st["steps"] += 1
            if now:
                pass_any = False
                for l, s in zip(lanes, spans):
                    if j < len(s) and s[j] < l.bound():
                        pass_any = True
                        l.insert(s[j])
                if pass_any:
                    st["nets"] += 1
            else:
                for l, s in zip(lanes, spans):
                    if j < len(s) and s[j] < l.bound():
                        l.queue.append(s[j])
                if max(len(l.queue) for l in lanes) >= B:
                    flush()
        if row_flush:
            flush()

    for (dy, dz) in inner:
        row_iter([l.span(l.c[1] + dy, l.c[2] + dz) for l in lanes])
    flush()  # the outer-row masks use the flushed bound
    marked = []
    for l in lanes:
        q = l.q
        sgy = -1 if q[1] - l.c[1] < 0.5 else 1
        sgz = -1 if q[2] - l.c[2] < 0.5 else 1
        t0 = l.bound()
        marked.append([(l.c[1] + sgy * oy, l.c[2] + sgz * oz) for (oy, oz) in outer
                       if slab(q[1], l.c[1] + sgy * oy) ** 2 + slab(q[2], l.c[2] + sgz * oz) ** 2 <= t0])
    n = max(len(m) for m in marked)
    for i in range(n):
        row_iter([l.span(*m[i]) if i < len(m) else np.zeros(0) for l, m in zip(lanes, marked)])
    flush()
    ref = [np.sort(((Ps[np.abs(Ps - l.q).max(1) < 3] - l.q) ** 2).sum(1))[:K + 1] for l in lanes]
    ok = all(np.allclose(l.keys[:K + 1], r) for l, r in zip(lanes, ref))
    st["ins"] = np.mean([l.ins for l in lanes])
    return st, ok


trng = np.random.default_rng(7)
tiles = [tuple(int(v) for v in trng.integers(3, G - 7, 3)) for _ in range(NT)]
waves = []
for (tx, ty, tz) in tiles:
    sel = np.where((P[:, 0] >= tx) & (P[:, 0] < tx + 4) & (P[:, 1] >= ty) & (P[:, 1] < ty + 4) &
                   (P[:, 2] >= tz) & (P[:, 2] < tz + 4))[0]
    Q = P[sel]
    k2 = (np.floor(Q[:, 2]) * G + np.floor(Q[:, 1])) * G * xs + np.floor(Q[:, 0] * xs)
    Q = Q[np.lexsort((sel, k2))]
    waves += [Q[c0:c0 + 64] for c0 in range(0, len(Q), 64)]
print(f"K={K} xsub={xs} KM={KM} waves={len(waves)}")
for pol in POL:
    acc = {"steps": 0, "nets": 0, "rows": 0, "flushes": 0, "ins": 0.0, "ri": 0}
    allok = True
    for w in waves:
        st, ok = run_wave(w, pol)
        allok &= ok
        for k in acc:
            acc[k] += st[k]
    nw = len(waves)
    d = pol != "now"
    cyc = (acc["steps"] * (25 + (9 if d else 0)) + acc["nets"] * (KM * 4 + (8 if d else 0)) + acc["rows"] * 150) / nw
    print(f"  {pol:6s} steps/wave {acc['steps'] / nw:6.1f} networks/wave {acc['nets'] / nw:6.1f} "
          f"rows/wave {acc['rows'] / nw:5.1f} flushes/wave {acc['flushes'] / nw:5.1f} "
          f"insertions/lane {acc['ins'] / nw:5.1f}  model cycles/wave {cyc:7.0f}  exact {allok}")
