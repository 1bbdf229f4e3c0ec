"""python -m cuda_knearests_amd -- the reference driver's flow from Python (reference
test_knearests.cu:117-235): load a ``.xyz`` file (count header + "x y z" lines, normalised to
[0,1000]^3 like test_knearests.cu:15-78), solve kNN of every point, optionally check against the
kd-tree oracle (distance-aware: ids must reproduce the oracle's distances) and write the rows.

  python -m cuda_knearests_amd points.xyz [--k 16] [--device cuda|cpu] [--check] [--out nb.txt]
                                          [--batch B] [--json]

GPU: the KNearests engine (grid / tree kernels); ``--batch B`` solves query ranges of B points
(no N x K device result). CPU (``--device cpu`` or no GPU): the native CPU grid solver.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m cuda_knearests_amd", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("xyz")
    ap.add_argument("--k", type=int, default=50, help="neighbours per point (reference default 50)")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--check", action="store_true", help="compare with the kd-tree oracle")
    ap.add_argument("--out", default="", help="write the neighbour rows (original ids, one row per point)")
    ap.add_argument("--batch", type=int, default=0, help="GPU: solve query ranges of this many points")
    ap.add_argument("--json", action="store_true", help="print one JSON summary line")
    a = ap.parse_args(argv)

    from . import KNearests, knn_cpu, read_xyz
    from .utils.check import assert_knn_exact

    pts = read_xyz(a.xyz, normalize=True)
    n, k = pts.size(0), a.k
    print(f"{n} points, K={k}, device {a.device}", file=sys.stderr)
    t0 = time.perf_counter()
    if a.device == "cpu":
        idx, d2, _ = knn_cpu(pts, k, "grid")
    else:
        dev = torch.device(a.device)
        m = KNearests(k=k, device=dev).prepare(pts.to(dev))
        if a.batch > 0:
            parts = [m.solve_range(f, min(a.batch, n - f)) for f in range(0, n, a.batch)]
            idx = torch.cat([p[0] for p in parts])
            d2 = torch.cat([p[1] for p in parts])
        else:
            m.solve()
            idx, d2 = m.neighbors, m.distances
        torch.cuda.synchronize(dev)
        idx, d2 = idx.cpu(), d2.cpu()
    ms = (time.perf_counter() - t0) * 1e3
    print(f"knn: {ms:.3f} ms (load excluded)", file=sys.stderr)
    ok = True
    if a.check:
        _, od = knn_cpu(pts, k, "kdtree")
        try:
            assert torch.equal(d2, od), "distances differ from the kd-tree oracle"
            assert_knn_exact(pts, torch.arange(n), idx, d2, od)
        except AssertionError as e:
            ok = False
            print(f"FAILED: {e}", file=sys.stderr)
    if a.out:
        with open(a.out, "w") as f:
            for row in idx.tolist():
                f.write(" ".join(str(v) for v in row) + "\n")
    if a.json:
        print(json.dumps({"n": n, "k": k, "device": a.device, "ms": round(ms, 3), "checked": a.check, "ok": ok}))
    print("ok" if ok else "FAILED", file=sys.stderr)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
