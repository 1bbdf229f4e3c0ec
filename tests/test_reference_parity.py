"""Parity with the reference's own oracle semantics on the reference's own fixture.

The reference validates its GPU result (test_knearests.cu:196-231) against its kd-tree with
K+1 neighbours, self dropped, rows compared as SETS (each row sorted by id). Its distance is the
non-fused float sum ((0 + dx^2) + dy^2) + dz^2 (kd_tree.cpp:13-19) and, at equal distances, the
first point found stays (kd_tree.h:102-117: strict `>=` rejection). Our oracles and kernels use
an fma chain and break ties by id. This test pins how far the two semantics can differ on
pts20K.xyz (normalised to [0,1000]^3 as test_knearests.cu:65-78 does): a brute force with the
reference arithmetic (numpy float32, same operation order) gives the reference's neighbour sets;
every row must equal ours as a set unless the reference's K-th and (K+1)-th distances are within
a few ulps (a near-tie where either arithmetic or tie rule may pick either point). Measured:
K=8 2 rows, K=16 0, K=50 1 of 20,626, each an exact tie or a 1-ulp fma/non-fused flip at the
K-th slot; every other row is the reference's set exactly.
"""
import numpy as np
import pytest
import torch

import cuda_knearests_amd as kn
from cuda_knearests_amd.utils import dataset


def _reference_sets(p: np.ndarray, k: int):
    """(n, k) neighbour ids with the reference's arithmetic and K+1 / drop-self protocol, plus
    the (K+1)-th / K-th distance gap per row (relative)."""
    n = p.shape[0]
    ids = np.empty((n, k), dtype=np.int64)
    gap = np.empty(n, dtype=np.float64)
    for c0 in range(0, n, 1024):
        q = p[c0:c0 + 1024]
        dx = p[None, :, 0] - q[:, None, 0]
        dy = p[None, :, 1] - q[:, None, 1]
        dz = p[None, :, 2] - q[:, None, 2]
        d = np.float32(0.0) + dx * dx
        d = d + dy * dy
        d = d + dz * dz  # float32 throughout: ((0 + dx^2) + dy^2) + dz^2, no fma
        part = np.argpartition(d, k + 1, axis=1)[:, :k + 2]
        dp = np.take_along_axis(d, part, 1)
        order = np.lexsort((part, dp), axis=1)
        part, dp = np.take_along_axis(part, order, 1), np.take_along_axis(dp, order, 1)
        # K+1 nearest including self (distance 0), self dropped (test_knearests.cu:205-211)
        rows = np.arange(c0, c0 + q.shape[0])
        keep = part[:, :k + 1]
        out = np.where(keep == rows[:, None], -1, keep)
        for i in range(out.shape[0]):
            r = out[i][out[i] >= 0][:k]
            ids[c0 + i] = r
        kth, nxt = dp[:, k].astype(np.float64), dp[:, k + 1].astype(np.float64)
        gap[c0:c0 + q.shape[0]] = (nxt - kth) / np.maximum(kth, 1e-30)
    return ids, gap


@pytest.mark.parametrize("k", [8, 16, 50])
def test_pts20k_sets_match_reference_semantics(k):
    pts = kn.read_xyz(str(dataset("pts20K.xyz")), normalize=True)
    ref_ids, gap = _reference_sets(pts.numpy().astype(np.float32), k)
    ours, _ = kn.knn_cpu(pts, k, "kdtree")  # bit-identical to the GPU kernels (tests/test_gpu.py)
    ours = np.sort(ours.numpy().astype(np.int64), axis=1)
    ref = np.sort(ref_ids, axis=1)
    diff = np.nonzero((ours != ref).any(1))[0]
    # a near-tie: the reference's K-th and (K+1)-th distances within 1e-6 relative (1-2 ulps at
    # these magnitudes), where fma vs non-fused rounding or the tie rule may pick either point
    near_tie = gap < 1e-6
    bad = [int(i) for i in diff if not near_tie[i]]
    assert not bad, f"{len(bad)} rows differ from the reference's semantics away from ties (first {bad[:5]})"
    # measured on this fixture: K=8 2 rows (one 1-ulp fma flip, one exact tie), K=16 none,
    # K=50 1 row (exact tie) -- out of 20,626; more would mean a semantic drift
    assert diff.size <= 3, f"{diff.size} rows differ (all at near-ties)"
