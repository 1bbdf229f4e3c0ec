"""Exactness check of kNN rows against an oracle, shared by the tests, the smoke and the bench.

A row is accepted when
  * its squared distances equal the oracle's bit for bit (same fp32 fma chain, ascending);
  * its empty slots (id < 0) are exactly the oracle's (infinite distance);
  * no id is the query itself and no id repeats inside the row;
  * every id reproduces its reported distance when recomputed from the points (float64 from the
    fp32 coordinate differences; the kernels' fma chain agrees to ~1 fp32 ulp), so an id can
    only differ from the oracle's inside a run of (near-)equal distances.

The third and fourth items are what make a wrong neighbour id fail: comparing ids only where the
oracle's distances differ cannot fail once the distances are known to be equal (the advisor's
round-1 finding on the old ``(idx == oi) | (d2 == od).any(-1)`` expression).
"""
from __future__ import annotations

import torch

# |recomputed - reported| <= REL * reported: the fp32 fma chain (3 roundings) vs an exact-ish f64
REL = 4e-7


def knn_row_errors(cloud: torch.Tensor, qids: torch.Tensor, idx: torch.Tensor, d2: torch.Tensor,
                   od: torch.Tensor | None = None) -> dict:
    """Counts of rows failing each check (all zero = exact). ``cloud`` (N, 3) fp32 points,
    ``qids`` (M,) index of each query in ``cloud``, ``idx`` (M, K) neighbour indices into
    ``cloud`` (-1 = empty), ``d2`` (M, K) reported squared distances, ``od`` (M, K) oracle
    squared distances (optional: without it only the id checks run)."""
    cloud = cloud.detach().float()
    dev = cloud.device
    qids = qids.to(dev).long()
    idx = idx.to(dev).long()
    d2 = d2.to(dev).float()
    out = {"rows": int(idx.size(0))}
    if idx.numel() == 0:
        return {**out, "dist": 0, "empty": 0, "self": 0, "dup": 0, "recompute": 0}
    valid = idx >= 0
    if od is not None:
        od = od.to(dev).float()
        out["dist"] = int((d2 != od).any(1).sum())
        out["empty"] = int((valid != torch.isfinite(od)).any(1).sum())
    else:
        out["dist"] = 0
        out["empty"] = int((valid != torch.isfinite(d2)).any(1).sum())
    out["self"] = int((valid & (idx == qids[:, None])).any(1).sum())
    s = torch.sort(torch.where(valid, idx, torch.full_like(idx, -1)), dim=1).values
    dup = (s[:, 1:] == s[:, :-1]) & (s[:, 1:] >= 0)
    out["dup"] = int(dup.any(1).sum())
    p = cloud[idx.clamp(min=0)]
    q = cloud[qids][:, None, :]
    diff = (p - q).double()  # fp32 differences, as the kernels form them
    rec = (diff * diff).sum(-1)
    ref = d2.double()
    bad = valid & ((rec - ref).abs() > REL * ref)
    out["recompute"] = int(bad.any(1).sum())
    return out


def assert_knn_exact(cloud: torch.Tensor, qids: torch.Tensor, idx: torch.Tensor, d2: torch.Tensor,
                     od: torch.Tensor) -> None:
    e = knn_row_errors(cloud, qids, idx, d2, od)
    bad = {k: v for k, v in e.items() if k != "rows" and v}
    assert not bad, f"kNN rows fail the exactness check ({e['rows']} rows): {bad}"


__all__ = ["knn_row_errors", "assert_knn_exact"]
