"""CPU-only tests: oracles, CPU grid solver, .xyz I/O, C++ unit binary."""
import math
import os
import subprocess

import numpy as np
import pytest
import torch

import cuda_knearests_amd as kn
from cuda_knearests_amd.utils import REPO, blue_cloud, clustered_cloud, dataset, uniform_cloud
from cuda_knearests_amd.utils.check import assert_knn_exact, knn_row_errors


def _same_up_to_ties(p, i1, d1, i2, d2):
    """(i1, d1) vs the reference (i2, d2): equal distances, valid ids (utils/check.py)."""
    assert torch.equal(d1, d2)
    assert_knn_exact(p, torch.arange(p.size(0)), i1, d1, d2)
    assert_knn_exact(p, torch.arange(p.size(0)), i2, d2, d2)


@pytest.mark.parametrize("k", [1, 8, 16, 50])
@pytest.mark.parametrize("gen", ["uniform", "blue", "clustered", "dupes"])
def test_oracles_agree(k, gen):
    if gen == "uniform":
        p = uniform_cloud(4000, 1)
    elif gen == "blue":
        p = blue_cloud(4000, 2)
    elif gen == "clustered":
        p = clustered_cloud(4000, 3)
    else:
        p = uniform_cloud(2000, 4)
        p = torch.cat([p, p])
    bi, bd = kn.knn_cpu(p, k, "brute")
    ki, kd = kn.knn_cpu(p, k, "kdtree")
    gi, gd, unc = kn.knn_cpu(p, k, "grid")
    assert unc.numel() == 0
    _same_up_to_ties(p, ki, kd, bi, bd)
    _same_up_to_ties(p, gi, gd, bi, bd)
    # ascending, no self
    assert bool((bd[:, 1:] >= bd[:, :-1]).all())
    assert not bool((bi == torch.arange(p.size(0)).unsqueeze(1)).any())


def test_self_excluded_by_index_with_duplicates():
    # the reference oracle drops neighbour 0 assuming it is the query (test_knearests.cu:210);
    # with exact duplicates the twin must stay in the result at distance 0.
    p = torch.tensor([[0, 0, 0], [0, 0, 0], [1, 0, 0], [5, 5, 5]], dtype=torch.float32)
    i, d = kn.knn_cpu(p, 2, "kdtree")
    assert i[0, 0] == 1 and d[0, 0] == 0 and i[1, 0] == 0


def test_small_n_fills_sentinel():
    p = torch.tensor([[0, 0, 0], [1, 0, 0], [0, 3, 0]], dtype=torch.float32)
    for m in ("brute", "kdtree"):
        i, d = kn.knn_cpu(p, 4, m)
        assert i[0].tolist() == [1, 2, -1, -1]
        assert math.isinf(d[0, 2].item())
    i, d, _ = kn.knn_cpu(p, 4, "grid")
    assert i[0].tolist() == [1, 2, -1, -1]


def test_pts20k_reference_dataset_k8():
    # BASELINE config 1: pts20K.xyz, k=8, CPU kd_tree path (plumbing, no GPU)
    p = kn.read_xyz(str(dataset("pts20K.xyz")), normalize=True)
    assert p.shape == (20626, 3)
    assert 0.0 < float(p.min()) and float(p.max()) < 1000.0
    ki, kd = kn.knn_cpu(p, 8, "kdtree")
    gi, gd, unc = kn.knn_cpu(p, 8, "grid")
    _same_up_to_ties(p, gi, gd, ki, kd)
    # blue noise: min NN spacing ~25 after x1000
    nn = kd[:, 0].sqrt()
    assert 20.0 < float(nn.min()) < 30.0


def test_xyz_roundtrip(tmp_path):
    p = uniform_cloud(1000, 5)
    f = tmp_path / "a.xyz"
    kn.write_xyz(str(f), p)
    q = kn.read_xyz(str(f))
    assert torch.equal(p, q)
    lines = f.read_text().splitlines()
    assert lines[0] == "1000"
    with pytest.raises(RuntimeError):
        bad = tmp_path / "b.xyz"
        bad.write_text("5\n1 2 3\n")
        kn.read_xyz(str(bad))


def test_normalize_matches_reference_rule():
    p = torch.tensor([[0, 0, 0], [2, 1, 0.5], [1, 1, 1]], dtype=torch.float32)
    q = kn.normalize_1000(p)
    # bbox inflated by 0.1% of the max side, uniform scale by the inflated max side
    d = 0.002
    side = 2 + 2 * d
    ref = (p - torch.tensor([-d, -d, -d])) * (1000.0 / side)
    assert torch.allclose(q, ref, rtol=1e-5, atol=1e-3)


def test_plan_auto_reference_density():
    p = kn.Plan.auto(900_000, 16)
    # ~3.4 points per cell (reference knearests.cu:249 uses 3.1), rounded to whole 4-cell tiles:
    # (900000/3.4)^(1/3) = 64.2 -> 64; K <= 16 grids split x into 2 sub-cells (AutoParams::xsub)
    assert p.xsub == 2 and p.dims == [128, 64, 64] and p.tile == [8, 4, 4]
    assert kn.Plan.auto(900_000, 16, xsub=1).dims == [64, 64, 64]
    q = kn.Plan.auto(10_000_000, 32)
    assert q.xsub == 1 and q.tile == [4, 4, 4] and all(d % t == 0 for d, t in zip(q.dims, q.tile))
    assert kn.Plan.auto(900_000, 50).halo == 2
    assert kn.Plan.auto(1000, 8).dims == [14, 7, 7]  # small grids are not rounded
    # x sub-cells keep the LDS plan within 4 workgroups per CU
    assert p.lds_bytes <= 40 * 1024
    assert p.halo >= 1 and p.lds_capacity >= 1024 and p.lds_bytes <= 160 * 1024


def test_cpp_unit_cpu():
    exe = REPO / "bin" / "knn_unit"
    if not exe.exists():
        from cuda_knearests_amd import _build

        _build.build(verbose=False)
    r = subprocess.run([str(exe), "cpu"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]


def test_cli_help():
    r = subprocess.run([str(REPO / "bin" / "knn_cli"), "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    assert "usage" in r.stderr


def test_cpp_unit_cpu_under_asan_ubsan():
    """SURVEY §5 race/sanitizer item: the host library (kd-tree, brute force, CPU grid solver,
    .xyz I/O, checker) runs clean under AddressSanitizer + UBSan (host-only build)."""
    from cuda_knearests_amd import _build

    exe = _build.build_asan()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), "cpu"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_kn_log_levels(monkeypatch):
    """KN_LOG drives the package logger (solve lines at INFO) and the native verbosity
    (kn_default_config().verbose: DEBUG -> 2, INFO -> 1, WARNING -> 0)."""
    import logging

    from cuda_knearests_amd import KNearests
    from cuda_knearests_amd.utils import get_logger, uniform_cloud

    records = []

    class H(logging.Handler):
        def emit(self, r):
            records.append(r)

    log = get_logger()
    h = H()
    log.addHandler(h)
    old = log.level
    try:
        log.setLevel(logging.INFO)
        KNearests(k=4, device="cpu").prepare(uniform_cloud(500, seed=1)).solve()
        assert any("kn_solve" in r.getMessage() for r in records)
        records.clear()
        log.setLevel(logging.WARNING)
        KNearests(k=4, device="cpu").prepare(uniform_cloud(500, seed=1)).solve()
        assert not any("kn_solve" in r.getMessage() for r in records)
    finally:
        log.removeHandler(h)
        log.setLevel(old)
    from test_capi import KnConfig  # the ctypes mirror of kn_config (size-checked there)

    from cuda_knearests_amd._ext import load_capi

    lib = load_capi()
    lib.kn_default_config.restype = KnConfig
    for val, want in (("DEBUG", 2), ("info", 1), ("WARNING", 0)):
        monkeypatch.setenv("KN_LOG", val)
        monkeypatch.delenv("KN_VERBOSE", raising=False)
        assert lib.kn_default_config().verbose == want, val


def test_python_cli_cpu(tmp_path):
    """python -m cuda_knearests_amd: the reference driver flow from Python (CPU grid solver),
    checked against the kd-tree oracle, rows written in original order."""
    import json
    import subprocess
    import sys

    from cuda_knearests_amd.utils import REPO, dataset

    out = tmp_path / "nb.txt"
    r = subprocess.run([sys.executable, "-m", "cuda_knearests_amd", str(dataset("pts20K.xyz")), "--k", "8",
                        "--device", "cpu", "--check", "--json", "--out", str(out)],
                       capture_output=True, text=True, timeout=300, cwd=str(REPO))
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["ok"] and line["n"] == 20626
    rows = out.read_text().splitlines()
    assert len(rows) == 20626 and len(rows[0].split()) == 8


def test_bench_prints_one_json_line():
    """bench.py's contract: exactly one JSON line on stdout (native libraries' own stdout prints,
    e.g. RCCL's version banner, are redirected to stderr)."""
    import json
    import subprocess
    import sys

    from cuda_knearests_amd.utils import REPO

    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--cpu-oracle", "--steps", "1", "--k", "8"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["unit"] == "queries/s" and d["value"] > 0


def test_tree_supports_bounds_padded_brick_space():
    """the tree path's brick counts live in a pow2(max bricks per axis)^3 cube, so an
    elongated grid must not be admitted by its per-axis cell count alone (8192 x 8 x 8 would need
    1024^3 slots, 4 GB per grid set). Admitted: up to 2^24 slots (2048 x 8 x 8 -- the GPU long-axis
    test -- and isotropic 2048^3); refused past it (the engine keeps such grids on the grid path)."""
    from cuda_knearests_amd._ext import load

    C = load()
    assert C.tree_supports([2048, 8, 8]) == (True, 256 ** 3)
    assert C.tree_supports([2048, 2048, 2048])[0]
    assert C.tree_supports([2049, 8, 8]) == (False, 512 ** 3)
    assert C.tree_supports([8192, 8, 8]) == (False, 1024 ** 3)
    assert C.tree_supports([64, 64, 64]) == (True, 8 ** 3)
