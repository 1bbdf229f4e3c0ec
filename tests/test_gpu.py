"""GPU tests (MI355X): HIP kernels vs the CPU oracles.

Every comparison is distance-aware: squared distances must equal the kd-tree oracle's bit for
bit (same fp32 fma chain); every returned id must be distinct, not the query, and reproduce its
distance from the points (cuda_knearests_amd/utils/check.py), so ids can differ from the
oracle's only inside runs of equal distance.
"""
import os
import subprocess
import sys

import pytest
import torch

import cuda_knearests_amd as kn
from cuda_knearests_amd.utils import REPO, blue_cloud, clustered_cloud, dataset, surface_cloud, uniform_cloud
from cuda_knearests_amd.utils.check import assert_knn_exact

pytestmark = pytest.mark.gpu


def _assert_matches_oracle(p, idx, d2, k):
    oi, od = kn.knn_cpu(p.cpu(), k, "kdtree")
    idx, d2 = idx.cpu(), d2.cpu()
    assert idx.shape == oi.shape
    mism = (d2 != od).any(1)
    assert int(mism.sum()) == 0, f"{int(mism.sum())} rows differ; first {int(mism.nonzero()[0, 0])}"
    # ids: distinct, not self, and each reproduces its distance (utils/check.py)
    assert_knn_exact(p.cpu(), torch.arange(p.size(0)), idx, d2, od)


def test_native_extension_loaded(cuda, ext):
    import cuda_knearests_amd._C as C

    assert C.__file__.startswith(str(REPO))


@pytest.mark.parametrize("k", [1, 4, 8, 16, 32, 50, 64])
def test_uniform_tile_vs_oracle(cuda, k):
    p = uniform_cloud(30000, seed=k, device=cuda)
    idx, d2 = kn.knn(p, k)
    _assert_matches_oracle(p, idx, d2, k)


@pytest.mark.parametrize("k", [6, 10, 12, 14, 30, 42, 45, 46, 48])
@pytest.mark.parametrize("gen", ["uniform", "clustered"])
def test_row_store_widths_vs_oracle(cuda, k, gen):
    # the re-rank and tree kernels write rows 4 positions per store when k % 4 == 0, 4 plus a
    # 2-position tail when k % 4 == 2 (8-byte aligned rows), else one entry per store
    # (kn/knn_device.h KN_VEC_OUT / KN_VEC_TAIL): every width, inside K buckets, on the grid
    # (uniform) and tree (clustered) paths
    mk = uniform_cloud if gen == "uniform" else clustered_cloud
    p = mk(30000, seed=300 + k, device=cuda)
    idx, d2 = kn.knn(p, k)
    _assert_matches_oracle(p, idx, d2, k)


@pytest.mark.parametrize("k", [1, 16, 50])
def test_forced_exact_rescan(cuda, k):
    # the wave-cooperative exact re-rank normally runs only for window overflows (long runs of
    # equal truncated distances) and truncation near-ties; force it for every query so the
    # branch is covered (rare data-dependent branches need their test). counters[3]
    # counts cooperative finishes: >= 1 per query (a near-tie adds its re-scan)
    p = uniform_cloud(20000, seed=200 + k, device=cuda)
    g = kn.build_grid(p, k)
    idx, d2, info = kn.query(g, k, return_info=True, flags=1)
    assert int(info["counters"][3]) >= p.size(0)
    _assert_matches_oracle(p, idx, d2, k)


@pytest.mark.parametrize("k,gen", [(1, "uniform"), (16, "uniform"), (50, "uniform"), (64, "uniform"),
                                   (16, "clustered"), (8, "blue")])
def test_stream_kernel_vs_oracle(cuda, k, gen):
    # staging-free stream kernel (query flags bit 1): same certification, rows read from global
    mk = {"uniform": uniform_cloud, "clustered": clustered_cloud, "blue": blue_cloud}[gen]
    p = mk(25000, seed=300 + k).to(cuda)
    g = kn.build_grid(p, k)
    idx, d2 = kn.query(g, k, flags=2)
    _assert_matches_oracle(p, idx, d2, k)
    # and it agrees with the LDS-staged tile kernel bit for bit
    i2, e2 = kn.query(g, k, flags=4)
    assert torch.equal(idx, i2) and torch.equal(d2, e2)


@pytest.mark.parametrize("k,gen", [(1, "uniform"), (8, "blue"), (16, "uniform"), (32, "uniform"), (50, "uniform"),
                                   (64, "uniform"), (16, "clustered"), (50, "clustered"), (48, "blue"),
                                   (64, "clustered"), (60, "blue")])
def test_lane_walk_vs_union_stream(cuda, k, gen):
    # per-lane walk (flags bit 3, the default) vs the wave-uniform union stream (bit 2) of the
    # same LDS-staged tile kernel: oracle-exact and bit-identical to each other
    mk = {"uniform": uniform_cloud, "clustered": clustered_cloud, "blue": blue_cloud}[gen]
    p = mk(30000, seed=500 + k).to(cuda)
    g = kn.build_grid(p, k)
    idx, d2 = kn.query(g, k, flags=8)
    _assert_matches_oracle(p, idx, d2, k)
    i2, e2 = kn.query(g, k, flags=4)
    assert torch.equal(idx, i2) and torch.equal(d2, e2)
    i3, e3 = kn.query(g, k)  # default algorithm
    assert torch.equal(idx, i3) and torch.equal(d2, e3)


@pytest.mark.parametrize("algo,k", [(4, 16), (8, 16), (8, 50)])
def test_tile_variants_forced_rescan(cuda, algo, k):
    # k=50: the lane walk's second phase (rest of the staged block, K buckets > 40) in the re-scan
    p = uniform_cloud(20000, seed=402, device=cuda)
    g = kn.build_grid(p, k)
    idx, d2, info = kn.query(g, k, return_info=True, flags=1 | algo)
    assert int(info["counters"][3]) >= p.size(0)
    _assert_matches_oracle(p, idx, d2, k)


def test_stream_kernel_forced_rescan(cuda):
    p = uniform_cloud(20000, seed=401, device=cuda)
    g = kn.build_grid(p, 16)
    idx, d2, info = kn.query(g, 16, return_info=True, flags=1 | 2)
    assert int(info["counters"][3]) == p.size(0)
    _assert_matches_oracle(p, idx, d2, 16)


@pytest.mark.parametrize("k", [8, 16, 96, 128])
def test_exact_path_vs_oracle(cuda, k):
    p = uniform_cloud(20000, seed=100 + k, device=cuda)
    idx, d2 = kn.knn(p, k, use_tiles=False)
    _assert_matches_oracle(p, idx, d2, k)


@pytest.mark.parametrize("gen", ["blue", "clustered"])
def test_distributions(cuda, gen):
    p = (blue_cloud if gen == "blue" else clustered_cloud)(40000, seed=7).to(cuda)
    idx, d2 = kn.knn(p, 16)
    _assert_matches_oracle(p, idx, d2, 16)


def test_duplicates_and_tiny(cuda):
    p = uniform_cloud(3000, seed=9)
    p = torch.cat([p, p]).to(cuda)
    idx, d2 = kn.knn(p, 8)
    _assert_matches_oracle(p, idx, d2, 8)
    for n in (1, 2, 3, 9, 17, 65):
        p = uniform_cloud(n, seed=n, device=cuda)
        idx, d2 = kn.knn(p, 8)
        _assert_matches_oracle(p, idx, d2, 8)


def test_pts20k_reference_dataset(cuda):
    p = kn.read_xyz(str(dataset("pts20K.xyz")), normalize=True).to(cuda)
    for k in (8, 50):
        idx, d2 = kn.knn(p, k)
        _assert_matches_oracle(p, idx, d2, k)


def test_engine_reference_semantics(cuda):
    p = uniform_cloud(25000, seed=11, device=cuda)
    e = kn.KNearests(k=16, device=cuda).prepare(p).solve()
    knn_s = e.get_knearests().cpu().long()
    perm = e.get_permutation().cpu().long()
    assert torch.equal(torch.sort(perm).values, torch.arange(p.size(0)))
    # stored-space rows remapped through the permutation == original-space result
    remap = torch.full_like(knn_s, -1)
    valid = knn_s >= 0
    remap[valid] = perm[knn_s[valid]]
    orig = torch.empty_like(remap)
    orig[perm] = remap
    assert torch.equal(orig, e.neighbors.cpu().long())
    sp = e.get_points().cpu()
    assert torch.equal(sp, p.cpu()[perm])
    s = e.stats()
    assert s["num_cells"] == 29 ** 3 or s["num_cells"] > 0
    assert s["min_cell"] >= 0 and s["max_cell"] >= s["avg_cell"]


def test_graph_replay_matches_eager(cuda):
    p = uniform_cloud(50000, seed=12, device=cuda)
    e = kn.KNearests(k=16, device=cuda).prepare(p).solve()
    ref_i, ref_d = e.neighbors.clone(), e.distances.clone()
    g = kn.KNearests(k=16, device=cuda)
    g.points = p
    for _ in range(3):
        g.step(p, capture=True)
    torch.cuda.synchronize()
    assert torch.equal(g.neighbors, ref_i) and torch.equal(g.distances, ref_d)
    # new data through the same graph
    q = uniform_cloud(50000, seed=13, device=cuda)
    g.step(q, capture=True)
    torch.cuda.synchronize()
    i2, d2 = kn.knn(q, 16)
    assert torch.equal(g.neighbors, i2) and torch.equal(g.distances, d2)


def test_deterministic_reruns(cuda):
    p = uniform_cloud(100000, seed=14, device=cuda)
    a = kn.knn(p, 16)
    b = kn.knn(p, 16)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("n,gen", [(1, "uniform"), (777, "uniform"), (20000, "uniform"),
                                   (60000, "clustered"), (65536, "surface")])
def test_small_build_matches_multikernel(cuda, n, gen, monkeypatch):
    # the one-workgroup build of small clouds (build.hip small_build_kernel) lays out exactly
    # what the deterministic multi-kernel build does
    p = {"uniform": uniform_cloud, "clustered": clustered_cloud, "surface": surface_cloud}[gen](n, seed=21, device=cuda)
    monkeypatch.setenv("KN_SMALL_BUILD", "1")  # opt-in (slower than the multi-kernel build)
    a = kn.build_grid(p, 8)
    monkeypatch.setenv("KN_SMALL_BUILD", "0")
    b = kn.build_grid(p, 8)
    monkeypatch.delenv("KN_SMALL_BUILD")
    assert torch.equal(a.geom[:14], b.geom[:14])  # kn::GridGeom is 14 words of the 16
    for f in ("cell_start", "perm", "sorted"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    i, d = kn.query(a, 8)
    _assert_matches_oracle(p, i, d, 8)


def test_set_k_and_save_load(cuda, tmp_path):
    p = uniform_cloud(20000, seed=15, device=cuda)
    e = kn.KNearests(k=8, device=cuda).prepare(p).solve()
    e.set_k(24).solve()
    _assert_matches_oracle(p, e.neighbors, e.distances, 24)
    f = tmp_path / "g.pt"
    e.save(str(f))
    e2 = kn.KNearests.load(str(f), device=cuda).solve()
    assert torch.equal(e2.neighbors, e.neighbors)


def test_large_uniform_subset(cuda):
    # 900K: the headline config (subset vs brute force on the GPU)
    p = uniform_cloud(900_000, seed=16, device=cuda)
    idx, d2, info = kn.query(kn.build_grid(p, 16), 16, return_info=True)
    sel = torch.randperm(p.size(0), device=cuda)[:1024]
    q = p[sel]
    diff = p.unsqueeze(0) - q.unsqueeze(1)  # exact differences (cdist's GEMM form is not exact)
    dd = (diff * diff).sum(-1)
    dd[torch.arange(1024, device=cuda), sel] = float("inf")
    ref = torch.topk(dd, 16, largest=False).values
    assert torch.allclose(d2[sel], ref, rtol=1e-5, atol=1e-4)
    c = info["counters"].cpu()
    assert int(c[1]) == 0  # nothing uncertified on a single GPU
    assert int(c[0]) < 0.01 * p.size(0), f"exact-path fraction too high: {int(c[0])}"


def test_cpp_unit_gpu(cuda):
    r = subprocess.run([str(REPO / "bin" / "knn_unit"), "gpu"], capture_output=True, text=True, timeout=900)
    print(r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]


def test_cli_reference_flow(cuda):
    r = subprocess.run([str(REPO / "bin" / "knn_cli"), str(dataset("pts20K.xyz")), "--k", "50", "--json"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert '"ok": true' in r.stdout


@pytest.mark.parametrize("mode", [["--batch", "7000"], ["--multi", "4"]])
def test_cli_batches_and_multi_rank(cuda, mode):
    """knn_cli --batch (kn_solve_range) and --multi (kn_prepare_multi: 4 ranks, virtual on one
    GPU) on the reference fixture, checked against the kd-tree oracle by the CLI itself."""
    r = subprocess.run([str(REPO / "bin" / "knn_cli"), str(dataset("pts20K.xyz")), "--k", "16", "--json"] + mode,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert '"ok": true' in r.stdout


@pytest.mark.parametrize("k", [16, 50])
def test_halo1_certification_and_fallback(cuda, k):
    """force a 1-ring halo -> many tile queries cannot be certified and must be
    finished by the exact kernel; results stay exact."""
    p = uniform_cloud(30000, seed=500 + k, device=cuda)
    plan = kn.Plan.auto(p.size(0), k, halo=1)
    assert plan.halo == 1
    g = kn.build_grid(p, k, plan=plan)
    idx, d2, info = kn.query(g, k, return_info=True)
    assert int(info["counters"][0]) > 0, "expected exact-path queries with a 1-ring halo"
    _assert_matches_oracle(p, idx, d2, k)


def test_grid_layout_and_cell_mapping(cuda):
    """Binning invariants: cell_start is an exclusive scan of per-cell counts (monotone, ends at
    N), perm is a bijection, every stored point lies in the cell range its coordinates map to
    (same fp32 arithmetic as the kernels), cells are ordered by original index (deterministic),
    and points exactly on the bounding box land in valid edge cells."""
    n = 50000
    p = uniform_cloud(n, seed=5, device=cuda)
    p[0] = torch.tensor([0.0, 0.0, 0.0], device=cuda)
    p[1] = torch.tensor([1000.0, 1000.0, 1000.0], device=cuda)
    p[2] = torch.tensor([0.0, 1000.0, 500.0], device=cuda)
    g = kn.build_grid(p, 16)
    cs = g.cell_start.cpu().long()
    assert cs[0] == 0 and cs[-1] == n and bool((cs[1:] >= cs[:-1]).all())
    perm = g.perm.cpu().long()
    assert torch.equal(torch.sort(perm).values, torch.arange(n))
    srt = g.sorted.cpu()
    assert torch.equal(srt[:, :3], p.cpu()[perm])
    assert torch.equal(srt[:, 3].contiguous().view(torch.int32).long(), perm)
    geom = g.geom.cpu()
    f = geom.view(torch.float32)
    origin, inv = f[0:3], f[6:9]
    dims = geom[10:13].long()
    c = torch.floor(torch.minimum(torch.maximum((srt[:, :3] - origin) * inv, torch.tensor(-1.0)), dims.float()))
    c = torch.minimum(torch.maximum(c.long(), torch.zeros(3, dtype=torch.long)), dims - 1)
    cell = c[:, 0] + dims[0] * (c[:, 1] + dims[1] * c[:, 2])
    pos = torch.arange(n)
    assert bool(((cs[cell] <= pos) & (pos < cs[cell + 1])).all()), "stored point outside its cell range"
    same = cell[1:] == cell[:-1]
    assert bool((perm[1:][same] > perm[:-1][same]).all()), "cells not ordered by original index"


@pytest.mark.parametrize("gen", ["surface", "clustered"])
def test_occupancy_adaptive_grid(cuda, ext, gen):
    """Over-occupied grids (points on surfaces, dense clusters) are re-binned with finer cells;
    results stay exact and far fewer queries spill to the exact kernel."""
    from cuda_knearests_amd.utils import surface_cloud

    mk = surface_cloud if gen == "surface" else clustered_cloud
    p = mk(60000, seed=11).to(cuda)
    g0 = kn.build_grid(p, 16)
    g1 = kn.build_grid(p, 16, adaptive=True)
    w0 = int(ext.occupancy(g0.cell_start).item()) / p.size(0)
    w1 = int(ext.occupancy(g1.cell_start).item()) / p.size(0)
    c0 = g0.plan.dims[0] * g0.plan.dims[1] * g0.plan.dims[2]
    c1 = g1.plan.dims[0] * g1.plan.dims[1] * g1.plan.dims[2]
    assert c1 > c0 and w1 < w0, (g0.plan.dims, g1.plan.dims, w0, w1)
    i0, d0, info0 = kn.query(g0, 16, return_info=True)
    i1, d1, info1 = kn.query(g1, 16, return_info=True)
    assert int(info1["counters"][0]) < int(info0["counters"][0])
    _assert_matches_oracle(p, i1, d1, 16)
    assert torch.equal(d0, d1)


def test_uniform_grid_not_refined(cuda):
    p = uniform_cloud(100000, seed=3, device=cuda)
    g0 = kn.build_grid(p, 16)
    g1 = kn.build_grid(p, 16, adaptive=True)
    assert g0.plan.dims == g1.plan.dims


def test_in_cell_order_does_not_change_results(cuda):
    """deterministic=False keeps the atomic (run-dependent) order inside cells: only the
    stored-space view changes; original-space neighbours and distances are identical (keys are
    re-ranked by (distance, original id) and certified), so the benchmarks may skip the sort."""
    p = uniform_cloud(20000, seed=8)
    p = torch.cat([p, p[:5000]]).to(cuda)  # exact duplicates -> distance ties
    for k in (8, 16, 50):
        i0, d0 = kn.knn(p, k, deterministic=True)
        i1, d1 = kn.knn(p, k, deterministic=False)
        assert torch.equal(i0, i1) and torch.equal(d0, d1)


def test_unaligned_points_slice(cuda):
    """A row slice whose base is not 16-B aligned (bbox scalar-load path) == an aligned copy."""
    import cuda_knearests_amd as kn
    from cuda_knearests_amd.utils import uniform_cloud

    p = uniform_cloud(20_003, seed=41, device=cuda)[3:]
    assert p.data_ptr() % 16 != 0
    i0, d0 = kn.knn(p, 8)
    i1, d1 = kn.knn(p.clone(), 8)
    assert torch.equal(i0, i1) and torch.equal(d0, d1)


def test_atomic_binning_fallback_matches(cuda):
    """KN_BUILD_ALGO=1 forces the global-atomic binning path (used when the bucketed plan does not
    fit); it must give the same results as the default bucketed binning."""
    code = (
        "import torch, cuda_knearests_amd as kn\n"
        "from cuda_knearests_amd.utils import uniform_cloud\n"
        "p = uniform_cloud(60_000, seed=8, device='cuda')\n"
        "i, d = kn.knn(p, 12)\n"
        "torch.save({'i': i.cpu(), 'd': d.cpu()}, '/tmp/kn_atomic_bin.pt')\n"
    )
    env = dict(os.environ, KN_BUILD_ALGO="1", PYTHONPATH=str(REPO))
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=240)
    ref = torch.load("/tmp/kn_atomic_bin.pt", weights_only=True)
    p = uniform_cloud(60_000, seed=8, device=cuda)
    i, d = kn.knn(p, 12)
    assert torch.equal(i.cpu(), ref["i"]) and torch.equal(d.cpu(), ref["d"])


def test_beyond_int32_point_offsets(cuda):
    """N > 715,827,882: 3*i and 16*i point offsets exceed 2^31 (round-1 finding: int32 `3*i`
    in the routing / fallback binning kernels). 725M uniform points, K=1 through the default
    build (bucketed binning or its global-atomic fallback) and query; the rows of queries whose
    stored AND original offsets lie beyond 2^31/3 are brute-forced on the GPU."""
    n = 725_000_000
    p = uniform_cloud(n, seed=21, device=cuda)
    g = kn.build_grid(p, 1)
    idx, d2, info = kn.query(g, 1, return_info=True)
    assert int(info["counters"][1]) == 0
    assert bool((idx >= 0).all())
    gen = torch.Generator(device="cpu").manual_seed(3)
    hi = torch.randint(716_000_000, n, (24,), generator=gen)
    lo = torch.randint(0, n, (8,), generator=gen)
    sel = torch.cat([hi, lo, torch.tensor([n - 1])]).to(cuda)
    # stored slots past 2^31/3 too: the last stored points of the cell order
    sel = torch.cat([sel, g.perm[-8:].long()])
    for q in sel.tolist():
        dd = p - p[q]
        dd = (dd * dd).sum(1)
        dd[q] = float("inf")
        j = int(torch.argmin(dd))
        assert float(dd[j]) == pytest.approx(float(d2[q, 0]), rel=1e-6), q
        # the returned id reproduces the reported distance (ties may pick another point)
        e = p[int(idx[q, 0])] - p[q]
        assert float((e * e).sum()) == pytest.approx(float(d2[q, 0]), rel=1e-6), q
    del p, g, idx, d2
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k", [8, 50])
def test_solve_range_matches_whole_solve(cuda, k):
    """Query ranges (kn_solve_range / KNearests.solve_range / Engine.solve_range): batches of
    original indices give the whole solve's rows bit for bit, also for a tree-path cloud (ranges
    run on the grid kernels)."""
    from cuda_knearests_amd._ext import load

    for gen in (uniform_cloud, clustered_cloud):
        p = gen(40000, seed=k, device=cuda)
        m = kn.KNearests(k=k, device=cuda).prepare(p).solve()
        whole_i, whole_d = m.neighbors.cpu(), m.distances.cpu()
        parts = [m.solve_range(f, min(9000, p.size(0) - f)) for f in range(0, p.size(0), 9000)]
        assert torch.equal(torch.cat([a for a, _ in parts]).cpu(), whole_i)
        assert torch.equal(torch.cat([b for _, b in parts]).cpu(), whole_d)
        e = load().Engine(k)
        e.prepare(p)
        ri, rd = e.solve_range(12345, 6000, cuda)  # before any whole solve: no N x K buffers
        assert torch.equal(ri.cpu(), whole_i[12345:18345]) and torch.equal(rd.cpu(), whole_d[12345:18345])


def test_python_cli_gpu_batches(cuda, tmp_path):
    r = subprocess.run([sys.executable, "-m", "cuda_knearests_amd", str(dataset("pts20K.xyz")), "--k", "16",
                        "--check", "--json", "--batch", "6000"],
                       capture_output=True, text=True, timeout=300, cwd=str(REPO))
    assert r.returncode == 0, r.stderr[-2000:]
    assert '"ok": true' in r.stdout


@pytest.mark.parametrize("k", [16, 24])
def test_grid_path_clustered_vs_oracle(cuda, k):
    """The grid kernels on a clustered cloud (no refinement: dense tiles go exact, sparse lanes
    keep an infinite bound after their 3x3 rows): exact against the kd-tree oracle. Caught the
    first packed-outer-row version, which took out-of-box rows for such lanes."""
    p = clustered_cloud(100000, seed=0).to(cuda)
    g = kn.build_grid(p, k)
    idx, d2 = kn.query(g, k, algo="grid")
    _assert_matches_oracle(p, idx, d2, k)
