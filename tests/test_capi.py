"""The reference-compatible C API (knearests.h) through ctypes (libknearests.so)."""
import ctypes as C

import numpy as np
import pytest

from cuda_knearests_amd._ext import load_capi
from cuda_knearests_amd.utils import dataset


class KnConfig(C.Structure):
    _fields_ = [("k", C.c_int), ("points_per_cell", C.c_float), ("tile", C.c_int * 3), ("halo", C.c_int),
                ("deterministic", C.c_int), ("device", C.c_int), ("verbose", C.c_int), ("exact_only", C.c_int),
                ("fixed_grid", C.c_int), ("algo", C.c_int)]


class KnProblem(C.Structure):
    # reference field names (reference knearests.h:3-16) + k, d_stored_points4, impl
    _fields_ = [("allocated_points", C.c_int), ("dimx", C.c_int), ("dimy", C.c_int), ("dimz", C.c_int),
                ("num_cell_offsets", C.c_int), ("d_cell_offsets", C.c_void_p), ("d_cell_offset_dists", C.c_void_p),
                ("d_cell_max", C.c_void_p), ("d_permutation", C.c_void_p), ("d_counters", C.c_void_p),
                ("d_ptrs", C.c_void_p), ("d_globcounter", C.c_void_p), ("d_stored_points", C.c_void_p),
                ("d_knearests", C.c_void_p), ("k", C.c_int), ("d_stored_points4", C.c_void_p),
                ("impl", C.c_void_p)]


class KnStats(C.Structure):
    _fields_ = [("num_points", C.c_int), ("k", C.c_int), ("dims", C.c_int * 3), ("num_cells", C.c_int),
                ("min_cell", C.c_int), ("max_cell", C.c_int), ("avg_cell", C.c_float), ("empty_cells", C.c_int),
                ("fallback_queries", C.c_int), ("uncertified_queries", C.c_int), ("ms_build", C.c_float),
                ("ms_solve", C.c_float), ("range_allocations", C.c_int)]


class KnMultiOptions(C.Structure):
    _fields_ = [("halo_factor", C.c_double), ("balance", C.c_int), ("forward", C.c_int), ("max_rounds", C.c_int)]


class KnMultiStats(C.Structure):
    _fields_ = [("ranks", C.c_int), ("rounds", C.c_int), ("halo_points", C.c_int), ("forwarded", C.c_int),
                ("uses_rccl", C.c_int), ("balanced", C.c_int), ("min_owned", C.c_int), ("max_owned", C.c_int),
                ("device_allocations", C.c_int), ("ms_total", C.c_float), ("host_syncs", C.c_int)]


def _lib():
    lib = load_capi()
    lib.kn_default_config.restype = KnConfig
    lib.kn_prepare_ex.restype = C.POINTER(KnProblem)
    lib.kn_prepare_ex.argtypes = [C.c_void_p, C.c_int, C.POINTER(KnConfig)]
    lib.kn_prepare.restype = C.POINTER(KnProblem)
    lib.kn_prepare.argtypes = [C.c_void_p, C.c_int]
    for f in ("kn_get_knearests", "kn_get_permutation", "kn_get_neighbors"):
        getattr(lib, f).restype = C.POINTER(C.c_uint)
        getattr(lib, f).argtypes = [C.POINTER(KnProblem)]
    lib.kn_get_points.restype = C.POINTER(C.c_float)
    lib.kn_get_points.argtypes = [C.POINTER(KnProblem)]
    lib.kn_get_distances.restype = C.POINTER(C.c_float)
    lib.kn_get_distances.argtypes = [C.POINTER(KnProblem)]
    lib.kn_solve.argtypes = [C.POINTER(KnProblem)]
    lib.kn_solve_ex.argtypes = [C.POINTER(KnProblem)]
    lib.kn_get_stats.argtypes = [C.POINTER(KnProblem), C.POINTER(KnStats)]
    lib.kn_free.argtypes = [C.POINTER(C.POINTER(KnProblem))]
    lib.kn_read_xyz.restype = C.POINTER(C.c_float)
    lib.kn_read_xyz.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.c_int]
    lib.kn_last_error.restype = C.c_char_p
    lib.kn_print_stats.argtypes = [C.POINTER(KnProblem)]
    lib.kn_struct_size.restype = C.c_size_t
    lib.kn_struct_size.argtypes = [C.c_int]
    return lib


def test_struct_layout_matches_library():
    """ctypes mirrors == the structs compiled into libknearests.so (drift fails loudly: a short
    KnConfig once let kn_default_config write past the ctypes buffer)."""
    lib = _lib()
    for which, cls in enumerate((KnConfig, KnProblem, KnStats, KnMultiOptions, KnMultiStats)):
        assert lib.kn_struct_size(which) == C.sizeof(cls), cls.__name__


def test_read_xyz_cpu():
    lib = _lib()
    libc = C.CDLL(None)
    n = C.c_int(0)
    p = lib.kn_read_xyz(str(dataset("pts20K.xyz")).encode(), C.byref(n), 1)
    assert n.value == 20626
    arr = np.ctypeslib.as_array(p, shape=(n.value * 3,)).copy()
    libc.free(p)
    assert 0 < arr.min() and arr.max() < 1000
    bad = lib.kn_read_xyz(b"/nonexistent.xyz", C.byref(n), 1)
    assert not bad and b"cannot open" in lib.kn_last_error()


def test_default_config_matches_reference_params():
    c = _lib().kn_default_config()
    assert c.k == 50 and c.deterministic == 1  # reference params.h:4 DEFAULT_NB_PLANES
    assert c.fixed_grid == 0 and c.exact_only == 0


@pytest.mark.gpu
def test_capi_reference_flow():
    import torch

    import cuda_knearests_amd as kn

    lib = _lib()
    libc = C.CDLL(None)
    rng = np.random.default_rng(0)
    pts = (rng.random((30000, 3), dtype=np.float32) * 1000).astype(np.float32)
    cfg = lib.kn_default_config()
    cfg.k = 16
    prob = lib.kn_prepare_ex(pts.ctypes.data, 30000, C.byref(cfg))
    assert prob, lib.kn_last_error()
    assert prob.contents.allocated_points == 30000 and prob.contents.dimx > 0
    lib.kn_solve(prob)
    pr = prob.contents
    # reference field semantics: after kn_solve the device fields hold the stored-space result
    # and the float3 stored points (reference knearests.cu:329-364, knearests.h:14-15)
    assert pr.d_knearests and pr.d_stored_points and pr.d_ptrs and pr.d_permutation
    assert not pr.d_cell_offsets and not pr.d_counters and pr.k == 16
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    dev_knn = np.empty((30000, 16), dtype=np.uint32)
    dev_pts = np.empty((30000, 3), dtype=np.float32)
    assert hip.hipMemcpy(dev_knn.ctypes.data, pr.d_knearests, dev_knn.nbytes, 2) == 0  # D2H
    assert hip.hipMemcpy(dev_pts.ctypes.data, pr.d_stored_points, dev_pts.nbytes, 2) == 0
    gk, gp, gs = lib.kn_get_knearests(prob), lib.kn_get_permutation(prob), lib.kn_get_points(prob)
    knn = np.ctypeslib.as_array(gk, shape=(30000 * 16,)).reshape(30000, 16).copy()
    perm = np.ctypeslib.as_array(gp, shape=(30000,)).copy()
    stored = np.ctypeslib.as_array(gs, shape=(30000 * 3,)).reshape(30000, 3).copy()
    for ptr in (gk, gp, gs):
        libc.free(ptr)  # getters return malloc'd buffers (reference knearests.cu:411,421,431)
    assert np.array_equal(dev_knn, knn)
    assert np.array_equal(dev_pts, stored)
    st = KnStats()
    assert lib.kn_get_stats(prob, C.byref(st)) == 0 and st.num_points == 30000 and st.k == 16
    lib.kn_print_stats(prob)
    pp = C.pointer(prob)
    lib.kn_free(pp)
    assert not pp.contents  # kn_free nulls the caller's pointer (reference knearests.cu:407)
    assert np.array_equal(np.sort(perm), np.arange(30000))
    assert np.array_equal(stored, pts[perm])
    nb = np.empty_like(knn)
    nb[perm] = perm[knn]  # reference remap (test_knearests.cu:158)
    oi, od = kn.knn_cpu(torch.from_numpy(pts), 16, "kdtree")
    q = torch.from_numpy(pts)
    d = ((q[torch.from_numpy(nb.astype(np.int64))] - q[:, None, :]) ** 2).sum(-1)
    assert torch.allclose(d, od, rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
def test_capi_solve_range_batches():
    """kn_solve_range: the cloud solved in query batches (no N x K device result) equals the
    whole solve row for row (original-space ids and distances)."""
    import torch

    import cuda_knearests_amd as kn

    lib = _lib()
    lib.kn_solve_range.argtypes = [C.POINTER(KnProblem), C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    lib.kn_get_neighbors.restype = C.POINTER(C.c_uint)
    lib.kn_get_neighbors.argtypes = [C.POINTER(KnProblem)]
    libc = C.CDLL(None)
    n, k = 25000, 12
    rng = np.random.default_rng(3)
    pts = (rng.random((n, 3), dtype=np.float32) * 1000).astype(np.float32)
    cfg = lib.kn_default_config()
    cfg.k = k
    prob = lib.kn_prepare_ex(pts.ctypes.data, n, C.byref(cfg))
    assert prob, lib.kn_last_error()
    ids = np.empty((n, k), dtype=np.uint32)
    d2 = np.empty((n, k), dtype=np.float32)
    for first in range(0, n, 7000):  # uneven last batch
        cnt = min(7000, n - first)
        assert lib.kn_solve_range(prob, first, cnt, ids[first:].ctypes.data, d2[first:].ctypes.data) == 0, \
            lib.kn_last_error()
    assert lib.kn_solve_range(prob, n - 5, 10, ids.ctypes.data, None) != 0  # out of range
    st = KnStats()
    assert lib.kn_get_stats(prob, C.byref(st)) == 0
    assert st.range_allocations == 1, st.range_allocations  # one grow-only scratch for all batches
    assert lib.kn_solve_ex(prob) == 0
    g = lib.kn_get_neighbors(prob)
    whole = np.ctypeslib.as_array(g, shape=(n * k,)).reshape(n, k).copy()
    libc.free(g)
    lib.kn_free(C.pointer(prob))
    assert np.array_equal(ids, whole)
    _, od = kn.knn_cpu(torch.from_numpy(pts), k, "kdtree")
    assert torch.equal(torch.from_numpy(d2), od)


def _multi_lib():
    lib = _lib()
    lib.kn_prepare_multi.restype = C.c_void_p
    lib.kn_prepare_multi.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_int, C.POINTER(KnConfig)]
    lib.kn_solve_multi.argtypes = [C.c_void_p]
    lib.kn_get_neighbors_multi.restype = C.POINTER(C.c_uint)
    lib.kn_get_neighbors_multi.argtypes = [C.c_void_p]
    lib.kn_get_distances_multi.restype = C.POINTER(C.c_float)
    lib.kn_get_distances_multi.argtypes = [C.c_void_p]
    lib.kn_get_multi_info.argtypes = [C.c_void_p] + [C.POINTER(C.c_int)] * 4
    lib.kn_free_multi.argtypes = [C.POINTER(C.c_void_p)]
    lib.kn_default_multi_options.restype = KnMultiOptions
    lib.kn_set_multi_options.argtypes = [C.c_void_p, C.POINTER(KnMultiOptions)]
    lib.kn_update_multi.argtypes = [C.c_void_p, C.c_void_p]
    lib.kn_get_multi_stats.argtypes = [C.c_void_p, C.POINTER(KnMultiStats)]
    return lib


def _multi_rows(lib, m, n, k):
    libc = C.CDLL(None)
    gi, gd = lib.kn_get_neighbors_multi(m), lib.kn_get_distances_multi(m)
    idx = np.ctypeslib.as_array(gi, shape=(n * k,)).reshape(n, k).astype(np.int64).copy()
    d2 = np.ctypeslib.as_array(gd, shape=(n * k,)).reshape(n, k).copy()
    libc.free(gi)
    libc.free(gd)
    return idx, d2


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0], [0] * 8])
def test_capi_multi_device(devices):
    """kn_prepare_multi / kn_solve_multi: one process, one rank per entry of `devices` (RCCL
    ncclSend/ncclRecv for distinct devices, device copies for virtual ranks on one GPU);
    original-order rows equal the kd-tree oracle."""
    import torch

    import cuda_knearests_amd as kn
    from cuda_knearests_amd.utils.check import assert_knn_exact

    lib = _multi_lib()
    libc = C.CDLL(None)
    n, k = 40000, 12
    rng = np.random.default_rng(len(devices))
    pts = (rng.random((n, 3), dtype=np.float32) * 1000).astype(np.float32)
    cfg = lib.kn_default_config()
    cfg.k = k
    devs = (C.c_int * len(devices))(*devices)
    m = lib.kn_prepare_multi(pts.ctypes.data, n, devs, len(devices), C.byref(cfg))
    assert m, lib.kn_last_error()
    assert lib.kn_solve_multi(m) == 0, lib.kn_last_error()
    info = [C.c_int(0) for _ in range(4)]
    lib.kn_get_multi_info(m, *[C.byref(x) for x in info])
    ranks, rounds, halo, rccl = (x.value for x in info)
    assert ranks == len(devices) and rounds >= 1
    assert rccl == (1 if len(set(devices)) == len(devices) else 0)
    gi, gd = lib.kn_get_neighbors_multi(m), lib.kn_get_distances_multi(m)
    idx = np.ctypeslib.as_array(gi, shape=(n * k,)).reshape(n, k).astype(np.int64).copy()
    d2 = np.ctypeslib.as_array(gd, shape=(n * k,)).reshape(n, k).copy()
    libc.free(gi)
    libc.free(gd)
    h = C.c_void_p(m)
    lib.kn_free_multi(C.byref(h))
    assert not h.value
    cloud = torch.from_numpy(pts)
    _, od = kn.knn_cpu(cloud, k, "kdtree")
    assert torch.equal(torch.from_numpy(d2), od)
    assert_knn_exact(cloud, torch.arange(n), torch.from_numpy(idx), torch.from_numpy(d2), od)


@pytest.mark.gpu
def test_capi_multi_balanced_forwarding_persistent():
    """The C++ multi-GPU runtime (multi.cpp) end to end on 4 virtual ranks: count-balanced boxes
    on a clustered cloud (owned counts within 2x, equal-volume boxes far worse), query forwarding
    of the uncertified queries of a narrow halo (exact rows, one round), halo growth rounds when
    forwarding is off, no device allocation on a repeated solve, kn_update_multi coordinates."""
    import torch

    import cuda_knearests_amd as kn
    from cuda_knearests_amd.utils import clustered_cloud
    from cuda_knearests_amd.utils.check import assert_knn_exact

    lib = _multi_lib()
    n, k, W = 60000, 16, 4
    cloud = clustered_cloud(n, seed=7)
    pts = cloud.numpy().astype(np.float32).copy()
    cfg = lib.kn_default_config()
    cfg.k = k
    devs = (C.c_int * W)(*([0] * W))
    m = lib.kn_prepare_multi(pts.ctypes.data, n, devs, W, C.byref(cfg))
    assert m, lib.kn_last_error()
    _, od = kn.knn_cpu(cloud, k, "kdtree")
    st = KnMultiStats()

    def check(c, o):
        idx, d2 = _multi_rows(lib, m, n, k)
        assert torch.equal(torch.from_numpy(d2), o)
        assert_knn_exact(c, torch.arange(n), torch.from_numpy(idx), torch.from_numpy(d2), o)

    opt = lib.kn_default_multi_options()
    assert opt.balance == 1 and opt.forward == 1
    # equal-volume boxes first: the clustered cloud's counts are far apart
    opt.balance = 0
    assert lib.kn_set_multi_options(m, C.byref(opt)) == 0
    assert lib.kn_solve_multi(m) == 0, lib.kn_last_error()
    lib.kn_get_multi_stats(m, C.byref(st))
    vol_ratio = st.max_owned / max(1, st.min_owned)
    check(cloud, od)
    # count-balanced + a narrow halo: forwarding answers the uncertified queries in one round
    opt.balance, opt.halo_factor = 1, 0.5
    assert lib.kn_set_multi_options(m, C.byref(opt)) == 0
    assert lib.kn_solve_multi(m) == 0, lib.kn_last_error()
    lib.kn_get_multi_stats(m, C.byref(st))
    assert st.balanced == 1 and st.rounds == 1 and st.forwarded > 0
    assert st.max_owned <= 2 * st.min_owned < 2 * vol_ratio * st.min_owned
    check(cloud, od)
    # the same solve again: every buffer fits, the kd splits are reused (no split histograms)
    assert lib.kn_solve_multi(m) == 0, lib.kn_last_error()
    lib.kn_get_multi_stats(m, C.byref(st))
    assert st.device_allocations == 0, st.device_allocations
    syncs_repeat = st.host_syncs
    check(cloud, od)
    # forwarding off: halo growth rounds instead, same rows
    opt.forward = 0
    assert lib.kn_set_multi_options(m, C.byref(opt)) == 0
    assert lib.kn_solve_multi(m) == 0, lib.kn_last_error()
    lib.kn_get_multi_stats(m, C.byref(st))
    assert st.rounds > 1 and st.forwarded == 0
    check(cloud, od)
    # new coordinates of the same points
    moved = cloud + 0.01 * torch.randn(n, 3, generator=torch.Generator().manual_seed(3))
    mp = moved.numpy().astype(np.float32).copy()
    assert lib.kn_update_multi(m, mp.ctypes.data) == 0, lib.kn_last_error()
    opt.forward = 1
    assert lib.kn_set_multi_options(m, C.byref(opt)) == 0
    assert lib.kn_solve_multi(m) == 0, lib.kn_last_error()
    lib.kn_get_multi_stats(m, C.byref(st))
    assert st.host_syncs > syncs_repeat, (st.host_syncs, syncs_repeat)  # moved: the splits are re-planned
    _, od2 = kn.knn_cpu(moved, k, "kdtree")
    check(moved, od2)
    h = C.c_void_p(m)
    lib.kn_free_multi(C.byref(h))


@pytest.mark.gpu
def test_capi_staged_host_copies_and_arena_cache(monkeypatch):
    """kn_prepare from host points and the malloc'd getters go through the pinned staging ring
    (csrc/runtime/hostio.cpp) for copies >= 1 MiB; kn_free parks the device arena for the next
    kn_prepare. Results equal those of the direct (unstaged, uncached) path byte for byte."""
    lib = _lib()
    lib.kn_release_cached_memory.restype = None
    libc = C.CDLL(None)
    libc.free.argtypes = [C.c_void_p]
    n, k = 300_000, 16  # 3.6 MB of points, 19 MB of rows: several 4 MiB chunks each way
    pts = (np.random.default_rng(7).random((n, 3), dtype=np.float32) * 1000.0).astype(np.float32)

    def run():
        cfg = lib.kn_default_config()
        cfg.k = k
        cfg.verbose = 0
        kp = lib.kn_prepare_ex(pts.ctypes.data, n, C.byref(cfg))
        assert kp, lib.kn_last_error()
        assert lib.kn_solve_ex(kp) == 0, lib.kn_last_error()
        out = []
        for getter, cnt, ty in (("kn_get_knearests", n * k, np.uint32), ("kn_get_permutation", n, np.uint32),
                                ("kn_get_points", n * 3, np.float32)):
            ptr = getattr(lib, getter)(kp)
            assert ptr, getter
            out.append(np.ctypeslib.as_array(ptr, shape=(cnt,)).astype(ty).copy())
            libc.free(C.cast(ptr, C.c_void_p))
        pp = C.pointer(kp)
        lib.kn_free(pp)
        return out

    monkeypatch.setenv("KN_HOST_STAGE", "0")
    monkeypatch.setenv("KN_ARENA_CACHE", "0")
    ref = run()
    monkeypatch.setenv("KN_HOST_STAGE", "1")
    monkeypatch.setenv("KN_ARENA_CACHE", "1")
    for _ in range(3):  # the second and third prepares take the cached arena
        got = run()
        for a, b in zip(ref, got):
            assert np.array_equal(a, b)
    # stored points are a permutation of the input
    assert np.array_equal(np.sort(got[2].reshape(-1, 3), axis=0), np.sort(pts, axis=0))
    lib.kn_release_cached_memory()
