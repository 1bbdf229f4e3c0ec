"""The reference-compatible C API (knearests.h) through ctypes (libknearests.so)."""
import ctypes as C

import numpy as np
import pytest

from cuda_knearests_amd._ext import load_capi
from cuda_knearests_amd.utils import dataset


class KnConfig(C.Structure):
    _fields_ = [("k", C.c_int), ("points_per_cell", C.c_float), ("tile", C.c_int * 3), ("halo", C.c_int),
                ("deterministic", C.c_int), ("device", C.c_int), ("verbose", C.c_int), ("exact_only", C.c_int)]


class KnProblem(C.Structure):
    _fields_ = [("allocated_points", C.c_int), ("dimx", C.c_int), ("dimy", C.c_int), ("dimz", C.c_int),
                ("num_cell_offsets", C.c_int), ("k", C.c_int), ("d_permutation", C.c_void_p),
                ("d_cell_start", C.c_void_p), ("d_stored_points", C.c_void_p), ("d_knearests", C.c_void_p),
                ("impl", C.c_void_p)]


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
    lib.kn_free.argtypes = [C.POINTER(C.POINTER(KnProblem))]
    lib.kn_read_xyz.restype = C.POINTER(C.c_float)
    lib.kn_read_xyz.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.c_int]
    lib.kn_last_error.restype = C.c_char_p
    lib.kn_print_stats.argtypes = [C.POINTER(KnProblem)]
    return lib


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
    knn = np.ctypeslib.as_array(lib.kn_get_knearests(prob), shape=(30000 * 16,)).reshape(30000, 16).copy()
    perm = np.ctypeslib.as_array(lib.kn_get_permutation(prob), shape=(30000,)).copy()
    stored = np.ctypeslib.as_array(lib.kn_get_points(prob), shape=(30000 * 3,)).reshape(30000, 3).copy()
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
