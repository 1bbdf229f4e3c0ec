"""Functional ops (GPU HIP kernels via the _C extension, CPU native host library)."""
from .knn_ops import Grid, Plan, build_grid, check_knn, expected_kth_radius, knn, knn_cpu, normalize_1000, query, read_xyz, to_stored_space, write_xyz

__all__ = ["Grid", "Plan", "build_grid", "query", "knn", "knn_cpu", "check_knn", "read_xyz", "write_xyz",
           "normalize_1000", "to_stored_space", "expected_kth_radius"]
