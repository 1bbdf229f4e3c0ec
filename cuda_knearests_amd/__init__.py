"""cuda_knearests_amd -- MI355X-native (gfx950) k-nearest-neighbour engine.

Same capabilities as ssloy/cuda_knearests (grid-binned exact kNN of 3-D point clouds, the
knearests.h C API, .xyz I/O, a CPU kd-tree oracle), re-designed for CDNA4: LDS-staged,
wave64-uniform query kernel with register-resident med3 top-K, deterministic scan-based
binning, hipGraph replay, and multi-GPU spatial decomposition with RCCL halo exchange.

Layout:
  models/    KNearests engine object (C-API mirror)
  ops/       functional GPU/CPU ops (build_grid, query, knn, knn_cpu, xyz I/O)
  parallel/  spatial decomposition + DistributedKNearests (torch.distributed / RCCL)
  utils/     synthetic clouds, timers, logging, result checking
"""
from ._ext import load as _load_ext
from .models.knearests import KNearests
from .ops.knn_ops import Grid, Plan, build_grid, build_tree, check_knn, knn, knn_cpu, normalize_1000, query, read_xyz, to_stored_space, write_xyz

__version__ = "0.1.0"

__all__ = [
    "KNearests", "Grid", "Plan", "build_grid", "build_tree", "query", "knn", "knn_cpu", "check_knn",
    "read_xyz", "write_xyz", "normalize_1000", "to_stored_space", "__version__",
]
