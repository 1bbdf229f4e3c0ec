"""Multi-GPU: spatial decomposition + RCCL (torch.distributed) halo exchange."""
from .decomposition import SpatialDecomposition, factor3
from .distributed import DistributedKNearests, DistResult

__all__ = ["SpatialDecomposition", "factor3", "DistributedKNearests", "DistResult"]
