"""Multi-GPU: spatial decomposition + one routing all-to-all (RCCL via torch.distributed, or loopback)."""
from .decomposition import SpatialDecomposition, factor3
from .distributed import DistributedKNearests, DistResult, halo_send_width, route_rows_torch
from .transport import CollectiveError, HostStagedTransport, LoopbackHub, LoopbackTransport, TorchDistTransport, run_loopback

__all__ = ["SpatialDecomposition", "factor3", "DistributedKNearests", "DistResult", "halo_send_width",
           "route_rows_torch", "CollectiveError", "HostStagedTransport", "LoopbackHub", "LoopbackTransport", "TorchDistTransport", "run_loopback"]
