"""admm_hip -- MI355X-native decentralized-ADMM tomography hot path.

Host side (PyTorch-ROCm for device memory / streams / torch.distributed) over
hand-written gfx950 HIP kernels behind the C-ABI of include/admm_tomo.h.
The reference-compatible entry points are the drop-in modules one directory up
(block_5_node_problem, block_6_admm_loop, block_6_admm_loop_ver2, ...).
"""
from .geometry import ParallelBeamGeometry, RayTransform, split_angles  # noqa: F401
from ._lib import AdmmError, AdmmLibraryError  # noqa: F401

__all__ = ["ParallelBeamGeometry", "RayTransform", "split_angles", "AdmmError", "AdmmLibraryError"]
