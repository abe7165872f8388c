"""nerf_amd — MI355X (gfx950) NeRF hot path behind the reference's render_rays / expert API.

Host side in Python/PyTorch-ROCm (device memory, streams, torch.distributed); every compute stage is a
hand-written HIP kernel in libnerf_amd.so reached through the C-ABI of include/nerf_amd.h.
"""
from ._lib import LIB_PATH, lib  # noqa: F401

__all__ = ["LIB_PATH", "lib"]
