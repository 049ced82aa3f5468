"""avz — MI355X-native mask-driven MVDR beamforming engine (host side).

The compute path is libavz.so (hand-written HIP kernels for gfx950, C ABI in
include/avz.h); PyTorch-ROCm supplies device memory, streams and
torch.distributed. Importing this package fails if libavz.so is missing: there is
no CPU fallback.
"""
from ._lib import AvzError, lib  # noqa: F401  (loads libavz.so or raises)
from .engine import MVDRPlan, PlanConfig, n_frames, out_length  # noqa: F401

__all__ = ["MVDRPlan", "PlanConfig", "AvzError", "n_frames", "out_length"]
