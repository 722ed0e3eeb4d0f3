"""The PyTorch-ROCm operator form of the boundary: torch.ops.polarcub.* (csrc/torch/torch_ops.cpp).

    from polarcub_amd import ops
    info, xhat = ops.sc_decode_bin_f64(xy, frozen_mask, frozen_val)   # xy [B, N, 2] f64 on device
    info, xhat = ops.sc_decode_qary_f64(q, xy, frozen_mask)           # xy [B, N, q] f64 on device
    x = ops.polar_encode_bin(u)                                       # u [B, N] 0/1 on device

These are the extension exports SURVEY.md:443 names, registered with the dispatcher (CUDA key) so
they compose with torch code and CUDA graphs like any other op.  They launch the same kernels as
the ctypes facade (polarcub_amd.sc) on torch's current stream.  Loading fails loudly when the
library is missing; there is no CPU implementation.
"""
import os

import torch

from . import _lib
from . import build as _build

_loaded = False


def load():
    """Register torch.ops.polarcub (building the library in-tree first if it is absent or stale)."""
    global _loaded
    if _loaded:
        return torch.ops.polarcub
    _lib.lib()  # the HIP library it links against, built and ABI-checked
    if not os.path.exists(_build.TORCH_LIB):
        _build.build_torch_ops()
    torch.ops.load_library(_build.TORCH_LIB)
    _loaded = True
    return torch.ops.polarcub


def sc_decode_bin_f64(xy, frozen_mask, frozen_val):
    """BinaryPolarEncoderDecoder.decode (BinaryPolarEncoderDecoder.py:71-99) of a batch, uniform
    prior: xy [B, N, 2] float64 joint probabilities on device, frozen_mask / frozen_val [N] 0/1
    (host or device) -> (info [B, K] uint8, xhat [B, N] uint8)."""
    return load().sc_decode_bin_f64(xy, torch.as_tensor(frozen_mask), torch.as_tensor(frozen_val))


def sc_decode_qary_f64(q, xy, frozen_mask):
    """QaryPolarEncoderDecoder.decode (QaryPolarEncoderDecoder.py:90-116) of a batch, frozen
    symbols 0: xy [B, N, q] float64 on device -> (info [B, K] uint8, xhat [B, N] uint8)."""
    return load().sc_decode_qary_f64(int(q), xy, torch.as_tensor(frozen_mask))


def polar_encode_bin(u):
    """The polar transform of each row of u [B, N] (0/1, device) -> x [B, N] uint8
    (polarTransformOfBits, BinaryPolarEncoderDecoder.py:494-516)."""
    return load().polar_encode_bin(u)
