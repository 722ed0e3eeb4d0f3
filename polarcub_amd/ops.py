"""The PyTorch-ROCm operator form of the boundary: torch.ops.polarcub.* (csrc/torch/torch_ops.cpp).

    from polarcub_amd import ops
    info, xhat = ops.sc_decode_bin_f64(xy, frozen_mask, frozen_val)   # xy [B, N, 2] f64 on device
    info, xhat = ops.sc_decode_qary_f64(q, xy, frozen_mask)           # xy [B, N, q] f64 on device
    x = ops.polar_encode_bin(u)                                       # u [B, N] 0/1 on device

    info, xhat, leaf_m = ops.sc_decode_bin_f64(xy, frozen_mask, frozen_val, leaf_m=True)
    counters = ops.mc_run(log2N, channel, param, frozen_mask, frozen_val, seed, cw_offset, count)

These are the extension exports SURVEY.md:443 names, registered with the dispatcher (CUDA key).
They launch the same kernels as the ctypes facade (polarcub_amd.sc) on torch's current stream.
The byte-mask forms count K on the host (the output shape depends on it), so they synchronise;
`sc_decode_bin_words` takes device-packed masks and K and never does, so it can be captured in a
HIP graph, and has a Meta kernel for shape inference.  Loading fails loudly when the library is
missing; there is no CPU implementation.
"""
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
    torch.ops.load_library(_build.torch_ops_current())
    _loaded = True
    return torch.ops.polarcub


def sc_decode_bin_f64(xy, frozen_mask, frozen_val, leaf_m=False):
    """BinaryPolarEncoderDecoder.decode (BinaryPolarEncoderDecoder.py:71-99) of a batch, uniform
    prior: xy [B, N, 2] float64 joint probabilities on device, frozen_mask / frozen_val [N] 0/1
    (host or device) -> (info [B, K] uint8, xhat [B, N] uint8), and with leaf_m=True also every
    leaf's marginal [B, N, 2] float64 (the reference's marginalizedUProbs, :268-273)."""
    ops = load()
    fm, fv = torch.as_tensor(frozen_mask), torch.as_tensor(frozen_val)
    if leaf_m:
        return ops.sc_decode_bin_f64.leaf(xy, fm, fv)
    return ops.sc_decode_bin_f64(xy, fm, fv)


def sc_decode_bin_words(xy, frozen_words, frozen_val_words, K):
    """sc_decode_bin_f64 with the masks packed on the device (int32 [ceil(N/32)], bit i of word
    i // 32) and K given: no host synchronisation (graph-capturable)."""
    return load().sc_decode_bin_words(xy, frozen_words, frozen_val_words, int(K))


def mc_run(log2N, channel, param, frozen_mask, frozen_val, seed, cw_offset, count, chunk=1 << 18):
    """encodeDecodeSimulation (BinaryPolarEncoderDecoder.py:328-387) as the device pipeline over
    global codewords [cw_offset, cw_offset + count): channel 0 = BI-AWGN (param = sigma^2), 1 = BSC
    (param = p); frozen_mask / frozen_val [N] 0/1 on the device that runs it ->
    int64 [4] {codewords, frame errors, bit errors, 0} on that device."""
    return load().mc_run(int(log2N), int(channel), float(param), frozen_mask, frozen_val, int(seed),
                         int(cw_offset), int(count), int(chunk))


def sc_decode_qary_f64(q, xy, frozen_mask):
    """QaryPolarEncoderDecoder.decode (QaryPolarEncoderDecoder.py:90-116) of a batch, frozen
    symbols 0: xy [B, N, q] float64 on device -> (info [B, K] uint8, xhat [B, N] uint8)."""
    return load().sc_decode_qary_f64(int(q), xy, torch.as_tensor(frozen_mask))


def polar_encode_bin(u):
    """The polar transform of each row of u [B, N] (0/1, device) -> x [B, N] uint8
    (polarTransformOfBits, BinaryPolarEncoderDecoder.py:494-516)."""
    return load().polar_encode_bin(u)
