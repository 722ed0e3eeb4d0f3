"""polarcub_amd -- MI355X-native polar successive-cancellation (SC) decoding.

The hot path (binary SC decode over a memoryless channel, uniform prior) runs in
hand-written HIP kernels for gfx950 behind the C ABI in include/polarcub_sc.h.
Python modules:
  polarcub_amd.sc        batched device API (CodeSpec, BinaryDecoder, encode)
  polarcub_amd._lib      ctypes binding of libpolarcub_hip.so (no CPU fallback)
  polarcub_amd.build     in-tree hipcc build
"""
__version__ = "0.1.0"
