"""Diagnostic: the compact Monte-Carlo pipeline one call at a time, synchronising after each."""
import sys
import os
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
from polarcub_amd import _lib, construction, mc, sc

L = _lib.lib()
n, K = 10, 512
s2 = construction.awgn_sigma2(2.0, 0.5)
fr = construction.bhattacharyya_frozen(n, K, s2)
code = sc.CodeSpec.from_frozen_set(1 << n, set(np.nonzero(fr)[0].tolist()), 1, device="cuda")
B = 4096
print("ws compact", L.pcub_sc_decode_bin_compact_workspace(B, n), "ws pairs", L.pcub_sc_decode_bin_workspace(B, n),
      "mc ws", L.pcub_mc_run_bin_workspace(B, n, K), flush=True)
info, xc = mc.philox_norm_batch(code, 7, 0, B, mc.CHANNEL_AWGN, s2, compact=True)
torch.cuda.synchronize()
print("channel_norm compact ok", float(xc.abs().mean()), flush=True)
info, pairs = mc.philox_norm_batch(code, 7, 0, B, mc.CHANNEL_AWGN, s2, compact=False)
torch.cuda.synchronize()
print("channel_norm pairs ok", flush=True)
dec = sc.BinaryDecoder(code)
i2, _, _ = dec.decode_native(pairs)
torch.cuda.synchronize()
print("pair decode ok", flush=True)
i1, _, _ = dec.decode_compact_native(xc)
torch.cuda.synchronize()
print("compact decode ok", torch.equal(i1, i2), flush=True)
print(mc.run_bin(code, 7, 0, B, mc.CHANNEL_AWGN, s2, chunk=4096), flush=True)
