"""A/B of the uniform-base root twin (pcub_sc_set_tiled_root) on the bench workload (C2, tiled rows):
decode times interleaved, outputs compared bit for bit.  Diagnostic, not a test."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polarcub_amd import _lib, construction, mc, sc  # noqa: E402

n, B = 10, 1 << 20
N, K = 1 << n, 512
s2 = construction.awgn_sigma2(2.0, 0.5)
fr = construction.bhattacharyya_frozen(n, K, s2)
code = sc.CodeSpec.from_frozen_set(N, set(np.nonzero(fr)[0].tolist()), 1)
dec = sc.BinaryDecoder(code)
gen = torch.Generator(device="cuda")
gen.manual_seed(1)
xy, info = mc.awgn_batch(code, B, s2, gen)
T = sc.bin_tile(n)
xy = sc.tile_rows(xy, T)
L = _lib.lib()
L.pcub_sc_set_tiled_root.argtypes = [ctypes.c_int]
res = {0: [], 1: []}
outs = {}
for rnd in range(4):
    for tr in (0, 1):
        L.pcub_sc_set_tiled_root(tr)
        o = (torch.empty((code.info_words, B), dtype=torch.int32, device="cuda"),
             torch.empty((code.n_words, B), dtype=torch.int32, device="cuda"), None)
        dec.decode_tiled_native(xy, B, out=o)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            dec.decode_tiled_native(xy, B, out=o)
        e1.record()
        torch.cuda.synchronize()
        res[tr].append(e0.elapsed_time(e1) / 5)
        outs[tr] = o
same = torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
for tr in (0, 1):
    v = res[tr][1:]
    print("tiled_root=%d: %s ms -> %.2f M cw/s (median)" % (tr, " ".join("%.3f" % x for x in res[tr]),
                                                             B / np.median(v) / 1e3))
print("identical outputs:", same)
assert same
