"""A/B of the binary decode's wave tiles from a counter (BinArgs::wtiles, pcub_sc_set_dynamic_tiles)
against the static stride, on the bench workload (C2, or --n 12 for C3's shape): decode times
interleaved, outputs (info, x_hat) compared bit for bit.  Diagnostic, not a test.

    python scripts/ab_dyn_tiles.py [--n 10] [--batch 1048576] [--rounds 6]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polarcub_amd import _lib, construction, mc, sc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10)
ap.add_argument("--batch", type=int, default=1 << 20)
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
n, B = a.n, a.batch
N, K = 1 << n, (1 << n) // 2
s2 = construction.awgn_sigma2(2.0, 0.5)
fr = construction.bhattacharyya_frozen(n, K, s2)
code = sc.CodeSpec.from_frozen_set(N, set(np.nonzero(fr)[0].tolist()), 1)
dec = sc.BinaryDecoder(code)
gen = torch.Generator(device="cuda")
gen.manual_seed(1)
xy, info = mc.awgn_batch(code, B, s2, gen)
xy = sc.tile_rows(xy, sc.bin_tile(n))
L = _lib.lib()
L.pcub_sc_set_dynamic_tiles.argtypes = [ctypes.c_int]
L.pcub_sc_set_dynamic_tiles.restype = ctypes.c_int
res = {m: [] for m in (1, 0)}
outs = {}
for rnd in range(a.rounds):
    for m in (1, 0):
        L.pcub_sc_set_dynamic_tiles(m)
        o = (torch.empty((code.info_words, B), dtype=torch.int32, device="cuda"),
             torch.empty((code.n_words, B), dtype=torch.int32, device="cuda"), None)
        dec.decode_tiled_native(xy, B, out=o)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            dec.decode_tiled_native(xy, B, out=o)
        e1.record()
        torch.cuda.synchronize()
        res[m].append(e0.elapsed_time(e1) / a.reps)
        outs[m] = o
L.pcub_sc_set_dynamic_tiles(1)
same = torch.equal(outs[1][0], outs[0][0]) and torch.equal(outs[1][1], outs[0][1])
for m in (1, 0):
    v = res[m][1:]
    print("%s: %s ms -> %.2f M cw/s (median)" % ("counter" if m else "stride ", " ".join("%.3f" % x for x in res[m]),
                                                 B / np.median(v) / 1e3), flush=True)
print("IDENTICAL" if same else "OUTPUTS DIFFER")
sys.exit(0 if same else 1)
