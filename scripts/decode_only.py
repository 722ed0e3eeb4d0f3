"""Minimal driver for profiling: generate the bench workload, run the decode kernel R times."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polarcub_amd import construction, mc, sc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10)
ap.add_argument("--batch", type=int, default=1 << 20)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--variant", type=int, default=None)
ap.add_argument("--exp", type=int, default=0, help="pcub_sc_set_experiment (A/B kernels, sc_bin_kx*.hip)")
ap.add_argument("--no-tile", action="store_true", help="root rows [N][B][2] instead of the kernel's tiles (bench.py)")
a = ap.parse_args()
N = 1 << a.n
K = N // 2
s2 = construction.awgn_sigma2(2.0, 0.5)
fr = construction.bhattacharyya_frozen(a.n, K, s2)
code = sc.CodeSpec.from_frozen_set(N, set(np.nonzero(fr)[0].tolist()), 1)
sc.set_variant(a.variant)
if a.exp:
    import ctypes
    from polarcub_amd import _lib
    _lib.lib().pcub_sc_set_experiment.argtypes = [ctypes.c_int]
    _lib.lib().pcub_sc_set_experiment(a.exp)
dec = sc.BinaryDecoder(code)
gen = torch.Generator(device="cuda")
gen.manual_seed(1)
xy, info = mc.awgn_batch(code, a.batch, s2, gen)
T = 0 if a.no_tile else sc.bin_tile(a.n)
if T:
    xy = sc.tile_rows(xy, T)
outs = (torch.empty((code.info_words, a.batch), dtype=torch.int32, device="cuda"),
        torch.empty((code.n_words, a.batch), dtype=torch.int32, device="cuda"), None)
for _ in range(a.reps):
    if T:
        dec.decode_tiled_native(xy, a.batch, out=outs)
    else:
        dec.decode_native(xy, out=outs)
torch.cuda.synchronize()
print("done")
