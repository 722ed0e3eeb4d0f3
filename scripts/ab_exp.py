"""A/B of experimental binary decode kernels (pcub_sc_set_experiment, sc_bin_kx*.hip) against the
shipped tiled-root twin on the bench workload (C2 unless --n): decode times interleaved, outputs
(info, x_hat) compared bit for bit with the shipped kernel's.  Diagnostic, not a test.

    python scripts/ab_exp.py 0 1 [2 ...] [--n 10] [--batch 1048576] [--rounds 4]
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
ap.add_argument("exps", type=int, nargs="+")
ap.add_argument("--n", type=int, default=10)
ap.add_argument("--batch", type=int, default=1 << 20)
ap.add_argument("--rounds", type=int, default=4)
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
L.pcub_sc_set_experiment.argtypes = [ctypes.c_int]
L.pcub_sc_set_experiment.restype = ctypes.c_int
res = {e: [] for e in a.exps}
outs = {}
for rnd in range(a.rounds):
    for e in a.exps:
        L.pcub_sc_set_experiment(e)
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
        res[e].append(e0.elapsed_time(e1) / a.reps)
        outs[e] = o
L.pcub_sc_set_experiment(0)
ref = outs[a.exps[0]]
ok = True
for e in a.exps:
    same = torch.equal(outs[e][0], ref[0]) and torch.equal(outs[e][1], ref[1])
    ok = ok and same
    v = res[e][1:] if len(res[e]) > 1 else res[e]
    print("exp %d: %s ms -> %.2f M cw/s (median)  identical=%s" % (
        e, " ".join("%.3f" % x for x in res[e]), B / np.median(v) / 1e3, same), flush=True)
fe = int((outs[a.exps[0]][0][: code.info_words] != 0).sum())
print("ALL IDENTICAL" if ok else "OUTPUTS DIFFER")
sys.exit(0 if ok else 1)
