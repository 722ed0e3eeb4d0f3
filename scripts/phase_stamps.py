"""Where a wave's time goes in the C2 decode: runs experiment kernel 9 (a stamped twin of the shipped
tiled-root kernel, linked in by scripts/exp_build.sh) on the bench workload and prints the share of
wave time per phase (s_memtime, accumulated per wave: root-pass chains, level-1 chains, the split
level's register subtrees, bookkeeping, tail).  Diagnostic, not a test."""
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
xy, _ = mc.awgn_batch(code, B, s2, gen)
T = sc.bin_tile(n)
xy = sc.tile_rows(xy, T)
L = _lib.lib()
L.pcub_sc_set_experiment.argtypes = [ctypes.c_int]
L.pcub_sc_set_experiment(9)
info = torch.empty((code.info_words, B), dtype=torch.int32, device="cuda")
xh = torch.empty((code.n_words, B), dtype=torch.int32, device="cuda")
st = torch.zeros(64, dtype=torch.int64, device="cuda")
ws = dec.workspace(B)
for rep in range(3):
    st.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    rc = L.pcub_sc_decode_bin_tiled(sc._p(xy), B, n, T, sc._p(code.fmask_dev), sc._p(code.fval_dev), K, sc._p(info),
                                    sc._p(xh), sc._p(st), sc._p(ws), ws.numel(), sc._stream())
    e1.record()
    torch.cuda.synchronize()
    assert rc == 0
    v = st.cpu().numpy()[:6].astype(np.float64)
    names = ["root-pass chains", "level-1 chains", "hl_run", "bookkeeping", "tail (info flush, x_hat)"]
    print("rep %d: %.3f ms; per-wave cycles %.3g" % (rep, e0.elapsed_time(e1), v[5]))
    for i, nm in enumerate(names):
        print("   %-26s %5.1f %%" % (nm, 100 * v[i] / v[5]))
    print("   %-26s %5.1f %%" % ("other", 100 * (v[5] - v[:5].sum()) / v[5]))
L.pcub_sc_set_experiment(0)
