"""Where a wave's time goes in the C4 q-ary decode: runs experiment kernel 9 (a stamped twin of the
shipped split-level tiled-root kernel, linked in by scripts/exp_build.sh) on the bench workload and
prints the share of wave time per phase.  Diagnostic, not a test."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polarcub_amd import _lib, mc, sc  # noqa: E402

from tests.conftest import ROOT  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "construct_qary.npz"), allow_pickle=False)
code = sc.QaryCode(4, 256, g["qsc4_n8_L64_frozen"].astype(np.uint8), device="cuda")
dec = sc.QaryDecoder(code)
B = 1 << 20
T = dec.tile()
info, xy = mc.philox_qsc_batch(code, 1, 0, B, 0.11, tile=T)
L = _lib.lib()
L.pcub_sc_set_experiment.argtypes = [ctypes.c_int]
L.pcub_sc_set_experiment(9)
ws = dec.workspace(B)
out_info = torch.empty((code.K, B), dtype=torch.uint8, device="cuda")
st = torch.zeros(64, dtype=torch.int64, device="cuda")
for rep in range(3):
    st.zero_()
    rc = L.pcub_sc_decode_qary_tiled(sc._p(xy), B, code.n, code.q, T, sc._p(code.frozen_dev), code.K,
                                     sc._p(out_info), sc._p(st), sc._p(ws), ws.numel(), sc._stream())
    torch.cuda.synchronize()
    assert rc == 0
    v = st.cpu().numpy()[:6].astype(np.float64)
    names = ["root chains", "other chains", "q_hl_run", "bookkeeping (symbols, combine)"]
    print("rep %d" % rep)
    for i, nm in enumerate(names):
        print("   %-32s %5.1f %%" % (nm, 100 * v[i] / v[5]))
    print("   %-32s %5.1f %%" % ("other", 100 * (v[5] - v[:4].sum()) / v[5]))
L.pcub_sc_set_experiment(0)
