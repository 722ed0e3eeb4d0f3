"""A/B of the q-ary split-level tiled-root kernel specialised on the C4 code length (pcub_sc_set_fixed_n) on C4: decode
times interleaved, outputs compared bit for bit.  Diagnostic, not a test."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polarcub_amd import _lib, mc, sc  # noqa: E402
from tests.conftest import load_golden  # noqa: E402

g = load_golden("construct_qary")
code = sc.QaryCode(4, 256, g["qsc4_n8_L64_frozen"].astype(np.uint8), device="cuda")
dec = sc.QaryDecoder(code)
B = 1 << 20
T = dec.tile()
info, xy = mc.philox_qsc_batch(code, 20250204, 0, B, 0.11, tile=T)
L = _lib.lib()
L.pcub_sc_set_fixed_n.argtypes = [ctypes.c_int]
res = {0: [], 1: []}
outs = {}
for rnd in range(4):
    for tr in (0, 1):
        L.pcub_sc_set_fixed_n(tr)
        o = dec.decode_tiled_native(xy, B)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            o = dec.decode_tiled_native(xy, B)
        e1.record()
        torch.cuda.synchronize()
        res[tr].append(e0.elapsed_time(e1) / 5)
        outs[tr] = o
same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]) if a is not None)
for tr in (0, 1):
    print("qary fixed_n=%d: %s ms -> %.2f M cw/s (median)" % (tr, " ".join("%.3f" % x for x in res[tr]),
                                                                  B / np.median(res[tr][1:]) / 1e3))
print("identical outputs:", same)
L.pcub_sc_set_fixed_n(1)
assert same
