"""A/B of an experimental q-ary decode kernel (pcub_sc_set_experiment, pcub_exp_qkernel linked in by
scripts/exp_build.sh) against the shipped C4 kernel on the bench's C4 batch: decode times
interleaved, outputs compared bit for bit.  Diagnostic, not a test.

    python scripts/ab_qexp.py 0 1 [--batch 1048576] [--rounds 4]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polarcub_amd import _lib, mc, sc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("exps", type=int, nargs="+")
ap.add_argument("--batch", type=int, default=1 << 20)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
g = np.load(os.path.join(root, "tests", "golden", "construct_qary.npz"), allow_pickle=False)
code = sc.QaryCode(4, 256, g["qsc4_n8_L64_frozen"].astype(np.uint8), device="cuda")
dec = sc.QaryDecoder(code)
T = dec.tile()
_, xy = mc.philox_qsc_batch(code, 20250204, 0, a.batch, 0.11, tile=T)
dec.workspace(a.batch)
L = _lib.lib()
res = {e: [] for e in a.exps}
outs = {}
for rnd in range(a.rounds):
    for e in a.exps:
        L.pcub_sc_set_experiment(e)
        o = dec.decode_tiled_native(xy, a.batch)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            o = dec.decode_tiled_native(xy, a.batch)
        e1.record()
        torch.cuda.synchronize()
        res[e].append(e0.elapsed_time(e1) / a.reps)
        outs[e] = [t.clone() for t in o]
L.pcub_sc_set_experiment(0)
ok = True
for e in a.exps:
    same = all(torch.equal(x, y) for x, y in zip(outs[e], outs[a.exps[0]]))
    ok = ok and same
    ms = sorted(res[e])[len(res[e]) // 2]
    print("exp %d: %s ms -> %.2f M cw/s (median)  identical=%s" % (e, " ".join("%.3f" % t for t in res[e]), a.batch / ms / 1e3, same))
print("ALL IDENTICAL" if ok else "MISMATCH")
sys.exit(0 if ok else 1)
