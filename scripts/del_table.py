"""Deletion decode layouts: n0 = 3 without the table (per-lane trellis levels), k_sc_del with the
table, and the table-driven 16-lanes-a-codeword layout (sc_del_dense.h); n0 = 2 lane vs dense.
Throughput at main_deletion.py's n0 = n // 3 shapes.  Diagnostic, not a test."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from polarcub_amd import mc, sc  # noqa: E402
from scripts.del_split import timed  # noqa: E402


def main():
    pd, xi = 0.1, 0.1
    dev = torch.device("cuda", 0)
    for n0, n, B in ((2, 8, 1 << 20), (2, 10, 1 << 18), (3, 9, 1 << 18), (3, 10, 1 << 18), (3, 11, 1 << 16)):
        N = 1 << n
        code = sc.CodeSpec.from_frozen_set(N, set(range(N - N // 4)), 200, device=dev)
        gen = torch.Generator(device=dev)
        gen.manual_seed(n)
        rx, ln, _ = mc.deletion_batch(code, B, n0, xi, pd, gen)
        res, outs = {}, {}
        modes = (("plain", False, False), ("lane+tab", True, False), ("dense", True, True)) if n0 == 3 else \
            (("lane", True, False), ("dense", True, True))
        for name, tab, dense in modes:
            if n0 == 3 and not tab and n >= 11:
                continue
            prev = sc.set_deletion_dense(dense)
            d = sc.DeletionDecoder(code, n0, pd, use_table=tab)
            res[name] = timed(d, rx, ln, reps=3)
            i0, x0 = d.decode_native(rx, ln)
            outs[name] = (i0.clone(), x0.clone())
            sc.set_deletion_dense(prev)
        ref = outs["dense"]
        same = all(torch.equal(a, b) for o in outs.values() for a, b in zip(o, ref))
        print("n=%2d n0=%d B=%7d  " % (n, n0, B) + " | ".join("%s %8.2f ms %8.3f M cw/s" % (k, v, B / v / 1e3)
                                                       for k, v in res.items()) + " | identical %s" % same,
              flush=True)


if __name__ == "__main__":
    main()
