"""Deletion kernel time split: the bench code vs all-frozen (memoryless subtrees skipped,
trellis stages only) vs all-information (nothing skipped).  Diagnostic, not a test."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from polarcub_amd import mc, sc  # noqa: E402


def timed(dec, rx, ln, reps=5):
    dec.decode_native(rx, ln)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dec.decode_native(rx, ln)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n, n0, pd, xi, B = 8, 2, 0.1, 0.1, 1 << 20
    N = 1 << n
    dev = torch.device("cuda", 0)
    g = np.load(os.path.join(ROOT, "tests", "golden", "deletion_n8.npz"), allow_pickle=False)
    score = g["genie_score"]
    order = sorted(range(N), key=lambda i: (score[i], i))
    codes = {"bench K=64": set(order[N // 4:]), "all frozen K=0": set(range(N)), "all info K=256": set()}
    base = sc.CodeSpec.from_frozen_set(N, codes["bench K=64"], 200, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    rx, ln, _ = mc.deletion_batch(base, B, n0, xi, pd, gen)
    for name, fr in codes.items():
        code = sc.CodeSpec.from_frozen_set(N, fr, 200, device=dev)
        ms = timed(sc.DeletionDecoder(code, n0, pd), rx, ln)
        print("%-16s %8.2f ms  %6.1f M cw/s" % (name, ms, B / ms / 1e3), flush=True)


if __name__ == "__main__":
    main()
