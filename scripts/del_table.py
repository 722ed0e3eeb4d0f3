"""n0 = 3 deletion decode with and without the segment-state table (pcub_sc_deletion_build_table):
throughput at n = 9..11 (main_deletion.py's n0 = n // 3).  Diagnostic, not a test."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from polarcub_amd import mc, sc  # noqa: E402
from scripts.del_split import timed  # noqa: E402


def main():
    pd, xi, n0 = 0.1, 0.1, 3
    dev = torch.device("cuda", 0)
    for n in (9, 10, 11):
        N = 1 << n
        B = 1 << (17 if n < 11 else 16)
        code = sc.CodeSpec.from_frozen_set(N, set(range(N - N // 4)), 200, device=dev)
        gen = torch.Generator(device=dev)
        gen.manual_seed(n)
        rx, ln, _ = mc.deletion_batch(code, B, n0, xi, pd, gen)
        res = {}
        for tab in (False, True):
            d = sc.DeletionDecoder(code, n0, pd, use_table=tab)
            res[tab] = timed(d, rx, ln, reps=3)
            i0, x0 = d.decode_native(rx, ln)
            res[(tab, "out")] = (i0.clone(), x0.clone())
        same = all(torch.equal(a, b) for a, b in zip(res[(False, "out")], res[(True, "out")]))
        print("n=%2d n0=3 B=%d  plain %8.2f ms %7.3f M cw/s | table %8.2f ms %7.3f M cw/s | identical %s"
              % (n, B, res[False], B / res[False] / 1e3, res[True], B / res[True] / 1e3, same), flush=True)


if __name__ == "__main__":
    main()
