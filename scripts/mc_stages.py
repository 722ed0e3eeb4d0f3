"""pcub_mc_run_bin stage times (run under rocprofv3 --kernel-trace --stats): the whole pipeline at
C2 (N=1024, K=512, BI-AWGN 2 dB) over 2^20 codewords, chunk from argv.  Diagnostic, not a test."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from polarcub_amd import construction, mc, sc  # noqa: E402

chunks = [int(a) for a in sys.argv[1:]] or [1 << 20]
n, K, B = 10, 512, 1 << 20
s2 = construction.awgn_sigma2(2.0, K / (1 << n))
fr = construction.bhattacharyya_frozen(n, K, s2)
code = sc.CodeSpec.from_frozen_set(1 << n, set(np.nonzero(fr)[0].tolist()), 1, device=torch.device("cuda", 0))
reps = int(os.environ.get("REPS", "2"))
res = {c: [] for c in chunks}
for rep, chunk in [(r, c) for r in range(reps) for c in chunks]:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c = mc.run_bin(code, 1, 0, B, mc.CHANNEL_AWGN, s2, chunk=chunk)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print("chunk %d: %.2f ms  %.1f M cw/s  counters %s" % (chunk, dt * 1e3, B / dt / 1e6, c), flush=True)
    if rep > 0:
        res[chunk].append(B / dt / 1e6)
for c, v in res.items():
    if v:
        print("chunk %d: median %.1f M cw/s over %d runs (min %.1f, max %.1f)" % (c, float(np.median(v)), len(v),
                                                                            min(v), max(v)))
