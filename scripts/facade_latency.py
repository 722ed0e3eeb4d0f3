"""Facade measurements (GPU): per-call latency of the reference-API single-codeword
BinaryPolarEncoderDecoder.decode at N=1024 (one upload, launch, download per call), the same
codewords through decode_batch, and the genie construction run over a BSC at N=1024 (the
user's per-trial Python closures included, as the reference API requires).

    python scripts/facade_latency.py [--calls 200] [--genie-trials 4096]
Prints one JSON line."""
import argparse
import contextlib
import io
import json
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polarcub_amd import coding, construction, scalar, vectors  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--genie-trials", type=int, default=4096)
    a = ap.parse_args()
    n, N = 10, 1024
    s2 = construction.awgn_sigma2(2.0, 0.5)
    frozen = construction.bhattacharyya_frozen(n, N // 2, s2)
    fs = set(int(i) for i in np.nonzero(frozen)[0])
    encdec = coding.BinaryPolarEncoderDecoder(N, fs, 1)
    rng = np.random.default_rng(7)
    xs = [rng.random((N, 2)) for _ in range(a.calls)]
    xvd = vectors.BinaryMemorylessVectorDistribution(N)
    xvd.probs[:] = 0.5

    def xyvd(p):
        v = vectors.BinaryMemorylessVectorDistribution(N)
        v.probs[:] = p
        return v

    vds = [xyvd(p) for p in xs]
    for v in vds[:5]:
        encdec.decode(xvd, v)
    torch.cuda.synchronize()
    t = time.perf_counter()
    outs = [encdec.decode(xvd, v) for v in vds]
    single = (time.perf_counter() - t) / a.calls
    xy = torch.from_numpy(np.stack(xs)).cuda()
    encdec.decode_batch(xy)
    torch.cuda.synchronize()
    t = time.perf_counter()
    bx, binfo = encdec.decode_batch(xy)
    torch.cuda.synchronize()
    batch = (time.perf_counter() - t) / a.calls
    same = all(np.array_equal(np.asarray(outs[i][1]), np.asarray(binfo[i])) for i in range(a.calls))

    bsc = scalar.makeBSC(0.11)
    crng = random.Random(1)

    def make_x():
        xd = scalar.BinaryMemorylessDistribution()
        xd.append([bsc.calcXMarginal(0), bsc.calcXMarginal(1)])
        return xd.makeBinaryMemorylessVectorDistribution(N, None)

    def channel(codeword):
        return [int(x) ^ (1 if crng.random() < 0.11 else 0) for x in codeword]

    t = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        fz = coding.genieEncodeDecodeSimulation(N, make_x, lambda e: e, channel,
                                                lambda r: bsc.makeBinaryMemorylessVectorDistribution(len(r), r),
                                                a.genie_trials, 0.1, 5, trustXYProbs=True)
    genie = time.perf_counter() - t
    print(json.dumps({"N": N, "single_decode_ms": single * 1e3, "single_decode_cw_s": 1.0 / single,
                      "decode_batch_B": a.calls, "decode_batch_us_per_cw": batch * 1e6,
                      "batch_equals_single": same, "genie_trials": a.genie_trials, "genie_s": genie,
                      "genie_trials_s": a.genie_trials / genie, "genie_frozen": len(fz)}))


if __name__ == "__main__":
    main()
