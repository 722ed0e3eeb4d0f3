#!/usr/bin/env python3
"""Frame-error rates of the reference itself at the BASELINE configurations C2, C4 and C5, for the
statistical FER parity tests (tests/test_gpu_fer.py).

TEST INFRASTRUCTURE ONLY -- runs in the build container, never on the GPU box (the reference tree
does not exist there).  Each worker process imports /root/reference with make_golden.py's two
runtime shims and runs the reference's own encoder / channel closures / decoder on its shard of
trials (the per-trial loop of encodeDecodeSimulation, BinaryPolarEncoderDecoder.py:328-387 and
QaryPolarEncoderDecoder.py:935-982, with every draw from a generator seeded per worker).  Output:
tests/golden/fer_ref.json = {config: {trials, frame_errors, bit_errors, meta}}.

  C2  N=1024, K=512, BI-AWGN Eb/N0 = 2 dB, frozen set = bench.py's (Bhattacharyya at the design
      sigma^2, common randomness seed 1); the channel rows are the joint P(x, y) of BPSK over AWGN
      (the reference has no AWGN factory); the reference decodes them.
  C3  N=4096, K=2048, BI-AWGN Eb/N0 = 2 dB, bench.py's frozen set for n=12 (Bhattacharyya at the
      design sigma^2, common randomness seed 1): configs[2]'s code, the same trial loop as C2.
  C4  q=4, N=256, QSC(0.11), the reference's own degrading construction (construct_qary.npz,
      K=128), frozen symbols 0; makeQSC's table, the reference's q-ary encoder and decoder.
  C5  deletion, main_deletion.py's configuration (n=8, n0=2, pd=0.1, xi=0.1, no ones), the frozen
      set of bench.py's C5 line (frozen_deletion_n8_g8000.txt, K=3) and the genie ranking at
      K=64; main_deletion's closures (guard bands, deletionChannelSimulation, the trellis
      collection) around the reference's encoder and decoder.

Usage:  python oracle/make_fer.py [--only C2 C3 C4 C5 C5k64] [--workers 7] [--trials-scale 1.0]
"""
import argparse
import json
import math
import os
import random
import sys
import time
from multiprocessing import get_context

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "tests", "golden", "fer_ref.json")

# trials per configuration (the binomial half-width at FER p is 4 sqrt(p (1 - p) / T))
# C2 at 96,000 trials: the 4-sigma band is +-3.8 % relative at FER 0.1 (round 5; 24,000 before)
TRIALS = {"C2": 96000, "C3": 24000, "C4": 24000, "C5": 60000, "C5k64": 24000}


def _ref():
    sys.path.insert(0, HERE)
    import make_golden
    return make_golden.load_reference()


def _genie_file(path):
    scores, frozen = {}, set()
    with open(path) as f:
        for line in f:
            if line.startswith("***"):
                _, i, c = line.split()
                scores[int(i)] = float(c)
            elif not line.startswith("*") and line.strip():
                frozen.add(int(line))
    return scores, frozen


def _c2_setup(n=10):
    sys.path.insert(0, ROOT)
    from polarcub_amd import construction
    N = 1 << n
    K = N // 2
    s2 = construction.awgn_sigma2(2.0, K / N)
    frozen = set(np.nonzero(construction.bhattacharyya_frozen(n, K, s2))[0].tolist())
    return N, K, s2, frozen


def work_c2(args):
    wid, T, seed = args[:3]
    n = args[3] if len(args) > 3 else 10
    R = _ref()
    BPED, BMVD = R["BPED"], R["BMVD"]
    N, K, s2, frozen = _c2_setup(n)
    enc = BPED.BinaryPolarEncoderDecoder(N, frozen, 1)
    xvd = BMVD.BinaryMemorylessVectorDistribution(N)
    xvd.probs[:] = np.array([0.5, 0.5])
    info_pos = [i for i in range(N) if i not in frozen]
    r = np.array(enc.randomlyGeneratedNumbers)
    u = np.where(0.5 >= r, 0, 1).astype(np.int64)  # frozen values under the uniform prior (:258-262)
    rng = np.random.default_rng([seed, wid])
    c = 0.5 / math.sqrt(2.0 * math.pi * s2)
    fe = be = 0
    for t in range(T):
        inf = rng.integers(0, 2, K)
        uu = u.copy()
        uu[info_pos] = inf
        x = np.array(BPED.polarTransformOfBits(list(int(v) for v in uu)), np.int64)
        if t < 2:  # the transform is the reference encoder's output under the uniform prior
            assert np.array_equal(x, np.array(enc.encode(xvd, list(int(v) for v in inf))))
        y = (1.0 - 2.0 * x) + math.sqrt(s2) * rng.standard_normal(N)
        xyvd = BMVD.BinaryMemorylessVectorDistribution(N)
        xyvd.probs[:, 0] = c * np.exp(-((y - 1.0) ** 2) / (2.0 * s2))
        xyvd.probs[:, 1] = c * np.exp(-((y + 1.0) ** 2) / (2.0 * s2))
        _, dec = enc.decode(xvd, xyvd)
        d = int(np.sum(np.array(dec) != inf))
        fe += d > 0
        be += d
    return T, fe, be


def work_c4(args):
    wid, T, seed = args
    R = _ref()
    QPED, QMD = R["QPED"], R["QMD"]
    g = np.load(os.path.join(ROOT, "tests", "golden", "construct_qary.npz"), allow_pickle=False)
    mask = g["qsc4_n8_L64_frozen"].astype(np.uint8)
    q, N, p = 4, 256, 0.11
    frozen = set(int(i) for i in np.nonzero(mask)[0])
    qsc = QMD.makeQSC(q, p)
    dec = QPED.QaryPolarEncoderDecoder(q, N, frozen, 1)
    xq = QMD.QaryMemorylessDistribution(q)
    xq.probs = [qsc.calcXMarginals()]
    xvd = xq.makeQaryMemorylessVectorDistribution(N, None)
    K = dec.k
    info_pos = [i for i in range(N) if i not in frozen]
    rng = np.random.default_rng([seed, wid])
    fe = be = 0
    for t in range(T):
        inf = rng.integers(0, q, K)
        uu = np.zeros(N, np.int64)  # frozen symbols are 0 (QaryPolarEncoderDecoder.py:351)
        uu[info_pos] = inf
        x = np.array(QPED.polarTransformOfQudits(q, list(int(v) for v in uu)), np.int64)
        if t < 2:
            assert np.array_equal(x, np.array(dec.encode(xvd, list(int(v) for v in inf))))
        flip = rng.random(N) < p
        y = np.where(flip, (x + rng.integers(1, q, N)) % q, x)
        xyvd = qsc.makeQaryMemorylessVectorDistribution(N, [int(v) for v in y])
        out = np.array(dec.decode(xvd, xyvd))
        d = int(np.sum(out != inf))
        fe += d > 0
        be += d
    return T, fe, be


def _c5_frozen(k64):
    scores, frozen = _genie_file(os.path.join(ROOT, "tests", "golden", "frozen_deletion_n8_g8000.txt"))
    if k64:
        order = sorted(range(256), key=lambda i: (scores[i], i))
        frozen = set(order[64:])
    return frozen


def work_c5(args):
    wid, T, seed, k64 = args
    R = _ref()
    sys.path.insert(0, HERE)
    import make_golden
    BPED = R["BPED"]
    n, n0, pd, xi, ones = 8, 2, 0.1, 0.1, 0
    N = 1 << n
    frozen = _c5_frozen(k64)
    make_x, make_codeword, channel, make_xy = make_golden.deletion_closures(R, n, n0, pd, xi, ones,
                                                                            seed * 1000 + wid)
    xvd = make_x()
    enc = BPED.BinaryPolarEncoderDecoder(N, frozen, 200)
    irng = random.Random(seed * 7919 + wid)
    fe = be = 0
    for t in range(T):
        inf = [0 if irng.random() < 0.5 else 1 for _ in range(enc.k)]
        rx = channel(make_codeword(enc.encode(xvd, inf)))
        _, di = enc.decode(xvd, make_xy(rx))
        d = int(sum(1 for a, b in zip(di, inf) if int(a) != int(b)))
        fe += d > 0
        be += d
    return T, fe, be


def run(name, workers, scale):
    T = int(TRIALS[name] * scale)
    per = [T // workers + (1 if i < T % workers else 0) for i in range(workers)]
    seed = {"C2": 2002, "C3": 3003, "C4": 4004, "C5": 5005, "C5k64": 5064}[name]
    if name == "C2":
        fn, jobs = work_c2, [(i, per[i], seed) for i in range(workers)]
    elif name == "C3":
        fn, jobs = work_c2, [(i, per[i], seed, 12) for i in range(workers)]
    elif name == "C4":
        fn, jobs = work_c4, [(i, per[i], seed) for i in range(workers)]
    else:
        fn, jobs = work_c5, [(i, per[i], seed, name == "C5k64") for i in range(workers)]
    t0 = time.time()
    with get_context("spawn").Pool(workers) as pool:
        res = pool.map(fn, jobs)
    trials, fe, be = (sum(r[i] for r in res) for i in range(3))
    meta = {"C2": "N=1024 K=512 BI-AWGN Eb/N0=2 dB, Bhattacharyya frozen set (bench.py), crs=1, reference decode",
            "C3": "N=4096 K=2048 BI-AWGN Eb/N0=2 dB, Bhattacharyya frozen set (bench.py), crs=1, reference decode",
            "C4": "q=4 N=256 K=128 QSC(0.11), reference degrading construction (construct_qary.npz), reference decode",
            "C5": "deletion n=8 n0=2 pd=0.1 xi=0.1, frozen_deletion_n8_g8000.txt (K=3), crs=200, main_deletion closures",
            "C5k64": "deletion n=8 n0=2 pd=0.1 xi=0.1, genie ranking K=64, crs=200, main_deletion closures"}[name]
    return {"trials": trials, "frame_errors": fe, "bit_errors": be, "fer": fe / trials, "meta": meta,
            "seed": seed, "workers": workers, "wall_s": round(time.time() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=["C2", "C3", "C4", "C5", "C5k64"])
    ap.add_argument("--workers", type=int, default=7)
    ap.add_argument("--trials-scale", type=float, default=1.0)
    a = ap.parse_args()
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in a.only:
        r = run(name, a.workers, a.trials_scale)
        out[name] = r
        print(name, r, flush=True)
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
