"""Statistical FER parity at the BASELINE configurations (BASELINE.json metric: "FER match vs
reference"): the device Monte-Carlo's frame-error rate over 2^20 codewords (Philox keyed by the
global codeword index) against the reference's own frame-error rate at the same code, channel and
decoder, run in the build container by oracle/make_fer.py (tests/golden/fer_ref.json: 24,000 to
60,000 reference trials per configuration).  The two runs draw independent channel noise, so the
test is a two-sample binomial test: |p_dev - p_ref| <= 4 sqrt(s_dev^2 + s_ref^2).

  C2  N=1024 K=512 BI-AWGN 2 dB (BinaryPolarEncoderDecoder.py:328-387's trial loop)
  C3  N=4096 K=2048 BI-AWGN 2 dB (configs[2]'s code: the same trial loop at n=12), through the
      chunked device pipeline mc.run_bin that bench.py's C3 line shards over ranks
  C4  q=4 N=256 K=128 QSC(0.11), the reference's degrading construction (QaryPolarEncoderDecoder.py:935-982)
  C5  deletion n=8 n0=2 pd=0.1 xi=0.1, main_deletion's construction (K=3) and the genie ranking at K=64
      (main_deletion.py:142-146)
"""
import json
import math
import os

import numpy as np
import pytest

from tests.conftest import ROOT

FIX = os.path.join(ROOT, "tests", "golden", "fer_ref.json")


def _ref(name):
    with open(FIX) as f:
        return json.load(f)[name]


def _close(fe_dev, n_dev, r):
    p_dev = fe_dev / n_dev
    p_ref = r["frame_errors"] / r["trials"]
    s = math.sqrt(p_dev * (1 - p_dev) / n_dev + p_ref * (1 - p_ref) / r["trials"])
    return abs(p_dev - p_ref) <= 4 * s, (p_dev, p_ref, s)


def test_fixture_is_complete():
    """CPU: the fixture holds every configuration with enough trials for a useful interval."""
    with open(FIX) as f:
        d = json.load(f)
    for name, need in (("C2", 20000), ("C3", 20000), ("C4", 20000), ("C5", 50000), ("C5k64", 20000)):
        r = d[name]
        assert r["trials"] >= need and 0 <= r["frame_errors"] <= r["trials"]
        assert r["bit_errors"] >= r["frame_errors"]
    # the C2 interval is tight enough to see a 12 % relative FER shift
    r = d["C2"]
    p = r["frame_errors"] / r["trials"]
    assert 4 * math.sqrt(p * (1 - p) / r["trials"] + p * (1 - p) / (1 << 20)) < 0.12 * p


@pytest.mark.gpu
def test_c2_awgn_fer_matches_reference():
    from polarcub_amd import construction, mc, sc
    n, K = 10, 512
    s2 = construction.awgn_sigma2(2.0, K / (1 << n))
    fr = construction.bhattacharyya_frozen(n, K, s2)
    code = sc.CodeSpec.from_frozen_set(1 << n, set(np.nonzero(fr)[0].tolist()), 1, device="cuda")
    n_cw, fe, be, _ = mc.run_bin(code, 20250204, 0, 1 << 20, mc.CHANNEL_AWGN, s2)
    ok, info = _close(fe, n_cw, _ref("C2"))
    assert ok, info


@pytest.mark.gpu
def test_c3_awgn_fer_matches_reference():
    """configs[2]'s code at N=4096: 2^20 codewords through mc.run_bin in 2^18-codeword chunks (the
    f32-channel pipeline, compact tiled rows into the N=4096 decode) against 24,000 reference trials."""
    from polarcub_amd import construction, mc, sc
    n, K = 12, 2048
    s2 = construction.awgn_sigma2(2.0, K / (1 << n))
    fr = construction.bhattacharyya_frozen(n, K, s2)
    code = sc.CodeSpec.from_frozen_set(1 << n, set(np.nonzero(fr)[0].tolist()), 1, device="cuda")
    n_cw, fe, be, _ = mc.run_bin(code, 20250205, 0, 1 << 20, mc.CHANNEL_AWGN, s2, chunk=1 << 18)
    ok, info = _close(fe, n_cw, _ref("C3"))
    assert ok, info


@pytest.mark.gpu
def test_c4_qsc_fer_matches_reference():
    import torch
    from polarcub_amd import mc, sc
    g = np.load(os.path.join(ROOT, "tests", "golden", "construct_qary.npz"), allow_pickle=False)
    mask = g["qsc4_n8_L64_frozen"].astype(np.uint8)
    code = sc.QaryCode(4, 256, mask, device="cuda")
    dec = sc.QaryDecoder(code)
    fe = n_cw = 0
    for off in range(0, 1 << 20, 1 << 18):
        info, xy = mc.philox_qsc_batch(code, 20250204, off, 1 << 18, 0.11)
        out = dec.decode_native(xy)[0]
        f, _ = mc.error_counts(out.t(), info.t())
        fe += f
        n_cw += 1 << 18
        del xy
        torch.cuda.empty_cache()
    ok, info = _close(fe, n_cw, _ref("C4"))
    assert ok, info


@pytest.mark.gpu
@pytest.mark.parametrize("k64", [False, True])
def test_c5_deletion_fer_matches_reference(k64):
    from polarcub_amd import mc, sc
    path = os.path.join(ROOT, "tests", "golden", "frozen_deletion_n8_g8000.txt")
    scores, frozen = {}, set()
    with open(path) as f:
        for line in f:
            if line.startswith("***"):
                _, i, c = line.split()
                scores[int(i)] = float(c)
            elif not line.startswith("*") and line.strip():
                frozen.add(int(line))
    if k64:
        frozen = set(sorted(range(256), key=lambda i: (scores[i], i))[64:])
    code = sc.CodeSpec.from_frozen_set(256, frozen, 200, device="cuda")
    dec = sc.DeletionDecoder(code, 2, 0.1)
    info_w, rx, ln = mc.philox_deletion_batch(code, 20250204, 0, 1 << 20, 2, 0.1, 0.1)
    out = dec.decode_native(rx, ln)[0]
    fe, _ = mc.error_counts(sc.unpack(out, code.K), sc.unpack(info_w, code.K))
    ok, info = _close(fe, 1 << 20, _ref("C5k64" if k64 else "C5"))
    assert ok, info
