"""q-ary list decoding (SCL / Fast-SSC, QaryPolarEncoderDecoder.py:118-227, 403-930) on CPU:
the oracle's restatement (oracle/scl_oracle.py) against runs of the reference itself
(tests/golden/scl.npz: 144 listDecode calls on tie-free inputs, two irSimulation runs), and the
host build of the kernel code (tests/emu/scl_emu.cpp over polarcub_amd/csrc/scl_body.h) against
the oracle, bit for bit, including inputs with ties (QSC rows).

Parity contract (include/polarcub_sc.h): the reference orders the list and breaks ties with
numpy's argpartition (x86-simd-sort on AVX-512 hosts, so CPU-dependent); the final path SET and
the metrics are compared with the reference (metrics within 1e-12 relative), everything --
order, ties included -- with the oracle."""
import ctypes
import math
import os
import random

import numpy as np
import pytest

from oracle import scl_oracle as so
from tests.conftest import ROOT, load_golden


@pytest.fixture(scope="module")
def emu():
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "emu")], check=True)
    return ctypes.CDLL(os.path.join(ROOT, "tests", "emu", "build", "libsclemu.so"))


def emu_decode(E, xy, q, L, frozen, fvals, actual, use_log=False):
    P = ctypes.c_void_p
    B, N, _ = xy.shape
    n = N.bit_length() - 1
    K = int((np.asarray(frozen) == 0).sum())
    nF = N - K
    x = np.ascontiguousarray(np.asarray(xy, np.float64).transpose(1, 0, 2))
    fv = np.ascontiguousarray(np.asarray(fvals, np.uint8).reshape(B, nF).T) if nF else np.zeros((1, B), np.uint8)
    act = None if actual is None else np.ascontiguousarray(np.asarray(actual, np.uint8).reshape(B, K).T)
    oi = np.zeros((L, max(K, 1), B), np.uint8)
    op = np.zeros((L, B))
    osz = np.zeros(B, np.int32)
    oa = np.zeros(B)
    fz = np.ascontiguousarray(np.asarray(frozen, np.uint8))
    E.emu_scl(x.ctypes.data_as(P), ctypes.c_longlong(B), q, n, L, fz.ctypes.data_as(P), fv.ctypes.data_as(P), nF,
              None if act is None else act.ctypes.data_as(P), K, oi.ctypes.data_as(P), op.ctypes.data_as(P),
              osz.ctypes.data_as(P), oa.ctypes.data_as(P), int(use_log))
    return osz, oi[:, :K].transpose(2, 0, 1), op.T, oa


def _cases():
    return load_golden("scl")["meta"]["cases"]


def _as_set(info, probs):
    return sorted(zip(map(tuple, info), probs))


@pytest.mark.parametrize("case", range(12))
def test_oracle_matches_reference_list_set(case):
    g = load_golden("scl")
    c = g["meta"]["cases"][case]
    t_, q, L = c["tag"], c["q"], c["L"]
    for t in range(g[t_ + "_xy"].shape[0]):
        k, info, probs, ap = so.list_decode(q, g[t_ + "_frozen"], L, g[t_ + "_xy"][t], g[t_ + "_fv"][t],
                                            g[t_ + "_actual"][t])
        rk = int(g[t_ + "_size"][t])
        assert k == rk
        ours = _as_set(info, probs)
        ref = _as_set(g[t_ + "_info"][t][:rk].tolist(), g[t_ + "_prob"][t][:rk].tolist())
        assert [a for a, _ in ours] == [a for a, _ in ref]
        assert np.allclose([p for _, p in ours], [p for _, p in ref], rtol=1e-12, atol=0)
        assert math.isclose(ap, g[t_ + "_aprob"][t], rel_tol=1e-12)


def _random_inputs(rng, q, n, B, ties):
    N = 1 << n
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    K = int((frozen == 0).sum())
    if ties:  # QSC rows: permutations of (1-p, p/(q-1), ...), the reference's IR channel
        p = 0.2
        y = rng.integers(0, q, (B, N))
        xy = np.where(np.arange(q)[None, None, :] == y[:, :, None], 1.0 - p, p / (q - 1))
    else:
        xy = rng.random((B, N, q)) * 0.98 + 0.02
    return frozen, xy, rng.integers(0, q, (B, N - K)), rng.integers(0, q, (B, K))


@pytest.mark.parametrize("q,n,L,ties", [(2, 3, 2, False), (3, 4, 4, False), (4, 5, 8, False), (2, 6, 16, False),
                                        (3, 4, 4, True), (4, 5, 8, True), (2, 5, 3, True), (5, 3, 4, False)])
def test_kernel_code_matches_oracle(emu, q, n, L, ties):
    rng = np.random.default_rng(100 * q + 10 * n + L + ties)
    frozen, xy, fv, act = _random_inputs(rng, q, n, 6, ties)
    size, info, prob, ap = emu_decode(emu, xy, q, L, frozen, fv, act)
    for b in range(xy.shape[0]):
        k, oinfo, oprob, oap = so.list_decode(q, frozen, L, xy[b], fv[b], act[b])
        assert size[b] == k
        assert info[b][:k].tolist() == oinfo
        assert np.array_equal(prob[b][:k], np.array(oprob))
        assert ap[b] == oap


def test_kernel_code_matches_oracle_on_reference_inputs(emu):
    g = load_golden("scl")
    for c in g["meta"]["cases"]:
        t_ = c["tag"]
        size, info, prob, ap = emu_decode(emu, g[t_ + "_xy"], c["q"], c["L"], g[t_ + "_frozen"], g[t_ + "_fv"],
                                          g[t_ + "_actual"])
        for b in range(g[t_ + "_xy"].shape[0]):
            k, oinfo, oprob, oap = so.list_decode(c["q"], g[t_ + "_frozen"], c["L"], g[t_ + "_xy"][b],
                                                  g[t_ + "_fv"][b], g[t_ + "_actual"][b])
            assert size[b] == k and info[b][:k].tolist() == oinfo
            assert np.array_equal(prob[b][:k], np.array(oprob)) and ap[b] == oap


def ir_closures(r):
    chan = random.Random(r["chan_seed"])
    q, sig, N = r["q"], r["sigma"], 1 << r["n"]
    from polarcub_amd import vectors

    def simulate(a):
        return [float(x) + chan.gauss(0.0, sig) for x in a]

    def make_xy(b):
        vd = vectors.QaryMemorylessVectorDistribution(q, N)
        for i, y in enumerate(b):
            vd.probs[i] = [math.exp(-((y - x) ** 2) / (2 * sig * sig)) for x in range(q)]
        return vd
    return simulate, make_xy


@pytest.mark.parametrize("which", [0, 1])
def test_ir_simulation_logic_with_oracle_matches_reference(which, monkeypatch, capsys):
    """The facade's batched irSimulation with the oracle standing in for the GPU list decoder:
    frame errors, per-trial ProbResults, rate and their printed lines equal to the reference run.
    The symbol-error line is not compared: on a failure the reference returns informationList[0],
    and that list's order is argpartition's (100 vs 108 and 359 vs 371 symbol errors here)."""
    from polarcub_amd import coding_qary
    g = load_golden("scl")
    r = g["meta"]["ir"][which]

    def oracle_batch(self, xy, fvals, L, actual):
        B = xy.shape[0]
        info = np.full((B, L, self.k), -1, np.int64)
        prob = np.zeros((B, L))
        size = np.zeros(B, np.int64)
        ap = np.zeros(B)
        for b in range(B):
            k, inf, p, a = so.list_decode(self.q, self._mask, L, xy[b], fvals[b], actual[b])
            size[b], ap[b] = k, a
            info[b, :k] = inf
            prob[b, :k] = p
        return info, prob, size, ap
    monkeypatch.setattr(coding_qary.QaryPolarEncoderDecoder, "list_decode_batch", oracle_batch)
    simulate, make_xy = ir_closures(r)
    frozen = set(int(i) for i in np.nonzero(g[r["name"] + "_frozen"])[0])
    np.random.seed(r["np_seed"])
    fe, se, rate, prl = coding_qary.irSimulation(r["q"], 1 << r["n"], simulate, make_xy, r["trials"], frozen, r["L"],
                                                 r["check_size"], verbosity=1)
    assert fe == r["frame_error_prob"] and rate == r["rate"]
    assert [p.name for p in prl] == r["prob_results"]
    lines = capsys.readouterr().out.splitlines()
    assert lines[:2] == r["printed"].splitlines()[:2]


# -- log domain (use_log=True: recursiveListDecode's use_log branches) -----------------------
LOG_RTOL, LOG_ATOL = 1e-12, 1e-9  # log-domain metrics: few-ulp exp/log1p/log differences


def _close_log(a, b):
    return np.allclose(a, b, rtol=LOG_RTOL, atol=LOG_ATOL)


@pytest.mark.parametrize("case", range(12))
def test_oracle_log_matches_reference_list_set(case):
    """The oracle's log domain against the reference's own use_log=True listDecode runs
    (tests/golden/scl_log.npz: the scl.npz cases on np.log rows)."""
    g = load_golden("scl_log")
    c = g["meta"]["cases"][case]
    t_, q, L = c["tag"], c["q"], c["L"]
    for t in range(g[t_ + "_xy"].shape[0]):
        k, info, probs, ap = so.list_decode(q, g[t_ + "_frozen"], L, g[t_ + "_xy"][t], g[t_ + "_fv"][t],
                                            g[t_ + "_actual"][t], use_log=True)
        rk = int(g[t_ + "_size"][t])
        assert k == rk
        ours = _as_set(info, probs)
        ref = _as_set(g[t_ + "_info"][t][:rk].tolist(), g[t_ + "_prob"][t][:rk].tolist())
        assert [a for a, _ in ours] == [a for a, _ in ref]
        assert _close_log([p for _, p in ours], [p for _, p in ref])
        assert _close_log(ap, g[t_ + "_aprob"][t])


def test_log_and_linear_reference_runs_agree():
    """The reference's two domains pick the same final path sets on these tie-free inputs (so the
    log-domain fixture exercises the same lists), with log metrics = log of the linear ones."""
    gl, g = load_golden("scl_log"), load_golden("scl")
    for c in g["meta"]["cases"]:
        t_ = c["tag"]
        assert np.array_equal(gl[t_ + "_size"], g[t_ + "_size"])
        for t in range(g[t_ + "_xy"].shape[0]):
            rk = int(g[t_ + "_size"][t])
            a = _as_set(g[t_ + "_info"][t][:rk].tolist(), np.log(g[t_ + "_prob"][t][:rk]).tolist())
            b = _as_set(gl[t_ + "_info"][t][:rk].tolist(), gl[t_ + "_prob"][t][:rk].tolist())
            assert [x for x, _ in a] == [x for x, _ in b]
            assert np.allclose([p for _, p in a], [p for _, p in b], rtol=1e-9, atol=1e-9)


def _log_inputs(rng, q, n, B, ties):
    frozen, xy, fv, act = _random_inputs(rng, q, n, B, ties)
    with np.errstate(divide="ignore"):
        lxy = np.log(xy)
    return frozen, lxy, fv, act


def _oracle_log_with_gap(monkeypatch, *args):
    """so.list_decode(..., use_log=True) and the smallest gap between the last kept and the first
    dropped candidate metric over its prunes (0 = an exact tie)."""
    gaps = [math.inf]
    orig = so._keep

    def keep(cand, L, use_log=False):
        if len(cand) > L:
            srt = sorted(cand, reverse=True)
            gaps.append(srt[L - 1] - srt[L])
        return orig(cand, L, use_log)
    monkeypatch.setattr(so, "_keep", keep)
    try:
        return so.list_decode(*args, use_log=True), min(gaps)
    finally:
        monkeypatch.setattr(so, "_keep", orig)


@pytest.mark.parametrize("q,n,L,ties", [(2, 3, 2, False), (3, 4, 4, False), (4, 5, 8, False), (2, 6, 16, False),
                                        (4, 8, 4, False), (2, 9, 2, False), (3, 4, 4, True), (4, 5, 8, True)])
def test_kernel_code_log_matches_oracle(emu, monkeypatch, q, n, L, ties):
    """The kernel's log domain (host build of scl_body.h) against the oracle's: the same lists in
    the same order (the tie rules are shared), metrics within the log tolerance.  n = 8, 9 take the
    rate-0 / repetition sums past numpy's 128-element pairwise blocks.  Log-domain values differ
    from the oracle's by ulps (its logsumexp runs numpy's vectorised exp), so a prune whose kept /
    dropped metrics are within 1e-9 may go either way (exact ties too: QSC rows, and random rows
    flattened to uniform by many minus levels; permuted rows' logsumexp differs by an ulp with the
    summation order, in the reference's numpy as here, so not even the reference's own tie pattern
    is reproducible): for such codewords only the list size and the normalisation are checked;
    without ties at least half the codewords compare in full."""
    rng = np.random.default_rng(300 * q + 10 * n + L + ties)
    frozen, xy, fv, act = _log_inputs(rng, q, n, 6, ties)
    if n >= 8:  # a long rate-0 node (the first half), then a rate-1 (n = 8) or repetition (n = 9) half
        N = 1 << n
        frozen[: N // 2] = 1
        frozen[N // 2:] = 0 if n == 8 else 1
        frozen[N - 1] = 0
        K = int((frozen == 0).sum())
        fv = rng.integers(0, q, (6, N - K))
        act = rng.integers(0, q, (6, K))
        y = rng.integers(0, q, (6, N))
        lin = np.where(np.arange(q)[None, None, :] == y[:, :, None], 0.9, 0.1 / (q - 1))
        xy = np.log(lin * (0.9 + 0.2 * rng.random(lin.shape)))
    size, info, prob, ap = emu_decode(emu, xy, q, L, frozen, fv, act, use_log=True)
    compared = 0
    for b in range(xy.shape[0]):
        (k, oinfo, oprob, oap), gap = _oracle_log_with_gap(monkeypatch, q, frozen, L, xy[b], fv[b], act[b])
        if gap < 1e-9:  # which of the (near-)tied candidates survive may differ, and so may what follows
            assert size[b] == k and prob[b][:k].max() == 0.0
            continue
        compared += 1
        assert size[b] == k
        assert info[b][:k].tolist() == oinfo
        assert _close_log(prob[b][:k], np.array(oprob))
        assert _close_log(ap[b], oap)
    assert ties or compared >= xy.shape[0] // 2


def test_kernel_code_log_matches_reference_sets(emu):
    g = load_golden("scl_log")
    for c in g["meta"]["cases"]:
        t_ = c["tag"]
        size, info, prob, ap = emu_decode(emu, g[t_ + "_xy"], c["q"], c["L"], g[t_ + "_frozen"], g[t_ + "_fv"],
                                          g[t_ + "_actual"], use_log=True)
        for t in range(g[t_ + "_xy"].shape[0]):
            rk = int(g[t_ + "_size"][t])
            assert size[t] == rk
            ours = _as_set(info[t][:rk].tolist(), prob[t][:rk].tolist())
            ref = _as_set(g[t_ + "_info"][t][:rk].tolist(), g[t_ + "_prob"][t][:rk].tolist())
            assert [a for a, _ in ours] == [a for a, _ in ref]
            assert _close_log([p for _, p in ours], [p for _, p in ref])
            assert _close_log(ap[t], g[t_ + "_aprob"][t])


def ir_closures_log(r):
    chan = random.Random(r["chan_seed"])
    q, sig, N = r["q"], r["sigma"], 1 << r["n"]
    from polarcub_amd import vectors

    def simulate(a):
        return [float(x) + chan.gauss(0.0, sig) for x in a]

    def make_xy(b):
        vd = vectors.QaryMemorylessVectorDistribution(q, N, use_log=True)
        for i, y in enumerate(b):
            vd.probs[i] = [-((y - x) ** 2) / (2 * sig * sig) for x in range(q)]
        return vd
    return simulate, make_xy


@pytest.mark.parametrize("which", [0, 1])
def test_ir_simulation_log_logic_with_oracle_matches_reference(which, monkeypatch, capsys):
    """irSimulation(use_log=True) with the oracle's log domain standing in for the GPU decoder:
    frame errors, rate, ProbResults and the printed lines of the reference's log-domain run."""
    from polarcub_amd import coding_qary
    g = load_golden("scl_log")
    r = g["meta"]["ir"][which]

    def oracle_batch(self, xy, fvals, L, actual):
        assert self.use_log
        B = xy.shape[0]
        info = np.full((B, L, self.k), -1, np.int64)
        prob = np.zeros((B, L))
        size = np.zeros(B, np.int64)
        ap = np.zeros(B)
        for b in range(B):
            k, inf, p, a = so.list_decode(self.q, self._mask, L, xy[b], fvals[b], actual[b], use_log=True)
            size[b], ap[b] = k, a
            info[b, :k] = inf
            prob[b, :k] = p
        return info, prob, size, ap
    monkeypatch.setattr(coding_qary.QaryPolarEncoderDecoder, "list_decode_batch", oracle_batch)
    simulate, make_xy = ir_closures_log(r)
    frozen = set(int(i) for i in np.nonzero(g[r["name"] + "_frozen"])[0])
    np.random.seed(r["np_seed"])
    fe, se, rate, prl = coding_qary.irSimulation(r["q"], 1 << r["n"], simulate, make_xy, r["trials"], frozen, r["L"],
                                                 r["check_size"], use_log=True, verbosity=1)
    assert fe == r["frame_error_prob"] and rate == r["rate"]
    assert [p.name for p in prl] == r["prob_results"]
    lines = capsys.readouterr().out.splitlines()
    assert lines[:2] == r["printed"].splitlines()[:2]
