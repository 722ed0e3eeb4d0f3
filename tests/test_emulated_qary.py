"""The q-ary kernel's schedule (polarcub_amd/csrc/sc_qary_body.h: register subtrees,
fused chain passes, rate-0 skipping) compiled for the host, against the reference's
golden vectors and the C oracle, every register-subtree size."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import orc
from tests.conftest import ROOT, load_golden

_L = None


def emu():
    global _L
    if _L is None:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "emu")], check=True)
        _L = ctypes.CDLL(os.path.join(ROOT, "tests", "emu", "build", "libqemu.so"))
    return _L


def run(xy, frozen, q, S):
    B, N, _ = xy.shape
    n = N.bit_length() - 1
    K = int(N - frozen.sum())
    native = np.ascontiguousarray(np.transpose(xy, (1, 0, 2)))
    fr = np.ascontiguousarray(frozen, np.uint8)
    info = np.zeros((max(K, 1), B), np.uint8)
    xh = np.zeros((N, B), np.uint8)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = emu().emu_decode_qary(P(native), ctypes.c_longlong(B), n, q, P(fr), P(info), P(xh), S)
    assert rc == 0
    return info[:K].T, xh.T


@pytest.mark.parametrize("S", [1, 2, 4, 8, 16, -1, -2, -4, -8])
def test_qsc_golden(S):
    """S < 0: the split-level schedule (HL) with |S| register positions."""
    g = load_golden("qsc_q4_n256")
    info, _ = run(g["table"][g["y"]], g["frozen"], 4, S)
    assert np.array_equal(info, g["info"])
    info, _ = run(g["xy_rand"], g["frozen"], 4, S)
    assert np.array_equal(info, g["info_rand"])


@pytest.mark.parametrize("q", [2, 3, 5, 8])
def test_random_vs_oracle(q):
    rng = np.random.default_rng(100 + q)
    for N, B in [(4, 9), (16, 40), (128, 60)]:
        frozen = (rng.random(N) < 0.4).astype(np.uint8)
        frozen[: N // 4] = 1  # rate-0 blocks
        xy = rng.random((B, N, q))
        xy[rng.random((B, N)) < 0.05] = 0.0
        ri, rx = orc.decode_qary(q, xy, frozen)
        for S in (1, 2, 4, 8, 16, -1, -2, -4):
            if N < (-4 * S if S < 0 else 2 * S):
                continue
            info, xh = run(xy, frozen, q, S)
            assert np.array_equal(info, ri), (q, N, S)
            assert np.array_equal(xh, rx), (q, N, S)


def test_qdiv_matches_ieee_division():
    """q_div (one correctly rounded reciprocal per vector + Markstein's correction per
    component, guarded range) returns exactly p / t: normalised sums of random products,
    raw channel rows, tiny / huge / zero components, all-ones significands, ties."""
    rng = np.random.default_rng(7)
    cases = []
    # what the transforms produce: sums of products of normalised vectors
    a = rng.dirichlet(np.ones(4), size=200000)
    b = rng.dirichlet(np.ones(4), size=200000)
    p = np.stack([a[:, 0] * b[:, 0] + a[:, 1] * b[:, 3], a[:, 2] * b[:, 1], a[:, 3] * b[:, 2], a[:, 1] * b[:, 1]], 1)
    cases.append(p)
    # wide dynamic range per component
    e = rng.integers(-1074, 30, size=(200000, 4)).astype(np.float64)
    cases.append(rng.random((200000, 4)) * np.exp2(e))
    cases.append(np.exp2(rng.integers(-900, 0, size=(100000, 4)).astype(np.float64)) * (1 + rng.random((100000, 4))))
    # significands near 1 and near 2 (reciprocal rounding edges), zeros, equal components
    m = 1.0 + rng.integers(0, 64, size=(100000, 4)) * 2.0 ** -52
    m2 = 2.0 - rng.integers(1, 64, size=(100000, 4)) * 2.0 ** -52
    cases.append(m * np.exp2(rng.integers(-60, 4, size=(100000, 4)).astype(np.float64)))
    cases.append(m2 * np.exp2(rng.integers(-60, 4, size=(100000, 4)).astype(np.float64)))
    z = rng.random((100000, 4))
    z[rng.random((100000, 4)) < 0.3] = 0.0
    z[:, 1] = np.where(rng.random(100000) < 0.2, z[:, 0], z[:, 1])
    cases.append(z)
    P = np.ascontiguousarray(np.concatenate(cases), np.float64)
    T = np.zeros(P.shape[0])
    for x in range(4):
        T = T + P[:, x]  # left-to-right sum, as the normaliser
    keep = T != 0
    P, T = np.ascontiguousarray(P[keep]), np.ascontiguousarray(T[keep])
    Pt = lambda v: v.ctypes.data_as(ctypes.c_void_p)
    emu().emu_qdiv_check.restype = ctypes.c_longlong
    bad = emu().emu_qdiv_check(Pt(P), Pt(T), ctypes.c_longlong(P.shape[0]))
    assert bad == 0
    # divisors far from the sums too (scaled t)
    T2 = np.ascontiguousarray(T * np.exp2(rng.integers(0, 300, size=T.shape[0]).astype(np.float64)))
    assert emu().emu_qdiv_check(Pt(P), Pt(T2), ctypes.c_longlong(P.shape[0])) == 0
