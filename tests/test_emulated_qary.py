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


@pytest.mark.parametrize("S", [1, 2, 4, 8])
def test_qsc_golden(S):
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
        for S in (1, 2, 4, 8):
            if N < 2 * S:
                continue
            info, xh = run(xy, frozen, q, S)
            assert np.array_equal(info, ri), (q, N, S)
            assert np.array_equal(xh, rx), (q, N, S)
