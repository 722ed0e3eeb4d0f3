"""The kernel's decode schedule (polarcub_amd/csrc/sc_bin_body.h) compiled for the
host (tests/emu) against the reference's golden vectors: catches schedule and
indexing bugs on CPU.  The emulator runs the one-lane-per-codeword paths."""
import ctypes
import os

import numpy as np
import pytest

from polarcub_amd.sc import pack_rows, unpack_rows
from tests.conftest import ROOT, edge_cases, load_golden

_L = None


def emu():
    global _L
    if _L is None:
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "emu")], check=True)
        _L = ctypes.CDLL(os.path.join(ROOT, "tests", "emu", "build", "libemu.so"))
    return _L


def run(xy, frozen, fval, S):
    B, N, _ = xy.shape
    n = N.bit_length() - 1
    K = int(N - frozen.sum())
    fm = pack_rows(frozen).reshape(-1).copy()
    fv = pack_rows(fval).reshape(-1).copy()
    xyt = np.ascontiguousarray(np.transpose(xy, (1, 0, 2)))
    info = np.zeros((max(1, (K + 31) // 32), B), np.uint32)
    xh = np.zeros((max(1, (N + 31) // 32), B), np.uint32)
    uo = np.zeros_like(xh)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = emu().emu_decode_bin(P(xyt), ctypes.c_longlong(B), n, P(fm), P(fv), P(info), P(xh), P(uo), S)
    assert rc == 0
    return unpack_rows(info, K), unpack_rows(xh, N), unpack_rows(uo, N)


@pytest.mark.parametrize("S", [8, 16, 32])
@pytest.mark.parametrize("name", ["bsc_n64", "awgn_n1024", "awgn_n256_lowsnr"])
def test_schedule_matches_reference(name, S):
    g = load_golden(name)
    xy = g["xy"] if "xy" in g else g["table"][g["y"]]
    if xy.shape[1] < 2 * S:
        pytest.skip("code shorter than two register subtrees")
    info, xhat, u = run(xy, g["frozen"], g["fval"], S)
    assert np.array_equal(info, g["info"])
    assert np.array_equal(xhat, g["xhat"])
    # u = decisions: information positions carry the info bits, frozen ones the frozen values
    assert np.array_equal(u[:, g["frozen"] == 0], g["info"])
    assert np.all(u[:, g["frozen"] == 1] == g["fval"][g["frozen"] == 1])


def test_schedule_awgn_4096():
    g = load_golden("awgn_n4096")
    info, xhat, _ = run(g["xy"], g["frozen"], g["fval"], 16)
    assert np.array_equal(info, g["info"]) and np.array_equal(xhat, g["xhat"])


@pytest.mark.parametrize("idx", range(24))
def test_schedule_edge_cases(idx):
    c = edge_cases()[idx]
    info, xhat, _ = run(c["xy"], c["frozen"], c["fval"], 8)
    assert np.array_equal(info, c["info"]) and np.array_equal(xhat, c["xhat"])


def test_bit_helpers():
    assert emu().emu_check_bits(ctypes.c_uint64(0x9E3779B97F4A7C15)) == 0


@pytest.mark.parametrize("S", [8, 16, 32])
@pytest.mark.parametrize("n", [6, 7, 8, 10])
def test_schedule_rate0_blocks(n, S):
    """Frozen sets full of aligned rate-0 blocks (skipped by the schedule) against the oracle."""
    from oracle import orc
    from tests.conftest import awgn_like, blocky_frozen
    N = 1 << n
    if N < 2 * S:
        pytest.skip("code shorter than two register subtrees")
    rng = np.random.default_rng(100 * n + S)
    for _ in range(3):
        frozen, fval = blocky_frozen(N, rng)
        xy = awgn_like(40, N, rng)
        info, xhat, u = run(xy, frozen, fval, S)
        ri, rx = orc.decode_bin(xy, frozen, fval)
        assert np.array_equal(info, ri) and np.array_equal(xhat, rx)
        assert np.all(u[:, frozen == 1] == fval[frozen == 1])


@pytest.mark.parametrize("S", [8, 16, 32])
@pytest.mark.parametrize("n", [6, 8, 10])
def test_compact_root_schedule_matches_pairs(n, S):
    """The compact-root schedule (CR: rows as compact normalised doubles) decodes exactly what the
    pair schedule decodes on the pairs they stand for (zeros, -0.0, ties and a (0, 0) row in)."""
    rng = np.random.default_rng(10 * n + S)
    N, B = 1 << n, 40
    if N < 2 * S:
        pytest.skip("code shorter than two register subtrees")
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    frozen[: N // 8] = 1
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    r = rng.random((B, N)) ** 3
    r[rng.random((B, N)) < 0.03] = 0.0
    r[rng.random((B, N)) < 0.02] = 1.0
    xc = np.where(rng.random((B, N)) < 0.5, r, -r)
    xc[0, 1] = -0.0
    xc[2, 3] = np.nan
    ab = np.abs(xc)
    pairs = np.where(np.signbit(xc)[..., None], np.stack([ab, np.ones_like(ab)], -1),
                     np.stack([np.ones_like(ab), ab], -1))
    pairs[2, 3] = 0.0
    info_p, xh_p, _ = run(pairs, frozen, fval, S)
    K = int(N - frozen.sum())
    fm = pack_rows(frozen).reshape(-1).copy()
    fv = pack_rows(fval).reshape(-1).copy()
    xct = np.ascontiguousarray(xc.T)
    info = np.zeros((max(1, (K + 31) // 32), B), np.uint32)
    xh = np.zeros((max(1, (N + 31) // 32), B), np.uint32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    assert emu().emu_decode_bin_compact(P(xct), ctypes.c_longlong(B), n, P(fm), P(fv), P(info), P(xh), S, 0) == 0
    assert np.array_equal(unpack_rows(info, K), info_p)
    assert np.array_equal(unpack_rows(xh, N), xh_p)
