"""The deletion kernel's trellis code (polarcub_amd/csrc/trellis_body.h) compiled for
the host (tests/emu/del_emu.cpp) against the reference's golden vectors: catches
ordering and capacity bugs of the trellis stages on CPU, before any GPU run."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from polarcub_amd.sc import pack_rows, unpack_rows
from tests.conftest import ROOT, load_golden
from tests.test_trellis_oracle import deletion_edge_cases

_L = None


def emu():
    global _L
    if _L is None:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "emu")], check=True)
        _L = ctypes.CDLL(os.path.join(ROOT, "tests", "emu", "build", "libdelemu.so"))
    return _L


def run(rx, rx_len, n, n0, pd, frozen, fval, ones=0):
    B = rx.shape[0]
    N = 1 << n
    K = int(N - frozen.sum())
    fm = pack_rows(frozen).reshape(-1).copy()
    fv = pack_rows(fval).reshape(-1).copy()
    rx = np.ascontiguousarray(rx, np.uint8)
    ln = np.ascontiguousarray(rx_len, np.int32)
    info = np.zeros((max(1, (K + 31) // 32), B), np.uint32)
    xh = np.zeros((max(1, (N + 31) // 32), B), np.uint32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = emu().emu_decode_deletion(P(rx), P(ln), ctypes.c_longlong(B), rx.shape[1], n, n0, ones, ctypes.c_double(pd),
                                   P(fm), P(fv), P(info), P(xh))
    assert rc == 0
    return unpack_rows(info, K), unpack_rows(xh, N)


@pytest.fixture(params=[False, True], ids=["general", "n02"])
def n02(request):
    """Both trellis representations: the general one (trellis_body.h) and, for n0 = 2,
    the register-resident one the kernel uses (trellis_n02.h)."""
    emu().emu_set_n02(int(request.param))
    yield request.param
    emu().emu_set_n02(0)


def test_c5_golden(n02):
    g = load_golden("deletion_n8")
    m = g["meta"]
    info, xhat = run(g["rx"], g["rx_len"], m["n"], m["n0"], m["pd"], g["frozen"], g["fval"])
    assert np.array_equal(info, g["info"])
    assert np.array_equal(xhat, g["xhat"])


@pytest.mark.parametrize("idx", range(11))
def test_edge_golden(idx, n02):
    c = deletion_edge_cases()[idx]
    n, n0, ones = (int(v) for v in c["shape"])
    if n02 and (n0 != 2 or ones != 0):
        pytest.skip("the register-resident representation covers n0 = 2 without guard-band ones")
    info, xhat = run(c["rx"], c["rx_len"], n, n0, float(c["pd"][0]), c["frozen"], c["fval"], ones)
    assert np.array_equal(info, c["info"])
    assert np.array_equal(xhat, c["xhat"])


@pytest.mark.parametrize("idx", range(11))
def test_edge_golden_implicit_base(idx, implicit_base):
    c = deletion_edge_cases()[idx]
    n, n0, ones = (int(v) for v in c["shape"])
    if n0 < 3 or ones != 0:
        pytest.skip("the implicit base trellis is the n0 >= 3 path without guard-band ones")
    info, xhat = run(c["rx"], c["rx_len"], n, n0, float(c["pd"][0]), c["frozen"], c["fval"], ones)
    assert np.array_equal(info, c["info"])
    assert np.array_equal(xhat, c["xhat"])


@pytest.mark.parametrize("n", [3, 5, 8])
def test_n02_random_vs_oracle(n):
    """Register-resident n0 = 2 path on random channel outputs and adversarial words."""
    import random

    from oracle import trellis_oracle as tro
    emu().emu_set_n02(1)
    try:
        N = 1 << n
        rng = np.random.default_rng(n)
        prng = random.Random(n)
        frozen = (rng.random(N) < 0.5).astype(np.uint8)
        fval = (rng.random(N) < 0.5).astype(np.uint8)
        words = []
        for t in range(40):
            x = [int(b) for b in rng.integers(0, 2, N)]
            words.append(tro.deletion_channel(tro.add_guard_bands(x, n, 2, 0.1), [0.05, 0.2, 0.5][t % 3], prng))
        words += [[], [1], [1, 1, 1, 1, 1], [int(b) for b in rng.integers(0, 2, 3 * N)]]
        W = max(len(w) for w in words)
        rx = np.zeros((len(words), W), np.uint8)
        for i, w in enumerate(words):
            rx[i, :len(w)] = w
        info, xhat = run(rx, np.array([len(w) for w in words], np.int32), n, 2, 0.1, frozen, fval)
        for i, w in enumerate(words):
            xr, ir = tro.decode_deletion(w, n, 2, 0.1, frozen, fval)
            assert list(info[i]) == ir and list(xhat[i]) == xr, i
    finally:
        emu().emu_set_n02(0)


def test_packed_segment_parse_matches_byte_parse():
    """The kernel parses guard bands on the bit-packed received word (segment_of_packed):
    same (start, length) as the byte-wise removeDeletionGuardBands restatement for every
    trellis of 1..6 levels on random words with long zero runs."""
    L = emu()
    L.emu_check_segments.restype = ctypes.c_longlong
    assert L.emu_check_segments(ctypes.c_uint64(12345), 3000) == 0


def test_dense_layout_host_pieces():
    """The table-driven layout (sc_del_dense.h): a lane's shared descent plus per-level splits
    (dense_segments) gives segment_of_packed's segment for each of its trellises at 16..256
    trellises on random words with long zero runs; enc_hist is DelNode's re-encoding; the history
    slots are the n0 = 2 and n0 = 3 tables' layouts."""
    L = emu()
    L.emu_check_dense.restype = ctypes.c_longlong
    assert L.emu_check_dense(ctypes.c_uint64(777), 600) == 0


@pytest.fixture(params=[False, True], ids=["stored-base", "implicit-base"])
def implicit_base(request):
    """n0 >= 3 without guard-band ones: the kernel never stores the base trellis (BaseT,
    trellis_body.h); the emulator then builds the top level's children from it and checks
    each one against the stored base's child, field by field."""
    emu().emu_set_base(int(request.param))
    yield request.param
    emu().emu_set_base(0)


@pytest.mark.parametrize("n0,n,ones", [(3, 10, 0), (3, 11, 0), (4, 12, 0), (4, 6, 0), (2, 5, 1), (1, 4, 2),
                                       (3, 6, 3), (4, 6, 2), (2, 9, 0), (3, 7, 0), (4, 8, 0)])
def test_wide_shapes_vs_oracle(n0, n, ones, implicit_base):
    """Shapes the widened kernel adds: more than 64 trellises (main_deletion.py's n0 = n // 3
    at n = 10..12), 16-input trellises and guard-band ones (capacities, vertex probabilities,
    the materialised collapse), against the oracle."""
    import random

    from oracle import trellis_oracle as tro
    N = 1 << n
    rng = np.random.default_rng(97 * n + 7 * n0 + ones)
    prng = random.Random(n + ones)
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    frozen[: N // 4] = 1
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    pd = [0.05, 0.1, 0.2][(n + ones) % 3]
    words = []
    for t in range(3 if n >= 10 else 8):
        x = [int(b) for b in rng.integers(0, 2, N)]
        words.append(tro.deletion_channel(tro.add_guard_bands(x, n, n0, 0.1, ones), pd, prng))
    words += [[], [1, 1, 1], [int(b) for b in rng.integers(0, 2, N // 2)]]
    W = max(len(w) for w in words)
    rx = np.zeros((len(words), W), np.uint8)
    for i, w in enumerate(words):
        rx[i, :len(w)] = w
    L = emu()
    L.emu_base_checks.restype = ctypes.c_longlong
    L.emu_n03_checks.restype = ctypes.c_longlong
    checks0 = L.emu_base_checks()
    n03_0 = L.emu_n03_checks()
    info, xhat = run(rx, np.array([len(w) for w in words], np.int32), n, n0, pd, frozen, fval, ones)
    if implicit_base and n0 >= 3 and ones == 0:
        assert L.emu_base_checks() > checks0
    if n0 == 3 and ones == 0:  # every n0 = 3 leaf value matched its segment-state table entry
        assert L.emu_n03_checks() > n03_0
    for i, w in enumerate(words):
        xr, ir = tro.decode_deletion(w, n, n0, pd, frozen, fval, ones=ones)
        assert list(info[i]) == ir and list(xhat[i]) == xr, i


def test_dense_trellis_matches_trel():
    """trellis_dense.h (the dense-slot trellises, test-only: tests/emu/, no guard-band ones)
    against trellis_body.h's Trel on random segments (n0 = 3 and 4, pd from 0 to 1, lengths around,
    below and above the trellis length) and random decision histories: every stage holds the same
    edges in the same creation order, the same vertices in the same insertion order, bit-identical
    probabilities and collapsed values (tests/emu/dtrel_check.cpp)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "emu")], check=True)
    exe = os.path.join(ROOT, "tests", "emu", "build", "dtrel_check")
    for seed in (11, 12):
        r = subprocess.run([exe, "100000", str(seed)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert " 0 mismatches" in r.stdout


def test_wave_trellises_match_trel():
    """trellis_wave.h (the n0 = 4 wave-per-task trellises of sc_del_w4.hip: edges at fixed slots, the
    reference's creation and insertion orders as ranks of first contributions) against
    trellis_body.h's Trel walk on random segments (lengths 0..16 and beyond, pd from 0 to 1) and random
    decision histories: every depth-3 node's three collapsed rows bit-identical, and the re-encoding of
    the 16 decisions equal to the recursion's (tests/emu/w4_check.cpp, its lanes run one after another)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "emu")], check=True)
    exe = os.path.join(ROOT, "tests", "emu", "build", "w4_check")
    for seed in (21, 22):
        r = subprocess.run([exe, "20000", str(seed)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert " 0 mismatches" in r.stdout
