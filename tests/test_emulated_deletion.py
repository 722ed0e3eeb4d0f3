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


def run(rx, rx_len, n, n0, pd, frozen, fval):
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
    rc = emu().emu_decode_deletion(P(rx), P(ln), ctypes.c_longlong(B), rx.shape[1], n, n0, ctypes.c_double(pd),
                                   P(fm), P(fv), P(info), P(xh))
    assert rc == 0
    return unpack_rows(info, K), unpack_rows(xh, N)


def test_c5_golden():
    g = load_golden("deletion_n8")
    m = g["meta"]
    info, xhat = run(g["rx"], g["rx_len"], m["n"], m["n0"], m["pd"], g["frozen"], g["fval"])
    assert np.array_equal(info, g["info"])
    assert np.array_equal(xhat, g["xhat"])


@pytest.mark.parametrize("idx", range(11))
def test_edge_golden(idx):
    c = deletion_edge_cases()[idx]
    n, n0, ones = (int(v) for v in c["shape"])
    if ones != 0 or n0 > 3:
        pytest.skip("outside the kernel's shapes (generic plugin path)")
    info, xhat = run(c["rx"], c["rx_len"], n, n0, float(c["pd"][0]), c["frozen"], c["fval"])
    assert np.array_equal(info, c["info"])
    assert np.array_equal(xhat, c["xhat"])
