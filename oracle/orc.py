"""ctypes front-end for the CPU parity oracle (oracle/sc_oracle.c, oracle/trellis_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product package (polarcub_amd) never imports
this module.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liborc.so")

_lib = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_f64p = ctypes.POINTER(ctypes.c_double)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_sc_decode_bin.restype = ctypes.c_int
        L.orc_sc_decode_bin.argtypes = [ctypes.c_int, _f64p, _f64p, _u8p, _f64p, _u8p, _u8p, _u8p, _f64p]
        L.orc_sc_decode_bin_batch.restype = None
        L.orc_sc_decode_bin_batch.argtypes = [ctypes.c_int, ctypes.c_int64, _f64p, _u8p, _u8p, ctypes.c_int,
                                              _u8p, _u8p, _f64p]
        L.orc_encode_bin.restype = None
        L.orc_encode_bin.argtypes = [ctypes.c_int, _f64p, _u8p, _f64p, _u8p, _u8p, _u8p]
        L.orc_polar_transform_bits.restype = None
        L.orc_polar_transform_bits.argtypes = [ctypes.c_int, _u8p, _u8p]
        L.orc_sc_decode_qary.restype = ctypes.c_int
        L.orc_sc_decode_qary.argtypes = [ctypes.c_int, ctypes.c_int, _f64p, _u8p, _u8p, _u8p, _f64p]
        L.orc_sc_decode_qary_batch.restype = None
        L.orc_sc_decode_qary_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, _f64p, _u8p,
                                               ctypes.c_int, _u8p, _u8p]
        L.orc_encode_qary.restype = None
        L.orc_encode_qary.argtypes = [ctypes.c_int, ctypes.c_int, _u8p, _u8p, _u8p]
        L.orc_decode_deletion_batch.restype = ctypes.c_int
        L.orc_decode_deletion_batch.argtypes = [_u8p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int64, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_double, _u8p, _u8p, ctypes.c_int,
                                                ctypes.c_int, _u8p, _u8p]
        _lib = L
    return _lib


def _p(a, t):
    if a is None:
        return None
    return a.ctypes.data_as(t)


def _log2(N):
    n = int(N).bit_length() - 1
    assert (1 << n) == N, "N must be a power of two"
    return n


def decode_bin(xy, frozen, fval, leaf=False):
    """Batch decode with a uniform prior. xy: [B,N,2] f64.  Returns (info [B,K], xhat [B,N][, leaf_m])."""
    xy = np.ascontiguousarray(xy, np.float64)
    B, N, _ = xy.shape
    frozen = np.ascontiguousarray(frozen, np.uint8)
    fval = np.ascontiguousarray(fval, np.uint8)
    K = int(N - frozen.sum())
    info = np.zeros((B, K), np.uint8)
    xhat = np.zeros((B, N), np.uint8)
    lm = np.zeros((B, N, 2)) if leaf else None
    lib().orc_sc_decode_bin_batch(_log2(N), B, _p(xy, _f64p), _p(frozen, _u8p), _p(fval, _u8p), K,
                                  _p(info, _u8p), _p(xhat, _u8p), _p(lm, _f64p))
    return (info, xhat, lm) if leaf else (info, xhat)


def decode_bin_general(xy, frozen, r, prior=None):
    """One codeword with the full two-tree recursion (a-priori x-tree + xy-tree)."""
    xy = np.ascontiguousarray(xy, np.float64)
    N = xy.shape[0]
    frozen = np.ascontiguousarray(frozen, np.uint8)
    r = np.ascontiguousarray(r, np.float64)
    K = int(N - frozen.sum())
    pr = None
    if prior is not None:
        pr = np.ascontiguousarray(np.broadcast_to(prior, (N, 2)), np.float64)
    info = np.zeros(K, np.uint8)
    xhat = np.zeros(N, np.uint8)
    lm = np.zeros((N, 2))
    lib().orc_sc_decode_bin(_log2(N), _p(xy, _f64p), _p(pr, _f64p), _p(frozen, _u8p), _p(r, _f64p), None,
                            _p(info, _u8p), _p(xhat, _u8p), _p(lm, _f64p))
    return info, xhat, lm


def encode_bin(info, frozen, r=None, fval=None, prior=None):
    info = np.ascontiguousarray(info, np.uint8)
    frozen = np.ascontiguousarray(frozen, np.uint8)
    N = frozen.shape[0]
    x = np.zeros(N, np.uint8)
    pr = None
    if prior is not None:
        pr = np.ascontiguousarray(np.broadcast_to(prior, (N, 2)), np.float64)
    rr = None if r is None else np.ascontiguousarray(r, np.float64)
    fv = None if fval is None else np.ascontiguousarray(fval, np.uint8)
    lib().orc_encode_bin(_log2(N), _p(pr, _f64p), _p(frozen, _u8p), _p(rr, _f64p), _p(fv, _u8p),
                         _p(info, _u8p), _p(x, _u8p))
    return x


def polar_transform_bits(x):
    x = np.ascontiguousarray(x, np.uint8)
    u = np.zeros_like(x)
    lib().orc_polar_transform_bits(_log2(x.shape[0]), _p(x, _u8p), _p(u, _u8p))
    return u


def decode_qary(q, xy, frozen):
    xy = np.ascontiguousarray(xy, np.float64)
    B, N, qq = xy.shape
    assert qq == q
    frozen = np.ascontiguousarray(frozen, np.uint8)
    K = int(N - frozen.sum())
    info = np.zeros((B, K), np.uint8)
    xhat = np.zeros((B, N), np.uint8)
    lib().orc_sc_decode_qary_batch(q, _log2(N), B, _p(xy, _f64p), _p(frozen, _u8p), K, _p(info, _u8p),
                                   _p(xhat, _u8p))
    return info, xhat


def encode_qary(q, info, frozen):
    info = np.ascontiguousarray(info, np.uint8)
    frozen = np.ascontiguousarray(frozen, np.uint8)
    x = np.zeros(frozen.shape[0], np.uint8)
    lib().orc_encode_qary(q, _log2(frozen.shape[0]), _p(frozen, _u8p), _p(info, _u8p), _p(x, _u8p))
    return x


def decode_deletion(rx, rx_len, n, n0, pd, frozen, fval, ones=0):
    """Deletion-channel SC decode of received words (oracle/trellis_oracle.c, the C restatement of
    oracle/trellis_oracle.py).  rx: [B, W] u8 padded words, rx_len: [B].  Returns (info [B, K],
    xhat [B, N])."""
    rx = np.ascontiguousarray(rx, np.uint8)
    ln = np.ascontiguousarray(rx_len, np.int32)
    B, W = rx.shape
    frozen = np.ascontiguousarray(frozen, np.uint8)
    fval = np.ascontiguousarray(fval, np.uint8)
    N = 1 << n
    K = int(N - frozen.sum())
    info = np.zeros((B, max(K, 1)), np.uint8)
    xhat = np.zeros((B, N), np.uint8)
    rc = lib().orc_decode_deletion_batch(_p(rx, _u8p), ln.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), B, W, n,
                                         n0, float(pd), _p(frozen, _u8p), _p(fval, _u8p), int(ones), K,
                                         _p(xhat, _u8p), _p(info, _u8p))
    assert rc == 0, "orc_decode_deletion_batch failed"
    return info[:, :K], xhat
