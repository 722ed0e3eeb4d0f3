"""Code construction (host side, one-time per code).

* The reference's Tal-Vardy degrading/upgrading construction
  (ScalarDistributions/BinaryMemorylessDistribution.py:287-427, :624-680, with the
  LinkedListHeap of ScalarDistributions/UpgradingDegrading/LinkedListHeap.py) runs in
  the native host library libpolarcub_construct.so (csrc/host/tv_construct.cpp, C ABI
  include/polarcub_construct.h), bit-identical to the reference, with the 2^m
  channels of each tree level on a thread pool: merge_equivalent / degrade /
  upgrade / tv_pe here, calcFrozenSet_degradingUpgrading in polarcub_amd.scalar.
* The q-ary degrading/upgrading construction (ScalarDistributions/QaryMemorylessDistribution.py:
  98-153, 218-260, 329-475, 934-991) in the same library (csrc/host/qary_construct.cpp):
  qmd_degrade / qmd_upgrade / qary_tv_pe here; the reference-named classes and
  calcFrozenSet_degradingUpgrading with its .npy cache in polarcub_amd.scalar_qary.
* bhattacharyya_frozen: the standard Bhattacharyya-parameter recursion for BI-AWGN
  in the reference's index convention (minus child = first half of the u range,
  BinaryPolarEncoderDecoder.py:289-317), used for the benchmark's code.
"""
import ctypes
import math
import os
import sys

import numpy as np

_HOST = None

# return codes of include/polarcub_construct.h -> the reference's exceptions
_ERRORS = {-1: ValueError, -10: AssertionError, -11: ZeroDivisionError, -12: IndexError, -13: AttributeError}


def host_lib():
    """libpolarcub_construct.so (built by polarcub_amd.build / __graft_entry__.build)."""
    global _HOST
    if _HOST is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libpolarcub_construct.so")
        if not os.path.exists(path):
            raise RuntimeError("libpolarcub_construct.so not built: run `python -m polarcub_amd.build`")
        lib = ctypes.CDLL(path)
        P, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        lib.pcub_bmd_merge_equivalent.argtypes = [P, I64, P, P, P]
        lib.pcub_bmd_degrade.argtypes = [P, I64, I64, P, P, P]
        lib.pcub_bmd_upgrade.argtypes = [P, I64, I64, P, P]
        lib.pcub_bin_construct.argtypes = [I32, I64, P, I64, P, I64, P, P, I32]
        lib.pcub_qmd_degrade.argtypes = [I32, P, I64, I64, P, I64, P]
        lib.pcub_qmd_upgrade.argtypes = [I32, P, I64, I64, P, I64, P]
        lib.pcub_qmd_error_prob.argtypes = [I32, P, I64, P, P]
        lib.pcub_qary_construct.argtypes = [I32, I32, I64, P, I64, P, I64, P, P, I32]
        for f in (lib.pcub_bmd_merge_equivalent, lib.pcub_bmd_degrade, lib.pcub_bmd_upgrade, lib.pcub_bin_construct,
                  lib.pcub_qmd_degrade, lib.pcub_qmd_upgrade, lib.pcub_qmd_error_prob, lib.pcub_qary_construct):
            f.restype = ctypes.c_int
        _HOST = lib
    return _HOST


def _check(rc, what):
    if rc != 0:
        raise _ERRORS.get(rc, RuntimeError)("%s failed (code %d)" % (what, rc))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _letters(probs):
    a = np.ascontiguousarray(np.asarray(probs, dtype=np.float64).reshape(-1, 2))
    return a


def merge_equivalent(probs):
    """mergeEquivalentSymbols on rows [p(y,0), p(y,1)] -> (merged rows, group) where
    group[i] is the merged letter of input letter i (-1: zero probability, dropped)."""
    a = _letters(probs)
    out = np.empty_like(a)
    grp = np.empty(len(a), np.int64)
    n = ctypes.c_int64(0)
    _check(host_lib().pcub_bmd_merge_equivalent(_ptr(a), len(a), _ptr(out), ctypes.byref(n), _ptr(grp)),
           "mergeEquivalentSymbols")
    return out[:n.value], grp


def degrade(merged, L):
    """degrade(L) of already-merged letters -> (letters, group of each merged letter)."""
    a = _letters(merged)
    out = np.empty_like(a)
    grp = np.empty(len(a), np.int64)
    n = ctypes.c_int64(0)
    _check(host_lib().pcub_bmd_degrade(_ptr(a), len(a), int(L), _ptr(out), ctypes.byref(n), _ptr(grp)), "degrade")
    return out[:n.value], grp


def upgrade(merged, L):
    """upgrade(L) of already-merged letters."""
    a = _letters(merged)
    out = np.empty_like(a)
    n = ctypes.c_int64(0)
    _check(host_lib().pcub_bmd_upgrade(_ptr(a), len(a), int(L), _ptr(out), ctypes.byref(n)), "upgrade")
    return out[:n.value]


def tv_pe(n, L, xprobs, xyprobs, threads=0):
    """(TV, Pe) vectors of calcFrozenSet_degradingUpgrading: Pe of the degraded xy
    channels, TV (total variation distance) of the upgraded x channels or zeros."""
    xy = _letters(xyprobs)
    x = None if xprobs is None else _letters(xprobs)
    N = 1 << n
    TV = np.empty(N)
    Pe = np.empty(N)
    _check(host_lib().pcub_bin_construct(int(n), int(L), _ptr(x), 0 if x is None else len(x), _ptr(xy), len(xy),
                                         _ptr(TV), _ptr(Pe), int(threads)), "calcFrozenSet_degradingUpgrading")
    return TV, Pe


def _qrows(q, probs):
    a = np.ascontiguousarray(np.asarray(probs, dtype=np.float64).reshape(-1, int(q)))
    return a


def calc_m(q, L):
    """calcMFromL (ScalarDistributions/QaryMemorylessDistribution.py:753-755)."""
    return math.floor(L ** (1.0 / (q - 1)) + sys.float_info.epsilon)


def _qmd(fn, what, q, probs, L):
    a = _qrows(q, probs)
    cap = max(1, calc_m(q, L)) ** (q - 1)
    out = np.empty((cap, q))
    n = ctypes.c_int64(0)
    _check(fn(int(q), _ptr(a), len(a), int(L), _ptr(out), cap, ctypes.byref(n)), what)
    return out[:n.value].copy()


def qmd_degrade(q, probs, L):
    """QaryMemorylessDistribution.degrade(L) (degrade_dynamic, :218-260) of rows [n][q]."""
    return _qmd(host_lib().pcub_qmd_degrade, "degrade", q, probs, L)


def qmd_upgrade(q, probs, L):
    """QaryMemorylessDistribution.upgrade(L) (upgrade_dynamic, :329-475) of rows [n][q]."""
    return _qmd(host_lib().pcub_qmd_upgrade, "upgrade", q, probs, L)


def qmd_error_prob_tv(q, probs):
    """(errorProb, totalVariation) of rows [n][q] (:53-61, :87-96)."""
    a = _qrows(q, probs)
    pe, tv = ctypes.c_double(0.0), ctypes.c_double(0.0)
    _check(host_lib().pcub_qmd_error_prob(int(q), _ptr(a), len(a), ctypes.byref(pe), ctypes.byref(tv)), "errorProb")
    return pe.value, tv.value


def qary_tv_pe(q, n, L, xprobs, xyprobs, threads=0):
    """(TV, Pe) of calcTVAndPe_degradingUpgrading (:934-991): Pe of the degraded xy tree, TV of
    the upgraded x tree (zeros when xprobs is None), leaves in u order."""
    xy = _qrows(q, xyprobs)
    x = None if xprobs is None else _qrows(q, xprobs)
    N = 1 << n
    TV = np.empty(N)
    Pe = np.empty(N)
    _check(host_lib().pcub_qary_construct(int(q), int(n), int(L), _ptr(x), 0 if x is None else len(x), _ptr(xy),
                                          len(xy), _ptr(TV), _ptr(Pe), int(threads)), "calcTVAndPe_degradingUpgrading")
    return TV, Pe


def awgn_sigma2(ebn0_db, rate):
    """Noise variance for BPSK at the given Eb/N0 (dB) and code rate."""
    return 1.0 / (2.0 * rate * 10.0 ** (ebn0_db / 10.0))


def bhattacharyya_z(n, sigma2):
    """Bhattacharyya parameters of the 2^n synthetic channels, u order."""
    z = np.array([math.exp(-1.0 / (2.0 * sigma2))])
    for _ in range(n):
        nz = np.empty(2 * len(z))
        nz[0::2] = 2 * z - z * z
        nz[1::2] = z * z
        z = nz
    return z


def bhattacharyya_frozen(n, K, sigma2):
    """Frozen mask (uint8[N], 1 = frozen) keeping the K most reliable indices."""
    z = bhattacharyya_z(n, sigma2)
    order = sorted(range(len(z)), key=lambda i: (z[i], i))
    mask = np.ones(len(z), np.uint8)
    mask[order[:K]] = 0
    return mask
