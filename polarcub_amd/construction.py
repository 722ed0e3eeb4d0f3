"""Code construction helpers (host side, one-time per code).

bhattacharyya_frozen follows the standard Bhattacharyya-parameter recursion for
BI-AWGN in the reference's index convention (minus child = first half of the
u range, BinaryPolarEncoderDecoder.py:289-317).  The reference's own
degrading/upgrading construction (ScalarDistributions/BinaryMemorylessDistribution.py:624-680)
is a separate, later component; frozen sets it produced are accepted as plain
index sets everywhere.
"""
import math

import numpy as np


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
