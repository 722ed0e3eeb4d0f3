"""Device-side channel simulation for Monte-Carlo runs (synthetic inputs).

BI-AWGN with BPSK 0 -> +1, 1 -> -1.  The joint probabilities handed to the
decoder are P(x, y) = 1/2 * (2 pi sigma^2)^-1/2 * exp(-(y - s_x)^2 / (2 sigma^2)),
the quantity the reference's memoryless vector distributions hold
(probs[i][x] = P(X=x, Y=y_i), VectorDistributions/BinaryMemorylessVectorDistribution.py:10-13).
The reference ships no AWGN factory (ScalarDistributions/QaryMemorylessDistribution.py:800-804
is a stub), so this module defines it.
"""
import math

import torch


def bits_from_words(words, N):
    """[W, B] int32 packed -> [N, B] uint8 (bit i of codeword b)."""
    idx = torch.arange(N, device=words.device)
    w = words.index_select(0, idx >> 5)
    return ((w >> (idx & 31).to(torch.int32).unsqueeze(1)) & 1).to(torch.uint8)


def awgn_pairs_native(x_nb, sigma2, generator=None, out=None):
    """x_nb: [N, B] 0/1 codeword bits -> [N, B, 2] float64 joint probabilities."""
    N, B = x_nb.shape
    s = 1.0 - 2.0 * x_nb.to(torch.float64)
    noise = torch.randn((N, B), dtype=torch.float64, device=x_nb.device, generator=generator)
    y = s + math.sqrt(sigma2) * noise
    c = 0.5 / math.sqrt(2.0 * math.pi * sigma2)
    if out is None:
        out = torch.empty((N, B, 2), dtype=torch.float64, device=x_nb.device)
    out[:, :, 0] = c * torch.exp(-((y - 1.0) ** 2) / (2.0 * sigma2))
    out[:, :, 1] = c * torch.exp(-((y + 1.0) ** 2) / (2.0 * sigma2))
    return out
