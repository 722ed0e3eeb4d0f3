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


def guard_band_positions(n, n0, xi, ones=0):
    """Positions of the N codeword bits inside the guard-banded word of
    Guardbands.addDeletionGuardBands (Guardbands.py:4-44), and its length."""
    from .deletion import addDeletionGuardBands
    N = 1 << n
    marked = addDeletionGuardBands([i + 2 for i in range(N)], n, n0, xi, ones)
    pos = [j for j, v in enumerate(marked) if v >= 2]
    assert len(pos) == N
    return pos, len(marked), [j for j, v in enumerate(marked) if v == 1]


def deletion_words(x_bn, n, n0, xi, pd, generator=None, ones=0):
    """x_bn: [B, N] 0/1 codewords (device) -> guard bands added (with `ones` ones at both
    ends of every guard band), every symbol deleted independently with probability pd
    (BinaryTrellis.deletionChannelSimulation's law, drawn with torch's Philox instead of
    MT19937), survivors packed to the left.
    Returns (rx [B, W] uint8, rx_len [B] int32), W = guard-banded length."""
    B, N = x_bn.shape
    pos, W, ones_pos = guard_band_positions(n, n0, xi, ones)
    dev = x_bn.device
    cw = torch.zeros((B, W), dtype=torch.uint8, device=dev)
    cw[:, torch.tensor(pos, device=dev)] = x_bn.to(torch.uint8)
    if ones_pos:
        cw[:, torch.tensor(ones_pos, device=dev)] = 1
    keep = torch.rand((B, W), device=dev, generator=generator) >= pd
    dest = torch.cumsum(keep, dim=1, dtype=torch.int32) - 1
    dest = torch.where(keep, dest, torch.full_like(dest, W))  # deleted symbols go to a trash column
    rx = torch.zeros((B, W + 1), dtype=torch.uint8, device=dev)
    rx.scatter_(1, dest.to(torch.int64), cw)
    return rx[:, :W].contiguous(), keep.sum(dim=1, dtype=torch.int32)


def qsc_pairs_native(x_nb, q, p, generator=None):
    """x_nb: [N, B] symbols in [0, q) -> q-ary symmetric channel output y and the joint table
    rows probs[y][x] (1-p if x == y else p/(q-1), ScalarDistributions/QaryMemorylessDistribution.py:780-784)
    as [N, B, q] float64."""
    N, B = x_nb.shape
    dev = x_nb.device
    err = torch.rand((N, B), device=dev, generator=generator, dtype=torch.float64) < p
    shift = torch.randint(1, q, (N, B), device=dev, generator=generator)
    y = torch.where(err, (x_nb.to(torch.int64) + shift) % q, x_nb.to(torch.int64))
    hit = y.unsqueeze(-1) == torch.arange(q, device=dev)
    return torch.where(hit, torch.tensor(1.0 - p, dtype=torch.float64, device=dev),
                       torch.tensor(p / (q - 1), dtype=torch.float64, device=dev))
