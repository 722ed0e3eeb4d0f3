"""Two-tree SC on the GPU (pcub_sc_prior_bin): a non-uniform a-priori distribution, the prior
tree beside the xy tree, frozen bits drawn against the common randomness
(BinaryPolarEncoderDecoder.py:223-325, :258-262).  Bit-exact against the reference's own
two-tree runs (prior_n64.npz) and against the oracle's general recursion on random cases:
skewed and per-position priors, priors with exact zeros, a per-codeword prior, ragged
batches, short codes, encode mode, leaf marginals."""
import numpy as np
import pytest
import torch

from oracle import orc
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sc():
    from polarcub_amd import _lib, sc as m
    _lib.lib()
    return m


def _code(sc, frozen):
    return sc.CodeSpec(len(frozen), frozen, None, device="cuda")


def test_prior_golden_through_the_facade():
    from polarcub_amd import coding, vectors
    g = load_golden("prior_n64")
    fs = set(int(i) for i in np.nonzero(g["frozen"])[0])
    enc = coding.BinaryPolarEncoderDecoder(64, fs, 11)
    assert np.array_equal(enc.randomlyGeneratedNumbers, g["r"])
    xvd = vectors.BinaryMemorylessVectorDistribution(64)
    xvd.probs[:] = np.tile(g["prior"], (64, 1))
    for b in range(g["xy"].shape[0]):
        xy = vectors.BinaryMemorylessVectorDistribution(64)
        xy.probs[:] = g["xy"][b]
        x, info = enc.decode(xvd, xy)
        assert np.array_equal(info, g["info"][b]) and np.array_equal(x, g["xhat"][b])
    for b in range(g["enc_info"].shape[0]):
        assert np.array_equal(enc.encode(xvd, list(g["enc_info"][b])), g["enc_x"][b])
    # the batched entry points agree with the per-word ones
    xb, ib = enc.decode_prior_batch(g["prior"][None, :].repeat(64, 0), g["xy"])
    assert np.array_equal(ib, g["info"]) and np.array_equal(xb, g["xhat"])
    assert np.array_equal(enc.encode_prior_batch(np.tile(g["prior"], (64, 1)), g["enc_info"]), g["enc_x"])


def test_prior_golden_leaf_marginals(sc):
    g = load_golden("prior_n64")
    pc = sc.PriorCoder(_code(sc, g["frozen"]), g["r"])
    info, xhat, m = pc.decode(torch.from_numpy(np.tile(g["prior"], (64, 1))).cuda(),
                              torch.from_numpy(g["xy"]).cuda(), want_marginals=True)
    m = m.cpu().numpy()
    ip = g["frozen"] == 0
    assert np.array_equal(m[:, ip], g["leaf_m"][:, ip])
    for b in range(0, g["xy"].shape[0], 7):
        _, _, lm = orc.decode_bin_general(g["xy"][b], g["frozen"], g["r"], prior=g["prior"])
        assert np.array_equal(m[b], lm)


def _random_case(rng, n, B, kind):
    N = 1 << n
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    r = rng.random(N)
    if kind == "iid":
        prior = np.tile([0.8, 0.2], (N, 1))
    elif kind == "positional":
        a = rng.random(N)
        prior = np.stack([a, 1.0 - a], 1)
    else:  # exact zeros and unnormalised rows
        prior = rng.random((N, 2)) * 3.0
        z = rng.random(N) < 0.2
        prior[z, rng.integers(0, 2, int(z.sum()))] = 0.0
    xy = rng.random((B, N, 2))
    xy[rng.random((B, N)) < 0.05, 0] = 0.0
    return frozen, r, prior, xy


@pytest.mark.parametrize("n,B,kind", [(1, 5, "iid"), (2, 33, "zeros"), (4, 64, "positional"), (6, 257, "zeros"),
                                      (8, 100, "iid"), (10, 17, "positional")])
def test_prior_decode_vs_oracle(sc, n, B, kind):
    rng = np.random.default_rng(1000 * n + B)
    frozen, r, prior, xy = _random_case(rng, n, B, kind)
    pc = sc.PriorCoder(_code(sc, frozen), r)
    info, xhat = pc.decode(torch.from_numpy(prior).cuda(), torch.from_numpy(xy).cuda())
    info, xhat = info.cpu().numpy(), xhat.cpu().numpy()
    for b in range(B):
        i2, x2, _ = orc.decode_bin_general(xy[b], frozen, r, prior=prior)
        assert np.array_equal(info[b], i2), b
        assert np.array_equal(xhat[b], x2), b


@pytest.mark.parametrize("n,B", [(1, 3), (3, 40), (7, 129), (9, 20)])
def test_prior_encode_vs_oracle(sc, n, B):
    rng = np.random.default_rng(7 * n + B)
    frozen, r, prior, _ = _random_case(rng, n, 1, "positional")
    code = _code(sc, frozen)
    info = rng.integers(0, 2, (B, code.K)).astype(np.uint8)
    x = sc.PriorCoder(code, r).encode(torch.from_numpy(prior).cuda(), torch.from_numpy(info).cuda()).cpu().numpy()
    for b in range(B):
        assert np.array_equal(x[b], orc.encode_bin(info[b], frozen, r=r, prior=prior)), b


def test_prior_per_codeword(sc):
    rng = np.random.default_rng(5)
    n, B = 5, 24
    frozen, r, _, xy = _random_case(rng, n, B, "iid")
    a = rng.random((B, 1 << n))
    priors = np.stack([a, 1.0 - a], 2)  # [B, N, 2]
    pc = sc.PriorCoder(_code(sc, frozen), r)
    px = torch.from_numpy(priors).cuda().transpose(0, 1).contiguous()  # [N, B, 2]
    info, xhat = pc.decode(px, torch.from_numpy(xy).cuda())
    info, xhat = info.cpu().numpy(), xhat.cpu().numpy()
    for b in range(B):
        i2, x2, _ = orc.decode_bin_general(xy[b], frozen, r, prior=priors[b])
        assert np.array_equal(info[b], i2) and np.array_equal(xhat[b], x2), b


def test_prior_mc_driver_matches_reference_line(capsys):
    """encodeDecodeSimulation under a non-uniform prior: GPU encode + decode batches give the
    same printed line as the generic recursion."""
    from polarcub_amd import coding, vectors
    N, frozen = 32, set(range(0, 32, 2)) | {1, 3}
    prior = [0.75, 0.25]

    def make_x():
        v = vectors.BinaryMemorylessVectorDistribution(N)
        v.probs[:] = np.tile(prior, (N, 1))
        return v

    rng = np.random.default_rng(3)

    def channel(c):
        return [int(b) ^ int(rng.random() < 0.1) for b in c]

    def make_xy(y):
        v = vectors.BinaryMemorylessVectorDistribution(N)
        for i, yi in enumerate(y):
            v.probs[i] = [prior[0] * (0.9 if yi == 0 else 0.1), prior[1] * (0.1 if yi == 0 else 0.9)]
        return v

    coding.encodeDecodeSimulation(N, make_x, lambda x: x, channel, make_xy, 300, frozen, 5, 9)
    gpu_line = capsys.readouterr().out.strip().splitlines()[-1]
    # the same run through the generic recursion (the reference's algorithm, restated)
    rng = np.random.default_rng(3)
    import random
    enc = coding.BinaryPolarEncoderDecoder(N, frozen, 5)
    rr = random.Random()
    rr.seed(9)
    errors = 0
    for t in range(300):
        info = [0 if rr.random() < 0.5 else 1 for _ in range(enc.k)]
        x, _, _ = enc.recursiveEncodeDecode(list(info), 0, 0, enc.randomlyGeneratedNumbers, make_x())
        dec = np.full(enc.k, -1, np.int64)
        enc.recursiveEncodeDecode(dec, 0, 0, enc.randomlyGeneratedNumbers, make_x(), make_xy(channel(x)))
        errors += int(np.any(dec != np.asarray(info)))
    assert gpu_line.split() == ["Error", "probability", "=", str(errors), "/", "300", "=", str(errors / 300)]
