"""The reference-compatible facade on the GPU: decode()/encode() and the
Monte-Carlo driver must reproduce the reference's outputs and printed line."""
import contextlib
import io
import random

import numpy as np
import pytest

from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


def test_facade_decode_matches_reference():
    from polarcub_amd import coding, scalar, vectors
    for name in ("bsc_n64", "awgn_n1024"):
        g = load_golden(name)
        N = g["frozen"].shape[0]
        xy = g["xy"] if "xy" in g else g["table"][g["y"]]
        fs = set(int(i) for i in np.nonzero(g["frozen"])[0])
        enc = coding.BinaryPolarEncoderDecoder(N, fs, g["meta"]["crs"])
        xvd = vectors.BinaryMemorylessVectorDistribution(N)
        xvd.probs[:] = 0.5
        for b in range(0, xy.shape[0], max(1, xy.shape[0] // 16)):
            yvd = vectors.BinaryMemorylessVectorDistribution(N)
            yvd.probs[:] = xy[b]
            x, info = enc.decode(xvd, yvd)
            assert x.dtype == np.int64 and info.dtype == np.int64
            assert np.array_equal(info, g["info"][b])
            assert np.array_equal(x, g["xhat"][b])
        X, I = enc.decode_batch(xy)
        assert np.array_equal(I, g["info"]) and np.array_equal(X, g["xhat"])


def test_facade_encode_matches_reference():
    from polarcub_amd import coding, vectors
    g = load_golden("encode_binary")
    for n in (3, 8, 10):
        N = 1 << n
        fs = set(int(i) for i in np.nonzero(g["n%d_frozen" % n])[0])
        # frozen values come from r_i; rebuild them through the seed-free path by checking equality
        enc = coding.BinaryPolarEncoderDecoder(N, fs, 0)
        enc.randomlyGeneratedNumbers = g["n%d_r" % n]
        xvd = vectors.BinaryMemorylessVectorDistribution(N)
        xvd.probs[:] = 0.5
        for b in range(g["n%d_info" % n].shape[0]):
            assert np.array_equal(enc.encode(xvd, list(g["n%d_info" % n][b])), g["n%d_x" % n][b])


def test_encode_decode_simulation_prints_reference_line():
    from polarcub_amd import coding, scalar
    g = load_golden("harness_bsc_n64")
    m = g["meta"]
    N = m["N"]
    fs = set(int(i) for i in np.nonzero(g["frozen"])[0])
    xy_dist = scalar.makeBSC(m["p"])

    def make_x():
        xd = scalar.BinaryMemorylessDistribution()
        xd.probs.append([xy_dist.calcXMarginal(0), xy_dist.calcXMarginal(1)])
        return xd.makeBinaryMemorylessVectorDistribution(N, None)

    def channel(codeword):
        out = []
        for x in codeword:
            rnd = random.random()
            s = 0.0
            for y in range(len(xy_dist.probs)):
                if s + xy_dist.probXGivenY(x, y) >= rnd:
                    out.append(y)
                    break
                s += xy_dist.probXGivenY(x, y)
        return out

    def make_xy(received):
        return xy_dist.makeBinaryMemorylessVectorDistribution(len(received), received)

    random.seed(m["global_seed"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        coding.encodeDecodeSimulation(N, make_x, lambda e: e, channel, make_xy, m["trials"], fs)
    assert buf.getvalue().strip().splitlines()[-1] == m["line"]


def test_encode_decode_simulation_verbose_printout():
    """verbosity=1 error printout (BinaryPolarEncoderDecoder.py:374-385) line for line."""
    from polarcub_amd import coding, scalar
    g = load_golden("harness_verbose")
    m = g["meta"]
    N = m["N"]
    fs = set(int(i) for i in np.nonzero(g["frozen"])[0])
    xy_dist = scalar.makeBSC(m["p"])

    def make_x():
        xd = scalar.BinaryMemorylessDistribution()
        xd.probs.append([xy_dist.calcXMarginal(0), xy_dist.calcXMarginal(1)])
        return xd.makeBinaryMemorylessVectorDistribution(N, None)

    def channel(codeword):
        out = []
        for x in codeword:
            rnd = random.random()
            s = 0.0
            for y in range(len(xy_dist.probs)):
                if s + xy_dist.probXGivenY(x, y) >= rnd:
                    out.append(y)
                    break
                s += xy_dist.probXGivenY(x, y)
        return out

    def make_xy(received):
        return xy_dist.makeBinaryMemorylessVectorDistribution(len(received), received)

    random.seed(m["global_seed"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        coding.encodeDecodeSimulation(N, make_x, lambda e: e, channel, make_xy, m["trials"], fs, verbosity=1)
    assert buf.getvalue() == m["stdout"]


@pytest.mark.parametrize("n", [15, 16])
def test_long_code_encode_matches_oracle(n):
    """Codes past the encoder's LDS tile (n > 14) take the global-scratch encoder: the
    facade's encode and the device Monte-Carlo pipeline accept them."""
    import torch

    from oracle import orc
    from polarcub_amd import coding, mc, sc, vectors
    N = 1 << n
    rng = np.random.default_rng(n)
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    fs = set(int(i) for i in np.nonzero(frozen)[0])
    enc = coding.BinaryPolarEncoderDecoder(N, fs, 3)
    xvd = vectors.BinaryMemorylessVectorDistribution(N)
    xvd.probs[:] = 0.5
    fval = np.where(0.5 >= enc.randomlyGeneratedNumbers, 0, 1).astype(np.uint8)
    infos = rng.integers(0, 2, size=(3, enc.k)).astype(np.uint8)
    for b in range(3):
        x = enc.encode(xvd, list(infos[b]))
        assert np.array_equal(x, orc.encode_bin(infos[b], frozen, fval=fval))
    X = enc.encode_batch(infos)
    for b in range(3):
        assert np.array_equal(X[b], orc.encode_bin(infos[b], frozen, fval=fval))
    code = sc.CodeSpec(N, frozen, fval, device="cuda:0")
    cnt = mc.run_bin(code, 5, 0, 96, mc.CHANNEL_BSC, 0.0, chunk=64)  # noiseless: every word decodes
    torch.cuda.synchronize()
    assert cnt[0] == 96 and cnt[1] == 0 and cnt[2] == 0


@pytest.mark.parametrize("n,B", [(4, 37), (6, 100), (10, 1000), (10, 16), (12, 77)])
def test_batch_decode_through_tiles_matches_native(n, B):
    """BinaryDecoder.decode ([B, N, 2], the reference API's layout) goes through pcub_tile_pairs and
    the tiled headline kernel: the same decisions as the untiled kernel on the transposed rows, and
    tile_pairs is the two-pass tile_rows(transpose_pairs(.)) in one pass."""
    import torch
    from polarcub_amd import construction, sc
    N, K = 1 << n, (1 << n) // 2
    s2 = construction.awgn_sigma2(2.0, 0.5)
    fr = construction.bhattacharyya_frozen(n, K, s2)
    code = sc.CodeSpec.from_frozen_set(N, set(np.nonzero(fr)[0].tolist()), 1, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(n * 1000 + B)
    xy = torch.rand((B, N, 2), dtype=torch.float64, device="cuda", generator=g)
    T = sc.bin_tile(n)
    assert torch.equal(sc.tile_pairs(xy, T), sc.tile_rows(sc.transpose_pairs(xy), T))
    dec = sc.BinaryDecoder(code)
    info, xh = dec.decode(xy)
    iw, xw, _ = dec.decode_native(sc.transpose_pairs(xy))
    assert torch.equal(info, sc.unpack(iw, K)) and torch.equal(xh, sc.unpack(xw, N))


def test_qary_batch_decode_through_tiles_matches_native():
    import torch
    from polarcub_amd import sc
    q, n, B = 4, 8, 333
    rng = np.random.default_rng(5)
    mask = (rng.random(1 << n) < 0.5).astype(np.uint8)
    code = sc.QaryCode(q, 1 << n, mask, device="cuda")
    xy = torch.as_tensor(rng.random((B, 1 << n, q)), device="cuda")
    dec = sc.QaryDecoder(code)
    info, xh = dec.decode(xy)
    i2, x2 = dec.decode_native(sc.transpose_pairs(xy))
    assert torch.equal(info, i2.t().contiguous()) and torch.equal(xh, x2.t().contiguous())
