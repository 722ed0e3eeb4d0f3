"""Leaf export on the GPU (pcub_sc_leaf_bin / pcub_sc_leaf_deletion): decisions identical
to the decoder's, and every leaf's xy marginal -- the LLR the north star compares
within 1e-6 relative, here bit-exact -- against the reference's golden marginals and
the oracle's.  Per-codeword frozen values (the genie's per-trial randomness) too."""
import numpy as np
import pytest
import torch

from oracle import orc
from oracle import trellis_oracle as tro
from tests.conftest import edge_cases, load_golden

pytestmark = pytest.mark.gpu

BIN_SETS = ["bsc_n64", "awgn_n1024", "awgn_n4096", "awgn_n256_lowsnr"]


@pytest.fixture(scope="module")
def sc():
    from polarcub_amd import _lib, sc as m
    _lib.lib()
    return m


def _xy(g):
    return g["xy"] if "xy" in g else g["table"][g["y"]]


def _llr(m):
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.log(m[..., 0]) - np.log(m[..., 1])


@pytest.mark.parametrize("name", BIN_SETS)
def test_leaves_match_reference(sc, name):
    g = load_golden(name)
    xy = _xy(g)
    N = xy.shape[1]
    code = sc.CodeSpec(N, g["frozen"], g["fval"], device="cuda")
    info, xhat, m = sc.LeafDecoder(code).decode(torch.from_numpy(xy).cuda())
    info, xhat, m = info.cpu().numpy(), xhat.cpu().numpy(), m.cpu().numpy()
    assert np.array_equal(info, g["info"]) and np.array_equal(xhat, g["xhat"])
    infopos = g["frozen"] == 0
    assert np.array_equal(m[:, infopos], g["leaf_m"][:, infopos])
    _, _, lm = orc.decode_bin(xy, g["frozen"], g["fval"], leaf=True)
    assert np.array_equal(m, lm)
    # the north-star LLR tolerance (bit-exact marginals give identical LLRs)
    a, b = _llr(m), _llr(lm)
    fin = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), fin)
    assert np.all(np.abs(a[fin] - b[fin]) <= 1e-6 * np.maximum(1.0, np.abs(b[fin])))


@pytest.mark.parametrize("idx", range(0, 24, 3))
def test_leaves_edge_cases(sc, idx):
    c = edge_cases()[idx]
    N = c["xy"].shape[1]
    code = sc.CodeSpec(N, c["frozen"], c["fval"], device="cuda")
    info, xhat, m = sc.LeafDecoder(code).decode(torch.from_numpy(c["xy"]).cuda())
    assert np.array_equal(info.cpu().numpy(), c["info"]) and np.array_equal(xhat.cpu().numpy(), c["xhat"])
    _, _, lm = orc.decode_bin(c["xy"], c["frozen"], c["fval"], leaf=True)
    assert np.array_equal(m.cpu().numpy(), lm)


def test_genie_per_codeword_frozen_values(sc):
    """All positions frozen, a different frozen-value vector per codeword (genie decode)."""
    g = load_golden("awgn_n1024")
    xy = g["xy"][:24]
    B, N, _ = xy.shape
    rng = np.random.default_rng(8)
    fv = (rng.random((B, N)) < 0.5).astype(np.uint8)
    code = sc.CodeSpec(N, np.ones(N, np.uint8), np.zeros(N, np.uint8), device="cuda")
    info, xhat, m = sc.LeafDecoder(code).decode(torch.from_numpy(xy).cuda(), torch.from_numpy(fv).cuda())
    m = m.cpu().numpy()
    for b in range(B):
        _, xr, lm = orc.decode_bin(xy[b:b + 1], np.ones(N, np.uint8), fv[b], leaf=True)
        assert np.array_equal(m[b], lm[0])
        assert np.array_equal(xhat.cpu().numpy()[b], xr[0])


def test_deletion_leaves_match_reference(sc):
    g = load_golden("deletion_n8")
    mt = g["meta"]
    n, n0, pd = mt["n"], mt["n0"], mt["pd"]
    code = sc.CodeSpec(1 << n, g["frozen"], g["fval"], device="cuda")
    d = sc.DeletionDecoder(code, n0, pd)
    info, xhat, m = d.decode_leaves(torch.from_numpy(g["rx"]).cuda(), torch.from_numpy(g["rx_len"]).cuda())
    info, xhat, m = info.cpu().numpy(), xhat.cpu().numpy(), m.cpu().numpy()
    assert np.array_equal(info, g["info"]) and np.array_equal(xhat, g["xhat"])
    infopos = g["frozen"] == 0
    assert np.array_equal(m[:, infopos], g["leaf_m"][:, infopos])
    for t in range(0, g["rx"].shape[0], 7):
        lm = []
        tro.decode_deletion(list(map(int, g["rx"][t, :g["rx_len"][t]])), n, n0, pd, g["frozen"], g["fval"],
                            leaf_m=lm)
        assert np.array_equal(m[t], np.array(lm))


def test_deletion_genie_per_codeword(sc):
    g = load_golden("deletion_n8")
    mt = g["meta"]
    n, n0, pd = mt["n"], mt["n0"], mt["pd"]
    N = 1 << n
    B = 12
    rng = np.random.default_rng(9)
    fv = (rng.random((B, N)) < 0.5).astype(np.uint8)
    code = sc.CodeSpec(N, np.ones(N, np.uint8), np.zeros(N, np.uint8), device="cuda")
    d = sc.DeletionDecoder(code, n0, pd)
    _, xhat, m = d.decode_leaves(torch.from_numpy(g["rx"][:B]).cuda(), torch.from_numpy(g["rx_len"][:B]).cuda(),
                                 torch.from_numpy(fv).cuda())
    m = m.cpu().numpy()
    for t in range(B):
        lm = []
        x, _ = tro.decode_deletion(list(map(int, g["rx"][t, :g["rx_len"][t]])), n, n0, pd, np.ones(N, np.uint8),
                                   fv[t], leaf_m=lm)
        assert np.array_equal(m[t], np.array(lm))
        assert list(xhat.cpu().numpy()[t]) == x
