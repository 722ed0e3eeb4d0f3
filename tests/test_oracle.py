"""The CPU oracle against the reference's own outputs (golden vectors made by
oracle/make_golden.py from the shimmed reference).  This pins the oracle before
any kernel is compared with it."""
import numpy as np
import pytest

from oracle import orc
from tests.conftest import edge_cases, edge_long_cases, load_golden

BIN_SETS = ["bsc_n64", "awgn_n1024", "awgn_n4096", "awgn_n256_lowsnr"]


def _xy(g):
    if "xy" in g:
        return g["xy"]
    return g["table"][g["y"]]


@pytest.mark.parametrize("name", BIN_SETS)
def test_binary_decode_matches_reference(name):
    g = load_golden(name)
    info, xhat, lm = orc.decode_bin(_xy(g), g["frozen"], g["fval"], leaf=True)
    assert np.array_equal(info, g["info"])
    assert np.array_equal(xhat, g["xhat"])
    infopos = g["frozen"] == 0
    # leaf marginals at information leaves are the xy marginals the reference decided on
    assert np.array_equal(lm[:, infopos], g["leaf_m"][:, infopos])


def test_binary_decode_general_two_tree_path():
    g = load_golden("bsc_n64")
    xy = _xy(g)
    for b in range(0, 1000, 97):
        info, xhat, _ = orc.decode_bin_general(xy[b], g["frozen"], g["r"], prior=np.array([0.5, 0.5]))
        assert np.array_equal(info, g["info"][b])
        assert np.array_equal(xhat, g["xhat"][b])


@pytest.mark.parametrize("idx", range(24))
def test_edge_cases(idx):
    c = edge_cases()[idx]
    info, xhat, lm = orc.decode_bin(c["xy"], c["frozen"], c["fval"], leaf=True)
    assert np.array_equal(info, c["info"])
    assert np.array_equal(xhat, c["xhat"])
    infopos = c["frozen"] == 0
    assert np.array_equal(lm[:, infopos], c["leaf_m"][:, infopos])
    # and the general path driven by r_i
    for b in range(0, c["xy"].shape[0], 5):
        i2, x2, _ = orc.decode_bin_general(c["xy"][b], c["frozen"], c["r"])
        assert np.array_equal(i2, c["info"][b])
        assert np.array_equal(x2, c["xhat"][b])


@pytest.mark.parametrize("idx", range(40))
def test_edge_long_cases(idx):
    """The oracle against the reference's decodes of the edge families at N = 1024 / 4096
    (edge_long.npz), before the GPU tests trust it on them."""
    c = edge_long_cases()[idx]
    info, xhat = orc.decode_bin(c["xy"], c["frozen"], c["fval"])
    assert np.array_equal(info, c["info"]), c["family_name"]
    assert np.array_equal(xhat, c["xhat"]), c["family_name"]


def test_nonuniform_prior_two_trees():
    g = load_golden("prior_n64")
    for b in range(g["xy"].shape[0]):
        info, xhat, lm = orc.decode_bin_general(g["xy"][b], g["frozen"], g["r"], prior=g["prior"])
        assert np.array_equal(info, g["info"][b])
        assert np.array_equal(xhat, g["xhat"][b])
        ip = g["frozen"] == 0
        assert np.array_equal(lm[ip], g["leaf_m"][b][ip])
    for b in range(g["enc_info"].shape[0]):
        x = orc.encode_bin(g["enc_info"][b], g["frozen"], r=g["r"], prior=g["prior"])
        assert np.array_equal(x, g["enc_x"][b])


@pytest.mark.parametrize("n", [1, 3, 5, 8, 10])
def test_encode_and_polar_transform(n):
    g = load_golden("encode_binary")
    fz, r, fv = g["n%d_frozen" % n], g["n%d_r" % n], g["n%d_fval" % n]
    for b in range(g["n%d_info" % n].shape[0]):
        x = orc.encode_bin(g["n%d_info" % n][b], fz, r=r)
        assert np.array_equal(x, g["n%d_x" % n][b])
        x2 = orc.encode_bin(g["n%d_info" % n][b], fz, fval=fv)
        assert np.array_equal(x2, x)
        assert np.array_equal(orc.polar_transform_bits(x), g["n%d_u" % n][b])


def test_qary_q4_decode_matches_reference():
    g = load_golden("qsc_q4_n256")
    xy = g["table"][g["y"]]
    info, _ = orc.decode_qary(4, xy, g["frozen"])
    assert np.array_equal(info, g["info"])
    info_r, _ = orc.decode_qary(4, g["xy_rand"], g["frozen"])
    assert np.array_equal(info_r, g["info_rand"])
    for t in range(0, g["tx_info"].shape[0], 16):
        assert np.array_equal(orc.encode_qary(4, g["tx_info"][t], g["frozen"]), g["x"][t])


def test_qary_q3():
    g = load_golden("qary_q3_n32")
    info, _ = orc.decode_qary(3, g["xy"], g["frozen"])
    assert np.array_equal(info, g["info"])
    for b in range(g["enc_info"].shape[0]):
        assert np.array_equal(orc.encode_qary(3, g["enc_info"][b], g["frozen"]), g["enc_x"][b])
