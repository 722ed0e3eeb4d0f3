"""Host-side parts of the reference-compatible facade (no GPU needed): plugin
classes, the generic plugin recursion, frozen-set helpers and the drop-in tree."""
import io
import os
import sys

import numpy as np
import pytest

from polarcub_amd import coding, scalar, vectors
from tests.conftest import ROOT, load_golden


def _bmvd(p):
    vd = vectors.BinaryMemorylessVectorDistribution(p.shape[0])
    vd.probs[:] = p
    return vd


def test_generic_recursion_matches_reference_uniform():
    g = load_golden("bsc_n64")
    xy = g["table"][g["y"]]
    fs = set(int(i) for i in np.nonzero(g["frozen"])[0])
    enc = coding.BinaryPolarEncoderDecoder(64, fs, g["meta"]["crs"])
    xvd = _bmvd(np.full((64, 2), 0.5))
    for b in range(0, 1000, 37):
        info = np.full(enc.k, -1, np.int64)
        x, nu, ni = enc.recursiveEncodeDecode(info, 0, 0, enc.randomlyGeneratedNumbers, xvd, _bmvd(xy[b]))
        assert nu == 64 and ni == enc.k
        assert np.array_equal(info, g["info"][b])
        assert np.array_equal(x, g["xhat"][b])


def test_nonuniform_prior_plugin_recursion():
    """The generic recursion (the path of non-memoryless priors) on the two-tree golden set."""
    g = load_golden("prior_n64")
    fs = set(int(i) for i in np.nonzero(g["frozen"])[0])
    enc = coding.BinaryPolarEncoderDecoder(64, fs, 11)
    xvd = _bmvd(np.tile(g["prior"], (64, 1)))
    for b in range(0, g["xy"].shape[0], 3):
        info = np.full(enc.k, -1, np.int64)
        x, nu, ni = enc.recursiveEncodeDecode(info, 0, 0, enc.randomlyGeneratedNumbers, xvd, _bmvd(g["xy"][b]))
        assert np.array_equal(info, g["info"][b])
        assert np.array_equal(x, g["xhat"][b])
    for b in range(g["enc_info"].shape[0]):
        x, nu, ni = enc.recursiveEncodeDecode(list(g["enc_info"][b]), 0, 0, enc.randomlyGeneratedNumbers, xvd)
        assert np.array_equal(x, g["enc_x"][b])


def test_prior_rows_dispatch_rule():
    assert coding._prior_rows(_bmvd(np.tile([0.7, 0.3], (8, 1))), 8) is not None
    assert coding._prior_rows(_bmvd(np.tile([0.7, 0.3], (1, 1))), 1) is None  # N = 1: recursion
    assert coding._prior_rows(_bmvd(np.tile([np.nan, 0.3], (8, 1))), 8) is None


def test_polar_transform_of_bits():
    g = load_golden("encode_binary")
    for n in (1, 3, 5, 8, 10):
        for b in range(g["n%d_x" % n].shape[0]):
            assert coding.polarTransformOfBits(list(g["n%d_x" % n][b])) == list(g["n%d_u" % n][b])


def test_frozen_set_from_tv_and_pe(capsys):
    tv = [0.0] * 8
    pe = [0.3, 0.01, 0.2, 0.001, 0.05, 0.0, 0.4, 0.02]
    fs = coding.frozenSetFromTVAndPe(tv, pe, 0.05)
    # sorted by TV+Pe: 5(0) 3(.001) 1(.01) 7(.02) | 4(.05) would exceed the bound
    assert fs == {0, 2, 4, 6}
    out = capsys.readouterr().out
    assert "frozen set =" in out and "fraction of non-frozen indices = 0.5" in out


def test_frozen_file_roundtrip(tmp_path):
    p = str(tmp_path / "frozen.txt")
    coding.write_frozen_file(p, {3, 1, 7}, 10, [0.1] * 8, [0.2] * 8, argv=["main_deletion.py", "-n", "3"])
    assert coding.read_frozen_file(p) == {1, 3, 7}
    text = open(p).read().splitlines()
    assert text[0] == "* main_deletion.py -n 3" and text[-1].startswith("*** 7 ")


def test_vector_plugin_methods_are_reference_arithmetic():
    rng = np.random.default_rng(0)
    p = rng.random((16, 2))
    vd = _bmvd(p)
    m = vd.minusTransform()
    a, b = p[0::2], p[1::2]
    assert np.array_equal(m.probs[:, 0], a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1])
    u = rng.integers(0, 2, 8)
    pl = vd.plusTransform(u)
    ref0 = np.where(u == 0, a[:, 0] * b[:, 0], a[:, 1] * b[:, 0])
    assert np.array_equal(pl.probs[:, 0], ref0)
    t = m.calcNormalizationVector()
    m.normalizeDistList(t)
    assert np.all(np.max(m.probs, axis=1) == 1.0)
    z = _bmvd(np.zeros((1, 2)))
    assert list(z.calcMarginalizedProbabilities()) == [0.5, 0.5]


def test_scalar_factories():
    bsc = scalar.makeBSC(0.11)
    assert bsc.probs == [[0.5 * (1.0 - 0.11), 0.5 * 0.11], [0.5 * 0.11, 0.5 * (1.0 - 0.11)]]
    vd = bsc.makeBinaryMemorylessVectorDistribution(4, [0, 1, 1, 0])
    assert np.array_equal(vd.probs, np.array(bsc.probs)[[0, 1, 1, 0]])
    assert bsc.calcXMarginal(0) == bsc.calcXMarginal(1)
    bec = scalar.makeBEC(0.3)
    assert len(bec.probs) == 3


def test_dropin_tree_imports():
    d = os.path.join(ROOT, "polarcub_amd", "dropin")
    sys.path.insert(0, d)
    try:
        import BinaryPolarEncoderDecoder as B
        from ScalarDistributions import BinaryMemorylessDistribution as S
        from VectorDistributions import BinaryMemorylessVectorDistribution as V
        assert B.BinaryPolarEncoderDecoder is coding.BinaryPolarEncoderDecoder
        assert S.makeBSC is scalar.makeBSC
        assert V.BinaryMemorylessVectorDistribution is vectors.BinaryMemorylessVectorDistribution
        assert S.calcFrozenSet_degradingUpgrading is scalar.calcFrozenSet_degradingUpgrading
        from ScalarDistributions.UpgradingDegrading import LinkedListHeap as H
        from polarcub_amd import heap
        assert H.LinkedListHeap is heap.LinkedListHeap
    finally:
        sys.path.remove(d)


def test_qary_polar_transform_and_generic_recursion():
    from polarcub_amd import coding_qary, scalar_qary
    g = load_golden("qsc_q4_n256")
    fz = g["frozen"]
    for t in range(0, 160, 40):
        u = coding_qary.polarTransformOfQudits(4, g["x"][t])
        assert np.array_equal(u[fz == 0], g["tx_info"][t]) and np.all(u[fz == 1] == 0)
    fs = set(int(i) for i in np.nonzero(fz)[0])
    encdec = coding_qary.QaryPolarEncoderDecoder(4, 256, fs, 1)
    qsc = scalar_qary.makeQSC(4, 0.11)
    xvd = vectors.QaryMemorylessVectorDistribution(4, 256)
    xvd.probs[:] = 0.25
    for t in range(0, 160, 53):
        yvd = qsc.makeQaryMemorylessVectorDistribution(256, [int(v) for v in g["y"][t]])
        info = np.full(encdec.k, -1, np.int64)
        encdec.recursiveEncodeDecode(info, 0, 0, xvd, yvd)
        assert np.array_equal(info, g["info"][t])


def test_qary_frozen_set_quirks():
    from polarcub_amd import coding_qary
    pe = [0.5, 0.1, 0.3, 0.0, 0.2, 0.05, 0.4, 0.01]
    fs = coding_qary.frozenSetFromTVAndPe([0.0] * 8, pe, numInfoIndices=2)
    # numInfoIndices=2 keeps 3 information indices (the reference's off-by-one)
    assert fs == {0, 2, 4, 6, 1}
