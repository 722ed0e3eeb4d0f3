"""q-ary degrading/upgrading construction on the native host library, bit-exact against the
reference's own runs (construct_qary.npz, construct_qary_up.npz from oracle/make_golden.py):
degrade / upgrade of QSC / QEC / a-priori distributions and their polar transforms, the
reference's failures (AttributeError when M = 1 leaves a letter without neighbours), whole-tree
TV / Pe vectors with and without an a-priori distribution, frozen sets, the .npy cache, and
the combine_codes.py counterpart."""
import os

import numpy as np
import pytest

from polarcub_amd import coding_qary, construction, scalar_qary
from tests.conftest import load_golden


@pytest.fixture(scope="module", autouse=True)
def _built():
    from polarcub_amd import build
    build.build_host()


def _dist(rows):
    d = scalar_qary.QaryMemorylessDistribution(rows.shape[1])
    d.probs = [list(map(float, r)) for r in rows]
    return d


def _cases(g):
    return g["meta"]["cases"]


def test_degrade_matches_reference():
    g = load_golden("construct_qary")
    n = 0
    for case in _cases(g):
        src = _dist(g[case + "_in"])
        for L in (4, 9, 16, 64):
            out = np.array(src.degrade(L).probs)
            assert np.array_equal(out, g["%s_deg%d" % (case, L)]), (case, L)
            n += 1
    assert n == 4 * len(_cases(g))


def test_upgrade_and_degrade_with_priors_match_reference():
    g = load_golden("construct_qary_up")
    errors = g["meta"]["errors"]
    seen_err = 0
    for case in _cases(g):
        src = _dist(g[case + "_in"])
        for L in (4, 9, 16, 64):
            for op in ("up", "deg"):
                key = "%s_%s%d" % (case, op, L)
                fn = src.upgrade if op == "up" else src.degrade
                if key in errors:
                    with pytest.raises(getattr(__builtins__, errors[key], None) or Exception) as ei:
                        fn(L)
                    assert type(ei.value).__name__ == errors[key]
                    seen_err += 1
                    continue
                assert np.array_equal(np.array(fn(L).probs).reshape(-1, src.q), g[key]), key
    assert seen_err == len(errors) > 0


def test_transforms_error_prob_and_tv_match_reference_semantics():
    g = load_golden("construct_qary")
    d = _dist(g["qsc3_in"])
    assert np.array_equal(np.array(d.minusTransform().probs), g["qsc3_m_in"])
    assert np.array_equal(np.array(d.plusTransform().probs), g["qsc3_p_in"])
    assert np.array_equal(np.array(d.minusTransform().plusTransform().probs), g["qsc3_mp_in"])
    for case in ("qsc4_p", "qec3_mp", "qsc5_p"):
        rows = g[case + "_in"]
        pe, tv = construction.qmd_error_prob_tv(rows.shape[1], rows)
        dd = _dist(rows)
        assert pe == dd.errorProb() and tv == dd.totalVariation()


@pytest.mark.parametrize("tree", ["qsc3_n4_L16", "qsc4_n3_L27", "qsc4_n5_L64", "qsc2_n6_L16", "qsc4_n8_L64"])
def test_tree_pe_and_frozen_set_match_reference(tree, tmp_path):
    g = load_golden("construct_qary")
    t = [x for x in g["meta"]["trees"] if x["name"] == tree][0]
    ch = scalar_qary.makeQSC(t["q"], t["p"])
    d = str(tmp_path) + "/"
    fz = scalar_qary.calcFrozenSet_degradingUpgrading(t["n"], t["L"], None, ch, d, t["bound"], t["numInfoIndices"])
    tv, pe = np.load(d + "DegradingUpgrading_L=%d_tv.npy" % t["L"]), np.load(d + "DegradingUpgrading_L=%d_pe.npy" % t["L"])
    assert np.array_equal(pe, g[tree + "_pe"]) and np.array_equal(tv, g[tree + "_tv"])
    mask = np.zeros(1 << t["n"], np.uint8)
    mask[sorted(fz)] = 1
    assert np.array_equal(mask, g[tree + "_frozen"])
    # a second call reads the cache (the files are the reference's np.save format)
    tv2, pe2 = scalar_qary.calcTVAndPe_degradingUpgrading(t["n"], t["L"], None, ch, d)
    assert isinstance(pe2, np.ndarray) and np.array_equal(pe2, pe)


@pytest.mark.parametrize("tree", ["j3_n4_L16", "j3_n5_L9", "j4_n3_L27"])
def test_tree_with_prior_matches_reference(tree):
    g = load_golden("construct_qary_up")
    t = [x for x in g["meta"]["trees"] if x["name"] == tree][0]
    xy, x = _dist(g[tree + "_xy"]), _dist(g[tree + "_x"])
    tv, pe = scalar_qary.calcTVAndPe_degradingUpgrading(t["n"], t["L"], x, xy)
    assert np.array_equal(np.array(tv), g[tree + "_tv"])
    assert np.array_equal(np.array(pe), g[tree + "_pe"])
    fz = coding_qary.frozenSetFromTVAndPe(tv, pe, t["bound"], t["numInfoIndices"])
    mask = np.zeros(1 << t["n"], np.uint8)
    mask[sorted(fz)] = 1
    assert np.array_equal(mask, g[tree + "_frozen"])


def test_input_distribution_and_m():
    d = scalar_qary.makeInputDistribution([2.0, 1.0, 1.0])
    assert d.probs == [[0.5, 0.25, 0.25]]
    assert scalar_qary.QaryMemorylessDistribution(4).calcMFromL(64) == 4
    assert scalar_qary.QaryMemorylessDistribution(3).calcMFromL(16) == 4


def test_combine_codes_matches_reference(tmp_path, capsys):
    from polarcub_amd.cli import combine_codes
    g = load_golden("combine_codes")
    files = []
    for k, text in enumerate(g["inputs"]):
        p = tmp_path / ("frozen%d.txt" % k)
        p.write_text(str(text))
        files.append(str(p))
    cwd = os.getcwd()
    try:
        os.chdir(tmp_path)
        combine_codes.main(files)
    finally:
        os.chdir(cwd)
    assert capsys.readouterr().out == str(g["stdout"])
    assert (tmp_path / "out").read_text() == str(g["out"])
