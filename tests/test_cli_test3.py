"""cli/test3.py on the CPU: test() and test_ir() fail where the reference's do (the bound lands
in getFrozenSet's snr slot, test3.py:130 / :169, and frozenSetFromTVAndPe compares a float with
None), and the construction cache follows the reference's layout."""
import os

import pytest

from polarcub_amd.cli import test3


def test_test_fails_like_the_reference(tmp_path, monkeypatch):
    monkeypatch.setenv("POLARCUB_CONSTRUCTIONS", str(tmp_path))
    with pytest.raises(TypeError, match="not supported between instances of 'float' and 'NoneType'"):
        test3.test(2)
    # the construction ran and was cached where the reference would put it
    d = test3.get_construction_path(2, 256, QER=0.99)
    assert d.startswith(str(tmp_path))
    assert os.path.isfile(d + "DegradingUpgrading_L=100_tv.npy") and os.path.isfile(d + "DegradingUpgrading_L=100_pe.npy")


def test_test_ir_fails_like_the_reference(tmp_path, monkeypatch):
    monkeypatch.setenv("POLARCUB_CONSTRUCTIONS", str(tmp_path))
    with pytest.raises(TypeError):
        test3.test_ir(2)


def test_key_rates():
    assert test3.calc_theoretic_key_rate(2, qer=0.0) == 1.0
    assert abs(test3.calc_theoretic_key_qrate(3, 0.01) - (1.0 + 0.99 * __import__("math").log(0.99, 3)
                                                          + 0.01 * __import__("math").log(0.005, 3))) < 1e-15
    assert 0.0 < test3.snr_to_qer(2, 2.0, 0.5) < 0.5
