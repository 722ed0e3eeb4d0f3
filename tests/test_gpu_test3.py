"""test3.py's q-ary harness counterpart (polarcub_amd/cli/test3.py) on the GPU.

* test()'s body (test3.py:118-150, getFrozenSet's bound passed by name) reproduces the
  reference's printed "Error probability" line on the same seeded channel
  (tests/golden/test3_body.npz, oracle/make_golden.py fx_test3_body), with the frozen set from
  the native q-ary construction equal to the reference's.
* encodeListDecodeSimulation (QaryPolarEncoderDecoder.py:985-1035), which fails in the
  reference itself (tests/test_dropin_names.py), runs its evident intent: the batched driver
  matches a trial-by-trial loop over listDecode with the same draws."""
import contextlib
import io
import os
import random

import numpy as np
import pytest

from polarcub_amd import coding_qary, scalar_qary
from polarcub_amd.cli import test3

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _runs():
    g = np.load(os.path.join(HERE, "golden", "test3_body.npz"), allow_pickle=False)
    import json
    return g, json.loads(str(g["meta"]))["runs"]


@pytest.mark.parametrize("idx", [0])
def test_body_matches_reference_line(idx, tmp_path, monkeypatch):
    g, runs = _runs()
    r = runs[idx]
    monkeypatch.setenv("POLARCUB_CONSTRUCTIONS", str(tmp_path))
    random.seed(r["global_seed"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        frozen = test3.body(r["q"], numberOfTrials=r["trials"])
    mask = np.zeros(2 ** r["n"], np.uint8)
    mask[sorted(frozen)] = 1
    assert np.array_equal(mask, g["q%d_frozen" % r["q"]])
    assert buf.getvalue().strip().splitlines()[-1] == r["line"]


def _loop_list_sim(q, N, xy, frozen, T, L, check, seed):
    """encodeListDecodeSimulation's intent, one listDecode call per trial (the reference's loop)."""
    encDec = coding_qary.QaryPolarEncoderDecoder(q, N, frozen, 1)
    rng = random.Random(1)
    xvd = test3.make_xVectorDistribution_fromQaryMemorylessDistribution(q, xy, N)()
    ch = test3.simulateChannel_fromQaryMemorylessDistribution(xy)
    mk = test3.make_xyVectorDistribution_fromQaryMemorylessDistribution(xy)
    random.seed(seed)
    np.random.seed(seed)
    bad = 0
    for _ in range(T):
        info = rng.choices(range(0, q), k=encDec.k)
        enc = encDec.encode(xvd, info)
        xyvd = mk(ch(enc))
        cm = np.random.choice(range(q), (encDec.k, check))
        cv = np.matmul(info, cm) % q
        dec, _ = encDec.listDecode(xyvd, np.zeros(len(encDec.frozenSet), np.int64), L, cm, cv, info)
        bad += not np.array_equal(info, dec)
    return bad


@pytest.mark.parametrize("q,L", [(2, 1), (3, 4), (4, 8)])
def test_list_simulation_batched_equals_loop(q, L):
    N, T, check, seed = 32, 60, 1, 17
    xy = scalar_qary.makeQSC(q, 0.12)
    rng = np.random.default_rng(q)
    frozen = set(int(i) for i in rng.choice(N, N // 2, replace=False))
    want = _loop_list_sim(q, N, xy, frozen, T, L, check, seed)
    random.seed(seed)
    np.random.seed(seed)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        coding_qary.encodeListDecodeSimulation(
            q, N, test3.make_xVectorDistribution_fromQaryMemorylessDistribution(q, xy, N),
            test3.make_codeword_noprocessing, test3.simulateChannel_fromQaryMemorylessDistribution(xy),
            test3.make_xyVectorDistribution_fromQaryMemorylessDistribution(xy), T, frozen, L, check, chunk=16)
    line = buf.getvalue().strip().splitlines()[-1]
    assert line == "Error probability =  %d / %d  =  %s" % (want, T, want / T)
