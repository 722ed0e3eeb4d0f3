"""q-ary parity holes closed with fixtures from runs of the reference itself
(oracle/make_golden.py): the log-domain decode (VectorDistributions/QaryMemorylessVectorDistribution.py:
40, 92-118: logaddexp transforms, logsumexp normalisation), the q-ary frozen-set picker on the
reference construction's own TV/Pe vectors (QaryPolarEncoderDecoder.py:1157-1191), and -- on the
GPU -- the q-ary Monte-Carlo driver's printed line (QaryPolarEncoderDecoder.py:935-982)."""
import contextlib
import io
import random

import numpy as np
import pytest

from tests.conftest import load_golden


def _log_sets():
    g = load_golden("qary_log")
    return g, [s["name"] for s in g["meta"]["sets"]]


@pytest.mark.parametrize("kind", ["chan", "rand"])
@pytest.mark.parametrize("name", ["q4_n6", "q3_n5", "q2_n4"])
def test_log_domain_restatement_matches_reference(name, kind):
    """polarcub_amd.vectors (log domain) through the generic recursion: decisions bit-exact and
    every information-leaf log-marginal equal to the reference's (same numpy/scipy calls)."""
    from polarcub_amd import coding_qary, vectors
    g, _ = _log_sets()
    meta = {s["name"]: s for s in g["meta"]["sets"]}[name]
    q, n = meta["q"], meta["n"]
    N = 1 << n
    frozen = set(int(i) for i in np.nonzero(g[name + "_frozen"])[0])
    dec = coding_qary.QaryPolarEncoderDecoder(q, N, frozen, 1, use_log=True)
    from polarcub_amd import scalar_qary
    qsc = scalar_qary.makeQSC(q, meta["p"])
    xd = scalar_qary.QaryMemorylessDistribution(q)
    xd.probs = [qsc.calcXMarginals()]
    xvd = xd.makeQaryMemorylessVectorDistribution(N, None, use_log=True)
    xy = g["%s_%s_xy" % (name, kind)]
    info = g["%s_%s_info" % (name, kind)]
    leaf = g["%s_%s_leaf" % (name, kind)]
    infos = [i for i in range(N) if i not in frozen]
    for t in range(xy.shape[0]):
        vd = vectors.QaryMemorylessVectorDistribution(q, N, use_log=True)
        vd.probs[:] = xy[t]
        marg = []
        got = np.full(dec.k, -1, np.int64)
        enc, nu, ni = dec.recursiveEncodeDecode(got, 0, 0, xvd, vd, marg)
        assert np.array_equal(got, info[t].astype(np.int64))
        # marg holds every leaf (frozen ones from the xy tree too); compare information leaves
        for i in infos:
            assert np.array_equal(np.asarray(marg[i], np.float64), leaf[t, i]), (t, i)
        # decode() itself runs the log-domain kernel: tests/test_gpu_qary_log.py


def test_frozen_set_from_reference_construction_vectors():
    from polarcub_amd import coding_qary
    g = load_golden("construct_qary")
    for tr in g["meta"]["trees"]:
        name = tr["name"]
        fz = coding_qary.frozenSetFromTVAndPe(g[name + "_tv"], g[name + "_pe"], tr["bound"], tr["numInfoIndices"])
        mask = np.zeros(1 << tr["n"], np.uint8)
        mask[sorted(fz)] = 1
        assert np.array_equal(mask, g[name + "_frozen"]), name
        assert (1 << tr["n"]) - mask.sum() == tr["K"]


def test_c4_code_is_the_reference_construction():
    """The C4 code (q=4, n=8, L=64, QSC(0.11), numInfoIndices=127) used by bench.py's qary
    workload: K = 128 from the reference's own degrading construction."""
    g = load_golden("construct_qary")
    m = g["qsc4_n8_L64_frozen"]
    assert m.shape == (256,) and int(256 - m.sum()) == 128


def _qary_closures(q, N, p):
    from polarcub_amd import scalar_qary
    qsc = scalar_qary.makeQSC(q, p)

    def make_x():
        xd = scalar_qary.QaryMemorylessDistribution(q)
        xd.probs = [qsc.calcXMarginals()]
        return xd.makeQaryMemorylessVectorDistribution(N, None)

    def channel(codeword):  # test3.py:35-55
        out = []
        for x in codeword:
            rnd = random.random()
            s = 0.0
            for y in range(len(qsc.probs)):
                if s + qsc.probXGivenY(int(x), y) >= rnd:
                    out.append(y)
                    break
                s += qsc.probXGivenY(int(x), y)
        return out

    def make_xy(rx):
        return qsc.makeQaryMemorylessVectorDistribution(len(rx), rx)

    return make_x, channel, make_xy


@pytest.mark.gpu
@pytest.mark.parametrize("run", [0, 1])
def test_qary_encode_decode_simulation_prints_reference_line(run):
    from polarcub_amd import coding_qary
    g = load_golden("qary_harness")
    r = g["meta"]["runs"][run]
    q, N = r["q"], 1 << r["n"]
    frozen = set(int(i) for i in np.nonzero(load_golden("construct_qary")[r["frozen_key"]])[0])
    make_x, channel, make_xy = _qary_closures(q, N, r["p"])
    random.seed(r["global_seed"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        coding_qary.encodeDecodeSimulation(q, N, make_x, lambda e: e, channel, make_xy, r["trials"], frozen)
    assert buf.getvalue().strip().splitlines()[-1] == r["line"]
