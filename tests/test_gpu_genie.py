"""Genie construction (genieEncodeDecodeSimulation) with the GPU leaf-export decoders,
against the reference's own genie runs: the TV / Pe vectors it derives the frozen set
from, and the frozen set, bit-exact (memoryless BSC with trusted probabilities; the
deletion channel of main_deletion.py with trustXYProbs=False)."""
import contextlib
import io
import random

import numpy as np
import pytest

from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


def _run_capturing(fn):
    from polarcub_amd import coding
    cap = {}
    orig = coding.frozenSetFromTVAndPe

    def capture(TV, Pe, b):
        cap["TV"], cap["Pe"] = np.array(TV, np.float64), np.array(Pe, np.float64)
        return orig(TV, Pe, b)

    coding.frozenSetFromTVAndPe = capture
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            frozen = fn()
    finally:
        coding.frozenSetFromTVAndPe = orig
    return frozen, cap


def test_genie_bsc_matches_reference():
    from polarcub_amd import coding, scalar
    g = load_golden("genie_bsc_n64")
    m = g["meta"]
    N = m["N"]
    bsc = scalar.makeBSC(m["p"])
    crng = random.Random(m["channel_seed"])

    def make_x():
        xd = scalar.BinaryMemorylessDistribution()
        xd.append([bsc.calcXMarginal(0), bsc.calcXMarginal(1)])
        return xd.makeBinaryMemorylessVectorDistribution(N, None)

    def channel(codeword):
        out = []
        for x in codeword:
            rnd = crng.random()
            acc = 0.0
            for y in range(2):
                if acc + bsc.probXGivenY(int(x), y) >= rnd:
                    out.append(y)
                    break
                acc += bsc.probXGivenY(int(x), y)
        return out

    frozen, cap = _run_capturing(lambda: coding.genieEncodeDecodeSimulation(
        N, make_x, lambda e: e, channel, lambda r: bsc.makeBinaryMemorylessVectorDistribution(len(r), r),
        m["trials"], m["bound"], m["genie_seed"], trustXYProbs=True))
    assert np.array_equal(cap["TV"], g["TV"])
    assert np.array_equal(cap["Pe"], g["Pe"])
    assert np.array_equal(np.array([1 if i in frozen else 0 for i in range(N)], np.uint8), g["frozen"])


def test_genie_deletion_matches_reference():
    from polarcub_amd import coding, deletion, vectors
    g = load_golden("deletion_n8")
    m = g["meta"]
    n, n0, pd, xi = m["n"], m["n0"], m["pd"], m["xi"]
    N = 1 << n
    crng = random.Random()
    crng.seed(m["channel_seed"])

    def make_x():
        v = vectors.BinaryMemorylessVectorDistribution(N)
        v.probs[:] = 0.5
        return v

    frozen, cap = _run_capturing(lambda: coding.genieEncodeDecodeSimulation(
        N, make_x, lambda e: deletion.addDeletionGuardBands(e, n, n0, xi, 0),
        lambda c: deletion.deletionChannelSimulation(c, pd, None, crng),
        lambda r: deletion.buildCollectionOfBinaryTrellises_uniformInput_deletion(r, pd, xi, n, n0, 0),
        m["genie_trials"], 0.1, m["genie_seed"], trustXYProbs=False))
    assert np.array_equal(cap["TV"] + cap["Pe"], g["genie_score"])
    assert np.array_equal(np.array([1 if i in frozen else 0 for i in range(N)], np.uint8), g["genie_frozen"])


def test_main_deletion_cli_matches_reference_run():
    """polarcub_amd.cli.main_deletion with the reference run's argv prints the same lines
    (the genie vectors aside, whose element repr differs between numpy scalars and floats)."""
    from polarcub_amd.cli import main_deletion
    g = load_golden("main_deletion_n8")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        main_deletion.main(list(g["meta"]["argv"]))
    lines = [l for l in buf.getvalue().strip().splitlines()
             if not l.startswith(("TVVec", "pevec", "HEncvec", "HDecvec"))]
    assert lines == g["meta"]["lines"]


def test_test2_cli_matches_reference_run():
    """polarcub_amd.cli.test2 (native Tal-Vardy construction + 4000 GPU-batched trials)
    with the reference run's channel seed prints the reference's lines, error count included."""
    from polarcub_amd.cli import test2
    g = load_golden("test2_run")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        test2.main(["--seed", str(g["meta"]["global_random_seed"])])
    assert buf.getvalue().strip().splitlines() == g["meta"]["lines"]


@pytest.mark.parametrize("ci", range(6))
def test_genie_deletion_wide_matches_reference(ci, monkeypatch):
    """Genie runs past 64 trellises per codeword (main_deletion's own n0 = n//3 at n = 10: 128;
    n0 = 1 at n = 8 / 9: 128 / 256) and with guard-band ones 1..3: every trial's leaves come from
    the GPU export kernel (the host recursion is disabled here), TV + Pe and the frozen set equal
    the reference run's."""
    from polarcub_amd import coding, deletion, sc, vectors
    g = load_golden("deletion_genie_wide")
    xi = g["meta"]["xi"]
    n, n0, ones, G = (int(v) for v in g["c%d_shape" % ci])
    pd = float(g["c%d_pd" % ci][0])
    N = 1 << n
    assert sc.leaf_deletion_supported(n, n0, ones)
    monkeypatch.setattr(coding.BinaryPolarEncoderDecoder, "genieSingleDecodeSimulatioan",
                        lambda *a, **k: pytest.fail("host genie decode used"))
    crng = random.Random()
    crng.seed(100 + ci)

    def make_x():
        v = vectors.BinaryMemorylessVectorDistribution(N)
        v.probs[:] = 0.5
        return v

    frozen, cap = _run_capturing(lambda: coding.genieEncodeDecodeSimulation(
        N, make_x, lambda e: deletion.addDeletionGuardBands(e, n, n0, xi, ones),
        lambda c: deletion.deletionChannelSimulation(c, pd, None, crng),
        lambda r: deletion.buildCollectionOfBinaryTrellises_uniformInput_deletion(r, pd, xi, n, n0, ones),
        G, 0.1, 300 + ci, trustXYProbs=n <= n0))
    assert np.array_equal(cap["TV"] + cap["Pe"], g["c%d_score" % ci])
    assert np.array_equal(np.array([1 if i in frozen else 0 for i in range(N)], np.uint8), g["c%d_frozen" % ci])


def test_main_deletion_cli_n10_matches_reference_run():
    """main_deletion -n 10 -g 6 -e 4 (n0 = 3: 128 trellises a codeword, genie and decode on the GPU)
    prints the reference run's lines."""
    from polarcub_amd.cli import main_deletion
    g = load_golden("deletion_genie_wide")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        main_deletion.main(list(g["meta"]["main_argv"]))
    lines = [l for l in buf.getvalue().strip().splitlines()
             if not l.startswith(("TVVec", "pevec", "HEncvec", "HDecvec"))]
    assert lines == g["meta"]["main_lines"]
