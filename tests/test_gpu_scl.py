"""q-ary list decoding on the GPU (pcub_scl_qary): bit for bit against the oracle's restatement
(oracle/scl_oracle.py, same tie rules; tie-free and QSC inputs), as a path set against runs of the
reference itself (tests/golden/scl.npz), and the batched irSimulation against the reference's
frame errors and ProbResults (see tests/test_scl.py for the list-order caveat)."""
import math

import numpy as np
import pytest

from oracle import scl_oracle as so
from tests.conftest import load_golden
from tests.test_scl import _as_set, _random_inputs, ir_closures

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sc():
    from polarcub_amd import _lib, sc as m
    _lib.lib()
    return m


@pytest.mark.parametrize("q,n,L,ties", [(2, 3, 2, False), (3, 4, 4, False), (4, 5, 8, False), (2, 6, 16, False),
                                        (3, 4, 4, True), (4, 5, 8, True), (2, 5, 3, True), (5, 3, 4, False),
                                        (4, 8, 8, False), (2, 10, 4, False)])
def test_gpu_list_decoder_matches_oracle(sc, q, n, L, ties):
    rng = np.random.default_rng(1000 * q + 10 * n + L + ties)
    B = 40 if n < 8 else 6
    frozen, xy, fv, act = _random_inputs(rng, q, n, B, ties)
    info, prob, size, ap = sc.QaryListDecoder(q, 1 << n, frozen, L).decode(xy, fv, act)
    for b in range(B):
        k, oinfo, oprob, oap = so.list_decode(q, frozen, L, xy[b], fv[b], act[b])
        assert size[b] == k, b
        assert info[b][:k].tolist() == oinfo, b
        assert np.array_equal(prob[b][:k], np.array(oprob)), b
        assert ap[b] == oap, b


def test_gpu_list_decoder_matches_reference_sets(sc):
    g = load_golden("scl")
    for c in g["meta"]["cases"]:
        t_, q, L = c["tag"], c["q"], c["L"]
        info, prob, size, ap = sc.QaryListDecoder(q, 1 << c["n"], g[t_ + "_frozen"], L).decode(
            g[t_ + "_xy"], g[t_ + "_fv"], g[t_ + "_actual"])
        for t in range(g[t_ + "_xy"].shape[0]):
            rk = int(g[t_ + "_size"][t])
            assert size[t] == rk
            ours = _as_set(info[t][:rk].tolist(), prob[t][:rk].tolist())
            ref = _as_set(g[t_ + "_info"][t][:rk].tolist(), g[t_ + "_prob"][t][:rk].tolist())
            assert [a for a, _ in ours] == [a for a, _ in ref]
            assert np.allclose([p for _, p in ours], [p for _, p in ref], rtol=1e-12, atol=0)
            assert math.isclose(ap[t], g[t_ + "_aprob"][t], rel_tol=1e-12)


@pytest.mark.parametrize("which", [0, 1])
def test_gpu_ir_simulation_matches_reference(which, capsys):
    from polarcub_amd import coding_qary
    g = load_golden("scl")
    r = g["meta"]["ir"][which]
    simulate, make_xy = ir_closures(r)
    frozen = set(int(i) for i in np.nonzero(g[r["name"] + "_frozen"])[0])
    np.random.seed(r["np_seed"])
    fe, se, rate, prl = coding_qary.irSimulation(r["q"], 1 << r["n"], simulate, make_xy, r["trials"], frozen, r["L"],
                                                 r["check_size"], verbosity=1)
    assert fe == r["frame_error_prob"] and rate == r["rate"]
    assert [p.name for p in prl] == r["prob_results"]
    assert capsys.readouterr().out.splitlines()[:2] == r["printed"].splitlines()[:2]


def test_list_decode_facade_single_word(sc):
    """QaryPolarEncoderDecoder.listDecode: the returned word and ProbResult follow the list."""
    from polarcub_amd import coding_qary, vectors
    g = load_golden("scl")
    c = g["meta"]["cases"][4]
    t_, q, L, N = c["tag"], c["q"], c["L"], 1 << c["n"]
    frozen = set(int(i) for i in np.nonzero(g[t_ + "_frozen"])[0])
    enc = coding_qary.QaryPolarEncoderDecoder(q, N, frozen, 1)
    for t in range(4):
        vd = vectors.QaryMemorylessVectorDistribution(q, N)
        vd.probs[:] = g[t_ + "_xy"][t]
        info, pr = enc.listDecode(vd, g[t_ + "_fv"][t], L, np.zeros((enc.k, 0), np.int64), np.zeros(0, np.int64),
                                  actualInformation=g[t_ + "_actual"][t])
        assert pr.name == c["prob_result"][t]
        if pr.name.startswith("Success"):
            assert np.array_equal(info, g[t_ + "_actual"][t])


def test_gpu_list_decoder_full_occupancy(sc):
    """A batch that fills every resident workgroup (2^17 codewords, q=4, N=256, L=8) at the
    runtime's default per-thread stack limit (the recursion is an explicit frame loop, the kernel
    has no dynamic stack, and the library no longer raises the limit), and the first codewords
    decode as they do alone."""
    import torch
    rng = np.random.default_rng(5)
    q, n, L, B = 4, 8, 8, 1 << 17
    N = 1 << n
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    dec = sc.QaryListDecoder(q, N, frozen, L)
    xy = torch.rand((N, B, q), dtype=torch.float64, device="cuda")
    fv = torch.zeros((int(frozen.sum()), B), dtype=torch.uint8, device="cuda")
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    limit = ctypes.c_size_t(0)
    assert hip.hipDeviceGetLimit(ctypes.byref(limit), 0) == 0  # hipLimitStackSize
    before = limit.value
    info, prob, size, _ = dec.decode_native(xy, fv)
    torch.cuda.synchronize()
    assert hip.hipDeviceGetLimit(ctypes.byref(limit), 0) == 0 and limit.value == before
    assert int(size.min()) >= 1
    info1, prob1, size1, _ = dec.decode_native(xy[:, :6].contiguous(), fv[:, :6].contiguous())
    assert torch.equal(size[:6], size1)
    assert torch.equal(info[:, :, :6], info1) and torch.equal(prob[:, :6], prob1)
