"""The PyTorch-ROCm operator form of the boundary (torch.ops.polarcub.*, csrc/torch/torch_ops.cpp;
SURVEY.md:443).  CPU: the library loads and registers the schemas, a host tensor is refused
(there is no CPU kernel), and the graph-capturable words form infers its shapes on Meta tensors.  GPU: the ops reproduce the reference's golden vectors and the
ctypes facade's outputs bit for bit."""
import numpy as np
import pytest
import torch

from tests.conftest import load_golden

BIN_SETS = ["bsc_n64", "awgn_n1024"]


def test_ops_register_the_extension_schemas():
    from polarcub_amd import ops
    o = ops.load()
    assert str(o.sc_decode_bin_f64.default._schema) == (
        "polarcub::sc_decode_bin_f64(Tensor xy, Tensor frozen_mask, Tensor frozen_val) -> (Tensor, Tensor)")
    assert str(o.sc_decode_qary_f64.default._schema) == (
        "polarcub::sc_decode_qary_f64(int q, Tensor xy, Tensor frozen_mask) -> (Tensor, Tensor)")
    assert str(o.polar_encode_bin.default._schema) == "polarcub::polar_encode_bin(Tensor u) -> Tensor"
    assert str(o.sc_decode_bin_f64.leaf._schema) == (
        "polarcub::sc_decode_bin_f64.leaf(Tensor xy, Tensor frozen_mask, Tensor frozen_val) -> (Tensor, Tensor, Tensor)")
    assert str(o.sc_decode_bin_words.default._schema) == (
        "polarcub::sc_decode_bin_words(Tensor xy, Tensor frozen_words, Tensor frozen_val_words, int K) -> (Tensor, Tensor)")
    assert str(o.mc_run.default._schema) == (
        "polarcub::mc_run(int log2N, int channel, float param, Tensor frozen_mask, Tensor frozen_val, int seed, "
        "int cw_offset, int count, int chunk=262144) -> Tensor")


def test_words_op_meta_shapes():
    from polarcub_amd import ops
    xy = torch.empty((300, 1024, 2), dtype=torch.float64, device="meta")
    w = torch.empty(32, dtype=torch.int32, device="meta")
    info, xhat = ops.sc_decode_bin_words(xy, w, w, 512)
    assert info.device.type == "meta" and tuple(info.shape) == (300, 512) and info.dtype == torch.uint8
    assert tuple(xhat.shape) == (300, 1024) and xhat.dtype == torch.uint8


def test_ops_have_no_cpu_kernel():
    from polarcub_amd import ops
    xy = torch.full((2, 8, 2), 0.25, dtype=torch.float64)
    m = torch.zeros(8, dtype=torch.uint8)
    with pytest.raises((NotImplementedError, RuntimeError)):
        ops.sc_decode_bin_f64(xy, m, m)


@pytest.mark.gpu
@pytest.mark.parametrize("name", BIN_SETS)
def test_op_decode_bin_matches_reference(name):
    from polarcub_amd import ops
    g = load_golden(name)
    xy = g["xy"] if "xy" in g else g["table"][g["y"]]
    info, xhat = ops.sc_decode_bin_f64(torch.from_numpy(xy).cuda(), g["frozen"], g["fval"])
    torch.cuda.synchronize()
    assert info.dtype == torch.uint8 and info.shape == g["info"].shape
    assert np.array_equal(info.cpu().numpy(), g["info"])
    assert np.array_equal(xhat.cpu().numpy(), g["xhat"])
    # a device-resident mask gives the same decode; an empty batch gives empty outputs
    info_d, _ = ops.sc_decode_bin_f64(torch.from_numpy(xy).cuda(), torch.from_numpy(g["frozen"]).cuda(),
                                      torch.from_numpy(g["fval"]).cuda())
    assert torch.equal(info_d, info)
    e_info, e_x = ops.sc_decode_bin_f64(torch.from_numpy(xy[:0]).cuda(), g["frozen"], g["fval"])
    assert e_info.shape == (0, info.shape[1]) and e_x.shape == (0, xhat.shape[1])


@pytest.mark.gpu
def test_op_decode_bin_matches_facade_on_a_ragged_batch():
    from polarcub_amd import ops, sc
    rng = np.random.default_rng(77)
    N, B = 1024, 1000  # not a multiple of the kernel's tile
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    xy = torch.from_numpy(rng.random((B, N, 2))).cuda()
    info, xhat = ops.sc_decode_bin_f64(xy, frozen, fval)
    info_f, xhat_f = sc.BinaryDecoder(sc.CodeSpec(N, frozen, fval)).decode(xy)
    torch.cuda.synchronize()
    assert torch.equal(info, info_f) and torch.equal(xhat, xhat_f)


@pytest.mark.gpu
def test_op_decode_qary_matches_reference():
    from polarcub_amd import ops
    g = load_golden("qsc_q4_n256")
    info, xhat = ops.sc_decode_qary_f64(4, torch.from_numpy(g["table"][g["y"]]).cuda(), g["frozen"])
    torch.cuda.synchronize()
    assert np.array_equal(info.cpu().numpy(), g["info"])
    info_r, _ = ops.sc_decode_qary_f64(4, torch.from_numpy(g["xy_rand"]).cuda(), g["frozen"])
    assert np.array_equal(info_r.cpu().numpy(), g["info_rand"])
    assert xhat.shape == (g["info"].shape[0], 256)


@pytest.mark.gpu
def test_op_polar_encode_matches_oracle():
    from oracle import orc
    from polarcub_amd import ops
    rng = np.random.default_rng(5)
    for n in (1, 5, 10):
        u = (rng.random((33, 1 << n)) < 0.5).astype(np.uint8)
        x = ops.polar_encode_bin(torch.from_numpy(u).cuda())
        torch.cuda.synchronize()
        ref = np.stack([orc.polar_transform_bits(row) for row in u])
        assert np.array_equal(x.cpu().numpy(), ref)


def _words(bits):
    """[N] 0/1 -> int32 [ceil(N/32)] words (bit i of word i // 32)"""
    b = np.asarray(bits, np.uint64).reshape(-1)
    W = max(1, (b.shape[0] + 31) // 32)
    out = np.zeros(W, np.uint64)
    for i in np.nonzero(b)[0]:
        out[i >> 5] |= np.uint64(1) << np.uint64(i & 31)
    return torch.from_numpy(out.astype(np.uint32).view(np.int32).copy())


@pytest.mark.gpu
def test_op_leaf_marginals_match_reference():
    """sc_decode_bin_f64.leaf: the reference's information-leaf marginals of awgn_n1024 bit for bit,
    every leaf equal to the oracle's, and the north star's LLR tolerance (1e-6 relative)."""
    from oracle import orc
    from polarcub_amd import ops
    g = load_golden("awgn_n1024")
    info, xhat, m = ops.sc_decode_bin_f64(torch.from_numpy(g["xy"]).cuda(), g["frozen"], g["fval"], leaf_m=True)
    torch.cuda.synchronize()
    m = m.cpu().numpy()
    assert m.shape == g["xy"].shape
    assert np.array_equal(info.cpu().numpy(), g["info"]) and np.array_equal(xhat.cpu().numpy(), g["xhat"])
    infopos = g["frozen"] == 0
    assert np.array_equal(m[:, infopos], g["leaf_m"][:, infopos])
    _, _, lm = orc.decode_bin(g["xy"], g["frozen"], g["fval"], leaf=True)
    assert np.array_equal(m, lm)
    with np.errstate(divide="ignore", invalid="ignore"):
        a, b = np.log(m[..., 0]) - np.log(m[..., 1]), np.log(lm[..., 0]) - np.log(lm[..., 1])
    fin = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), fin)
    assert np.all(np.abs(a[fin] - b[fin]) <= 1e-6 * np.maximum(1.0, np.abs(b[fin])))


@pytest.mark.gpu
def test_op_words_form_matches_byte_form_and_captures():
    """sc_decode_bin_words on device-packed masks = sc_decode_bin_f64, and it replays from a HIP graph."""
    from polarcub_amd import ops
    g = load_golden("awgn_n1024")
    xy = torch.from_numpy(g["xy"]).cuda()
    K = int((g["frozen"] == 0).sum())
    fw, vw = _words(g["frozen"]).cuda(), _words(g["fval"]).cuda()
    info, xhat = ops.sc_decode_bin_words(xy, fw, vw, K)
    info_b, xhat_b = ops.sc_decode_bin_f64(xy, g["frozen"], g["fval"])
    assert torch.equal(info, info_b) and torch.equal(xhat, xhat_b)
    assert np.array_equal(info.cpu().numpy(), g["info"])
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.sc_decode_bin_words(xy, fw, vw, K)  # warm the caching allocator on the capture stream
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        gi, gx = ops.sc_decode_bin_words(xy, fw, vw, K)
    xy.copy_(torch.from_numpy(g["xy"][::-1].copy()).cuda())
    graph.replay()
    torch.cuda.synchronize()
    assert np.array_equal(gi.cpu().numpy(), g["info"][::-1])
    assert np.array_equal(gx.cpu().numpy(), g["xhat"][::-1])


@pytest.mark.gpu
def test_op_mc_run_matches_pipeline():
    """mc_run = mc.run_bin's counters (the same pcub_mc_run_bin pipeline) over a sharded range."""
    from polarcub_amd import mc, ops, sc
    rng = np.random.default_rng(8)
    N = 256
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    code = sc.CodeSpec(N, frozen, fval)
    sigma2 = 0.630957
    ref = mc.run_bin(code, 99, 1000, 5000, 0, sigma2, chunk=2048)
    c = ops.mc_run(8, 0, sigma2, torch.from_numpy(frozen).cuda(), torch.from_numpy(fval).cuda(), 99, 1000, 5000,
                   chunk=2048)
    assert c.dtype == torch.int64 and c.is_cuda
    assert c.cpu().tolist() == ref
    a = ops.mc_run(8, 0, sigma2, torch.from_numpy(frozen).cuda(), torch.from_numpy(fval).cuda(), 99, 1000, 2500)
    b = ops.mc_run(8, 0, sigma2, torch.from_numpy(frozen).cuda(), torch.from_numpy(fval).cuda(), 99, 3500, 2500)
    assert (a + b).cpu().tolist() == ref
    bsc = ops.mc_run(8, 1, 0.11, torch.from_numpy(frozen).cuda(), torch.from_numpy(fval).cuda(), 5, 0, 3000)
    assert bsc.cpu().tolist() == mc.run_bin(code, 5, 0, 3000, 1, 0.11)
