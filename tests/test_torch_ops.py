"""The PyTorch-ROCm operator form of the boundary (torch.ops.polarcub.*, csrc/torch/torch_ops.cpp;
SURVEY.md:443).  CPU: the library loads and registers the three schemas, and a host tensor is
refused (there is no CPU kernel).  GPU: the ops reproduce the reference's golden vectors and the
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
