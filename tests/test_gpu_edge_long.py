"""GPU parity at the BASELINE code lengths on the reference's edge families (edge_long.npz,
oracle/make_golden.py fx_edge_long): discrete, subnormal, random, one-sided zeros, ties, underflow,
quantised BI-AWGN at 2 dB (the rate-1 shortcut's common case), the same scaled to subnormal root
products, a high-SNR channel whose ratios underflow, and 2 dB rows with 1 % defect letters — at
N = 1024 and 4096, C2 / C3 Bhattacharyya and random frozen sets — through every built binary
variant, including the shipped defaults 26 (N = 1024) and 31 (N = 4096) whose minus-transform
division (`div_den12`) and rate-1 shortcut are exact by argument exactly at these inputs
(sc_common.h, sc_bin_body.h; reference BinaryPolarEncoderDecoder.py:223-325,
VectorDistributions/BinaryMemorylessVectorDistribution.py:15-87).  Bit-exact."""
import numpy as np
import pytest

from tests.conftest import edge_cases, edge_long_cases

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

VARIANTS = [0, 1, 10, 13, 14, 17, 24, 26, 30, 31, 33]


@pytest.fixture(scope="module")
def sc():
    from polarcub_amd import sc as _sc
    yield _sc
    _sc.set_variant()


@pytest.mark.parametrize("variant", VARIANTS)
def test_edge_long_all_variants(sc, variant):
    sc.set_variant(variant)
    try:
        for c in edge_long_cases():
            N = 1 << int(c["n"])
            code = sc.CodeSpec(N, c["frozen"], c["fval"])
            info, xhat = sc.BinaryDecoder(code).decode(torch.from_numpy(c["xy"]).cuda())
            assert np.array_equal(info.cpu().numpy(), c["info"]), (N, c["family_name"])
            assert np.array_equal(xhat.cpu().numpy(), c["xhat"]), (N, c["family_name"])
    finally:
        sc.set_variant()


def test_edge_long_bench_path(sc):
    """The bench's own entry (decode_tiled_native on tiles of the kernel's wave width, the shipped
    tiled-root twin) on every long edge case, packed outputs unpacked against the reference."""
    sc.set_variant()
    for c in edge_long_cases():
        N = 1 << int(c["n"])
        n = int(c["n"])
        code = sc.CodeSpec(N, c["frozen"], c["fval"])
        dec = sc.BinaryDecoder(code)
        B = c["xy"].shape[0]
        native = torch.from_numpy(np.ascontiguousarray(c["xy"].transpose(1, 0, 2))).cuda()
        ti, tx, _ = dec.decode_tiled_native(sc.tile_rows(native, sc.bin_tile(n)), B)
        assert np.array_equal(sc.unpack(ti, code.K).cpu().numpy(), c["info"]), (N, c["family_name"])
        assert np.array_equal(sc.unpack(tx, N).cpu().numpy(), c["xhat"]), (N, c["family_name"])


@pytest.mark.parametrize("variant", [17, 26, 31])
@pytest.mark.parametrize("idx", range(24))
def test_edge_short_shipped_variants(sc, idx, variant):
    """The 24 short edge cases (N = 2..256) with the defaults selected: short codes take the
    launcher's fallback, which is what a user of the default gets there."""
    sc.set_variant(variant)
    try:
        c = edge_cases()[idx]
        N = 1 << int(c["n"])
        code = sc.CodeSpec(N, c["frozen"], c["fval"])
        info, xhat = sc.BinaryDecoder(code).decode(torch.from_numpy(c["xy"]).cuda())
        assert np.array_equal(info.cpu().numpy(), c["info"])
        assert np.array_equal(xhat.cpu().numpy(), c["xhat"])
    finally:
        sc.set_variant()


@pytest.mark.parametrize("variant", [24, 26, 31])
def test_rate1_subnormal_ratios_n4096(sc, variant):
    """N = 4096 rate-1 blocks at very high reliability, so that the products of ratios inside the
    register subtrees reach the subnormal range and zero (the numerators `div_den12`'s exactness
    argument singles out), mixed in the same waves with ties, (0, 0) rows and subnormal letters;
    bit-exact against the oracle."""
    from oracle import orc
    sc.set_variant(variant)
    try:
        rng = np.random.default_rng(4096 + variant)
        N, B = 4096, 96
        frozen = (rng.random(N) < 0.5).astype(np.uint8)
        w = N // 4
        while w >= 16:
            for _ in range(2):
                s = int(rng.integers(N // (2 * w), N // w)) * w
                frozen[s:s + w] = 0
            w //= 2
        frozen[: N // 8] = 1
        fval = (rng.random(N) < 0.5).astype(np.uint8)
        mu = rng.choice([30.0, 200.0, 600.0, 740.0], size=(B, 1))
        llr = rng.normal(mu, 5.0, (B, N)) * np.where(rng.random((B, N)) < 0.5, 1, -1)
        p1 = np.exp(-np.abs(llr))                 # subnormal and zero ratios at |llr| > 708 / 745
        xy = np.where(llr[..., None] >= 0, np.stack([np.ones_like(p1), p1], -1), np.stack([p1, np.ones_like(p1)], -1))
        odd = rng.random((B, N))
        xy[odd < 0.0005] = 0.0                    # (0, 0)
        xy[(odd >= 0.0005) & (odd < 0.001)] = 0.5  # exact ties
        xy[(odd >= 0.001) & (odd < 0.0015)] = (4.9e-324, 1.0)
        xy = np.ascontiguousarray(xy)
        code = sc.CodeSpec(N, frozen, fval)
        info, xhat = sc.BinaryDecoder(code).decode(torch.from_numpy(xy).cuda())
        ri, rx = orc.decode_bin(xy, frozen, fval)
        assert np.array_equal(info.cpu().numpy(), ri)
        assert np.array_equal(xhat.cpu().numpy(), rx)
    finally:
        sc.set_variant()
