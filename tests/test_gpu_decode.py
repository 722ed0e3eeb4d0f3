"""GPU parity: the HIP decoder (through the C ABI) against the reference's
golden vectors, bit-exact for information bits and re-encoded codewords."""
import numpy as np
import pytest

from tests.conftest import edge_cases, load_golden

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

BIN_SETS = ["bsc_n64", "awgn_n1024", "awgn_n4096", "awgn_n256_lowsnr"]
# the kernel variants the library builds (sc_bin_kern.h; the ones pick_variant can launch): 24 and 26
# keep the re-encoded bits in LDS, 26 and 31 split their last level (LDS + registers)
VARIANTS = [0, 1, 10, 13, 14, 17, 24, 26, 30, 31, 33]


def _xy(g):
    return g["xy"] if "xy" in g else g["table"][g["y"]]


@pytest.fixture(scope="module")
def sc():
    from polarcub_amd import sc as _sc
    return _sc


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("name", BIN_SETS)
def test_decode_matches_reference(sc, name, variant):
    sc.set_variant(variant)
    g = load_golden(name)
    code = sc.CodeSpec(g["frozen"].shape[0], g["frozen"], g["fval"])
    dec = sc.BinaryDecoder(code)
    xy = torch.from_numpy(_xy(g)).cuda()
    info, xhat = dec.decode(xy)
    torch.cuda.synchronize()
    assert np.array_equal(info.cpu().numpy(), g["info"])
    assert np.array_equal(xhat.cpu().numpy(), g["xhat"])
    sc.set_variant()


@pytest.mark.parametrize("variant", [0, 1, 10, 13, 14, 24])
@pytest.mark.parametrize("idx", range(24))
def test_edge_cases(sc, idx, variant):
    sc.set_variant(variant)
    c = edge_cases()[idx]
    N = 1 << int(c["n"])
    code = sc.CodeSpec(N, c["frozen"], c["fval"])
    info, xhat = sc.BinaryDecoder(code).decode(torch.from_numpy(c["xy"]).cuda())
    assert np.array_equal(info.cpu().numpy(), c["info"])
    assert np.array_equal(xhat.cpu().numpy(), c["xhat"])


@pytest.mark.parametrize("variant", VARIANTS)
def test_ragged_batches_and_slot_reuse(sc, variant):
    """Batch sizes that are not tile multiples, and more tiles than resident slots."""
    from oracle import orc
    sc.set_variant(variant)
    rng = np.random.default_rng(3 + variant)
    # N = 8192: past the LDS budget of the re-encoded-bits variants (their fallback runs)
    for N, B in [(64, 1), (128, 257), (256, 1000), (1024, 300), (512, 70000), (2048, 33), (8192, 40)]:
        frozen = (rng.random(N) < 0.5).astype(np.uint8)
        fval = (rng.random(N) < 0.5).astype(np.uint8)
        xy = rng.random((B, N, 2))
        xy[rng.random((B, N)) < 0.05] = 0.0
        code = sc.CodeSpec(N, frozen, fval)
        info, xhat = sc.BinaryDecoder(code).decode(torch.from_numpy(xy).cuda())
        sub = slice(0, B) if B <= 2000 else np.r_[0:500, B - 500:B]
        ri, rx = orc.decode_bin(xy[sub], frozen, fval)
        assert np.array_equal(info.cpu().numpy()[sub], ri), (N, B)
        assert np.array_equal(xhat.cpu().numpy()[sub], rx), (N, B)
    sc.set_variant()


@pytest.mark.parametrize("variant", VARIANTS)
def test_rate0_blocks(sc, variant):
    """Frozen sets full of aligned rate-0 blocks (skipped by every variant's schedule,
    at the stage levels and inside the register and cross-lane subtrees)."""
    from oracle import orc
    from tests.conftest import awgn_like, blocky_frozen
    sc.set_variant(variant)
    rng = np.random.default_rng(7 + variant)
    for n, B in [(6, 70), (7, 300), (8, 513), (10, 1000), (11, 200), (12, 64)]:
        N = 1 << n
        frozen, fval = blocky_frozen(N, rng)
        xy = awgn_like(B, N, rng)
        code = sc.CodeSpec(N, frozen, fval)
        info, xhat = sc.BinaryDecoder(code).decode(torch.from_numpy(xy).cuda())
        ri, rx = orc.decode_bin(xy, frozen, fval)
        assert np.array_equal(info.cpu().numpy(), ri), (n, B)
        assert np.array_equal(xhat.cpu().numpy(), rx), (n, B)
    sc.set_variant()


@pytest.mark.parametrize("variant", VARIANTS)
def test_rate1_blocks(sc, variant):
    """Frozen sets with large aligned all-information (rate-1) blocks, decoded through the rate-1
    shortcut (sc_bin_body.h: hard decisions when every codeword of the wave passes the reliability
    test) and through the recursion when one does not: per-codeword reliabilities from near-certain
    to noise, exact ties, near ties and (0, 0) rows in the same waves, bit-exact against the oracle."""
    from oracle import orc
    sc.set_variant(variant)
    rng = np.random.default_rng(19 + variant)
    for n, B in [(6, 300), (8, 700), (10, 900), (12, 160)]:
        N = 1 << n
        frozen = (rng.random(N) < 0.5).astype(np.uint8)
        w = N // 4
        while w >= 16:
            for _ in range(2):
                s = int(rng.integers(N // (2 * w), N // w)) * w
                frozen[s:s + w] = 0
            w //= 2
        frozen[: N // 8] = 1
        fval = (rng.random(N) < 0.5).astype(np.uint8)
        mu = rng.choice([1.0, 6.0, 20.0, 60.0], size=(B, 1), p=[0.1, 0.3, 0.3, 0.3])
        llr = rng.normal(mu, 2.0, (B, N)) * np.where(rng.random((B, N)) < 0.5, 1, -1)
        llr[rng.random((B, N)) < 0.002] = 0.0      # exact ties
        llr[rng.random((B, N)) < 0.002] = 1e-13    # near ties
        p1 = 1.0 / (1.0 + np.exp(llr))
        xy = np.stack([1.0 - p1, p1], axis=-1)
        xy[rng.random((B, N)) < 0.001] = 0.0       # (0, 0) rows
        code = sc.CodeSpec(N, frozen, fval)
        info, xhat = sc.BinaryDecoder(code).decode(torch.from_numpy(xy).cuda())
        ri, rx = orc.decode_bin(xy, frozen, fval)
        assert np.array_equal(info.cpu().numpy(), ri), (n, B)
        assert np.array_equal(xhat.cpu().numpy(), rx), (n, B)
    sc.set_variant()


@pytest.mark.parametrize("n", [1, 3, 5, 8, 10])
def test_encode_matches_reference(sc, n):
    g = load_golden("encode_binary")
    N = 1 << n
    code = sc.CodeSpec(N, g["n%d_frozen" % n], g["n%d_fval" % n])
    info = torch.from_numpy(g["n%d_info" % n]).cuda()
    x = sc.encode(code, info)
    assert np.array_equal(x.cpu().numpy(), g["n%d_x" % n])


def test_decode_then_reencode_roundtrip_large(sc):
    """Noiseless round trip at N=4096: decode(encode(u)) == u, x_hat == x (size-independent property).
    Certain observations (P(x,y) = 1 for the sent bit, 0 otherwise) make every SC
    decision exact, whatever the frozen set."""
    rng = np.random.default_rng(11)
    N, B = 4096, 2048
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    code = sc.CodeSpec(N, frozen, fval)
    info = torch.from_numpy(rng.integers(0, 2, size=(B, code.K)).astype(np.uint8)).cuda()
    x = sc.encode(code, info)
    xf = x.to(torch.float64)
    xy = torch.stack([1.0 - xf, xf], dim=-1)
    di, dx = sc.BinaryDecoder(code).decode(xy)
    assert torch.equal(di, info)
    assert torch.equal(dx, x)


@pytest.mark.parametrize("variant", [0, 1, 17, 24, 26, 30, 31, 33])
def test_tiled_root_layout(sc, variant):
    """pcub_sc_decode_bin_tiled: the root rows in tiles of T codewords ([ceil(B/T), N, T, 2], the
    kernel's own wave width and others, ragged last tiles) decode exactly as the [N, B, 2] rows, for
    the short-code kernels too, and the compact rows' tiled entry likewise."""
    from oracle import orc
    sc.set_variant(variant)
    rng = np.random.default_rng(100 + variant)
    try:
        for N, B in [(16, 77), (64, 300), (1024, 333), (4096, 70)]:
            n = N.bit_length() - 1
            frozen = (rng.random(N) < 0.5).astype(np.uint8)
            fval = (rng.random(N) < 0.5).astype(np.uint8)
            xy = rng.random((B, N, 2))
            xy[rng.random((B, N)) < 0.05] = 0.0
            code = sc.CodeSpec(N, frozen, fval)
            dec = sc.BinaryDecoder(code)
            native = torch.from_numpy(np.ascontiguousarray(xy.transpose(1, 0, 2))).cuda()
            ref_i, ref_x, _ = dec.decode_native(native)
            for T in sorted({sc.bin_tile(n), 1, 5, 64}):
                ti, tx, _ = dec.decode_tiled_native(sc.tile_rows(native, T), B)
                assert torch.equal(ti, ref_i) and torch.equal(tx, ref_x), (N, T)
            ri, rx = orc.decode_bin(xy[:40], frozen, fval)
            assert np.array_equal(sc.unpack(ref_i, code.K).cpu().numpy()[:40], ri)
            # compact rows (normalised pairs' ratios with the orientation in the sign)
            p0, p1 = xy[..., 0], xy[..., 1]
            with np.errstate(invalid="ignore", divide="ignore"):
                xc = np.where(p1 > p0, -(p0 / p1), p1 / p0)
            xct = torch.from_numpy(np.ascontiguousarray(xc.T)).cuda()
            ci, cx, _ = dec.decode_compact_native(xct)
            T = sc.bin_tile(n)
            tiled = sc.tile_rows(xct, T)
            from polarcub_amd import _lib
            L = _lib.lib()
            nt = (B + T - 1) // T
            ws = torch.empty(int(L.pcub_sc_decode_bin_compact_workspace(nt * T, n)), dtype=torch.uint8, device="cuda")
            info = torch.empty_like(ci)
            xh = torch.empty_like(cx)
            rc = L.pcub_sc_decode_bin_compact_tiled(sc._p(tiled), B, n, T, sc._p(code.fmask_dev), sc._p(code.fval_dev),
                                                    code.K, sc._p(info), sc._p(xh), None, sc._p(ws), ws.numel(),
                                                    sc._stream())
            assert rc == 0
            assert torch.equal(info, ci) and torch.equal(xh, cx), N
    finally:
        sc.set_variant()
