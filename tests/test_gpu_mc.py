"""Device Monte-Carlo (sc_mc.hip): codewords keyed by their global index, so any
sharding of [0, total) over ranks / chunks gives identical codewords and identical
summed counters; the pipeline decodes error-free on clean channels; FER agrees
with the reference-pinned host run within sampling error."""
import math

import numpy as np
import pytest
import torch

from tests.conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def code():
    from polarcub_amd import construction, sc
    n, K = 10, 512
    s2 = construction.awgn_sigma2(2.0, 0.5)
    fr = construction.bhattacharyya_frozen(n, K, s2)
    return sc.CodeSpec.from_frozen_set(1 << n, set(np.nonzero(fr)[0].tolist()), 1, device="cuda"), s2


def test_batches_keyed_by_global_index(code):
    from polarcub_amd import mc
    c, s2 = code
    info_a, xy_a = mc.philox_batch(c, 99, 1000, 300, mc.CHANNEL_AWGN, s2)
    info_b, xy_b = mc.philox_batch(c, 99, 1100, 50, mc.CHANNEL_AWGN, s2)
    assert torch.equal(info_a[:, 100:150], info_b)
    assert torch.equal(xy_a[:, 100:150, :], xy_b)
    info_c, _ = mc.philox_batch(c, 100, 1100, 50, mc.CHANNEL_AWGN, s2)
    assert not torch.equal(info_b, info_c)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_counters_match_single_run(code, world):
    """The counters of ranks 0..G-1 (each its own [r*B, (r+1)*B)) sum to the 1-GPU run over
    [0, G*B), for any chunking."""
    from polarcub_amd import mc
    c, s2 = code
    total = 3 * 8192
    one = mc.run_bin(c, 7, 0, total, mc.CHANNEL_AWGN, s2, chunk=4096)
    parts = []
    for r in range(world):
        lo, hi = mc.shard_range(total, r, world)
        parts.append(mc.run_bin(c, 7, lo, hi - lo, mc.CHANNEL_AWGN, s2, chunk=1000))
    summed = [sum(p[i] for p in parts) for i in range(4)]
    assert summed == one
    assert one[0] == total and 0 < one[1] < total


def test_sharded_counters_match_single_run_n4096():
    """C3's decomposition at its own code length (N=4096, K=2048): 8 ranks' shards of [0, total),
    each run in chunks that do not divide it, sum to one run over [0, total) in other chunks."""
    from polarcub_amd import construction, mc, sc
    n, K = 12, 2048
    s2 = construction.awgn_sigma2(2.0, K / (1 << n))
    fr = construction.bhattacharyya_frozen(n, K, s2)
    c = sc.CodeSpec.from_frozen_set(1 << n, set(np.nonzero(fr)[0].tolist()), 1, device="cuda")
    total = 8 * 6000 + 5
    one = mc.run_bin(c, 11, 0, total, mc.CHANNEL_AWGN, s2, chunk=16384)
    parts = []
    for r in range(8):
        lo, hi = mc.shard_range(total, r, 8)
        parts.append(mc.run_bin(c, 11, lo, hi - lo, mc.CHANNEL_AWGN, s2, chunk=2500))
    summed = [sum(p[i] for p in parts) for i in range(4)]
    assert summed == one
    assert one[0] == total and 0 < one[1] < total


def test_clean_channels_decode_error_free(code):
    from polarcub_amd import mc
    c, _ = code
    assert mc.run_bin(c, 3, 0, 20000, mc.CHANNEL_BSC, 0.0)[1:3] == [0, 0]
    assert mc.run_bin(c, 3, 0, 20000, mc.CHANNEL_AWGN, 0.05)[1:3] == [0, 0]


def test_norm_rows_high_snr_stay_soft(code):
    """at 20 dB (sigma^2 = 0.01, |2y/s2| around 200) the f32 exp would underflow to exact
    zeros -- hard rows the f64 reference never produces.  Every compact row must be finite and
    non-zero, its log-ratio -ln|r| = |2y/s2| (y = +-1 + sigma z), and its orientation = the sign of y."""
    from polarcub_amd import mc
    c, _ = code
    s2 = 0.01
    info, rows = mc.philox_norm_batch(c, 5, 0, 4096, mc.CHANNEL_AWGN, s2)
    r = rows.abs()
    assert bool(torch.isfinite(rows).all()) and bool((r > 0).all())
    l = -torch.log(r)  # |2y / s2|
    y = l * s2 / 2.0
    assert abs(float(y.mean()) - 1.0) < 0.01  # |y| ~ 1 + sigma z, z ~ N(0, 1): mean 1, sd 0.1
    assert abs(float(y.std()) - 0.1) < 0.01
    assert float(l.max()) > 103.0  # past the f32 exp's underflow point, still soft


def test_norm_rows_channel_law(code):
    """The normalised AWGN rows (53-bit Box-Muller radii) against the pair generator's law: the
    fraction of rows whose orientation disagrees with the sent bit is Q(1/sigma), and z = (|y| - 1) /
    sigma has unit variance with the Gaussian's fourth moment (3)."""
    from polarcub_amd import mc, sc
    c, _ = code
    s2 = 0.5
    B = 1 << 14
    info, rows = mc.philox_norm_batch(c, 9, 0, B, mc.CHANNEL_AWGN, s2)
    x = sc.encode_native(c, info).cpu().numpy().view(np.uint32)
    bits = ((x[:, None, :] >> np.arange(32, dtype=np.uint32)[None, :, None]) & 1).reshape(-1, B)[:c.N]
    v = rows.cpu().numpy()
    y = -np.log(np.abs(v)) * s2 / 2.0 * np.where(np.signbit(v), -1.0, 1.0)  # 2y/s2 = -ln r, signed
    flips = float(np.mean((y < 0) != (bits == 1)))
    q = 0.5 * math.erfc(1.0 / math.sqrt(2.0 * s2))
    n = y.size
    assert abs(flips - q) < 5 * math.sqrt(q * (1 - q) / n)
    z = (y * np.where(bits == 1, -1.0, 1.0) - 1.0) / math.sqrt(s2)
    assert abs(float(z.mean())) < 0.01 and abs(float(z.var()) - 1.0) < 0.01
    assert abs(float(np.mean(z ** 4)) - 3.0) < 0.05


def test_bsc_fer_agrees_with_reference_run():
    """C1 (N=64, K=32, BSC(0.11), the reference's degrade construction): device MC FER vs the
    reference's own 1000-trial FER (tests/golden/bsc_n64.npz), within 4 sigma."""
    from polarcub_amd import mc, sc
    g = load_golden("bsc_n64")
    c = sc.CodeSpec(64, g["frozen"], g["fval"], device="cuda")
    n_cw, fe, _, _ = mc.run_bin(c, 11, 0, 400000, mc.CHANNEL_BSC, 0.11)
    p_dev = fe / n_cw
    p_ref = g["meta"]["frame_errors"] / g["meta"]["trials"]
    sigma = math.sqrt(p_dev * (1 - p_dev) / g["meta"]["trials"])
    assert abs(p_dev - p_ref) <= 4 * sigma + 1e-3, (p_dev, p_ref)


def _x_bits(code, info):
    """x [N, B] u8 of the device encoder for native information words."""
    from polarcub_amd import sc
    xw = sc.encode_native(code, info).cpu().numpy().view(np.uint32)  # [ceil(N/32), B]
    bits = (xw[:, None, :] >> np.arange(32, dtype=np.uint32)[None, :, None]) & 1
    return bits.reshape(-1, xw.shape[1])[:code.N].astype(np.uint8)


def test_awgn_channel_law(code):
    """BI-AWGN pairs: the joint rows are 0.5 N(y; +-1, s2), so y = s2/2 ln(p0/p1) and
    (1 - 2x) y ~ N(1, s2) whatever x; both Box-Muller branches (even / odd elements)
    follow it and are uncorrelated."""
    from polarcub_amd import mc
    c, s2 = code
    info, xy = mc.philox_batch(c, 5, 0, 2048, mc.CHANNEL_AWGN, s2)
    xy = xy.cpu().numpy()
    x = _x_bits(c, info)
    y = 0.5 * s2 * np.log(xy[..., 0] / xy[..., 1])
    z = ((1.0 - 2.0 * x) * y - 1.0) / math.sqrt(s2)  # ~ N(0, 1)
    n = z.size
    assert abs(z.mean()) < 5 / math.sqrt(n)
    assert abs(z.var() - 1.0) < 5 * math.sqrt(2.0 / n)
    for half in (z[0::2], z[1::2]):
        assert abs(half.mean()) < 5 / math.sqrt(half.size)
        assert abs(half.var() - 1.0) < 5 * math.sqrt(2.0 / half.size)
    assert abs(np.mean(z[0::2] * z[1::2])) < 5 / math.sqrt(z[0::2].size)
    # the density constant: p0 + p1 integrates the joint law, p0 = 0.5 phi(y - 1)
    dens = 0.5 / math.sqrt(2 * math.pi * s2) * np.exp(-(y - 1.0) ** 2 / (2 * s2))
    np.testing.assert_allclose(xy[..., 0], dens, rtol=1e-9, atol=1e-300)


def test_bsc_channel_law(code):
    """BSC pairs are makeBSC's rows for y = x ^ flip, flips ~ Bernoulli(p) on both branches."""
    from polarcub_amd import mc
    c, _ = code
    p = 0.11
    info, xy = mc.philox_batch(c, 6, 0, 1024, mc.CHANNEL_BSC, p)
    xy = xy.cpu().numpy()
    x = _x_bits(c, info)
    hi, lo = 0.5 * (1 - p), 0.5 * p
    yb = (xy[..., 0] == lo).astype(np.uint8)
    assert np.all(np.where(yb == 1, xy[..., 1] == hi, (xy[..., 0] == hi) & (xy[..., 1] == lo)))
    flips = yb ^ x
    for half in (flips[0::2], flips[1::2]):
        f = half.mean()
        assert abs(f - p) < 5 * math.sqrt(p * (1 - p) / half.size)


# -- q-ary and deletion inputs keyed by the global codeword index --------------------------------

@pytest.fixture(scope="module")
def qcode():
    from polarcub_amd import sc
    g = load_golden("construct_qary")
    return sc.QaryCode(4, 256, g["qsc4_n8_L64_frozen"].astype(np.uint8), device="cuda")


def test_qsc_batches_keyed_by_global_index(qcode):
    from polarcub_amd import mc
    info_a, xy_a = mc.philox_qsc_batch(qcode, 5, 1000, 300, 0.11)
    info_b, xy_b = mc.philox_qsc_batch(qcode, 5, 1100, 50, 0.11)
    assert torch.equal(info_a[:, 100:150], info_b) and torch.equal(xy_a[:, 100:150], xy_b)
    info_c, _ = mc.philox_qsc_batch(qcode, 6, 1100, 50, 0.11)
    assert not torch.equal(info_b, info_c)


def test_qsc_channel_law(qcode):
    """Symbols uniform on Z_q; a position is in error with probability p, its wrong symbol
    uniform over the q - 1 others; rows are makeQSC's table."""
    from polarcub_amd import mc, sc
    B, p, q = 1 << 14, 0.11, 4
    info, xy = mc.philox_qsc_batch(qcode, 9, 0, B, p)
    counts = torch.bincount(info.reshape(-1).long(), minlength=q).double()
    assert torch.all((counts / counts.sum() - 1 / q).abs() < 5e-3)
    x = sc.encode_qary(qcode, info.t().contiguous()).t()  # [N, B]
    y = xy.argmax(dim=2)
    assert torch.all((xy.max(dim=2).values == 1 - p)) and torch.all(xy.sum(dim=2).sub(1.0).abs() < 1e-12)
    err = (y != x.long())
    rate = err.double().mean().item()
    n = err.numel()
    assert abs(rate - p) < 5 * math.sqrt(p * (1 - p) / n)
    shift = ((y - x.long()) % q)[err]
    sc_ = torch.bincount(shift, minlength=q).double()[1:]
    assert torch.all((sc_ / sc_.sum() - 1 / (q - 1)).abs() < 0.01)


def test_qsc_sharded_counters_match_single_run(qcode):
    """q-ary decode over [0, 2B) in one batch and in two shards: identical frame / symbol errors."""
    from polarcub_amd import mc, sc
    B = 4096
    dec = sc.QaryDecoder(qcode)

    def run(off, b):
        info, xy = mc.philox_qsc_batch(qcode, 21, off, b, 0.11)
        out = dec.decode_native(xy)
        return mc.error_counts(out[0].t(), info.t())
    one = run(0, 2 * B)
    a, b = run(0, B), run(B, B)
    assert one == (a[0] + b[0], a[1] + b[1]) and one[0] > 0


@pytest.fixture(scope="module")
def dcode():
    from polarcub_amd import construction, sc
    N = 256
    fr = construction.bhattacharyya_frozen(8, 64, 0.5)
    return sc.CodeSpec.from_frozen_set(N, set(np.nonzero(fr)[0].tolist()), 200, device="cuda")


def test_deletion_batches_keyed_by_global_index(dcode):
    from polarcub_amd import mc
    ia, ra, la = mc.philox_deletion_batch(dcode, 3, 500, 200, 2, 0.1, 0.1)
    ib, rb, lb = mc.philox_deletion_batch(dcode, 3, 550, 40, 2, 0.1, 0.1)
    assert torch.equal(ia[:, 50:90], ib) and torch.equal(ra[50:90], rb) and torch.equal(la[50:90], lb)


@pytest.mark.parametrize("ones", [0, 2])
def test_deletion_channel_law(dcode, ones):
    """pd = 0 gives the guard-banded codeword itself (Guardbands.addDeletionGuardBands of the
    GPU-encoded word); pd > 0 keeps each symbol with probability 1 - pd."""
    from polarcub_amd import deletion, mc, sc
    B = 2048
    info_w, rx, ln = mc.philox_deletion_batch(dcode, 11, 0, B, 2, 0.1, 0.0, ones)
    x = sc.unpack(sc.encode_native(dcode, info_w), dcode.N).cpu().numpy()
    for b in (0, 1, B - 1):
        want = deletion.addDeletionGuardBands([int(v) for v in x[b]], 8, 2, 0.1, ones)
        assert int(ln[b]) == len(want) and rx[b, :len(want)].cpu().tolist() == list(want)
    pd = 0.1
    _, rx, ln = mc.philox_deletion_batch(dcode, 12, 0, B, 2, 0.1, pd, ones)
    W = rx.shape[1]
    kept = ln.double().sum().item() / (B * W)
    assert abs(kept - (1 - pd)) < 5 * math.sqrt(pd * (1 - pd) / (B * W))
    assert torch.all(rx[torch.arange(W, device="cuda")[None, :] >= ln[:, None]] == 0)


def test_deletion_sharded_counters_match_single_run(dcode):
    from polarcub_amd import mc, sc
    dec = sc.DeletionDecoder(dcode, 2, 0.1)
    B = 2048

    def run(off, b):
        info_w, rx, ln = mc.philox_deletion_batch(dcode, 31, off, b, 2, 0.1, 0.1)
        iw, _ = dec.decode_native(rx, ln)
        return mc.error_counts(sc.unpack(iw, dcode.K), sc.unpack(info_w, dcode.K))
    one = run(0, 2 * B)
    a, b = run(0, B), run(B, B)
    assert one == (a[0] + b[0], a[1] + b[1]) and one[0] > 0


# -- mc_run for q-ary and deletion: the device pipelines count what the composed calls count -------

def test_run_qary_matches_composed_pipeline(qcode):
    """pcub_mc_run_qary over [off, off + B) in chunks = philox_qsc_batch -> QaryDecoder -> symbol
    errors on the same codewords; sharding the range over two calls adds up."""
    from polarcub_amd import mc, sc
    B, off, p = 5000, 700, 0.11
    got = mc.run_qary(qcode, 17, off, B, p, chunk=1536)
    info, xy = mc.philox_qsc_batch(qcode, 17, off, B, p)
    out = sc.QaryDecoder(qcode).decode_native(xy)[0]
    fe, se = mc.error_counts(out.t(), info.t())
    assert got[:3] == [B, fe, se] and fe > 0
    a = mc.run_qary(qcode, 17, off, 2000, p)
    b = mc.run_qary(qcode, 17, off + 2000, B - 2000, p)
    assert [x + y for x, y in zip(a, b)] == got


@pytest.mark.parametrize("n,n0,ones", [(8, 2, 0), (8, 2, 1), (10, 3, 0)])
def test_run_deletion_matches_composed_pipeline(n, n0, ones):
    """pcub_mc_run_deletion = philox_deletion_batch -> DeletionDecoder (table where it has one) ->
    bit errors on the same codewords, for main_deletion's shapes and with guard-band ones."""
    from polarcub_amd import construction, mc, sc
    N = 1 << n
    fr = construction.bhattacharyya_frozen(n, N // 4, 0.5)
    code = sc.CodeSpec.from_frozen_set(N, set(np.nonzero(fr)[0].tolist()), 200, device="cuda")
    dec = sc.DeletionDecoder(code, n0, 0.1, ones)
    B, off = 3000, 123
    tab = dec.table(code.device)
    got = mc.run_deletion(code, 29, off, B, n0, 0.1, 0.1, ones, table=tab, chunk=1024)
    info_w, rx, ln = mc.philox_deletion_batch(code, 29, off, B, n0, 0.1, 0.1, ones)
    iw, _ = dec.decode_native(rx, ln)
    fe, be = mc.error_counts(sc.unpack(iw, code.K), sc.unpack(info_w, code.K))
    assert got[:3] == [B, fe, be] and fe > 0
    if tab is not None:  # the table-less launch decides the same
        assert mc.run_deletion(code, 29, off, B, n0, 0.1, 0.1, ones, table=None) == got


# -- compact normalised rows: the end-to-end pipeline's format ------------------------------------

@pytest.mark.parametrize("n", [4, 6, 8, 10, 11, 12])
def test_compact_decode_matches_pair_decode(n):
    """pcub_sc_decode_bin_compact on compact rows = pcub_sc_decode_bin on the pairs they stand for
    (compact-root kernels at N = 1024, 2048, 4096; expansion into the workspace elsewhere), zeros,
    -0.0, ties (1.0) and a NaN (0, 0) row included."""
    from polarcub_amd import sc
    rng = np.random.default_rng(n)
    N, B = 1 << n, 700
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    frozen[: N // 8] = 1
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    code = sc.CodeSpec(N, frozen, fval, device="cuda")
    r = rng.random((N, B)) ** 3
    r[rng.random((N, B)) < 0.02] = 0.0
    r[rng.random((N, B)) < 0.01] = 1.0
    xc = np.where(rng.random((N, B)) < 0.5, r, -r)
    xc[0, 3] = -0.0
    xc[5, 7] = np.nan
    xct = torch.from_numpy(xc).cuda()
    ab = np.abs(xc)
    pairs = np.where(np.signbit(xc)[..., None], np.stack([ab, np.ones_like(ab)], -1), np.stack([np.ones_like(ab), ab], -1))
    pairs[5, 7] = 0.0
    dec = sc.BinaryDecoder(code)
    i1, x1, _ = dec.decode_compact_native(xct)
    i2, x2, _ = dec.decode_native(torch.from_numpy(pairs).cuda())
    assert torch.equal(i1, i2) and torch.equal(x1, x2)


def test_run_bin_matches_pair_pipeline(code):
    """pcub_mc_run_bin (compact normalised rows -> compact-root decode) counts exactly what the
    pair pipeline counts on the same normalised rows: info -> encode -> pcub_mc_channel_norm (pairs)
    -> pcub_sc_decode_bin -> errors."""
    from polarcub_amd import mc, sc
    c, s2 = code
    B = 5000
    for ch, param in ((mc.CHANNEL_AWGN, s2), (mc.CHANNEL_BSC, 0.11)):
        got = mc.run_bin(c, 44, 1000, B, ch, param, chunk=2048)
        info, pairs = mc.philox_norm_batch(c, 44, 1000, B, ch, param, compact=False)
        iw, _, _ = sc.BinaryDecoder(c).decode_native(pairs)
        fe, be = mc.error_counts(sc.unpack(iw, c.K), sc.unpack(info, c.K))
        assert got[:3] == [B, fe, be] and fe > 0
        _, xc = mc.philox_norm_batch(c, 44, 1000, B, ch, param, compact=True)
        ab = xc.abs()
        assert torch.equal(torch.where(torch.signbit(xc), ab, torch.ones_like(ab)), pairs[..., 0])
        assert torch.equal(torch.where(torch.signbit(xc), torch.ones_like(ab), ab), pairs[..., 1])


@pytest.mark.parametrize("n", [5, 15])
def test_run_bin_without_a_compact_kernel(n):
    """Code lengths whose variant has no compact-root twin (n <= 5, n >= 15): the pipeline
    generates normalised pairs and decodes them with pcub_sc_decode_bin (no expansion buffer), and
    counts exactly what the pair pipeline does on the same rows."""
    from polarcub_amd import _lib, construction, mc, sc
    assert _lib.lib().pcub_sc_decode_bin_compact_direct(n) == 0
    N = 1 << n
    s2 = construction.awgn_sigma2(1.0, 0.5)
    fr = construction.bhattacharyya_frozen(n, N // 2, s2)
    c = sc.CodeSpec.from_frozen_set(N, set(np.nonzero(fr)[0].tolist()), 1, device="cuda")
    B = 700 if n == 15 else 5000
    got = mc.run_bin(c, 45, 300, B, mc.CHANNEL_AWGN, s2, chunk=256)
    info, pairs = mc.philox_norm_batch(c, 45, 300, B, mc.CHANNEL_AWGN, s2, compact=False)
    iw, _, _ = sc.BinaryDecoder(c).decode_native(pairs)
    fe, be = mc.error_counts(sc.unpack(iw, c.K), sc.unpack(info, c.K))
    assert got[:3] == [B, fe, be] and be > 0


def test_normalised_awgn_rows_follow_the_channel_law(code):
    """The normalised BI-AWGN row of y is (1, exp(-2y/s2)) or (exp(2y/s2), 1): the implied
    (1 - 2x) y ~ N(1, s2)."""
    from polarcub_amd import mc
    c, s2 = code
    info, xc = mc.philox_norm_batch(c, 5, 0, 2048, mc.CHANNEL_AWGN, s2)
    x = _x_bits(c, info)
    v = xc.cpu().numpy()
    y = np.where(np.signbit(v), 1.0, -1.0) * np.log(np.abs(v)) * s2 / 2.0
    z = ((1.0 - 2.0 * x) * y - 1.0) / math.sqrt(s2)
    fin = np.isfinite(z)
    assert fin.mean() > 0.999
    z = z[fin]
    assert abs(z.mean()) < 5 / math.sqrt(z.size) and abs(z.var() - 1.0) < 5 * math.sqrt(2.0 / z.size)
