"""Deletion-channel SC decode on the GPU (pcub_sc_decode_deletion) against the
reference's golden vectors and the CPU oracle: info bits and x_hat bit-exact."""
import contextlib
import io
import random

import numpy as np
import pytest
import torch

from oracle import trellis_oracle as tro
from tests.conftest import load_golden
from tests.test_trellis_oracle import deletion_edge_cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sc():
    from polarcub_amd import _lib, sc as m
    _lib.lib()
    return m


def _dec(sc, n, n0, pd, frozen, fval, rx, rx_len, ones=0):
    code = sc.CodeSpec(1 << n, frozen, fval, device="cuda")
    d = sc.DeletionDecoder(code, n0, pd, ones)
    info, xhat = d.decode(torch.from_numpy(np.ascontiguousarray(rx, np.uint8)).cuda(),
                          torch.from_numpy(np.asarray(rx_len, np.int32)).cuda())
    torch.cuda.synchronize()
    return info.cpu().numpy(), xhat.cpu().numpy()


def test_c5_golden(sc):
    g = load_golden("deletion_n8")
    m = g["meta"]
    info, xhat = _dec(sc, m["n"], m["n0"], m["pd"], g["frozen"], g["fval"], g["rx"], g["rx_len"])
    assert np.array_equal(info, g["info"])
    assert np.array_equal(xhat, g["xhat"])


@pytest.mark.parametrize("idx", range(11))
def test_edge_golden(sc, idx):
    c = deletion_edge_cases()[idx]
    n, n0, ones = (int(v) for v in c["shape"])
    assert sc.deletion_supported(n, n0, ones)  # every golden shape (n0 = 4, guard-band ones) has a kernel
    info, xhat = _dec(sc, n, n0, float(c["pd"][0]), c["frozen"], c["fval"], c["rx"], c["rx_len"], ones)
    assert np.array_equal(info, c["info"])
    assert np.array_equal(xhat, c["xhat"])


SHAPES = ([(n0, n0 + tb, 0) for n0 in (1, 2, 3) for tb in range(1, 9)] + [(4, 4 + tb, 0) for tb in (1, 3, 5, 7, 8)]
          + [(n0, n0 + tb, ones) for n0, tb, ones in ((1, 2, 1), (2, 3, 2), (3, 4, 3), (2, 7, 1), (4, 2, 2), (3, 8, 1))])


@pytest.mark.parametrize("n0,n,ones", SHAPES)
def test_random_vs_oracle(sc, n0, n, ones):
    """Every kernel shape (2 .. 256 trellises of 2 .. 16 inputs, with and without
    guard-band ones): channel outputs at several deletion rates plus adversarial words,
    random frozen sets (incl. all-frozen and all-information windows) vs the oracle."""
    N = 1 << n
    rng = np.random.default_rng(1000 * n0 + 10 * n + ones)
    prng = random.Random(n + 100 * ones)
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    frozen[: N // 4] = 1
    frozen[-(N // 8) or -1:] = 0
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    pd = [0.05, 0.1, 0.3][n % 3]
    words = []
    ntx = 10 if n <= 9 else 4
    for t in range(ntx):
        x = [int(b) for b in rng.integers(0, 2, N)]
        cw = tro.add_guard_bands(x, n, n0, 0.1, ones)
        words.append(tro.deletion_channel(cw, pd if t < ntx - 2 else 0.6, prng))
    words += [[], [1], [0] * 9, [int(b) for b in rng.integers(0, 2, 3 * N)]]
    W = max(len(w) for w in words)
    rx = np.zeros((len(words), W), np.uint8)
    for i, w in enumerate(words):
        rx[i, :len(w)] = w
    info, xhat = _dec(sc, n, n0, pd, frozen, fval, rx, [len(w) for w in words], ones)
    for i, w in enumerate(words):
        x_ref, i_ref = tro.decode_deletion(w, n, n0, pd, frozen, fval, ones=ones)
        assert list(info[i]) == i_ref, (i, w)
        assert list(xhat[i]) == x_ref, (i, w)


@pytest.mark.parametrize("n", [13, 14])
def test_wide_shapes_vs_c_oracle(sc, n):
    """main_deletion's n0 = n // 3 at n = 13, 14: 512 / 1024 trellises of 16 inputs, one codeword a
    workgroup of T threads.  Channel outputs at pd 0.1 and 0.3, an empty, a one-symbol and an
    all-zeros word and a random overlong one, random frozen set, against the C oracle
    (oracle/trellis_oracle.c, pinned to the reference's goldens and the Python oracle)."""
    from oracle import orc
    n0 = 4
    assert sc.deletion_supported(n, n0, 0)
    N = 1 << n
    rng = np.random.default_rng(77 + n)
    prng = random.Random(n)
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    frozen[: N // 4] = 1
    frozen[-(N // 8):] = 0
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    pd = 0.1
    words = []
    for t in range(3):
        x = [int(b) for b in rng.integers(0, 2, N)]
        cw = tro.add_guard_bands(x, n, n0, 0.1, 0)
        words.append(tro.deletion_channel(cw, 0.1 if t < 2 else 0.3, prng))
    words += [[], [1], [0] * 9, [int(b) for b in rng.integers(0, 2, 2 * N)]]
    W = max(len(w) for w in words)
    rx = np.zeros((len(words), W), np.uint8)
    for i, w in enumerate(words):
        rx[i, :len(w)] = w
    ln = np.array([len(w) for w in words], np.int32)
    info, xhat = _dec(sc, n, n0, pd, frozen, fval, rx, ln)
    i_ref, x_ref = orc.decode_deletion(rx, ln, n, n0, pd, frozen, fval)
    assert np.array_equal(info, i_ref)
    assert np.array_equal(xhat, x_ref)


@pytest.mark.parametrize("n", [10, 11, 12, 13, 14])
def test_wave_kernel_matches_lane_kernel(sc, n):
    """n0 = 4 (main_deletion's n0 = n // 3 at n = 12 .. 14): the wave-per-task kernel
    (sc_del_w4.hip, trellis_wave.h) against the lane-per-trellis kernel k_sc_del and the C oracle
    (oracle/trellis_oracle.c): channel outputs at pd 0.05 .. 0.4 (segments from 0 to 16 symbols and
    overlong ones), an empty, a one-symbol, an all-zeros and an overlong random word, a frozen set
    with rate-0 depth-3 nodes (their tasks skipped) and one with none.  Bit-exact."""
    from oracle import orc
    n0 = 4
    N = 1 << n
    rng = np.random.default_rng(500 + n)
    prng = random.Random(900 + n)
    for fs in range(2):
        if fs == 0:
            frozen = (rng.random(N) < 0.5).astype(np.uint8)
            frozen[: N // 4] = 1  # the first four collapse points' nodes are rate-0
        else:
            frozen = (rng.random(N) < 0.3).astype(np.uint8)
            frozen[:: N // 16] = 0  # no rate-0 node
        fval = (rng.random(N) < 0.5).astype(np.uint8)
        pd = (0.05, 0.1, 0.25, 0.4)[(n + fs) % 4]
        words = []
        for t in range(6):
            x = [int(b) for b in rng.integers(0, 2, N)]
            cw = tro.add_guard_bands(x, n, n0, 0.1, 0)
            words.append(tro.deletion_channel(cw, (0.05, 0.1, 0.2, 0.3, 0.4, 0.1)[t], prng))
        words += [[], [1], [0] * 9, [int(b) for b in rng.integers(0, 2, N + N // 2)]]
        W = max(len(w) for w in words)
        rx = np.zeros((len(words), W), np.uint8)
        for i, w in enumerate(words):
            rx[i, :len(w)] = w
        ln = np.array([len(w) for w in words], np.int32)
        old = sc.set_deletion_wave(2)  # the wave kernel at every size
        try:
            info_w, xhat_w = _dec(sc, n, n0, pd, frozen, fval, rx, ln)
            sc.set_deletion_wave(0)
            info_l, xhat_l = _dec(sc, n, n0, pd, frozen, fval, rx, ln)
        finally:
            sc.set_deletion_wave(old)
        assert np.array_equal(info_w, info_l), (n, fs)
        assert np.array_equal(xhat_w, xhat_l), (n, fs)
        if n <= 12:
            i_ref, x_ref = orc.decode_deletion(rx, ln, n, n0, pd, frozen, fval)
            assert np.array_equal(info_w, i_ref), (n, fs)
            assert np.array_equal(xhat_w, x_ref), (n, fs)


def test_ragged_batches_match_single(sc):
    """A large batch (padding groups in the last workgroup) equals per-codeword results."""
    g = load_golden("deletion_n8")
    m = g["meta"]
    reps = np.concatenate([np.arange(g["rx"].shape[0])] * 7)[:301]
    info, xhat = _dec(sc, m["n"], m["n0"], m["pd"], g["frozen"], g["fval"], g["rx"][reps], g["rx_len"][reps])
    assert np.array_equal(info, g["info"][reps])
    assert np.array_equal(xhat, g["xhat"][reps])


def test_facade_dispatch_and_mc_line():
    """BinaryPolarEncoderDecoder.decode on a received-word collection runs the kernel (the
    trellises are never built on the host) and encodeDecodeSimulation with the
    main_deletion.py closures prints the reference's line."""
    from polarcub_amd import coding, deletion, vectors
    g = load_golden("deletion_n8")
    m = g["meta"]
    n, n0, pd, xi = m["n"], m["n0"], m["pd"], m["xi"]
    N = 1 << n
    enc = coding.BinaryPolarEncoderDecoder(N, set(int(i) for i in np.nonzero(g["frozen"])[0]), m["crs"])
    xvd = vectors.BinaryMemorylessVectorDistribution(N)
    xvd.probs[:] = 0.5
    for t in range(4):
        w = list(map(int, g["rx"][t, :g["rx_len"][t]]))
        coll = deletion.buildCollectionOfBinaryTrellises_uniformInput_deletion(w, pd, xi, n, n0, 0)
        x, info = enc.decode(xvd, coll)
        assert coll._lazy is not None, "host trellises were built: the kernel path did not run"
        assert np.array_equal(info, g["info"][t]) and np.array_equal(x, g["xhat"][t])

    frozen = set(int(i) for i in np.nonzero(g["genie_frozen"])[0])
    crng = random.Random()
    crng.seed(m["channel_seed"])

    def make_x():
        v = vectors.BinaryMemorylessVectorDistribution(N)
        v.probs[:] = 0.5
        return v

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        coding.encodeDecodeSimulation(
            N, make_x, lambda e: deletion.addDeletionGuardBands(e, n, n0, xi, 0),
            lambda c: deletion.deletionChannelSimulation(c, pd, None, crng),
            lambda r: deletion.buildCollectionOfBinaryTrellises_uniformInput_deletion(r, pd, xi, n, n0, 0),
            m["mc_trials"], frozen, commonRandomnessSeed=m["crs"], randomInformationSeed=m["info_seed"])
    assert buf.getvalue().strip().splitlines()[-1] == m["line"]


@pytest.mark.parametrize("n", [5, 10, 11])
def test_n03_table_paths_agree(sc, n):
    """n0 = 3: the segment-state table (pcub_sc_deletion_build_table, the table-driven layout), the
    per-lane trellis levels (no table), a table built for another pd and an n0 = 2 table's buffer
    (both rejected by the kernel's header check: the gated fallback decodes without them) decode
    identically, and agree with the oracle."""
    n0, pd = 3, 0.1
    N = 1 << n
    rng = np.random.default_rng(31 + n)
    prng = random.Random(n)
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    words = [tro.deletion_channel([int(b) for b in rng.integers(0, 2, N)], pd, prng) for _ in range(40)]
    words += [[], [0] * 7, [1] * (N + 9)]
    rxt, ln = sc.pad_words(words)
    code = sc.CodeSpec(N, frozen, fval, device="cuda")
    outs = []
    for mode in ("table", "plain", "stale", "n02"):
        d = sc.DeletionDecoder(code, n0, pd, use_table=(mode != "plain"))
        if mode == "stale":
            d._tables[str(rxt.device)] = sc.DeletionDecoder(code, n0, 0.2).table(rxt.device)
        if mode == "n02":  # an n0 = 2 table for this very pd: its header says n0 = 2
            d._tables[str(rxt.device)] = sc.DeletionDecoder(
                sc.CodeSpec(256, np.ones(256, np.uint8), np.zeros(256, np.uint8), device="cuda"), 2, pd).table(rxt.device)
        if mode == "table":
            tab = d.table(rxt.device).cpu().numpy()
            assert tab.shape == (8 + 512 * 256,) and tab[1] == 3.0 and tab[2] == pd
        info, xhat = d.decode(rxt, ln)
        outs.append((info.cpu().numpy(), xhat.cpu().numpy()))
    for o in outs[1:]:
        assert np.array_equal(o[0], outs[0][0]) and np.array_equal(o[1], outs[0][1])
    for i in list(range(0, len(words), 7)) + [len(words) - 1]:
        x_ref, i_ref = tro.decode_deletion(words[i], n, n0, pd, frozen, fval)
        assert list(outs[0][0][i]) == i_ref and list(outs[0][1][i]) == x_ref, i


def test_n02_foreign_tables_rejected(sc):
    """n0 = 2 given an n0 = 3 table (for this pd) or an n0 = 2 table for another pd: the header check
    rejects both and the gated fallback (the table-driven kernel building its own table) decodes
    exactly as the table-less path."""
    n, n0, pd = 8, 2, 0.1
    N = 1 << n
    rng = np.random.default_rng(5)
    prng = random.Random(5)
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    words = [tro.deletion_channel(tro.add_guard_bands([int(b) for b in rng.integers(0, 2, N)], n, n0, 0.1, 0), pd,
                                  prng) for _ in range(300)]
    rxt, ln = sc.pad_words(words)
    code = sc.CodeSpec(N, frozen, fval, device="cuda")
    ref = sc.DeletionDecoder(code, n0, pd, use_table=False).decode(rxt, ln)
    for other in (sc.DeletionDecoder(sc.CodeSpec(1024, np.ones(1024, np.uint8), np.zeros(1024, np.uint8), device="cuda"),
                                     3, pd), sc.DeletionDecoder(code, n0, 0.3)):
        d = sc.DeletionDecoder(code, n0, pd)
        d._tables[str(rxt.device)] = other.table(rxt.device)
        assert d.dense_layout(rxt.shape[1], rxt.device)
        info, xhat = d.decode(rxt, ln)
        assert np.array_equal(info.cpu().numpy(), ref[0].cpu().numpy())
        assert np.array_equal(xhat.cpu().numpy(), ref[1].cpu().numpy())


@pytest.mark.parametrize("n0,n", [(2, 6), (2, 8), (2, 9), (2, 10), (3, 7), (3, 9), (3, 10), (3, 11)])
def test_dense_layout_matches_lane_layout(sc, n0, n):
    """The table-driven layout (16 lanes a codeword, sc_del_dense.h; with and without a built table)
    and k_sc_del's lane-per-trellis layout decode identically (a ragged batch: padding codewords in the last workgroup), and
    agree with the oracle on a sample."""
    N = 1 << n
    pd = 0.1
    rng = np.random.default_rng(7 * n + n0)
    prng = random.Random(3 * n + n0)
    frozen = (rng.random(N) < 0.6).astype(np.uint8)
    frozen[: N // 8] = 1
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    words = []
    for _ in range(37):
        x = [int(b) for b in rng.integers(0, 2, N)]
        words.append(tro.deletion_channel(tro.add_guard_bands(x, n, n0, 0.1, 0), pd, prng))
    words += [[], [1], [0] * 5, [int(b) for b in rng.integers(0, 2, 2 * N)]]
    rxt, ln = sc.pad_words(words)
    code = sc.CodeSpec(N, frozen, fval, device="cuda")
    outs = []
    # table-driven with a built table, table-driven without one (n0 = 2 builds it per workgroup,
    # n0 = 3 falls back to k_sc_del), and the lane layout
    for dense, use_table in ((True, True), (True, False), (False, True)):
        d = sc.DeletionDecoder(code, n0, pd, use_table=use_table)
        prev = sc.set_deletion_dense(dense)
        try:
            if dense and use_table:
                assert d.dense_layout(rxt.shape[1], rxt.device)
            info, xhat = d.decode(rxt, ln)
            torch.cuda.synchronize()
        finally:
            sc.set_deletion_dense(prev)
        outs.append((info.cpu().numpy(), xhat.cpu().numpy()))
    for o in outs[1:]:
        assert np.array_equal(outs[0][0], o[0]) and np.array_equal(outs[0][1], o[1])
    for i in list(range(0, len(words), 9)) + [len(words) - 3, len(words) - 1]:
        x_ref, i_ref = tro.decode_deletion(words[i], n, n0, pd, frozen, fval)
        assert list(outs[0][0][i]) == i_ref and list(outs[0][1][i]) == x_ref, i


@pytest.mark.parametrize("n0,n", [(2, 8), (2, 10), (3, 10), (3, 11)])
def test_dense_staging_any_stride(sc, n0, n):
    """The table-driven kernel stages its group's received rows into LDS in chunks of R rows, each
    from the 16-byte boundary below its first byte (sc_del_dense.h): widening the rows by zero
    columns (strides that move every chunk's start off the boundary, and R with them) and a batch
    base off 16 bytes (no staging: pack_rows) decode identically."""
    N = 1 << n
    rng = np.random.default_rng(11 * n + n0)
    prng = random.Random(5 * n + n0)
    frozen = (rng.random(N) < 0.55).astype(np.uint8)
    frozen[: N // 8] = 1
    fval = np.zeros(N, np.uint8)
    words = [tro.deletion_channel(tro.add_guard_bands([int(b) for b in rng.integers(0, 2, N)], n, n0, 0.1, 0), 0.1, prng)
             for _ in range(45)]
    rxt, ln = sc.pad_words(words)
    d = sc.DeletionDecoder(sc.CodeSpec(N, frozen, fval, device="cuda"), n0, 0.1)
    assert d.dense_layout(rxt.shape[1], rxt.device)
    ref = [t.cpu().numpy() for t in d.decode(rxt, ln)]
    for extra in (1, 5, 13, 16 * 16 + 3):
        wide = torch.cat([rxt, torch.zeros(rxt.shape[0], extra, dtype=rxt.dtype, device=rxt.device)], 1).contiguous()
        out = [t.cpu().numpy() for t in d.decode(wide, ln)]
        assert np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]), extra
    buf = torch.zeros(rxt.numel() + 16, dtype=rxt.dtype, device=rxt.device)
    off = buf[3: 3 + rxt.numel()].view(rxt.shape)
    off.copy_(rxt)
    out = [t.cpu().numpy() for t in d.decode(off, ln)]
    assert np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1])
    for i in (0, 22, 44):
        x_ref, i_ref = tro.decode_deletion(words[i], n, n0, 0.1, frozen, fval)
        assert list(ref[0][i]) == i_ref and list(ref[1][i]) == x_ref, i


@pytest.mark.parametrize("n0,n", [(2, 6), (2, 7), (2, 8), (3, 7), (3, 8), (3, 9)])
def test_dense_layout_lanes(sc, n0, n):
    """The table-driven layout with 16, 8 (the default up to 64 trellises) and 4 lanes a codeword
    (pcub_sc_set_deletion_lanes: four, three and two cross-lane subtree levels), and 8 without the
    rate-1 shortcut (pcub_sc_set_deletion_rate1), decodes identically:
    ragged batch, the n0 = 2 table built per workgroup and given, n0 = 3 with its table; and agrees
    with the oracle on a sample."""
    N = 1 << n
    pd = 0.1
    rng = np.random.default_rng(5 * n + n0)
    prng = random.Random(9 * n + n0)
    frozen = (rng.random(N) < 0.5).astype(np.uint8)
    frozen[: N // 8] = 1
    fval = (rng.random(N) < 0.5).astype(np.uint8)
    words = [tro.deletion_channel(tro.add_guard_bands([int(b) for b in rng.integers(0, 2, N)], n, n0, 0.1, 0), pd, prng)
             for _ in range(75)]
    words += [[], [1], [0] * 5, [int(b) for b in rng.integers(0, 2, 2 * N)]]
    rxt, ln = sc.pad_words(words)
    code = sc.CodeSpec(N, frozen, fval, device="cuda")
    for use_table in ((True, False) if n0 == 2 else (True,)):
        d = sc.DeletionDecoder(code, n0, pd, use_table=use_table)
        outs = []
        for g, r1 in ((16, 1), (8, 1), (4, 1), (8, 0)):
            prev = sc.set_deletion_lanes(g)
            prev_r1 = sc.set_deletion_rate1(r1)  # 0: the 8-lane subtrees without the rate-1 shortcut
            try:
                info, xhat = d.decode(rxt, ln)
                torch.cuda.synchronize()
            finally:
                sc.set_deletion_lanes(prev)
                sc.set_deletion_rate1(prev_r1)
            outs.append((info.cpu().numpy(), xhat.cpu().numpy()))
        for o in outs[1:]:
            assert np.array_equal(outs[0][0], o[0]) and np.array_equal(outs[0][1], o[1]), use_table
    for i in (0, 40, len(words) - 3, len(words) - 1):
        x_ref, i_ref = tro.decode_deletion(words[i], n, n0, pd, frozen, fval)
        assert list(outs[1][0][i]) == i_ref and list(outs[1][1][i]) == x_ref, i
