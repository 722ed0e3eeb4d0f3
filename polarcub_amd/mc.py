"""Monte-Carlo batches and the multi-GPU plumbing around the decoder.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on ROCm,
"gloo" for CPU tests).  Codewords are independent and SC is sequential within a
codeword, so a Monte-Carlo run shards by codeword: rank r owns its own batch and
the only collective is one all_reduce of the int64 counters {codewords, frame
errors, bit errors, symbol errors} plus a max-reduce of the elapsed time.  There is
no data-path collective because none is needed.

The batch generators below produce synthetic channel outputs on the device
(torch Philox): random information -> GPU polar encoder -> channel.
"""
import os

import torch
import torch.distributed as dist

from . import channel, sc


def dist_env():
    """(world_size, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_seed(seed, rank):
    """Generator seed of rank r's shard (distinct streams per rank)."""
    return int(seed) + 7919 * int(rank)


def shard_range(total, rank, world):
    """Rank r's slice [lo, hi) of `total` codewords: contiguous, sizes differ by at most one."""
    lo = (total * rank) // world
    hi = (total * (rank + 1)) // world
    return lo, hi


def rank_offset(rank, batch):
    """First global codeword index of rank r under weak scaling (every rank owns `batch`
    codewords: [r*batch, (r+1)*batch)); the Philox streams are keyed by this index, so the
    union over ranks is the single-process run over [0, world*batch)."""
    return int(rank) * int(batch)


def gather_floats(values, device=None):
    """all_gather of one small float vector per rank -> [world][len] list (identity when not
    distributed)."""
    v = torch.tensor([float(x) for x in values], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        out = [torch.empty_like(v) for _ in range(dist.get_world_size())]
        dist.all_gather(out, v)
        return [o.tolist() for o in out]
    return [v.tolist()]


def reduce_counters(counters, elapsed, device=None):
    """Sum the int64 counters and max the elapsed time over all ranks (no-op when not
    distributed).  device: where the collective's tensors live (a CUDA device for RCCL,
    None = CPU for gloo).  Returns (list of ints, float)."""
    c = torch.tensor([int(v) for v in counters], dtype=torch.int64, device=device)
    e = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return [int(v) for v in c.tolist()], float(e.item())


def error_counts(decoded, sent):
    """(frame errors, bit/symbol errors) between [B, K] decoded and sent information."""
    if decoded.shape[1] == 0:
        return 0, 0
    diff = decoded != sent
    return int(diff.any(dim=1).sum().item()), int(diff.sum().item())


def awgn_batch(code, B, sigma2, generator, chunk=1 << 18):
    """Uniform information -> GPU encoder -> BI-AWGN joint pairs, native [N, B, 2] layout.
    Returns (xy, info [B, K] uint8)."""
    dev = code.device
    xy = torch.empty((code.N, B, 2), dtype=torch.float64, device=dev)
    info = torch.empty((B, code.K), dtype=torch.uint8, device=dev)
    for b0 in range(0, B, chunk):
        b1 = min(B, b0 + chunk)
        inf = torch.randint(0, 2, (b1 - b0, code.K), dtype=torch.uint8, device=dev, generator=generator)
        info[b0:b1] = inf
        xw = sc.encode_native(code, sc.pack(inf))
        channel.awgn_pairs_native(channel.bits_from_words(xw, code.N), sigma2, generator=generator,
                                  out=xy[:, b0:b1, :])
    return xy, info


def deletion_batch(code, B, n0, xi, pd, generator, chunk=1 << 17, ones=0):
    """Uniform information -> GPU encoder -> guard bands -> deletion channel.
    Returns (rx [B, W] uint8, rx_len [B] int32, info [B, K] uint8)."""
    dev = code.device
    rxs, lens, infos = [], [], []
    for b0 in range(0, B, chunk):
        b1 = min(B, b0 + chunk)
        inf = torch.randint(0, 2, (b1 - b0, code.K), dtype=torch.uint8, device=dev, generator=generator)
        x = sc.encode(code, inf)
        rx, ln = channel.deletion_words(x, code.n, n0, xi, pd, generator=generator, ones=ones)
        rxs.append(rx)
        lens.append(ln)
        infos.append(inf)
    return torch.cat(rxs), torch.cat(lens), torch.cat(infos)


def qsc_batch(code, B, p, generator, chunk=1 << 16):
    """Uniform q-ary information -> GPU q-ary encoder -> QSC(p) joint rows, native [N, B, q].
    Returns (xy, info [B, K] uint8)."""
    dev = code.device
    xy = torch.empty((code.N, B, code.q), dtype=torch.float64, device=dev)
    info = torch.empty((B, code.K), dtype=torch.uint8, device=dev)
    for b0 in range(0, B, chunk):
        b1 = min(B, b0 + chunk)
        inf = torch.randint(0, code.q, (b1 - b0, code.K), dtype=torch.uint8, device=dev, generator=generator)
        info[b0:b1] = inf
        x = sc.encode_qary(code, inf)  # [b, N]
        xy[:, b0:b1, :] = channel.qsc_pairs_native(x.t(), code.q, p, generator=generator)
    return xy, info


# ----------------------------------------------------------------------------- device Monte-Carlo (Philox)
# Codeword g's information bits and channel draws are keyed by (seed, g): a batch
# [offset, offset + B) is identical whichever rank / chunk generates it.

CHANNEL_AWGN, CHANNEL_BSC = 0, 1


def philox_batch(code, seed, offset, B, channel, param, tile=0):
    """Information words [ceil(K/32), B] and channel pairs for global codewords [offset, offset + B)
    (pcub_mc_info -> pcub_polar_encode_bin -> pcub_mc_channel): [N, B, 2], or with tile = T > 0 the
    tiled layout [ceil(B/T), N, T, 2] (BinaryDecoder.decode_tiled_native; padding columns zero)."""
    from . import _lib
    L = _lib.lib()
    dev = code.device
    info = torch.zeros((max(1, code.info_words), B), dtype=torch.int32, device=dev)
    _lib.check(L.pcub_mc_info(int(seed), int(offset), B, code.K, sc._p(info), sc._stream()), "pcub_mc_info")
    x = sc.encode_native(code, info)
    if tile:
        xy = torch.zeros(((B + tile - 1) // tile, code.N, tile, 2), dtype=torch.float64, device=dev)
    else:
        xy = torch.empty((code.N, B, 2), dtype=torch.float64, device=dev)
    _lib.check(L.pcub_mc_channel_tiled(int(seed), int(offset), B, code.n, int(channel), float(param), sc._p(x),
                                       sc._p(xy), int(tile), sc._stream()), "pcub_mc_channel_tiled")
    return info, xy


def philox_norm_batch(code, seed, offset, B, channel, param, compact=True):
    """Information words and the normalised channel rows of global codewords [offset, offset + B)
    (pcub_mc_channel_norm: four elements a Philox counter, f32 row arithmetic, each row divided by its
    larger entry — the channel law of philox_batch, not its draws):
    compact [N, B] float64, or the pairs they stand for [N, B, 2]."""
    from . import _lib
    L = _lib.lib()
    dev = code.device
    info = torch.zeros((max(1, code.info_words), B), dtype=torch.int32, device=dev)
    _lib.check(L.pcub_mc_info(int(seed), int(offset), B, code.K, sc._p(info), sc._stream()), "pcub_mc_info")
    x = sc.encode_native(code, info)
    shape = (code.N, B) if compact else (code.N, B, 2)
    out = torch.empty(shape, dtype=torch.float64, device=dev)
    _lib.check(L.pcub_mc_channel_norm(int(seed), int(offset), B, code.n, int(channel), float(param), sc._p(x),
                                      sc._p(out), 1 if compact else 0, sc._stream()), "pcub_mc_channel_norm")
    return info, out


def run_bin(code, seed, offset, count, channel, param, chunk=1 << 18):
    """encodeDecodeSimulation as one device pipeline (pcub_mc_run_bin: normalised channel rows in
    compact form into the compact-root decode) over global codewords [offset, offset + count);
    returns [codewords, frame errors, bit errors, 0]."""
    from . import _lib
    L = _lib.lib()
    chunk = int(max(1, min(chunk, count)))
    need = int(L.pcub_mc_run_bin_workspace(chunk, code.n, code.K))
    ws = torch.empty(max(need, 16), dtype=torch.uint8, device=code.device)
    counters = torch.zeros(4, dtype=torch.int64, device=code.device)
    rc = L.pcub_mc_run_bin(int(seed), int(offset), int(count), code.n, int(channel), float(param),
                           sc._p(code.fmask_dev), sc._p(code.fval_dev), code.K, chunk, sc._p(counters), sc._p(ws),
                           ws.numel(), sc._stream())
    _lib.check(rc, "pcub_mc_run_bin")
    return [int(v) for v in counters.tolist()]


def run_qary(code, seed, offset, count, p, chunk=1 << 18):
    """QaryPolarEncoderDecoder's QSC trial loop as one device pipeline (pcub_mc_run_qary: the
    philox_qsc_batch generators, the tiled decode, symbol-error counting) over global codewords
    [offset, offset + count); returns [codewords, frame errors, symbol errors, 0]."""
    from . import _lib
    L = _lib.lib()
    chunk = int(max(1, min(chunk, count)))
    need = int(L.pcub_mc_run_qary_workspace(chunk, code.n, code.q, code.K))
    if need == 0:
        raise ValueError("pcub_mc_run_qary: no decode kernel for q=%d N=%d" % (code.q, code.N))
    ws = torch.empty(need, dtype=torch.uint8, device=code.device)
    counters = torch.zeros(4, dtype=torch.int64, device=code.device)
    _lib.check(L.pcub_mc_run_qary(int(seed), int(offset), int(count), code.n, code.q, float(p), sc._p(code.frozen_dev),
                                  code.K, chunk, sc._p(counters), sc._p(ws), ws.numel(), sc._stream()),
               "pcub_mc_run_qary")
    return [int(v) for v in counters.tolist()]


def run_deletion(code, seed, offset, count, n0, xi, pd, ones=0, table=None, chunk=1 << 18):
    """main_deletion's trial loop as one device pipeline (pcub_mc_run_deletion: the
    philox_deletion_batch generators, the deletion decode with trellises built for pd, bit-error
    counting) over global codewords [offset, offset + count); returns [codewords, frame errors,
    bit errors, 0]."""
    from . import _lib
    L = _lib.lib()
    t = guard_template(code.n, n0, xi, ones, code.device)
    W = int(t.numel())
    chunk = int(max(1, min(chunk, count)))
    need = int(L.pcub_mc_run_deletion_workspace(chunk, code.n, W, code.K))
    ws = torch.empty(max(need, 16), dtype=torch.uint8, device=code.device)
    counters = torch.zeros(4, dtype=torch.int64, device=code.device)
    _lib.check(L.pcub_mc_run_deletion(int(seed), int(offset), int(count), code.n, int(n0), sc._p(t), W, int(ones),
                                      float(pd), sc._p(code.fmask_dev), sc._p(code.fval_dev), code.K,
                                      sc._p(table) if table is not None else None, chunk, sc._p(counters), sc._p(ws),
                                      ws.numel(), sc._stream()), "pcub_mc_run_deletion")
    return [int(v) for v in counters.tolist()]


def philox_qsc_batch(code, seed, offset, B, p, tile=0):
    """q-ary information [K, B] u8 and QSC(p) joint rows [N, B, q] for global codewords
    [offset, offset + B) (pcub_mc_info_qary -> pcub_polar_encode_qary -> pcub_mc_channel_qsc);
    the same codewords whichever rank or chunk generates them.  tile = T > 0: the rows in the tiled
    layout [ceil(B/T), N, T, q] (QaryDecoder.decode_tiled_native)."""
    from . import _lib
    L = _lib.lib()
    dev = code.device
    info = torch.zeros((max(1, code.K), B), dtype=torch.uint8, device=dev)
    _lib.check(L.pcub_mc_info_qary(int(seed), int(offset), B, code.K, code.q, sc._p(info), sc._stream()),
               "pcub_mc_info_qary")
    x = torch.empty((code.N, B), dtype=torch.uint8, device=dev)
    _lib.check(L.pcub_polar_encode_qary(sc._p(info), B, code.n, code.q, sc._p(code.frozen_dev), code.K, sc._p(x),
                                        sc._stream()), "pcub_polar_encode_qary")
    if tile:
        xy = torch.zeros(((B + tile - 1) // tile, code.N, tile, code.q), dtype=torch.float64, device=dev)
    else:
        xy = torch.empty((code.N, B, code.q), dtype=torch.float64, device=dev)
    _lib.check(L.pcub_mc_channel_qsc_tiled(int(seed), int(offset), B, code.n, code.q, float(p), sc._p(x), sc._p(xy),
                                           int(tile), sc._stream()), "pcub_mc_channel_qsc_tiled")
    return info[:code.K], xy


_TEMPLATES = {}


def guard_template(n, n0, xi, ones, device):
    """The guard-banded word's template for pcub_mc_deletion (codeword bit index, -1 zero, -2 one)."""
    key = (n, n0, float(xi), ones, str(device))
    t = _TEMPLATES.get(key)
    if t is None:
        pos, W, ones_pos = channel.guard_band_positions(n, n0, xi, ones)
        a = [-1] * W
        for i, j in enumerate(pos):
            a[j] = i
        for j in ones_pos:
            a[j] = -2
        t = _TEMPLATES[key] = torch.tensor(a, dtype=torch.int32, device=device)
    return t


def philox_deletion_batch(code, seed, offset, B, n0, xi, pd, ones=0):
    """Information words [ceil(K/32), B], received words rx [B, W] u8 and rx_len [B] i32 for global
    codewords [offset, offset + B): pcub_mc_info -> pcub_polar_encode_bin -> guard bands ->
    pcub_mc_deletion."""
    from . import _lib
    L = _lib.lib()
    dev = code.device
    info = torch.zeros((max(1, code.info_words), B), dtype=torch.int32, device=dev)
    _lib.check(L.pcub_mc_info(int(seed), int(offset), B, code.K, sc._p(info), sc._stream()), "pcub_mc_info")
    x = sc.encode_native(code, info)
    t = guard_template(code.n, n0, xi, ones, dev)
    W = int(t.numel())
    rx = torch.empty((B, W), dtype=torch.uint8, device=dev)
    ln = torch.empty(B, dtype=torch.int32, device=dev)
    _lib.check(L.pcub_mc_deletion(int(seed), int(offset), B, code.n, sc._p(t), W, float(pd), sc._p(x), sc._p(rx),
                                  sc._p(ln), sc._stream()), "pcub_mc_deletion")
    return info, rx, ln
