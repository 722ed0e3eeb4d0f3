"""Batched binary SC decode / encode on MI355X through the HIP C-ABI.

This is the batch entry point underneath the reference-compatible facade
(polarcub_amd.coding.BinaryPolarEncoderDecoder).  Tensors are torch CUDA (HIP)
tensors; every call is asynchronous on torch's current stream.

Layouts (see include/polarcub_sc.h):
  * joint probabilities, native:  [N, B, 2] float64  (element-major, codeword-minor)
  * joint probabilities, per-cw:  [B, N, 2] float64  (the reference's probs[i][x], stacked)
  * bit vectors, packed:          [ceil(nbits/32), B] int32 words (bit t of word w = bit 32w+t)
  * bit vectors, unpacked:        [B, nbits] uint8
"""
import ctypes
import random

import numpy as np
import torch

from . import _lib


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _log2(N):
    n = int(N).bit_length() - 1
    if N < 1 or (1 << n) != N:
        raise ValueError("code length must be a power of two, got %r" % (N,))
    return n


def pack_rows(bits):
    """Host helper: [B, nbits] 0/1 -> [ceil(nbits/32), B] uint32 (numpy)."""
    bits = np.asarray(bits, dtype=np.uint8)
    if bits.ndim == 1:
        bits = bits[None, :]
    B, nb = bits.shape
    W = max(1, (nb + 31) // 32)
    pad = np.zeros((B, W * 32), np.uint64)
    pad[:, :nb] = bits & 1
    words = (pad.reshape(B, W, 32) << np.arange(32, dtype=np.uint64)).sum(-1).astype(np.uint32)
    return np.ascontiguousarray(words.T)


def unpack_rows(words, nbits):
    """Host helper: [W, B] uint32 words -> [B, nbits] uint8."""
    words = np.asarray(words).view(np.uint32) if np.asarray(words).dtype == np.int32 else np.asarray(words, np.uint32)
    W, B = words.shape
    b = ((words.T[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1).astype(np.uint8).reshape(B, W * 32)
    return b[:, :nbits]


def common_randomness(N, seed):
    """r_i of BinaryPolarEncoderDecoder.initializeFrozenOrInformationAndRandomlyGeneratedNumbers
    (BinaryPolarEncoderDecoder.py:33-44): MT19937 draws for every index, or 1.0 for seed -1."""
    if seed == -1:
        return np.ones(N)
    rng = random.Random()
    rng.seed(seed)
    return np.array([rng.random() for _ in range(N)])


class CodeSpec:
    """One binary polar code: length, frozen positions and frozen values, resident on the device.

    frozen_values follow the reference's uniform-prior rule u_i = 0 if 0.5 >= r_i else 1
    (BinaryPolarEncoderDecoder.py:258-262); use from_frozen_set() to derive them from
    commonRandomnessSeed exactly as the reference does.
    """

    def __init__(self, N, frozen_mask, frozen_values=None, device=None):
        self.N = int(N)
        self.n = _log2(self.N)
        mask = np.asarray(frozen_mask, dtype=np.uint8).reshape(-1)
        if mask.shape[0] != self.N:
            raise ValueError("frozen mask has %d entries, expected N=%d" % (mask.shape[0], self.N))
        mask = (mask != 0).astype(np.uint8)
        vals = np.zeros(self.N, np.uint8) if frozen_values is None else (np.asarray(frozen_values) != 0).astype(np.uint8)
        vals = vals & mask
        self.frozen_mask = mask
        self.frozen_values = vals
        self.K = int(self.N - int(mask.sum()))
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self.fmask_dev = torch.from_numpy(pack_rows(mask).reshape(-1).view(np.int32).copy()).to(self.device)
        self.fval_dev = torch.from_numpy(pack_rows(vals).reshape(-1).view(np.int32).copy()).to(self.device)

    @classmethod
    def from_frozen_set(cls, N, frozen_set, common_randomness_seed, device=None):
        mask = np.zeros(int(N), np.uint8)
        for i in frozen_set:
            mask[int(i)] = 1
        r = common_randomness(int(N), common_randomness_seed)
        vals = np.where(0.5 >= r, 0, 1).astype(np.uint8)
        return cls(N, mask, vals, device=device)

    @property
    def info_words(self):
        return (self.K + 31) // 32

    @property
    def n_words(self):
        return max(1, (self.N + 31) // 32)


def default_variant():
    """The decode kernel variant the library picks unless told otherwise."""
    return int(_lib.lib().pcub_sc_default_variant())


def variant_for(n):
    """The decode kernel variant a code of length 2^n launches (the selected variant, or the
    fallback the launcher picks where it does not fit)."""
    return int(_lib.lib().pcub_sc_variant_for(int(n)))


def set_variant(v=None):
    """Select the decode kernel variant (see variants()); None restores the default."""
    if v is None:
        v = default_variant()
    _lib.check(_lib.lib().pcub_sc_set_variant(int(v)), "pcub_sc_set_variant")


def set_max_blocks_per_cu(b):
    """Cap resident decode workgroups per CU (0 = as many as fit); a tuning knob that
    trades latency hiding against the cache footprint of the codewords in flight."""
    _lib.check(_lib.lib().pcub_sc_set_max_blocks_per_cu(int(b)), "pcub_sc_set_max_blocks_per_cu")


def set_qary_lanes(g):
    """Lanes per codeword of the q-ary decode kernel (1, 2, 4, 8 or 16; reduced for
    short codes; 8 and 16 only where instantiated, else 4).  Returns the previous setting."""
    old = int(_lib.lib().pcub_sc_set_qary_lanes(int(g)))
    if old < 0:
        raise ValueError("q-ary lanes per codeword must be 1, 2, 4, 8 or 16")
    return old


def set_qary_hl(on):
    """Split last level of the q-ary decode kernel (2S positions per lane at a chain's end, S of
    them in LDS: one stored stage depth fewer) where it exists and fits (True, the default) or
    not (False).  Returns the previous setting."""
    old = int(_lib.lib().pcub_sc_set_qary_hl(1 if on else 0))
    if old < 0:
        raise ValueError("pcub_sc_set_qary_hl")
    return bool(old)


def set_qary_lds(on):
    """Re-encoded symbols of the q-ary decode kernel in LDS where a kernel for it exists and
    fits (True, the default) or in the per-slot workspace (False).  Returns the previous setting."""
    old = int(_lib.lib().pcub_sc_set_qary_lds(1 if on else 0))
    if old < 0:
        raise ValueError("pcub_sc_set_qary_lds")
    return bool(old)


def set_qary_regs(s):
    """Cap on the q-ary decode kernel's register positions per lane (0 = default, 2, 4 or
    8).  Returns the previous setting."""
    old = int(_lib.lib().pcub_sc_set_qary_regs(int(s)))
    if old < 0:
        raise ValueError("q-ary register positions must be 0, 2, 4 or 8")
    return old


def variants():
    """[(S, G, W)] per decode kernel variant: register-subtree values per lane,
    lanes per codeword, minimum waves per SIMD."""
    L = _lib.lib()
    out = []
    for v in range(L.pcub_sc_num_variants()):
        S, G, W = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(L.pcub_sc_variant_info(v, ctypes.byref(S), ctypes.byref(G), ctypes.byref(W)), "variant_info")
        out.append((S.value, G.value, W.value))
    return out


def bin_tile(n):
    """Codewords one wave of the binary decode kernel at N = 2^n decodes (pcub_sc_bin_tile): the tile
    width of the tiled root layout [ceil(B/T), N, T, 2] that BinaryDecoder.decode_tiled_native reads
    as one contiguous block per wave."""
    return int(_lib.lib().pcub_sc_bin_tile(int(n)))


def tile_rows(native, T):
    """[N, B, ...] rows (codeword-minor) -> the tiled layout [ceil(B/T), N, T, ...] (zero-padded)."""
    N, B = native.shape[0], native.shape[1]
    nt = (B + T - 1) // T
    pad = nt * T - B
    if pad:
        native = torch.cat([native, native.new_zeros((N, pad) + tuple(native.shape[2:]))], dim=1)
    return native.reshape((N, nt, T) + tuple(native.shape[2:])).transpose(0, 1).contiguous()


class BinaryDecoder:
    """Batched SC decoder for one CodeSpec; owns its device workspace."""

    def __init__(self, code):
        self.code = code
        self._ws = None

    def workspace(self, B):
        need = int(_lib.lib().pcub_sc_decode_bin_workspace(int(B), self.code.n))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 16), dtype=torch.uint8, device=self.code.device)
        return self._ws

    def decode_native(self, xy, want_xhat=True, want_u=False, out=None):
        """xy: [N, B, 2] float64 on device.  Returns packed (info_words, xhat_words|None, u_words|None)."""
        c = self.code
        if xy.dtype != torch.float64 or xy.dim() != 3 or xy.shape[0] != c.N or xy.shape[2] != 2:
            raise ValueError("xy must be float64 [N, B, 2] with N=%d" % c.N)
        if not xy.is_cuda:
            raise ValueError("xy must be a device tensor")
        xy = xy.contiguous()
        B = xy.shape[1]
        dev = xy.device
        if out is None:
            info = torch.empty((max(1, c.info_words), B), dtype=torch.int32, device=dev)
            xh = torch.empty((c.n_words, B), dtype=torch.int32, device=dev) if want_xhat else None
            uo = torch.empty((c.n_words, B), dtype=torch.int32, device=dev) if want_u else None
        else:
            info, xh, uo = out
        ws = self.workspace(B)
        rc = _lib.lib().pcub_sc_decode_bin(_p(xy), B, c.n, _p(c.fmask_dev), _p(c.fval_dev), c.K, _p(info), _p(xh),
                                           _p(uo), _p(ws), ws.numel(), _stream())
        _lib.check(rc, "pcub_sc_decode_bin")
        return info, xh, uo

    def decode_tiled_native(self, xy_t, B, want_xhat=True, out=None):
        """xy_t: the tiled root layout [ceil(B/T), N, T, 2] float64 on device (codeword b at tile b // T,
        column b % T; tile_rows), B codewords.  The same decode as decode_native on the untiled rows;
        each wave reads its codewords' rows as one contiguous block.  Returns packed
        (info_words, xhat_words|None, None)."""
        c = self.code
        if xy_t.dtype != torch.float64 or xy_t.dim() != 4 or xy_t.shape[1] != c.N or xy_t.shape[3] != 2:
            raise ValueError("xy_t must be float64 [ceil(B/T), N, T, 2] with N=%d" % c.N)
        if not xy_t.is_cuda:
            raise ValueError("xy_t must be a device tensor")
        T = xy_t.shape[2]
        if xy_t.shape[0] != (B + T - 1) // T:
            raise ValueError("xy_t holds %d tiles of %d codewords, B=%d needs %d" % (xy_t.shape[0], T, B,
                                                                                     (B + T - 1) // T))
        xy_t = xy_t.contiguous()
        dev = xy_t.device
        if out is None:
            info = torch.empty((max(1, c.info_words), B), dtype=torch.int32, device=dev)
            xh = torch.empty((c.n_words, B), dtype=torch.int32, device=dev) if want_xhat else None
        else:
            info, xh, _ = out
        ws = self.workspace(B)
        rc = _lib.lib().pcub_sc_decode_bin_tiled(_p(xy_t), B, c.n, T, _p(c.fmask_dev), _p(c.fval_dev), c.K, _p(info),
                                                 _p(xh), None, _p(ws), ws.numel(), _stream())
        _lib.check(rc, "pcub_sc_decode_bin_tiled")
        return info, xh, None

    def decode_compact_native(self, xc, want_xhat=True, out=None):
        """xc: [N, B] float64 compact normalised rows on device (+r: (1, r), -r: (r, 1)), the same
        decode as decode_native on those pairs (pcub_sc_decode_bin_compact).  Returns packed
        (info_words, xhat_words | None, None)."""
        c = self.code
        if xc.dtype != torch.float64 or xc.dim() != 2 or xc.shape[0] != c.N or not xc.is_cuda:
            raise ValueError("xc must be a float64 [N, B] device tensor with N=%d" % c.N)
        xc = xc.contiguous()
        B = xc.shape[1]
        if out is None:
            info = torch.empty((max(1, c.info_words), B), dtype=torch.int32, device=xc.device)
            xh = torch.empty((c.n_words, B), dtype=torch.int32, device=xc.device) if want_xhat else None
        else:
            info, xh, _ = out
        need = int(_lib.lib().pcub_sc_decode_bin_compact_workspace(B, c.n))
        if getattr(self, "_cws", None) is None or self._cws.numel() < need:
            self._cws = torch.empty(max(need, 16), dtype=torch.uint8, device=xc.device)
        rc = _lib.lib().pcub_sc_decode_bin_compact(_p(xc), B, c.n, _p(c.fmask_dev), _p(c.fval_dev), c.K, _p(info),
                                                   _p(xh), None, _p(self._cws), self._cws.numel(), _stream())
        _lib.check(rc, "pcub_sc_decode_bin_compact")
        return info, xh, None

    def decode(self, xy):
        """xy: [B, N, 2] float64 (per-codeword rows, as the reference's probs).
        Returns (info [B, K] uint8, xhat [B, N] uint8).  The rows go in one pass into the tiled root
        layout (pcub_tile_pairs) and through the headline kernel (decode_tiled_native); the same
        decisions as decode_native on the transposed rows."""
        B = xy.shape[0]
        T = bin_tile(self.code.n)
        info_w, xh_w, _ = self.decode_tiled_native(tile_pairs(xy, T), B)
        return unpack(info_w, self.code.K), unpack(xh_w, self.code.N)


class LeafDecoder:
    """Binary SC with every leaf exported (pcub_sc_leaf_bin): the xy marginals the reference
    collects in marginalizedUProbs (LLR checks, genie runs).  Optional per-codeword frozen
    values ([B, N] 0/1) override the code's."""

    def __init__(self, code):
        self.code = code
        self._ws = None

    def decode_native(self, xy, fval_cw=None):
        """xy [N, B, 2] float64 (device) -> (info_words, xhat_words, leaf [N, B] compact float64)."""
        c = self.code
        if xy.dtype != torch.float64 or xy.dim() != 3 or xy.shape[0] != c.N or xy.shape[2] != 2 or not xy.is_cuda:
            raise ValueError("xy must be a float64 [N, B, 2] device tensor with N=%d" % c.N)
        if c.n < 1:
            raise ValueError("leaf export needs N >= 2")
        xy = xy.contiguous()
        B = xy.shape[1]
        need = int(_lib.lib().pcub_sc_leaf_bin_workspace(B, c.n))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 16), dtype=torch.uint8, device=xy.device)
        fw = None if fval_cw is None else pack(fval_cw.to(device=xy.device, dtype=torch.uint8))
        info = torch.empty((max(1, c.info_words), B), dtype=torch.int32, device=xy.device)
        xh = torch.empty((c.n_words, B), dtype=torch.int32, device=xy.device)
        leaf = torch.empty((c.N, B), dtype=torch.float64, device=xy.device)
        rc = _lib.lib().pcub_sc_leaf_bin(_p(xy), B, c.n, _p(c.fmask_dev), _p(c.fval_dev), _p(fw), c.K, _p(info),
                                         _p(xh), _p(leaf), _p(self._ws), self._ws.numel(), _stream())
        _lib.check(rc, "pcub_sc_leaf_bin")
        return info, xh, leaf

    def decode(self, xy, fval_cw=None):
        """xy [B, N, 2] -> (info [B, K] uint8, xhat [B, N] uint8, marginals [B, N, 2] float64)."""
        info, xh, leaf = self.decode_native(transpose_pairs(xy), fval_cw)
        return unpack(info, self.code.K), unpack(xh, self.code.N), leaf_marginals(leaf)


class PriorCoder:
    """Two-tree SC for a non-uniform a-priori distribution (pcub_sc_prior_bin): decode with
    (prior, xy) or encode with the prior alone, frozen bits drawn against the common randomness
    r_i (BinaryPolarEncoderDecoder.py:223-325, :258-262).  The code's frozen values are not
    used: they follow from the prior tree."""

    def __init__(self, code, rnd):
        self.code = code
        r = np.asarray(rnd, dtype=np.float64).reshape(-1)
        if r.shape[0] != code.N:
            raise ValueError("common randomness has %d entries, expected N=%d" % (r.shape[0], code.N))
        self.rnd_dev = torch.from_numpy(r.copy()).to(code.device)
        self._ws = None

    def _prior(self, px, B):
        c = self.code
        px = torch.as_tensor(px, dtype=torch.float64, device=c.device)
        if px.dim() == 2:  # [N, 2]: one prior for the whole batch
            px = px[:, None, :]
        if px.dim() != 3 or px.shape[0] != c.N or px.shape[2] != 2 or px.shape[1] not in (1, B):
            raise ValueError("prior must be float64 [N, 2], [N, 1, 2] or [N, B, 2] with N=%d" % c.N)
        return px.contiguous()

    def run_native(self, px, xy=None, info_words=None, B=None, want_leaf=False):
        """Decode (xy [N, B, 2] given) or encode (info_words [ceil(K/32), B] given).
        Returns (info_words, xhat_words, leaf [N, B] compact | None)."""
        c = self.code
        if c.n < 1:
            raise ValueError("two-tree SC needs N >= 2")
        if xy is not None:
            if xy.dtype != torch.float64 or xy.dim() != 3 or xy.shape[0] != c.N or xy.shape[2] != 2 or not xy.is_cuda:
                raise ValueError("xy must be a float64 [N, B, 2] device tensor with N=%d" % c.N)
            xy = xy.contiguous()
            B = xy.shape[1]
        else:
            B = info_words.shape[1] if info_words is not None else int(B)
        px = self._prior(px, B)
        dev = c.device
        need = int(_lib.lib().pcub_sc_prior_bin_workspace(B, c.n))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 16), dtype=torch.uint8, device=dev)
        if xy is not None:
            info = torch.empty((max(1, c.info_words), B), dtype=torch.int32, device=dev)
        else:
            info = info_words.contiguous() if info_words is not None else torch.zeros((1, B), dtype=torch.int32,
                                                                                      device=dev)
        xh = torch.empty((c.n_words, B), dtype=torch.int32, device=dev)
        leaf = torch.empty((c.N, B), dtype=torch.float64, device=dev) if want_leaf else None
        rc = _lib.lib().pcub_sc_prior_bin(_p(xy), _p(px), px.shape[1], B, c.n, _p(c.fmask_dev), _p(self.rnd_dev), c.K,
                                          _p(info), _p(xh), _p(leaf), _p(self._ws), self._ws.numel(), _stream())
        _lib.check(rc, "pcub_sc_prior_bin")
        return info, xh, leaf

    def decode(self, px, xy, want_marginals=False):
        """xy [B, N, 2] per-codeword rows -> (info [B, K] uint8, xhat [B, N] uint8[, marginals [B, N, 2]])."""
        info, xh, leaf = self.run_native(px, xy=transpose_pairs(xy), want_leaf=want_marginals)
        out = (unpack(info, self.code.K), unpack(xh, self.code.N))
        return out + (leaf_marginals(leaf),) if want_marginals else out

    def encode(self, px, info):
        """info [B, K] uint8 -> codewords [B, N] uint8 under the prior."""
        c = self.code
        if info.shape[1] != c.K:
            raise ValueError("info has %d columns, code has K=%d" % (info.shape[1], c.K))
        words = pack(info) if c.K > 0 else None
        _, xh, _ = self.run_native(px, info_words=words, B=info.shape[0])
        return unpack(xh, c.N)


def leaf_marginals(leaf):
    """Compact leaves [N, B] -> the reference's leaf marginals [B, N, 2] (pcub_leaf_marginals)."""
    N, B = leaf.shape
    t = leaf.t().contiguous()
    m = torch.empty((B, N, 2), dtype=torch.float64, device=leaf.device)
    _lib.check(_lib.lib().pcub_leaf_marginals(_p(t), t.numel(), _p(m), _stream()), "pcub_leaf_marginals")
    return m


def transpose_pairs(xy):
    """[B, N, q] float64 -> [N, B, q] float64 on device."""
    if xy.dtype != torch.float64 or xy.dim() != 3:
        raise ValueError("expected float64 [B, N, q]")
    xy = xy.contiguous()
    B, N, q = xy.shape
    out = torch.empty((N, B, q), dtype=torch.float64, device=xy.device)
    _lib.check(_lib.lib().pcub_transpose_pairs(_p(xy), B, N, q, _p(out), _stream()), "pcub_transpose_pairs")
    return out


def tile_pairs(xy, T):
    """[B, N, q] float64 on device -> the tiled layout [ceil(B/T), N, T, q] (pcub_tile_pairs; padding
    columns zero): the same array as tile_rows(transpose_pairs(xy), T) in one pass."""
    if xy.dtype != torch.float64 or xy.dim() != 3:
        raise ValueError("expected float64 [B, N, q]")
    xy = xy.contiguous()
    B, N, q = xy.shape
    out = torch.empty(((B + T - 1) // T, N, T, q), dtype=torch.float64, device=xy.device)
    _lib.check(_lib.lib().pcub_tile_pairs(_p(xy), B, N, q, int(T), _p(out), _stream()), "pcub_tile_pairs")
    return out


def unpack(words, nbits):
    """[W, B] int32 words -> [B, nbits] uint8 on device."""
    W, B = words.shape
    out = torch.empty((B, nbits), dtype=torch.uint8, device=words.device)
    _lib.check(_lib.lib().pcub_unpack_bits(_p(words.contiguous()), B, int(nbits), _p(out), _stream()),
               "pcub_unpack_bits")
    return out


def pack(bits):
    """[B, nbits] uint8 -> [ceil(nbits/32), B] int32 on device."""
    bits = bits.to(torch.uint8).contiguous()
    B, nb = bits.shape
    out = torch.empty((max(1, (nb + 31) // 32), B), dtype=torch.int32, device=bits.device)
    _lib.check(_lib.lib().pcub_pack_bits(_p(bits), B, int(nb), _p(out), _stream()), "pcub_pack_bits")
    return out


def encode_native(code, info_words):
    """Packed info [ceil(K/32), B] -> packed codewords [ceil(N/32), B] (uniform prior)."""
    B = info_words.shape[1]
    x = torch.empty((code.n_words, B), dtype=torch.int32, device=info_words.device)
    rc = _lib.lib().pcub_polar_encode_bin(_p(info_words.contiguous()), B, code.n, _p(code.fmask_dev),
                                          _p(code.fval_dev), code.K, _p(x), _stream())
    _lib.check(rc, "pcub_polar_encode_bin")
    return x


def encode(code, info):
    """info [B, K] uint8 -> codewords [B, N] uint8."""
    if info.shape[1] != code.K:
        raise ValueError("info has %d columns, code has K=%d" % (info.shape[1], code.K))
    if code.K == 0:
        words = torch.zeros((1, info.shape[0]), dtype=torch.int32, device=info.device)
    else:
        words = pack(info)
    return unpack(encode_native(code, words), code.N)


class QaryCode:
    """One q-ary polar code (2 <= q <= 8): length, frozen positions (frozen symbols are 0,
    QaryPolarEncoderDecoder.py:347-351), resident on the device."""

    def __init__(self, q, N, frozen_mask, device=None):
        self.q = int(q)
        if not 2 <= self.q <= 8:
            raise ValueError("q must be in [2, 8] for the device decoder")
        self.N = int(N)
        self.n = _log2(self.N)
        if self.n < 2:
            raise ValueError("q-ary device decoder needs N >= 4")
        mask = (np.asarray(frozen_mask, dtype=np.uint8).reshape(-1) != 0).astype(np.uint8)
        if mask.shape[0] != self.N:
            raise ValueError("frozen mask has %d entries, expected N=%d" % (mask.shape[0], self.N))
        self.frozen_mask = mask
        self.K = int(self.N - int(mask.sum()))
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self.frozen_dev = torch.from_numpy(mask.copy()).to(self.device)


class QaryDecoder:
    """Batched q-ary SC decoder for one QaryCode (linear-domain probabilities)."""

    def __init__(self, code):
        self.code = code
        self._ws = None

    def workspace(self, B):
        c = self.code
        need = int(_lib.lib().pcub_sc_decode_qary_workspace(int(B), c.n, c.q))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 16), dtype=torch.uint8, device=c.device)
        return self._ws

    def decode_native(self, xy, want_xhat=True):
        """xy: [N, B, q] float64 on device -> (info [K, B] uint8, xhat [N, B] uint8 | None)."""
        c = self.code
        if xy.dtype != torch.float64 or xy.dim() != 3 or xy.shape[0] != c.N or xy.shape[2] != c.q:
            raise ValueError("xy must be float64 [N, B, q] with N=%d, q=%d" % (c.N, c.q))
        xy = xy.contiguous()
        B = xy.shape[1]
        info = torch.empty((max(1, c.K), B), dtype=torch.uint8, device=xy.device)
        xh = torch.empty((c.N, B), dtype=torch.uint8, device=xy.device) if want_xhat else None
        ws = self.workspace(B)
        rc = _lib.lib().pcub_sc_decode_qary(_p(xy), B, c.n, c.q, _p(c.frozen_dev), c.K, _p(info), _p(xh), _p(ws),
                                            ws.numel(), _stream())
        _lib.check(rc, "pcub_sc_decode_qary")
        return info[:c.K], xh

    def tile(self):
        """The native tile width of the tiled root layout (pcub_sc_qary_tile)."""
        return int(_lib.lib().pcub_sc_qary_tile(self.code.q, self.code.n))

    def decode_tiled_native(self, xy_t, B, want_xhat=True):
        """xy_t: [ceil(B/T), N, T, q] float64 on device (tile_rows of the [N, B, q] rows), B codewords:
        the same decode as decode_native, each wave's codewords read as one contiguous block."""
        c = self.code
        if xy_t.dtype != torch.float64 or xy_t.dim() != 4 or xy_t.shape[1] != c.N or xy_t.shape[3] != c.q:
            raise ValueError("xy_t must be float64 [ceil(B/T), N, T, q] with N=%d, q=%d" % (c.N, c.q))
        T = xy_t.shape[2]
        if xy_t.shape[0] != (B + T - 1) // T:
            raise ValueError("xy_t holds %d tiles of %d codewords; B=%d" % (xy_t.shape[0], T, B))
        xy_t = xy_t.contiguous()
        info = torch.empty((max(1, c.K), B), dtype=torch.uint8, device=xy_t.device)
        xh = torch.empty((c.N, B), dtype=torch.uint8, device=xy_t.device) if want_xhat else None
        ws = self.workspace(B)
        rc = _lib.lib().pcub_sc_decode_qary_tiled(_p(xy_t), B, c.n, c.q, T, _p(c.frozen_dev), c.K, _p(info), _p(xh),
                                                  _p(ws), ws.numel(), _stream())
        _lib.check(rc, "pcub_sc_decode_qary_tiled")
        return info[:c.K], xh

    def decode(self, xy):
        """xy: [B, N, q] float64 -> (info [B, K] uint8, xhat [B, N] uint8), through the tiled layout
        (pcub_tile_pairs, decode_tiled_native)."""
        B = xy.shape[0]
        info, xh = self.decode_tiled_native(tile_pairs(xy, self.tile()), B)
        return info.t().contiguous(), xh.t().contiguous()


class QaryLogDecoder:
    """Batched q-ary SC in the log domain (pcub_sc_decode_qary_log): use_log=True vector
    distributions, log-probabilities in, symbols and log leaf marginals out.  Values agree
    with the reference within a few ulps (device exp/log1p/log), decisions exactly wherever
    no two marginals are that close."""

    def __init__(self, q, N, frozen_mask, device=None):
        self.q = int(q)
        if not 2 <= self.q <= 8:
            raise ValueError("q must be in [2, 8] for the device decoder")
        self.N = int(N)
        self.n = _log2(self.N)
        if not 1 <= self.n <= 16:
            raise ValueError("log-domain device decoder needs 2 <= N <= 2^16")
        mask = (np.asarray(frozen_mask, dtype=np.uint8).reshape(-1) != 0).astype(np.uint8)
        if mask.shape[0] != self.N:
            raise ValueError("frozen mask has %d entries, expected N=%d" % (mask.shape[0], self.N))
        self.K = int(self.N - int(mask.sum()))
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self.fwords = torch.from_numpy(pack_rows(mask).reshape(-1).view(np.int32).copy()).to(self.device)
        self._ws = None

    def decode_native(self, xy, want_xhat=True, want_leaf=False):
        """xy [N, B, q] log-probabilities (device) -> (info [K, B] u8, xhat [N, B] u8 | None,
        leaf [N, B, q] f64 | None)."""
        if xy.dtype != torch.float64 or xy.dim() != 3 or xy.shape[0] != self.N or xy.shape[2] != self.q:
            raise ValueError("xy must be float64 [N, B, q] with N=%d, q=%d" % (self.N, self.q))
        xy = xy.contiguous()
        B = xy.shape[1]
        need = int(_lib.lib().pcub_sc_decode_qary_log_workspace(B, self.q, self.n))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(max(need, 16), dtype=torch.uint8, device=xy.device)
        info = torch.empty((max(1, self.K), B), dtype=torch.uint8, device=xy.device)
        xh = torch.empty((self.N, B), dtype=torch.uint8, device=xy.device) if want_xhat else None
        leaf = torch.empty((self.N, B, self.q), dtype=torch.float64, device=xy.device) if want_leaf else None
        rc = _lib.lib().pcub_sc_decode_qary_log(_p(xy), B, self.q, self.n, _p(self.fwords), self.K, _p(info), _p(xh),
                                                _p(leaf), _p(self._ws), self._ws.numel(), _stream())
        _lib.check(rc, "pcub_sc_decode_qary_log")
        return info[:self.K], xh, leaf

    def decode(self, xy, want_leaf=False):
        """xy [B, N, q] -> (info [B, K] u8, xhat [B, N] u8[, leaf log marginals [B, N, q]])."""
        info, xh, leaf = self.decode_native(transpose_pairs(xy), want_leaf=want_leaf)
        out = (info.t().contiguous(), xh.t().contiguous())
        return out + (leaf.transpose(0, 1).contiguous(),) if want_leaf else out


class QaryListDecoder:
    """Batched q-ary SCL / Fast-SSC list decoding (pcub_scl_qary): QaryPolarEncoderDecoder.listDecode
    for B codewords of one code at list size L, with optional actual information words."""

    def __init__(self, q, N, frozen_mask, L, device=None, use_log=False):
        self.q, self.N, self.L = int(q), int(N), int(L)
        self.use_log = bool(use_log)  # log-probability rows and metrics (pcub_scl_qary_log)
        self.n = _log2(self.N)
        if not 2 <= self.q <= 8 or not 1 <= self.L <= 64 or self.n > 12:
            raise ValueError("list decoder needs 2 <= q <= 8, 1 <= L <= 64, N <= 4096")
        mask = (np.asarray(frozen_mask, dtype=np.uint8).reshape(-1) != 0).astype(np.uint8)
        if mask.shape[0] != self.N:
            raise ValueError("frozen mask has %d entries, expected N=%d" % (mask.shape[0], self.N))
        self.K = int(self.N - int(mask.sum()))
        self.nF = self.N - self.K
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self.frozen_dev = torch.from_numpy(mask.copy()).to(self.device)
        self._ws = None

    def decode_native(self, xy, frozen_vals, actual=None, max_workspace_bytes=None):
        """xy [N, B, q] f64, frozen_vals [nF, B] u8, actual [K, B] u8 or None (device tensors)
        -> (info [L, K, B] u8, prob [L, B] f64, size [B] i32, actual_prob [B] f64 | None).
        The slot slab is capped at max_workspace_bytes (default: half the free device memory);
        fewer resident slots then stride over the batch."""
        if xy.dtype != torch.float64 or xy.dim() != 3 or xy.shape[0] != self.N or xy.shape[2] != self.q:
            raise ValueError("xy must be float64 [N, B, q] with N=%d, q=%d" % (self.N, self.q))
        xy = xy.contiguous()
        B = xy.shape[1]
        dev = xy.device
        fv = frozen_vals.to(device=dev, dtype=torch.uint8).contiguous() if self.nF else \
            torch.zeros((1, B), dtype=torch.uint8, device=dev)
        act = None if actual is None else actual.to(device=dev, dtype=torch.uint8).contiguous()
        need = int(_lib.lib().pcub_scl_qary_workspace(B, self.q, self.n, self.L, self.K))
        # The full resident grid of slots can exceed device memory at large N*L*q: cap the slab at
        # half of the free memory (at least one workgroup's slots); pcub_scl_qary then clips the grid.
        block = int(_lib.lib().pcub_scl_qary_workspace(1, self.q, self.n, self.L, self.K))
        free = torch.cuda.mem_get_info(dev)[0] + (0 if self._ws is None else self._ws.numel())
        need = min(need, max(block, free // 2 if max_workspace_bytes is None else int(max_workspace_bytes)))
        if self._ws is None or self._ws.numel() < need:
            self._ws = None
            self._ws = torch.empty(max(need, 16), dtype=torch.uint8, device=dev)
        info = torch.empty((self.L, max(1, self.K), B), dtype=torch.uint8, device=dev)
        prob = torch.empty((self.L, B), dtype=torch.float64, device=dev)
        size = torch.empty(B, dtype=torch.int32, device=dev)
        ap = torch.empty(B, dtype=torch.float64, device=dev) if act is not None else None
        fn = _lib.lib().pcub_scl_qary_log if self.use_log else _lib.lib().pcub_scl_qary
        rc = fn(_p(xy), B, self.q, self.n, self.L, _p(self.frozen_dev), _p(fv), self.nF, _p(act), self.K, _p(info),
                _p(prob), _p(size), _p(ap), _p(self._ws), self._ws.numel(), _stream())
        _lib.check(rc, "pcub_scl_qary_log" if self.use_log else "pcub_scl_qary")
        return info[:, :self.K], prob, size, ap

    def decode(self, xy, frozen_vals, actual=None):
        """xy [B, N, q], frozen_vals [B, nF], actual [B, K] or None -> numpy (info [B, L, K],
        prob [B, L], size [B], actual_prob [B] | None)."""
        dev = self.device
        x = transpose_pairs(torch.as_tensor(np.ascontiguousarray(xy, np.float64), device=dev))
        B = x.shape[1]
        fv = torch.as_tensor(np.ascontiguousarray(np.asarray(frozen_vals, np.uint8).reshape(B, self.nF).T),
                             device=dev)
        act = None if actual is None else torch.as_tensor(
            np.ascontiguousarray(np.asarray(actual, np.uint8).reshape(B, self.K).T), device=dev)
        info, prob, size, ap = self.decode_native(x, fv, act)
        return (info.permute(2, 0, 1).cpu().numpy(), prob.t().cpu().numpy(), size.cpu().numpy(),
                None if ap is None else ap.cpu().numpy())


def encode_qary(code, info):
    """info [B, K] uint8 symbols -> codewords [B, N] uint8."""
    B = info.shape[0]
    if info.shape[1] != code.K:
        raise ValueError("info has %d columns, code has K=%d" % (info.shape[1], code.K))
    inf = info.to(torch.uint8).t().contiguous() if code.K else torch.zeros((1, B), dtype=torch.uint8,
                                                                          device=code.device)
    x = torch.empty((code.N, B), dtype=torch.uint8, device=code.device)
    rc = _lib.lib().pcub_polar_encode_qary(_p(inf), B, code.n, code.q, _p(code.frozen_dev), code.K, _p(x), _stream())
    _lib.check(rc, "pcub_polar_encode_qary")
    return x.t().contiguous()


def deletion_supported(n, n0, ones=0):
    """True when pcub_sc_decode_deletion has a kernel for 2^(n-n0) trellises of 2^n0 inputs
    with `ones` guard-band ones."""
    return bool(_lib.lib().pcub_sc_deletion_supported(int(n), int(n0), int(ones)))


def leaf_deletion_supported(n, n0, ones=0):
    """True when pcub_sc_leaf_deletion (every leaf exported: the genie) covers the shape."""
    return bool(_lib.lib().pcub_sc_leaf_deletion_supported(int(n), int(n0), int(ones)))


def set_deletion_rate1(on):
    """Diagnostic: 0 runs the 8-lane deletion subtrees without the rate-1 shortcut where that twin is
    built (pcub_sc_set_deletion_rate1, not part of the stable ABI); returns the previous setting.
    Decisions are identical either way."""
    import ctypes
    f = _lib.lib().pcub_sc_set_deletion_rate1
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int32]
    return int(f(int(on)))


def set_deletion_wave(on):
    """Diagnostic: 0 sends n0 = 4 deletion decodes (64 .. 1024 trellises) back to the lane-per-trellis
    kernel instead of the wave-per-task kernel (pcub_sc_set_deletion_wave, not part of the stable ABI);
    returns the previous setting.  Decisions are identical either way."""
    import ctypes
    f = _lib.lib().pcub_sc_set_deletion_wave
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int32]
    return int(f(int(on)))


def set_dynamic_tiles(on):
    """Diagnostic: 0 makes the binary, q-ary and deletion decode kernels stride over their tiles
    statically instead of taking them from a per-launch counter (pcub_sc_set_dynamic_tiles, not part of
    the stable ABI); returns the previous setting.  Decisions are identical either way."""
    import ctypes
    f = _lib.lib().pcub_sc_set_dynamic_tiles
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int]
    return int(f(int(on)))


def set_deletion_lanes(g):
    """Lanes a codeword of the table-driven deletion layout: 8 (default), 16, or 4 (up to 64
    trellises; 8 beyond) (pcub_sc_set_deletion_lanes); returns the previous value.  Decisions are
    identical either way."""
    old = int(_lib.lib().pcub_sc_set_deletion_lanes(int(g)))
    if old < 0:
        raise ValueError("deletion lanes: 4, 8 or 16")
    return old


def set_deletion_dense(on):
    """Allow (default) or forbid the table-driven deletion layout (pcub_sc_set_deletion_dense);
    returns the previous setting.  Decisions are identical either way."""
    return bool(_lib.lib().pcub_sc_set_deletion_dense(1 if on else 0))


class DeletionDecoder:
    """Batched SC decoder over the deletion channel (CollectionOfBinaryTrellises built from
    each received word with buildCollectionOfBinaryTrellises_uniformInput_deletion, with
    `ones` guard-band ones) for one CodeSpec.  With use_table (the default), n0 = 2 or 3 and
    ones = 0 the decoder builds the segment-state table for (n0, pd) once per device
    (pcub_sc_deletion_build_table) and every decode passes it; the kernels check its header
    (magic, n0, pd) on the device and decode without it when it does not match.  Decisions are
    identical without a table: n0 = 3 then rebuilds the trellis levels per lane, n0 = 2 builds
    the table per workgroup."""

    def __init__(self, code, n0, pd, ones=0, use_table=True):
        self.code = code
        self.n0 = int(n0)
        self.pd = float(pd)
        self.ones = int(ones)
        self.use_table = bool(use_table)
        self._tables = {}
        if not deletion_supported(code.n, self.n0, self.ones):
            raise ValueError("no deletion kernel for n=%d, n0=%d, ones=%d" % (code.n, self.n0, self.ones))

    def table(self, device):
        """The segment-state table on `device` (a float64 device tensor), or None when the shape
        has none or use_table is off."""
        if not self.use_table or self.ones != 0:
            return None
        L = _lib.lib()
        nbytes = int(L.pcub_sc_deletion_table_bytes(self.n0))
        if nbytes == 0:
            return None
        key = str(device)
        t = self._tables.get(key)
        if t is None:
            t = torch.empty(nbytes // 8, dtype=torch.float64, device=device)
            _lib.check(L.pcub_sc_deletion_build_table(self.n0, self.pd, _p(t), _stream()),
                       "pcub_sc_deletion_build_table")
            self._tables[key] = t
        return t

    def dense_layout(self, stride, device):
        """True when decodes of rows of `stride` symbols run the table-driven layout
        (k_sc_del_dense) rather than k_sc_del."""
        return bool(_lib.lib().pcub_sc_deletion_dense_layout(self.code.n, self.n0, self.ones, int(stride),
                                                             _p(self.table(device)), self.pd))

    def decode_native(self, rx, rx_len, want_xhat=True):
        """rx: [B, W] uint8 received symbols on device, rx_len: [B] int32.
        Returns packed (info_words [ceil(K/32), B], xhat_words [ceil(N/32), B] | None)."""
        c = self.code
        if rx.dtype != torch.uint8 or rx.dim() != 2 or not rx.is_cuda:
            raise ValueError("rx must be a uint8 [B, W] device tensor")
        rx = rx.contiguous()
        B, W = rx.shape
        ln = rx_len.to(device=rx.device, dtype=torch.int32).contiguous()
        if ln.numel() != B:
            raise ValueError("rx_len must have B entries")
        info = torch.empty((max(1, c.info_words), B), dtype=torch.int32, device=rx.device)
        xh = torch.empty((c.n_words, B), dtype=torch.int32, device=rx.device) if want_xhat else None
        rc = _lib.lib().pcub_sc_decode_deletion_tab(_p(rx), _p(ln), B, W, c.n, self.n0, self.ones, self.pd,
                                                    _p(c.fmask_dev), _p(c.fval_dev), c.K, _p(info), _p(xh),
                                                    _p(self.table(rx.device)), _stream())
        _lib.check(rc, "pcub_sc_decode_deletion_tab")
        return info, xh

    def decode(self, rx, rx_len):
        """Returns (info [B, K] uint8, xhat [B, N] uint8) on device."""
        info_w, xh_w = self.decode_native(rx, rx_len)
        return unpack(info_w, self.code.K), unpack(xh_w, self.code.N)

    def decode_leaves(self, rx, rx_len, fval_cw=None):
        """Export mode (pcub_sc_leaf_deletion): (info [B, K], xhat [B, N], marginals [B, N, 2])."""
        c = self.code
        if not leaf_deletion_supported(c.n, self.n0, self.ones):
            raise ValueError("no leaf-export deletion kernel for n=%d, n0=%d, ones=%d" % (c.n, self.n0, self.ones))
        rx = rx.contiguous()
        B, W = rx.shape
        ln = rx_len.to(device=rx.device, dtype=torch.int32).contiguous()
        fw = None if fval_cw is None else pack(fval_cw.to(device=rx.device, dtype=torch.uint8))
        info = torch.empty((max(1, c.info_words), B), dtype=torch.int32, device=rx.device)
        xh = torch.empty((c.n_words, B), dtype=torch.int32, device=rx.device)
        leaf = torch.empty((c.N, B), dtype=torch.float64, device=rx.device)
        rc = _lib.lib().pcub_sc_leaf_deletion_tab(_p(rx), _p(ln), B, W, c.n, self.n0, self.ones, self.pd,
                                                  _p(c.fmask_dev), _p(c.fval_dev), _p(fw), c.K, _p(info), _p(xh),
                                                  _p(leaf), _p(self.table(rx.device)), _stream())
        _lib.check(rc, "pcub_sc_leaf_deletion_tab")
        return unpack(info, c.K), unpack(xh, c.N), leaf_marginals(leaf)


def pad_words(words, device=None):
    """List of received words (0/1 sequences of varying length) -> ([B, W] uint8, [B] int32) on device."""
    B = len(words)
    W = max([len(w) for w in words] + [1])
    a = np.zeros((B, W), np.uint8)
    for b, w in enumerate(words):
        a[b, :len(w)] = np.asarray(w, dtype=np.uint8)
    dev = torch.device("cuda") if device is None else device
    return (torch.from_numpy(a).to(dev), torch.tensor([len(w) for w in words], dtype=torch.int32, device=dev))
