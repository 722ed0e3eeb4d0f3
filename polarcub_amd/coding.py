"""Reference-compatible binary polar encoder/decoder (BinaryPolarEncoderDecoder.py).

Same class, method and function names, argument order and return types as the
reference, so harnesses written against polarcub run unchanged:

  BinaryPolarEncoderDecoder(length, frozenSet, commonRandomnessSeed)   :15-44
      .encode(xVD, information) -> int64[N]                           :46-69
      .decode(xVD, xyVD) -> (int64[N], int64[k])                      :71-99
      .genieSingleDecodeSimulatioan / .genieSingleEncodeSimulatioan   :101-221
      .recursiveEncodeDecode(...)                                     :223-325
  encodeDecodeSimulation(...)                                         :328-387
  genieEncodeDecodeSimulation(...)                                    :390-491
  polarTransformOfBits(xvec)                                          :494-516
  frozenSetFromTVAndPe(TVvec, Pevec, bound)                           :519-548

Dispatch.  Under a *uniform* a-priori distribution (every row p0 == p1: the
a-priori tree is then (1,1) at every node) decode() runs on the GPU through the
HIP C ABI, bit-identical to the reference, for
  * a memoryless binary xy distribution (pcub_sc_decode_bin), and
  * a deletion-channel collection of trellises built from a received word by
    buildCollectionOfBinaryTrellises_uniformInput_deletion, in the shapes the
    deletion kernel covers (pcub_sc_decode_deletion).
Under a non-uniform memoryless binary prior, encode() and decode() of memoryless
xy run the two-tree kernel (pcub_sc_prior_bin: prior and xy trees side by side,
frozen bits drawn against the common randomness).  Any other plugin (other
trellis shapes, user classes, non-memoryless priors) goes through
recursiveEncodeDecode, which drives the plugin's own methods exactly as the
reference does.  Additions: decode_batch / encode_batch / decode_deletion_batch /
decode_prior_batch / encode_prior_batch.
"""
import random
import sys
from enum import Enum

import numpy as np

from . import deletion, vectors


class uIndexType(Enum):
    frozen = 0
    information = 1


def _is_memoryless_binary(vd):
    return (isinstance(vd, vectors.BinaryMemorylessVectorDistribution)
            or (type(vd).__name__ == "BinaryMemorylessVectorDistribution" and hasattr(vd, "probs")))


def _is_uniform_prior(xvd):
    if not _is_memoryless_binary(xvd):
        return False
    p = np.asarray(xvd.probs, dtype=np.float64)
    return p.ndim == 2 and p.shape[1] == 2 and bool(np.all(p[:, 0] == p[:, 1])) and bool(np.all(np.isfinite(p)))


def _prior_rows(xvd, length):
    """The prior rows [N, 2] when xvd is a memoryless binary prior the two-tree kernel takes
    (finite, non-negative; N >= 2), else None."""
    if length < 2 or not _is_memoryless_binary(xvd):
        return None
    p = np.asarray(xvd.probs, dtype=np.float64)
    if p.shape != (length, 2) or not np.all(np.isfinite(p)) or not np.all(p >= 0):
        return None
    return p


def _deletion_kernel_shape(xyvd, leaves=False):
    """(pd, n, n0, ones) when xyvd is a received-word trellis collection the deletion kernel
    decodes (leaves=True: the leaf-export kernel, for the genie)."""
    if not deletion.is_deletion_collection(xyvd):
        return None
    word, pd, n, n0, ones = xyvd.deletion_source
    from . import sc
    ok = sc.leaf_deletion_supported(n, n0, ones) if leaves else sc.deletion_supported(n, n0, ones)
    return (pd, n, n0, ones) if ok else None


def _check_joint(p):
    p = np.asarray(p, dtype=np.float64)
    # the reference asserts t >= 0 in normalize (BinaryMemorylessVectorDistribution.py:82)
    assert np.all(p >= 0) and np.all(np.isfinite(p)), "joint probabilities must be finite and non-negative"
    return p


def eta(p):
    """-p log2 p with eta(0) = 0 (ScalarDistributions/BinaryMemorylessDistribution.py:451-459)."""
    import math
    assert 0.0 <= p <= 1.0 + 10 * sys.float_info.epsilon
    p = min(1.0, p)
    return 0.0 if p == 0.0 else -p * math.log2(p)


class BinaryPolarEncoderDecoder:
    def __init__(self, length, frozenSet, commonRandomnessSeed):
        self.commonRandomnessSeed = commonRandomnessSeed
        self.frozenSet = frozenSet
        self.length = length
        self.frozenOrInformation = np.empty(length, uIndexType)
        self._device_code = None
        self._device_key = None
        self._decoder = None
        self._del_decoders = {}
        self.initializeFrozenOrInformationAndRandomlyGeneratedNumbers()

    def initializeFrozenOrInformationAndRandomlyGeneratedNumbers(self):
        mask = np.zeros(self.length, np.uint8)
        for i in range(self.length):
            if i in self.frozenSet:
                mask[i] = 1
        self.frozenOrInformation[:] = [uIndexType.frozen if m else uIndexType.information for m in mask]
        self.k = int(self.length - mask.sum())
        self._frozen_mask = mask
        r = np.empty(self.length)
        if self.commonRandomnessSeed != -1:
            rng = random.Random()
            rng.seed(self.commonRandomnessSeed)
            for i in range(self.length):
                r[i] = rng.random()
        else:
            r[:] = 1.0
        self.randomlyGeneratedNumbers = r

    # -- device code tables ---------------------------------------------------
    def _code(self):
        from . import sc
        key = (self._frozen_mask.tobytes(), self.randomlyGeneratedNumbers.tobytes())
        if self._device_key != key:
            fval = np.where(0.5 >= self.randomlyGeneratedNumbers, 0, 1).astype(np.uint8)
            self._device_code = sc.CodeSpec(self.length, self._frozen_mask, fval)
            self._decoder = sc.BinaryDecoder(self._device_code)
            self._del_decoders = {}
            self._device_key = key
        return self._device_code

    def _prior(self):
        from . import sc
        code = self._code()
        if getattr(self, "_prior_key", None) != self._device_key:
            self._prior_coder = sc.PriorCoder(code, self.randomlyGeneratedNumbers)
            self._prior_key = self._device_key
        return self._prior_coder

    # -- batched device entry points -------------------------------------------
    def decode_prior_batch(self, prior, xy):
        """Two-tree decode under a non-uniform prior: prior [N, 2] (or [B, N, 2] per codeword),
        xy [B, N, 2].  Returns (encodedVectors int64[B, N], information int64[B, k])."""
        import torch
        pc = self._prior()
        dev = pc.code.device
        px = torch.as_tensor(np.asarray(prior, dtype=np.float64), device=dev)
        if px.dim() == 3:
            px = px.transpose(0, 1)
        info, xh = pc.decode(px, torch.as_tensor(np.asarray(xy, dtype=np.float64), device=dev))
        return xh.cpu().numpy().astype(np.int64), info.cpu().numpy().astype(np.int64)

    def encode_prior_batch(self, prior, information):
        """Encode [B, k] information bits under a non-uniform prior [N, 2]; frozen bits follow
        the prior tree and the common randomness (BinaryPolarEncoderDecoder.py:46-69, 258-262)."""
        import torch
        pc = self._prior()
        dev = pc.code.device
        inf = torch.as_tensor(np.asarray(information, dtype=np.uint8).reshape(-1, self.k), device=dev)
        return pc.encode(torch.as_tensor(np.asarray(prior, dtype=np.float64), device=dev), inf).cpu().numpy().astype(
            np.int64)

    def decode_batch(self, xy):
        """xy: [B, N, 2] joint probabilities (numpy or torch), uniform prior.
        Returns (encodedVectors int64[B, N], information int64[B, k]) as numpy arrays."""
        import torch
        code = self._code()
        if isinstance(xy, torch.Tensor):
            t = xy.to(device=code.device, dtype=torch.float64)
        else:
            t = torch.from_numpy(_check_joint(xy)).to(code.device)
        assert t.dim() == 3 and t.shape[1] == self.length and t.shape[2] == 2
        info, xhat = self._decoder.decode(t)
        return xhat.cpu().numpy().astype(np.int64), info.cpu().numpy().astype(np.int64)

    def decode_deletion_batch(self, receivedWords, deletionProb, n0, ones=0):
        """Received words (0/1 sequences) of the deletion channel -> (encodedVectors int64[B, N],
        information int64[B, k]); the same result as decode() on each word's
        buildCollectionOfBinaryTrellises_uniformInput_deletion(word, deletionProb, xi, n, n0, ones)."""
        from . import sc
        code = self._code()
        key = (int(n0), float(deletionProb), int(ones))
        dec = self._del_decoders.get(key)
        if dec is None:
            dec = self._del_decoders[key] = sc.DeletionDecoder(code, n0, deletionProb, ones)
        rx, ln = sc.pad_words(receivedWords, code.device)
        info, xhat = dec.decode(rx, ln)
        return xhat.cpu().numpy().astype(np.int64), info.cpu().numpy().astype(np.int64)

    def encode_batch(self, information):
        """information: [B, k] bits -> encoded vectors int64[B, N] (uniform prior)."""
        import torch

        from . import sc
        code = self._code()
        inf = torch.as_tensor(np.asarray(information, dtype=np.uint8).reshape(-1, self.k), device=code.device)
        return sc.encode(code, inf).cpu().numpy().astype(np.int64)

    # -- reference API -----------------------------------------------------------
    def encode(self, xVectorDistribution, information):
        assert len(xVectorDistribution) == self.length
        assert len(information) == self.k
        if _is_uniform_prior(xVectorDistribution):
            return self.encode_batch(np.asarray(information, dtype=np.uint8)[None, :])[0]
        prior = _prior_rows(xVectorDistribution, self.length)
        if prior is not None:
            return self.encode_prior_batch(prior, np.asarray(information, dtype=np.uint8)[None, :])[0]
        (enc, nu, ni) = self.recursiveEncodeDecode(information, 0, 0, self.randomlyGeneratedNumbers,
                                                   xVectorDistribution)
        assert nu == len(enc) == len(xVectorDistribution)
        assert ni == len(information)
        return enc

    def decode(self, xVectorDistribution, xyVectorDistribution):
        assert len(xVectorDistribution) == len(xyVectorDistribution) == self.length
        if _is_memoryless_binary(xyVectorDistribution) and _is_uniform_prior(xVectorDistribution):
            xy = _check_joint(xyVectorDistribution.probs)
            enc, info = self.decode_batch(xy[None, :, :])
            return (enc[0], info[0])
        shape = _deletion_kernel_shape(xyVectorDistribution)
        if shape is not None and _is_uniform_prior(xVectorDistribution):
            enc, info = self.decode_deletion_batch([xyVectorDistribution.deletion_source[0]], shape[0], shape[2],
                                                   shape[3])
            return (enc[0], info[0])
        prior = _prior_rows(xVectorDistribution, self.length)
        if prior is not None and _is_memoryless_binary(xyVectorDistribution):
            enc, info = self.decode_prior_batch(prior, _check_joint(xyVectorDistribution.probs)[None, :, :])
            return (enc[0], info[0])
        information = np.empty(self.k, np.int64)
        information[:] = -1
        (enc, nu, ni) = self.recursiveEncodeDecode(information, 0, 0, self.randomlyGeneratedNumbers,
                                                   xVectorDistribution, xyVectorDistribution)
        assert nu == len(enc) == self.length
        assert ni == len(information)
        return (enc, information)

    def geniePreSteps(self, genieSingleRunSeed):
        self.backupFrozenSet = self.frozenSet
        self.backupCommonRandomnessSeed = self.commonRandomnessSeed
        self.frozenSet = set(range(self.length))
        self.commonRandomnessSeed = genieSingleRunSeed
        self.initializeFrozenOrInformationAndRandomlyGeneratedNumbers()

    def geniePostSteps(self):
        self.frozenSet = self.backupFrozenSet
        self.commonRandomnessSeed = self.backupCommonRandomnessSeed
        self.initializeFrozenOrInformationAndRandomlyGeneratedNumbers()

    def genieSingleDecodeSimulatioan(self, xVectorDistribution, xyVectorDistribution, genieSingleRunSeed,
                                     trustXYProbs):
        marg = []
        self.geniePreSteps(genieSingleRunSeed)
        assert len(xVectorDistribution) == self.length
        (decoded, nu, ni) = self.recursiveEncodeDecode([], 0, 0, self.randomlyGeneratedNumbers, xVectorDistribution,
                                                       xyVectorDistribution, marg)
        assert nu == len(decoded) == len(xVectorDistribution)
        assert ni == 0 and len(marg) == self.length
        Pevec, Hvec = [], []
        if trustXYProbs:
            for m0, m1 in marg:
                Pevec.append(min(m0, m1))
                Hvec.append(eta(m0) + eta(m1))
        else:
            u = polarTransformOfBits(decoded)
            for i, pair in enumerate(marg):
                d = u[i]
                if pair[d] > pair[1 - d]:
                    Pevec.append(0.0)
                elif pair[d] == pair[1 - d]:
                    Pevec.append(0.5)
                else:
                    Pevec.append(1.0)
        self.geniePostSteps()
        return (decoded, Pevec, Hvec)

    def genieSingleEncodeSimulatioan(self, xVectorDistribution, genieSingleRunSeed):
        marg = []
        self.geniePreSteps(genieSingleRunSeed)
        assert len(xVectorDistribution) == self.length
        (encoded, nu, ni) = self.recursiveEncodeDecode([], 0, 0, self.randomlyGeneratedNumbers, xVectorDistribution,
                                                       None, marg)
        assert nu == len(encoded) == len(xVectorDistribution)
        assert ni == 0 and len(marg) == self.length
        TVvec = [abs(m0 - m1) for m0, m1 in marg]
        Hvec = [eta(m0) + eta(m1) for m0, m1 in marg]
        self.geniePostSteps()
        return (encoded, TVvec, Hvec)

    def recursiveEncodeDecode(self, information, uIndex, informationVectorIndex, randomlyGeneratedNumbers,
                              xVectorDistribution, xyVectorDistribution=None, marginalizedUProbs=None):
        """Generic SC recursion over any VectorDistribution plugin (BinaryPolarEncoderDecoder.py:223-325).

        Returns (encodedVector int64[len], next_uIndex, next_informationVectorIndex)."""
        n = len(xVectorDistribution)
        out = np.full(n, -1, np.int64)
        if n == 1:
            if self.frozenOrInformation[uIndex] == uIndexType.information:
                if xyVectorDistribution is not None:
                    m = xyVectorDistribution.calcMarginalizedProbabilities()
                    information[informationVectorIndex] = 0 if m[0] >= m[1] else 1
                out[0] = information[informationVectorIndex]
                nxt_info = informationVectorIndex + 1
            else:
                m = xVectorDistribution.calcMarginalizedProbabilities()
                out[0] = 0 if m[0] >= randomlyGeneratedNumbers[uIndex] else 1
                nxt_info = informationVectorIndex
            if marginalizedUProbs is not None:
                src = xyVectorDistribution if xyVectorDistribution is not None else xVectorDistribution
                m = src.calcMarginalizedProbabilities()
                marginalizedUProbs.append([m[0], m[1]])
            return (out, uIndex + 1, nxt_info)

        def child(vd, decisions=None):
            if vd is None:
                return None
            c = vd.minusTransform() if decisions is None else vd.plusTransform(decisions)
            c.normalizeDistList(c.calcNormalizationVector())
            return c

        (minus, uIndex, informationVectorIndex) = self.recursiveEncodeDecode(
            information, uIndex, informationVectorIndex, randomlyGeneratedNumbers, child(xVectorDistribution),
            child(xyVectorDistribution), marginalizedUProbs)
        (plus, uIndex, informationVectorIndex) = self.recursiveEncodeDecode(
            information, uIndex, informationVectorIndex, randomlyGeneratedNumbers, child(xVectorDistribution, minus),
            child(xyVectorDistribution, minus), marginalizedUProbs)
        out[0::2] = (minus + plus) % 2
        out[1::2] = plus
        return (out, uIndex, informationVectorIndex)


def encodeDecodeSimulation(length, make_xVectorDistribution, make_codeword, simulateChannel,
                           make_xyVectrorDistribution, numberOfTrials, frozenSet, commonRandomnessSeed=1,
                           randomInformationSeed=1, verbosity=0):
    """Monte-Carlo SC run (BinaryPolarEncoderDecoder.py:328-387), batched.

    Information bits are drawn from the same seeded MT19937 stream in the same
    order; the user's make_codeword / simulateChannel / make_xyVectrorDistribution
    closures are called once per trial in trial order (so they consume their
    RNGs exactly as in the reference); encoding and decoding of memoryless
    trials run as GPU batches.  Prints the reference's result line."""
    xvd = make_xVectorDistribution()
    encDec = BinaryPolarEncoderDecoder(length, frozenSet, commonRandomnessSeed)
    rng = random.Random()
    rng.seed(randomInformationSeed)
    errors = 0
    chunk = 1 << 16
    uniform = _is_uniform_prior(xvd)
    prior = None if uniform else _prior_rows(xvd, length)
    for t0 in range(0, numberOfTrials, chunk):
        T = min(chunk, numberOfTrials - t0)
        infos = np.array([[0 if rng.random() < 0.5 else 1 for _ in range(encDec.k)] for _ in range(T)],
                         dtype=np.int64).reshape(T, encDec.k)
        if uniform:
            encoded = encDec.encode_batch(infos)
        elif prior is not None:
            encoded = encDec.encode_prior_batch(prior, infos)
        else:
            encoded = np.stack([encDec.encode(xvd, list(infos[t])) for t in range(T)])
        batch_xy, batch_del, pending = [], {}, []
        for t in range(T):
            codeword = make_codeword(encoded[t])
            received = simulateChannel(codeword)
            xyvd = make_xyVectrorDistribution(received)
            shape = _deletion_kernel_shape(xyvd) if uniform else None
            if (uniform or prior is not None) and _is_memoryless_binary(xyvd):
                pending.append((t, codeword, received, ("bin", len(batch_xy))))
                batch_xy.append(_check_joint(xyvd.probs))
            elif shape is not None:
                words = batch_del.setdefault(shape, [])
                pending.append((t, codeword, received, (shape, len(words))))
                words.append(xyvd.deletion_source[0])
            else:
                pending.append((t, codeword, received, encDec.decode(xvd, xyvd)[1]))
        results = {}
        if batch_xy and uniform:
            results["bin"] = encDec.decode_batch(np.stack(batch_xy))[1]
        elif batch_xy:
            results["bin"] = encDec.decode_prior_batch(prior, np.stack(batch_xy))[1]
        for shape, words in batch_del.items():
            results[shape] = encDec.decode_deletion_batch(words, shape[0], shape[2], shape[3])[1]
        for (t, codeword, received, info_t) in pending:
            if isinstance(info_t, tuple):
                info_t = results[info_t[0]][info_t[1]]
            if np.any(info_t != infos[t]):
                errors += 1
                if verbosity > 0:
                    s = str(t0 + t) + ") error, transmitted inforamtion:\n" + str(infos[t].tolist())
                    s += "\ndecoded information:\n" + str(info_t)
                    s += "\nencoded vector before guard bands added:\n" + str(encoded[t])
                    s += "\ncodeword:\n" + str(codeword)
                    s += "\nreceived word:\n" + str(received)
                    print(s)
    print("Error probability = ", errors, "/", numberOfTrials, " = ", errors / numberOfTrials)


def _genie_u(length, seed):
    """The genie's frozen values for one trial: u_i = 0 if 0.5 >= r_i else 1 with r_i the
    MT19937 draws of Random(seed) (BinaryPolarEncoderDecoder.py:33-44, 258-262; uniform prior)."""
    rng = random.Random()
    rng.seed(seed)
    return np.array([0 if 0.5 >= rng.random() else 1 for _ in range(length)], np.uint8)


def _genie_stats(m, u, trustXYProbs):
    """Pe / H of one genie decode from its leaf marginals m [N, 2] and the genie's u
    (genieSingleDecodeSimulatioan, BinaryPolarEncoderDecoder.py:114-178)."""
    if trustXYProbs:
        pe = [float(min(a, b)) for a, b in m]
        h = [eta(float(a)) + eta(float(b)) for a, b in m]
        return pe, h
    mu = m[np.arange(len(u)), u]
    mo = m[np.arange(len(u)), 1 - u]
    pe = np.where(mu > mo, 0.0, np.where(mu == mo, 0.5, 1.0))
    return [float(v) for v in pe], []


def genieEncodeDecodeSimulation(length, make_xVectorDistribution, make_codeword, simulateChannel,
                                make_xyVectrorDistribution, numberOfTrials, errorUpperBoundForFrozenSet, genieSeed,
                                trustXYProbs=True, filename=None):
    """Genie construction run (BinaryPolarEncoderDecoder.py:390-491); returns the frozen set
    and optionally writes the frozen-set file in the reference's format.

    Batched: the per-trial seeds, common randomness and the user's closures run on the
    host in trial order (consuming their RNGs exactly as the reference does); under a
    uniform prior the genie encoder is the GPU polar transform and the genie decodes of
    memoryless and deletion-collection trials run on the GPU with every leaf exported
    (pcub_sc_leaf_bin / pcub_sc_leaf_deletion, per-trial frozen values).  Other plugins
    use the generic per-trial recursion.  Statistics are accumulated in trial order."""
    xvd = make_xVectorDistribution()
    encDec = BinaryPolarEncoderDecoder(length, set(), 0)
    seed_rng = random.Random()
    seed_rng.seed(genieSeed)
    uniform = _is_uniform_prior(xvd)
    TV = Pe = HEnc = HDec = None
    codeword = []
    chunk = 1 << 12
    for t0 in range(0, numberOfTrials, chunk):
        T = min(chunk, numberOfTrials - t0)
        seeds = [seed_rng.randint(1, 1000000) for _ in range(T)]
        enc_stats = []
        if uniform:
            U = np.stack([_genie_u(length, s) for s in seeds])
            enc_all = BinaryPolarEncoderDecoder(length, set(), 0).encode_batch(U)  # K = N: x = polar(u)
            h_half = eta(0.5) + eta(0.5)
            for t in range(T):
                enc_stats.append((enc_all[t], [abs(0.5 - 0.5)] * length, [h_half] * length))
        else:
            U = None
            for s in seeds:
                enc_stats.append(encDec.genieSingleEncodeSimulatioan(xvd, s))
        items, bin_rows, del_rows = [], [], {}
        for t in range(T):
            codeword = make_codeword(enc_stats[t][0])
            received = simulateChannel(codeword)
            xyvd = make_xyVectrorDistribution(received)
            shape = _deletion_kernel_shape(xyvd, leaves=True) if uniform else None
            if uniform and _is_memoryless_binary(xyvd) and length >= 2:
                items.append(("bin", len(bin_rows)))
                bin_rows.append(_check_joint(xyvd.probs))
            elif shape is not None:
                rows = del_rows.setdefault(shape, [])
                items.append((shape, len(rows)))
                rows.append((t, xyvd.deletion_source[0]))
            else:
                items.append(("host", encDec.genieSingleDecodeSimulatioan(xvd, xyvd, seeds[t], trustXYProbs)))
        marg = {}
        if bin_rows:
            marg["bin"] = _device_genie_bin(length, np.stack(bin_rows), U[[t for t, it in enumerate(items)
                                                                            if it[0] == "bin"]])
        for shape, rows in del_rows.items():
            marg[shape] = _device_genie_deletion(length, shape, [w for _, w in rows], U[[t for t, _ in rows]])
        for t in range(T):
            kind, val = items[t]
            if kind == "host":
                _, pe, hdec = val
            else:
                pe, hdec = _genie_stats(marg[kind][val], U[t], trustXYProbs)
            _, tv, henc = enc_stats[t]
            if TV is None:
                TV, Pe, HEnc, HDec = list(tv), list(pe), list(henc), list(hdec)
            else:
                for i in range(len(TV)):
                    TV[i] += tv[i]
                    Pe[i] += pe[i]
                    HEnc[i] += henc[i]
                    if trustXYProbs:
                        HDec[i] += hdec[i]
    hes = hds = 0.0
    for i in range(len(TV)):
        TV[i] /= numberOfTrials
        Pe[i] /= numberOfTrials
        HEnc[i] /= numberOfTrials
        hes += HEnc[i]
        if trustXYProbs:
            HDec[i] /= numberOfTrials
            hds += HDec[i]
    print("TVVec = ", TV)
    print("pevec = ", Pe)
    print("HEncvec = ", HEnc)
    if trustXYProbs:
        print("HDecvec = ", HDec)
    print("Normalized HEncsum = ", hes / len(HEnc))
    if trustXYProbs:
        print("Normalized HDecsum = ", hds / len(HDec))
    frozenSet = frozenSetFromTVAndPe(TV, Pe, errorUpperBoundForFrozenSet)
    print("code rate = ", (len(TV) - len(frozenSet)) / len(codeword))
    print("codeword length = ", len(codeword))
    if filename is not None:
        write_frozen_file(filename, frozenSet, numberOfTrials, TV, Pe)
    return frozenSet


def _device_genie_bin(length, xy, U):
    """Genie decodes of memoryless trials on the GPU: all positions frozen to the trial's u.
    Returns leaf marginals [T, N, 2] (numpy)."""
    import torch

    from . import sc
    code = sc.CodeSpec(length, np.ones(length, np.uint8), np.zeros(length, np.uint8))
    _, _, m = sc.LeafDecoder(code).decode(torch.from_numpy(xy).to(code.device), torch.from_numpy(U).to(code.device))
    return m.cpu().numpy()


def _device_genie_deletion(length, shape, words, U):
    import torch

    from . import sc
    pd, n, n0, ones = shape
    code = sc.CodeSpec(length, np.ones(length, np.uint8), np.zeros(length, np.uint8))
    rx, ln = sc.pad_words(words, code.device)
    _, _, m = sc.DeletionDecoder(code, n0, pd, ones).decode_leaves(rx, ln, torch.from_numpy(U).to(code.device))
    return m.cpu().numpy()


def write_frozen_file(filename, frozenSet, numberOfTrials, TVvec, Pevec, argv=None):
    """Frozen-set file format of BinaryPolarEncoderDecoder.py:471-489."""
    with open(filename, "w") as f:
        f.write("* " + " ".join(sys.argv[:] if argv is None else argv) + "\n")
        for i in frozenSet:
            f.write(str(i) + "\n")
        f.write("** number of trials = " + str(numberOfTrials) + "\n")
        f.write("* (TotalVariation+errorProbability) * (number of trials)\n")
        for i in range(len(TVvec)):
            f.write("*** " + str(i) + " " + str((TVvec[i] + Pevec[i]) * numberOfTrials) + "\n")


def read_frozen_file(filename):
    """Reader of the same format (main_deletion.py:149-159): every line not starting with '*'."""
    frozen = set()
    with open(filename) as f:
        for line in f:
            if line[0] == "*":
                continue
            frozen.add(int(line))
    return frozen


def polarTransformOfBits(xvec):
    """x -> u for the adjacent-pair convention (BinaryPolarEncoderDecoder.py:494-516); list in, list out."""
    x = np.asarray(list(xvec), dtype=np.int64)
    N = len(x)
    if N == 1:
        return list(xvec)
    assert N % 2 == 0
    # each level splits every vector v into [v0^v1, v2^v3, ...] and [v1, v3, ...],
    # kept in order (first part before second), until vectors have length 1
    cur = x.reshape(1, N)
    while cur.shape[1] > 1:
        a, b = cur[:, 0::2], cur[:, 1::2]
        cur = np.stack([(a + b) % 2, b], axis=1).reshape(-1, cur.shape[1] // 2)
    return [int(v) for v in cur[:, 0]]


def frozenSetFromTVAndPe(TVvec, Pevec, errorUpperBoundForFrozenSet):
    """Frozen-set picker (BinaryPolarEncoderDecoder.py:519-548)."""
    tvpe = [TVvec[i] + Pevec[i] for i in range(len(TVvec))]
    order = sorted(range(len(tvpe)), key=lambda k: tvpe[k])
    total = 0.0
    last = -1
    while total < errorUpperBoundForFrozenSet and last + 1 < len(tvpe):
        i = order[last + 1]
        if tvpe[i] + total <= errorUpperBoundForFrozenSet:
            total += tvpe[i]
            last += 1
        else:
            break
    frozenSet = set(order[j] for j in range(last + 1, len(tvpe)))
    print("frozen set =", frozenSet)
    print("fraction of non-frozen indices =", 1.0 - len(frozenSet) / len(tvpe))
    return frozenSet
