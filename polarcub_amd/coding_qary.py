"""Reference-compatible q-ary polar encoder/decoder (QaryPolarEncoderDecoder.py), SC part.

  QaryPolarEncoderDecoder(q, length, frozenSet, commonRandomnessSeed, use_log=False)   :27-53
      .encode(xVD, information) -> int64[N]                                           :65-88
      .decode(xVD, xyVD) -> int64[k]                                                  :90-116
      .recursiveEncodeDecode(...)                                                     :318-401
  encodeDecodeSimulation(q, length, ...)                                              :935-982
  polarTransformOfQudits(q, xvec)                                                     :1136-1154
  frozenSetFromTVAndPe(TVvec, Pevec, errorUpperBoundForFrozenSet, numInfoIndices, verbosity) :1157-1191

decode() of a linear-domain QaryMemorylessVectorDistribution (2 <= q <= 8,
N >= 4) runs on the GPU (pcub_sc_decode_qary), bit-identical to the
reference; the a-priori tree never influences q-ary decisions (frozen symbols
are 0), so any prior is accepted.  decode() of a log-domain (use_log=True)
memoryless distribution (2 <= q <= 8, 2 <= N <= 2^16) runs on the GPU log-domain
kernel (pcub_sc_decode_qary_log: numpy's logaddexp and scipy's logsumexp restated
over the device's exp/log1p/log, so within a few ulps of the reference rather than
bit-identical).  Other plugins use the generic recursion over the plugin's own
methods.  List decoding and the IR simulation (:118-227, :403-930) are not part of
this module.
"""
import random

import numpy as np

from . import vectors


class uIndexType:
    frozen = 0
    information = 1


def _is_qary_memoryless(vd):
    return (isinstance(vd, vectors.QaryMemorylessVectorDistribution)
            or (type(vd).__name__ == "QaryMemorylessVectorDistribution" and hasattr(vd, "probs")))


class QaryPolarEncoderDecoder:
    def __init__(self, q, length, frozenSet, commonRandomnessSeed, use_log=False):
        self.q = q
        self.commonRandomnessSeed = commonRandomnessSeed
        self.frozenSet = sorted(frozenSet)
        self.infoSet = sorted(set(i for i in range(length) if i not in set(self.frozenSet)))
        self.length = length
        self.k = length - len(self.frozenSet)
        self.frozenOrInformation = np.full(length, uIndexType.information, dtype=object)
        self.frozenOrInformation[list(self.frozenSet)] = uIndexType.frozen
        if commonRandomnessSeed != -1:
            rng = random.Random(commonRandomnessSeed)
            self.randomlyGeneratedNumbers = np.array([rng.random() for _ in range(length)])
        else:
            self.randomlyGeneratedNumbers = np.full(length, 1.0)
        self.use_log = use_log
        self._mask = np.zeros(length, np.uint8)
        self._mask[list(self.frozenSet)] = 1
        self._dev = None

    def _device(self):
        from . import sc
        if self._dev is None:
            code = sc.QaryCode(self.q, self.length, self._mask)
            self._dev = (code, sc.QaryDecoder(code))
        return self._dev

    def _device_ok(self):
        return 2 <= self.q <= 8 and self.length >= 4

    def _log_device(self):
        from . import sc
        if getattr(self, "_logdev", None) is None:
            self._logdev = sc.QaryLogDecoder(self.q, self.length, self._mask)
        return self._logdev

    def decode_log_batch(self, xy):
        """xy: [B, N, q] log-domain rows (use_log=True) -> information int64[B, k]."""
        import torch
        dec = self._log_device()
        t = xy if isinstance(xy, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(xy, np.float64))
        info, _ = dec.decode(t.to(dec.device, torch.float64))
        return info.cpu().numpy().astype(np.int64)

    def decode_batch(self, xy):
        """xy: [B, N, q] linear-domain joint probabilities -> information int64[B, k]."""
        import torch
        code, dec = self._device()
        t = xy if isinstance(xy, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(xy, np.float64))
        info, _ = dec.decode(t.to(code.device, torch.float64))
        return info.cpu().numpy().astype(np.int64)

    def encode_batch(self, information):
        import torch

        from . import sc
        code, _ = self._device()
        inf = torch.as_tensor(np.asarray(information, dtype=np.uint8).reshape(-1, self.k), device=code.device)
        return sc.encode_qary(code, inf).cpu().numpy().astype(np.int64)

    def encode(self, xVectorDistribution, information):
        assert len(xVectorDistribution) == self.length
        assert len(information) == self.k
        if self._device_ok():
            return self.encode_batch(np.asarray(information)[None, :])[0]
        (enc, nu, ni) = self.recursiveEncodeDecode(information, 0, 0, xVectorDistribution)
        assert nu == len(enc) == self.length and ni == self.k
        return enc

    def decode(self, xVectorDistribution, xyVectorDistribution):
        assert len(xVectorDistribution) == len(xyVectorDistribution) == self.length
        if (self._device_ok() and _is_qary_memoryless(xyVectorDistribution)
                and not getattr(xyVectorDistribution, "use_log", False)):
            p = np.asarray(xyVectorDistribution.probs, dtype=np.float64)
            assert np.all(p >= 0) and np.all(np.isfinite(p)), "probabilities must be finite and non-negative"
            return self.decode_batch(p[None])[0]
        if (2 <= self.q <= 8 and 2 <= self.length <= 1 << 16 and _is_qary_memoryless(xyVectorDistribution)
                and getattr(xyVectorDistribution, "use_log", False)):
            p = np.asarray(xyVectorDistribution.probs, dtype=np.float64)
            assert not np.any(np.isnan(p)) and not np.any(p == np.inf), "log-probabilities must be < +inf"
            return self.decode_log_batch(p[None])[0]
        information = np.full(self.k, -1, dtype=np.int64)
        (enc, nu, ni) = self.recursiveEncodeDecode(information, 0, 0, xVectorDistribution, xyVectorDistribution)
        assert nu == len(enc) == self.length and ni == self.k
        return information

    def recursiveEncodeDecode(self, information, uIndex, informationVectorIndex, xVectorDistribution,
                              xyVectorDistribution=None, marginalizedUProbs=None):
        """Generic q-ary SC recursion over plugin methods (QaryPolarEncoderDecoder.py:318-401)."""
        n = len(xVectorDistribution)
        q = self.q
        out = np.full(n, -1, dtype=np.int64)
        decoding = xyVectorDistribution is not None
        if n == 1:
            if self.frozenOrInformation[uIndex] == uIndexType.information:
                if decoding:
                    information[informationVectorIndex] = np.argmax(
                        xyVectorDistribution.calcMarginalizedProbabilities())
                out[0] = information[informationVectorIndex]
                ni = informationVectorIndex + 1
            else:
                out[0] = 0
                ni = informationVectorIndex
            if marginalizedUProbs is not None:
                marginalizedUProbs.append((xyVectorDistribution or xVectorDistribution).calcMarginalizedProbabilities())
            return (out, uIndex + 1, ni)

        def child(vd, decisions=None):
            if vd is None:
                return None
            c = vd.minusTransform() if decisions is None else vd.plusTransform(decisions)
            c.normalize()
            return c

        (m, uIndex, informationVectorIndex) = self.recursiveEncodeDecode(
            information, uIndex, informationVectorIndex, child(xVectorDistribution), child(xyVectorDistribution),
            marginalizedUProbs)
        (p, uIndex, informationVectorIndex) = self.recursiveEncodeDecode(
            information, uIndex, informationVectorIndex, child(xVectorDistribution, m),
            child(xyVectorDistribution, m) if decoding else None, marginalizedUProbs)
        out[0::2] = (m + p) % q
        out[1::2] = (q - p) % q
        return (out, uIndex, informationVectorIndex)


def encodeDecodeSimulation(q, length, make_xVectorDistribution, make_codeword, simulateChannel,
                           make_xyVectorDistribution, numberOfTrials, frozenSet, commonRandomnessSeed=1,
                           randomInformationSeed=1, verbosity=0):
    """q-ary Monte-Carlo SC run (QaryPolarEncoderDecoder.py:935-982), batched like the binary driver:
    trials in chunks of 2^14 (information from the seeded stream in trial order, the user's
    closures once per trial in trial order, one GPU encode and one GPU decode per chunk)."""
    xvd = make_xVectorDistribution()
    encDec = QaryPolarEncoderDecoder(q, length, frozenSet, commonRandomnessSeed)
    rng = random.Random(randomInformationSeed)
    errors = 0
    chunk = 1 << 14
    for t0 in range(0, numberOfTrials, chunk):
        T = min(chunk, numberOfTrials - t0)
        infos = [rng.choices(range(0, q), k=encDec.k) for _ in range(T)]
        if encDec._device_ok():
            encoded = encDec.encode_batch(np.array(infos, dtype=np.int64).reshape(T, encDec.k))
        else:
            encoded = [encDec.encode(xvd, inf) for inf in infos]
        batch, slots = [], []
        decoded = [None] * T
        for t in range(T):
            xyvd = make_xyVectorDistribution(simulateChannel(make_codeword(encoded[t])))
            if encDec._device_ok() and _is_qary_memoryless(xyvd) and not getattr(xyvd, "use_log", False):
                batch.append(np.asarray(xyvd.probs, dtype=np.float64))
                slots.append(t)
            else:
                decoded[t] = encDec.decode(xvd, xyvd)
        if batch:
            dec = encDec.decode_batch(np.stack(batch))
            for i, t in enumerate(slots):
                decoded[t] = dec[i]
        for t in range(T):
            if not np.array_equal(infos[t], decoded[t]):
                errors += 1
    print("Error probability = ", errors, "/", numberOfTrials, " = ", errors / numberOfTrials)


def polarTransformOfQudits(q, xvec):
    """x -> u for the q-ary convention (QaryPolarEncoderDecoder.py:1136-1154)."""
    x = np.asarray(xvec, dtype=np.int64)
    if len(x) == 1:
        return x
    assert len(x) % 2 == 0
    cur = x.reshape(1, -1)
    while cur.shape[1] > 1:
        a, b = cur[:, 0::2], cur[:, 1::2]
        cur = np.stack([(a + b) % q, (q - b) % q], axis=1).reshape(-1, cur.shape[1] // 2)
    return cur[:, 0]


def frozenSetFromTVAndPe(TVvec, Pevec, errorUpperBoundForFrozenSet=None, numInfoIndices=None, verbosity=False):
    """q-ary frozen-set picker (QaryPolarEncoderDecoder.py:1157-1191), including its
    quirks: with numInfoIndices the number of information indices is numInfoIndices + 1
    (:1173-1176), and the single-frozen-segment fix-up never fires (:1180)."""
    tvpe = np.add(TVvec, Pevec)
    N = len(tvpe)
    order = sorted(range(N), key=lambda k: tvpe[k])
    if numInfoIndices is None:
        total = 0.0
        last = -1
        while total < errorUpperBoundForFrozenSet and last + 1 < N:
            i = order[last + 1]
            if tvpe[i] + total <= errorUpperBoundForFrozenSet:
                total += tvpe[i]
                last += 1
            else:
                break
    else:
        last = numInfoIndices
    frozen = set(order[last + 1:])
    if verbosity:
        print("frozen set =", frozen)
        if numInfoIndices is None:
            print("fraction of info indices =", 1.0 - len(frozen) / N)
    return frozen
