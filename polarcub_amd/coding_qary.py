"""Reference-compatible q-ary polar encoder/decoder (QaryPolarEncoderDecoder.py), SC part.

  QaryPolarEncoderDecoder(q, length, frozenSet, commonRandomnessSeed, use_log=False)   :27-53
      .encode(xVD, information) -> int64[N]                                           :65-88
      .decode(xVD, xyVD) -> int64[k]                                                  :90-116
      .recursiveEncodeDecode(...)                                                     :318-401
  encodeDecodeSimulation(q, length, ...)                                              :935-982
  encodeListDecodeSimulation(q, length, ..., maxListSize, checkSize)                  :985-1035
  irSimulation(q, length, ...), ProbResult, hamming                                   :18-24, 887-933
  normalize / calcNormalizationVector / normalizeDistList                             :867-885
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
methods.  List decoding (listDecode, :118-227, 403-820) runs on the GPU list decoder
(pcub_scl_qary; pcub_scl_qary_log for use_log=True, within a few ulps of the reference's
log-domain metrics) and irSimulation / ir (:822-930) batch it; the list's
tie-breaking and order are documented in include/polarcub_sc.h.
"""
import math
import random
from enum import Enum

import numpy as np

from . import vectors


class uIndexType:
    frozen = 0
    information = 1


def _is_qary_memoryless(vd):
    return (isinstance(vd, vectors.QaryMemorylessVectorDistribution)
            or (type(vd).__name__ == "QaryMemorylessVectorDistribution" and hasattr(vd, "probs")))


class ProbResult(Enum):
    SuccessActualIsMax = 0
    SuccessActualSmallerThanMax = 1
    FailActualLargerThanMax = 2
    FailActualIsMax = 3
    FailActualWithinRange = 4
    FailActualSmallerThanMin = 5


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

    # -- list decoding and information reconciliation (:118-242, 822-865) --------------------
    def list_decode_batch(self, xy, frozenValues, maxListSize, actualInformation=None):
        """Batched listDecode core on the GPU (pcub_scl_qary, or pcub_scl_qary_log when use_log):
        xy [B, N, q] rows in the decoder's domain, frozenValues [B, nF], actualInformation [B, K]
        or None -> (info [B, L, K] int64 with -1 rows past each list's size, prob [B, L], size [B],
        actual_prob [B] | None)."""
        from . import sc
        if not hasattr(self, "_scl"):
            self._scl = {}
        key = (int(maxListSize), bool(self.use_log))
        dec = self._scl.get(key)
        if dec is None:
            dec = self._scl[key] = sc.QaryListDecoder(self.q, self.length, self._mask, int(maxListSize),
                                                      use_log=bool(self.use_log))
        info, prob, size, ap = dec.decode(xy, frozenValues, actualInformation)
        info = info.astype(np.int64)
        info[info == 0xff] = -1
        return info, prob, size, ap

    def _list_result(self, infos, probs, size, actual_prob, maxListSize, check_matrix, check_value,
                     actualInformation):
        """listDecode's return value from its final list (QaryPolarEncoderDecoder.py:172-227)."""
        prob_list = probs[:size]
        if actualInformation is not None:
            actual = np.asarray(actualInformation)
            for i, information in enumerate(infos[:maxListSize]):
                if np.array_equal(information, actual):
                    return information, (ProbResult.SuccessActualIsMax if prob_list[i] == max(prob_list)
                                         else ProbResult.SuccessActualSmallerThanMax)
            mx = max(prob_list)
            if actual_prob > mx:
                pr = ProbResult.FailActualLargerThanMax
            elif actual_prob == mx:
                pr = ProbResult.FailActualIsMax
            elif actual_prob >= min(prob_list):
                pr = ProbResult.FailActualWithinRange
            else:
                pr = ProbResult.FailActualSmallerThanMin
            return infos[0], pr
        for information in infos[:maxListSize]:
            if np.array_equal(np.matmul(information, check_matrix) % self.q, check_value):
                return information, None
        return infos[0], None

    def listDecode(self, xyVectorDistribution, frozenValues, maxListSize, check_matrix, check_value,
                   actualInformation=None, verbosity=0):
        """QaryPolarEncoderDecoder.listDecode (:118-227) on the GPU list decoder, linear or log
        domain (use_log); the list's tie-breaking and order are documented in include/polarcub_sc.h."""
        self._check_domain(xyVectorDistribution)
        assert len(xyVectorDistribution) == self.length
        xy = np.asarray(xyVectorDistribution.probs, dtype=np.float64)[None]
        act = None if actualInformation is None else np.asarray(actualInformation)[None]
        info, prob, size, ap = self.list_decode_batch(xy, np.asarray(frozenValues).reshape(1, -1), maxListSize, act)
        self.prob_list = prob[0, :size[0]]
        self.actual_prob = None if ap is None else float(ap[0])
        return self._list_result(info[0], prob[0], int(size[0]), self.actual_prob, maxListSize, check_matrix,
                                 check_value, actualInformation)

    def _check_domain(self, xyvd):
        """The kernels run one domain end to end; the reference lets the vector distribution's
        use_log drive the transforms and the decoder's the path metrics, so a mixed pair would
        combine log rows with linear metrics (or the reverse) there: refused here."""
        if bool(getattr(xyvd, "use_log", False)) != bool(self.use_log):
            raise NotImplementedError("list decoding needs the decoder and the vector distribution in the same "
                                      "domain (use_log=%s vs %s)" % (self.use_log, getattr(xyvd, "use_log", False)))

    def mergeInfoAndFrozen(self, actualInformation, frozenValues):
        merged = np.empty(self.length, dtype=np.int64)
        merged[list(self.infoSet)] = actualInformation
        merged[list(self.frozenSet)] = frozenValues
        return merged

    def calc_explicit_prob(self, information, frozenValues, xyVectorDistribution):
        guess = polarTransformOfQudits(self.q, self.mergeInfoAndFrozen(information, frozenValues))
        vals = [row[guess[i]] for i, row in enumerate(xyVectorDistribution.probs)]
        return sum(vals) if self.use_log else np.prod(vals)

    def calculate_syndrome_and_complement(self, u_message):
        y = polarTransformOfQudits(self.q, u_message)
        w = np.copy(y)
        w[list(self.infoSet)] = 0
        w[list(self.frozenSet)] *= self.q - 1
        w[list(self.frozenSet)] %= self.q
        u = y
        u[list(self.frozenSet)] = 0
        return w, u

    def get_message_info_bits(self, u_message):
        return np.asarray(u_message)[list(self.infoSet)]

    def get_message_frozen_bits(self, u_message):
        return np.asarray(u_message)[list(self.frozenSet)]

    def _ir_inputs(self, a, b, make_xyVectorDistribution, check_size):
        """ir()'s preparation (:841-855), consuming the global numpy RNG as the reference does."""
        w, u = self.calculate_syndrome_and_complement(a)
        a_key = self.get_message_info_bits(u)
        frozen_values = (self.get_message_frozen_bits(w) * (self.q - 1)) % self.q
        check_matrix = np.random.choice(range(self.q), (self.k, check_size))
        check_value = np.matmul(a_key, check_matrix) % self.q
        xyvd = make_xyVectorDistribution(b)
        return a_key, frozen_values, check_matrix, check_value, xyvd

    def ir(self, a, b, make_xyVectorDistribution, list_size=1, check_size=0, verbosity=0):
        """Information reconciliation of one pair (:841-858)."""
        a_key, frozen_values, check_matrix, check_value, xyvd = self._ir_inputs(a, b, make_xyVectorDistribution,
                                                                                check_size)
        b_key, prob_result = self.listDecode(xyvd, frozen_values, list_size, check_matrix, check_value,
                                             actualInformation=a_key, verbosity=verbosity)
        return a_key, b_key, prob_result

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


def encodeListDecodeSimulation(q, length, make_xVectorDistribution, make_codeword, simulateChannel,
                               make_xyVectorDistribution, numberOfTrials, frozenSet, maxListSize, checkSize,
                               commonRandomnessSeed=1, randomInformationSeed=1, verbosity=0, chunk=4096):
    """q-ary Monte-Carlo run with the list decoder (QaryPolarEncoderDecoder.py:985-1035), batched.

    Per trial, in trial order and exactly as the reference consumes them: the information from
    random.Random(randomInformationSeed) (:1017), the user's make_codeword / simulateChannel /
    make_xyVectorDistribution closures (:1020-1023) and the check matrix from the global numpy
    RNG (:1025-1026); the encodes (one per chunk) and the list decodes (one per chunk) run on
    the GPU.  Prints the reference's "Error probability = " line.

    The reference itself fails on its first trial: its call listDecode(xyVectorDistribution,
    maxListSize, check_matrix, check_value, information, ...) (:1028) predates listDecode's
    frozenValues parameter (:118), so every argument lands one slot over -- the check matrix in
    maxListSize, whose np.full((maxListSize * q, k), -1) (:131) raises TypeError ("only integer
    scalar arrays can be converted to a scalar index"; tests/golden/harness_names.json).  This runs what the driver
    evidently means: the encoder's frozen symbols (0, :351) as frozenValues, maxListSize,
    check_matrix / check_value as named, the trial's information as actualInformation, and a
    frame error when listDecode's decided information (its first return value) differs."""
    xvd = make_xVectorDistribution()
    encDec = QaryPolarEncoderDecoder(q, length, frozenSet, commonRandomnessSeed)
    if maxListSize < 1:
        raise ValueError("maxListSize must be >= 1")
    informationRNG = random.Random(randomInformationSeed)
    misdecodedWords = 0
    nF = len(encDec.frozenSet)
    for t0 in range(0, numberOfTrials, chunk):
        T = min(chunk, numberOfTrials - t0)
        infos = [informationRNG.choices(range(0, q), k=encDec.k) for _ in range(T)]
        if encDec._device_ok():
            encoded = encDec.encode_batch(np.array(infos, dtype=np.int64).reshape(T, encDec.k))
        else:
            encoded = [encDec.encode(xvd, inf) for inf in infos]
        xys, checks = [], []
        for t in range(T):
            xyvd = make_xyVectorDistribution(simulateChannel(make_codeword(encoded[t])))
            check_matrix = np.random.choice(range(q), (encDec.k, checkSize))
            check_value = np.matmul(infos[t], check_matrix) % q
            checks.append((check_matrix, check_value))
            if getattr(xyvd, "use_log", False) or not hasattr(xyvd, "probs"):
                raise NotImplementedError("list decoding runs on linear-domain memoryless distributions")
            assert len(xyvd) == encDec.length
            xys.append(np.asarray(xyvd.probs, dtype=np.float64))
        act = np.array(infos, dtype=np.int64).reshape(T, encDec.k)
        info, prob, size, ap = encDec.list_decode_batch(np.stack(xys), np.zeros((T, nF), np.int64), maxListSize,
                                                        act)
        for t in range(T):
            decoded, _ = encDec._list_result(info[t], prob[t], int(size[t]), float(ap[t]), maxListSize,
                                             checks[t][0], checks[t][1], act[t])
            if not np.array_equal(infos[t], decoded):
                misdecodedWords += 1
    print("Error probability = ", misdecodedWords, "/", numberOfTrials, " = ", misdecodedWords / numberOfTrials)


def genieEncodeDecodeSimulation(length, make_xVectorDistribution, make_codeword, simulateChannel,
                                make_xyVectorDistribution, numberOfTrials, errorUpperBoundForFrozenSet, genieSeed,
                                trustXYProbs=True, filename=None):
    """QaryPolarEncoderDecoder.genieEncodeDecodeSimulation (:1038-1133) as the reference runs it:
    it builds QaryPolarEncoderDecoder(length, set(range(length)), 0) without q (:1061), which
    raises TypeError before the first trial (after make_xVectorDistribution() has run).  The
    q-ary genie has no working reference behaviour to reproduce; the binary genie
    (coding.genieEncodeDecodeSimulation) is the supported one."""
    make_xVectorDistribution()
    raise TypeError("QaryPolarEncoderDecoder.__init__() missing 1 required positional argument: "
                    "'commonRandomnessSeed'")


def normalize(prob_list, use_log=False):
    """Max-normalisation of a path-metric list (:867-872): (prob_list / max, max), or in the log
    domain (prob_list - max, max)."""
    maxProb = np.max(prob_list)
    if use_log:
        return prob_list - maxProb, maxProb
    return prob_list / maxProb, maxProb


def calcNormalizationVector(dist_list):
    """Per position, the largest entry over a list of vector distributions (:874-879)."""
    segment_size = len(dist_list[0].probs)
    normalization = np.zeros(segment_size)
    for i in range(segment_size):
        normalization[i] = max([np.asarray(dist.probs[i]).max(axis=0) for dist in dist_list])
    return normalization


def normalizeDistList(dist_list):
    """Normalise every distribution of the list by the shared vector (:881-885)."""
    normalization_vector = calcNormalizationVector(dist_list)
    for dist in dist_list:
        dist.normalize(normalization_vector)
    return dist_list, normalization_vector


def hamming(x, y):
    return sum(np.asarray(x) != np.asarray(y))


def irSimulation(q, length, simulateChannel, make_xyVectorDistribution, numberOfTrials, frozenSet, maxListSize=1,
                 checkSize=0, commonRandomnessSeed=1, randomInformationSeed=1, use_log=False, verbosity=0,
                 ir_version=1, chunk=4096):
    """Information-reconciliation simulation (QaryPolarEncoderDecoder.py:887-930), batched: the
    per-trial draws (information RNG, the channel closure, the global numpy RNG of the check
    matrix) run on the host in trial order exactly as the reference consumes them, the list
    decodes run on the GPU in chunks.  Returns (frame_error_prob, symbol_error_prob, rate,
    probResultList) and prints the reference's lines when verbosity is set."""
    if ir_version != 1:
        raise TypeError("ir2 (ir_version=2) fails in the reference itself (listDecode argument mismatch)")
    encDec = QaryPolarEncoderDecoder(q, length, frozenSet, commonRandomnessSeed, use_log=use_log)
    informationRNG = random.Random(randomInformationSeed)
    badKeys = badSymbols = 0
    probResultList = []
    a_key = None
    for t0 in range(0, numberOfTrials, chunk):
        T = min(chunk, numberOfTrials - t0)
        keys, fvs, xys = [], [], []
        for _ in range(T):
            a = informationRNG.choices(range(0, q), k=encDec.length)
            b = simulateChannel(a)
            a_key, fv, _, _, xyvd = encDec._ir_inputs(a, b, make_xyVectorDistribution, checkSize)
            encDec._check_domain(xyvd)
            keys.append(a_key)
            fvs.append(fv)
            xys.append(np.asarray(xyvd.probs, dtype=np.float64))
        info, prob, size, ap = encDec.list_decode_batch(np.stack(xys), np.stack(fvs), maxListSize, np.stack(keys))
        for t in range(T):
            b_key, pr = encDec._list_result(info[t], prob[t], int(size[t]), float(ap[t]), maxListSize, None, None,
                                            keys[t])
            probResultList.append(pr)
            if not np.array_equal(keys[t], b_key):
                badKeys += 1
                badSymbols += hamming(keys[t], b_key)
    assert len(a_key) == length - len(frozenSet)
    rate = (math.log2(q) * len(a_key) - math.log2(maxListSize)) / length
    frame_error_prob = badKeys / numberOfTrials
    symbol_error_prob = badSymbols / (numberOfTrials * encDec.length)
    if verbosity:
        print("Rate: ", rate)
        print("Frame error probability = ", badKeys, "/", numberOfTrials, " = ", frame_error_prob)
        print("Symbol error probability = ", badSymbols, "/ (", numberOfTrials, " * ", encDec.length, ") = ",
              symbol_error_prob)
    return frame_error_prob, symbol_error_prob, rate, probResultList


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
