"""VectorDistribution plugin protocol and the memoryless implementations.

Mirrors the reference's plugin API (VectorDistribution.py:1-29) so user plugins
and harness code keep working.  The memoryless classes hold the same public
`probs` float64 array ([length][q], NaN-initialised) that factories and
harnesses write directly, and their methods reproduce the reference arithmetic
elementwise (numpy float64, no fused multiply-add):

  BinaryMemorylessVectorDistribution   VectorDistributions/BinaryMemorylessVectorDistribution.py:15-87
  QaryMemorylessVectorDistribution     VectorDistributions/QaryMemorylessVectorDistribution.py:26-118

These host methods are the plugin API (used by the generic recursion for
arbitrary plugins and by user code); the decoder never calls them for
memoryless inputs -- BinaryPolarEncoderDecoder.decode sends those to the HIP
kernel (polarcub_amd/csrc).
"""
import math

import numpy as np
from scipy.special import logsumexp


class VectorDistribution:
    """Abstract plugin protocol (VectorDistribution.py:1-29).  Methods are 'pure virtual'."""

    def minusTransform(self):
        raise NotImplementedError

    def plusTransform(self, uminusDecisions):
        raise NotImplementedError

    def __len__(self):
        raise NotImplementedError

    def calcMarginalizedProbabilities(self):
        raise NotImplementedError

    def calcNormalizationVector(self):
        raise NotImplementedError

    def normalize(self, normalization):
        raise NotImplementedError

    # The reference's binary decoder calls normalizeDistList (BinaryPolarEncoderDecoder.py:279,285,299,305);
    # every concrete class here answers to both names.
    def normalizeDistList(self, normalization):
        return self.normalize(normalization)


class BinaryMemorylessVectorDistribution(VectorDistribution):
    def __init__(self, length):
        assert length > 0
        self.probs = np.empty((length, 2))
        self.probs[:] = np.nan
        self.length = length

    def __len__(self):
        return self.length

    def minusTransform(self):
        assert self.length % 2 == 0
        a, b = self.probs[0::2], self.probs[1::2]
        out = BinaryMemorylessVectorDistribution(self.length // 2)
        out.probs[:, 0] = a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1]
        out.probs[:, 1] = a[:, 0] * b[:, 1] + a[:, 1] * b[:, 0]
        return out

    def plusTransform(self, uminusDecisions):
        assert self.length % 2 == 0
        u = np.asarray(uminusDecisions).astype(bool)
        a, b = self.probs[0::2], self.probs[1::2]
        out = BinaryMemorylessVectorDistribution(self.length // 2)
        out.probs[:, 0] = np.where(u, a[:, 1], a[:, 0]) * b[:, 0]
        out.probs[:, 1] = np.where(u, a[:, 0], a[:, 1]) * b[:, 1]
        return out

    def calcMarginalizedProbabilities(self):
        assert len(self) == 1
        s = 0.0
        s += self.probs[0][0]
        s += self.probs[0][1]
        if s > 0.0:
            return np.array([self.probs[0][0] / s, self.probs[0][1] / s])
        return np.array([0.5, 0.5])

    def calcNormalizationVector(self):
        return np.maximum(self.probs[:, 0], self.probs[:, 1])

    def normalize(self, normalization):
        t = np.asarray(normalization, dtype=np.float64).copy()
        assert np.all(t >= 0)
        t[t == 0] = 1.0
        self.probs /= t[:, None]


class QaryMemorylessVectorDistribution(VectorDistribution):
    def __init__(self, q, length, use_log=False):
        assert q > 1
        assert length > 0
        self.q = q
        self.probs = np.empty((length, q), dtype=np.float64)
        self.probs[:] = np.nan
        self.length = length
        self.use_log = use_log
        if use_log:
            self.default_marginal_probs = [-math.log(q)] * q
        else:
            self.default_marginal_probs = [1 / q] * q

    def __len__(self):
        return self.length

    def minusTransform(self):
        assert self.length % 2 == 0
        q = self.q
        out = QaryMemorylessVectorDistribution(q, self.length // 2, use_log=self.use_log)
        out.probs[:] = -math.inf if self.use_log else 0.0
        a, b = self.probs[0::2], self.probs[1::2]
        for x1 in range(q):  # x1 outer, x2 inner: the reference's accumulation order (:36-42)
            for x2 in range(q):
                u1 = (x1 + x2) % q
                if self.use_log:
                    out.probs[:, u1] = np.logaddexp(out.probs[:, u1], a[:, x1] + b[:, x2])
                else:
                    out.probs[:, u1] += a[:, x1] * b[:, x2]
        return out

    def plusTransform(self, uminusDecisions):
        assert self.length % 2 == 0
        q = self.q
        out = QaryMemorylessVectorDistribution(q, self.length // 2, use_log=self.use_log)
        out.probs[:] = -math.inf if self.use_log else 0.0
        u1 = np.asarray(uminusDecisions, dtype=np.int64)
        rows = np.arange(self.length // 2)
        a, b = self.probs[0::2], self.probs[1::2]
        for u2 in range(q):
            x1 = (u1 + u2) % q
            x2 = (-u2) % q
            if self.use_log:
                out.probs[:, u2] = np.logaddexp(out.probs[:, u2], a[rows, x1] + b[:, x2])
            else:
                out.probs[:, u2] += a[rows, x1] * b[:, x2]
        return out

    def calcMarginalizedProbabilities(self):
        assert len(self) == 1
        row = self.probs[0]
        if self.use_log:
            s = logsumexp(row)
            if s > -math.inf:
                return row - s
            return np.array(self.default_marginal_probs)
        s = 0
        for v in row:
            s = s + v
        if s > 0.0:
            return row / s
        return np.array(self.default_marginal_probs)

    def calcNormalizationVector(self):
        if self.use_log:
            return np.array([logsumexp(r) for r in self.probs])
        t = np.zeros(self.length)
        for x in range(self.q):  # python sum(): left to right
            t = t + self.probs[:, x]
        return t

    def normalize(self, normalization=None):
        if normalization is None:
            normalization = self.calcNormalizationVector()
        t = np.asarray(normalization, dtype=np.float64)
        if self.use_log:
            keep = t != -math.inf
            self.probs[keep] -= t[keep, None]
        else:
            assert np.all(t >= 0)
            nz = t != 0
            self.probs[nz] /= t[nz, None]
