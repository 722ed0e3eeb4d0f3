"""Scalar binary channels and the vector-distribution factories that feed the decoder.

Counterpart of ScalarDistributions/BinaryMemorylessDistribution.py for what the
hot path needs:
  class BinaryMemorylessDistribution: probs[y][x] = P(X=x, Y=y)
      makeBinaryMemorylessVectorDistribution(length, yvec)     :245-258
      calcXMarginal / calcYMarginal / probXGivenY               :429-443
      errorProb / bhattacharyya / totalVariationDistance / conditionalEntropy / mmse
      minusTransform / plusTransform (scalar channel transforms) :261-285
  makeBSC(p) :485-490, makeBEC(p) :493-499
The Tal-Vardy degrading/upgrading construction (:287-427, :624-680) is not part
of the decode hot path; frozen sets it produced are accepted everywhere.
"""
import math

from . import vectors


def eta(p):
    assert 0 <= p <= 1
    return 0.0 if p == 0 else -p * math.log2(p)


def hxgiveny(data):
    s = data[0] + data[1]
    return 0.0 if s == 0 else eta(data[0] / s) * s + eta(data[1] / s) * s


class BinaryMemorylessDistribution:
    def __init__(self):
        self.probs = []  # probs[yindex][xindex]
        self.auxiliary = None

    def __str__(self):
        s = "Binary memoryless channel with " + str(len(self.probs)) + " symbols. The error probability is " + str(
            self.errorProb()) + ". The conditional entropy is " + str(self.conditionalEntropy()) + \
            ". [p(y,x=0), p(y,x=1)]: "
        s += ", ".join("[" + str(p[0]) + ", " + str(p[1]) + "]" for p in self.probs)
        return s

    def append(self, item):
        self.probs.append(item)

    def errorProb(self):
        total = 0.0
        for pair in self.probs:
            total += min(pair)
        return total

    def bhattacharyya(self):
        total = 0.0
        for pair in self.probs:
            total += math.sqrt(pair[0] * pair[1])
        return 2.0 * total

    def totalVariationDistance(self):
        total = 0.0
        for pair in self.probs:
            total += abs(pair[0] - pair[1])
        return total

    def conditionalEntropy(self):
        total = 0.0
        for pair in self.probs:
            total += eta(pair[0]) + eta(pair[1]) - eta(pair[0] + pair[1])
        return total

    def mmse(self):
        total = 0.0
        for pair in self.probs:
            py = pair[0] + pair[1]
            if py == 0.0:
                continue
            e = (pair[0] - pair[1]) / py
            for x in range(2):
                total += pair[x] * ((1 - 2 * x) - e) ** 2
        return total

    def normalize(self):
        s = sum(sum(self.probs, []))
        self.probs = [[p / s for p in pair] for pair in self.probs]

    def calcXMarginal(self, x):
        s = 0.0
        for y in range(len(self.probs)):
            s += self.probs[y][x]
        return s

    def calcYMarginal(self, y):
        return sum(self.probs[y])

    def probXGivenY(self, x, y):
        return self.probs[y][x] / sum(self.probs[y])

    def minusTransform(self):
        out = BinaryMemorylessDistribution()
        for y1 in self.probs:
            for y2 in self.probs:
                out.append([y1[0] * y2[0] + y1[1] * y2[1], y1[0] * y2[1] + y1[1] * y2[0]])
        return out

    def plusTransform(self):
        out = BinaryMemorylessDistribution()
        for y1 in self.probs:
            for y2 in self.probs:
                out.append([y1[0] * y2[0], y1[1] * y2[1]])
                out.append([y1[1] * y2[0], y1[0] * y2[1]])
        return out

    def makeBinaryMemorylessVectorDistribution(self, length, yvec):
        vd = vectors.BinaryMemorylessVectorDistribution(length)
        if yvec is not None:
            assert len(yvec) == length
            for i in range(length):
                vd.probs[i][0] = self.probs[yvec[i]][0]
                vd.probs[i][1] = self.probs[yvec[i]][1]
        else:
            vd.probs[:, 0] = self.probs[0][0]
            vd.probs[:, 1] = self.probs[0][1]
        return vd


def makeBSC(p):
    bsc = BinaryMemorylessDistribution()
    bsc.append([0.5 * (1.0 - p), 0.5 * p])
    bsc.append([0.5 * p, 0.5 * (1.0 - p)])
    return bsc


def makeBEC(p):
    bec = BinaryMemorylessDistribution()
    bec.append([0.5 * (1.0 - p), 0])
    bec.append([0, 0.5 * (1.0 - p)])
    bec.append([0.5 * p, 0.5 * p])
    return bec
