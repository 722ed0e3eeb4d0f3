"""Scalar binary channels and the vector-distribution factories that feed the decoder.

Counterpart of ScalarDistributions/BinaryMemorylessDistribution.py for what the
hot path needs:
  class BinaryMemorylessDistribution: probs[y][x] = P(X=x, Y=y)
      makeBinaryMemorylessVectorDistribution(length, yvec)     :245-258
      calcXMarginal / calcYMarginal / probXGivenY               :429-443
      errorProb / bhattacharyya / totalVariationDistance / conditionalEntropy / mmse
      minusTransform / plusTransform (scalar channel transforms) :261-285
      removeZeroProbOutput / sortProbs / mergeEquivalentSymbols  :92-208
      degrade(L) / upgrade(L) (Tal-Vardy)                        :287-427
  makeBSC(p) :485-490, makeBEC(p) :493-499, makeBernoulli(p) :502-506
  calcFrozenSet_degradingUpgrading(n, L, bound, xDistribution, xyDistribution) :624-680
  eta / eta_list / naturalEta / hxgiveny                        :450-477
mergeEquivalentSymbols, degrade, upgrade and the construction run in the native
host library (polarcub_amd.construction, csrc/host/tv_construct.cpp).
"""
import math
import sys

from . import construction, vectors


def eta(p):
    assert 0.0 <= p <= 1.0 + 10 * sys.float_info.epsilon
    p = min(1.0, p)
    return 0.0 if p == 0.0 else -p * math.log2(p)


def eta_list(p_list):
    return sum([eta(p) for p in p_list])


def naturalEta(p):
    assert 0.0 <= p <= 1.0
    return 0.0 if p == 0.0 else -p * math.log(p)


def hxgiveny(data):
    py = data[0] + data[1]
    return py * (eta(data[0] / py) + eta(data[1] / py))


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

    # letter bookkeeping (the auxiliary list, when set, holds one set per letter)
    def removeZeroProbOutput(self):
        keep = [i for i, pair in enumerate(self.probs) if sum(pair) > 0.0]
        self.probs = [self.probs[i] for i in keep]
        if self.auxiliary is not None:
            self.auxiliary = [self.auxiliary[i] for i in keep]

    def sortProbs(self):
        """Ascending p(x=0|y): letters with p(x=0|y) > 1/2 first (by p(x=1|y)), then the
        rest (by -p(x=0|y)); stable, like the reference's list.sort."""
        aux = self.auxiliary if self.auxiliary is not None else [None] * len(self.probs)
        zero = [(p, a) for p, a in zip(self.probs, aux) if p[0] / sum(p) > 0.5]
        one = [(p, a) for p, a in zip(self.probs, aux) if not p[0] / sum(p) > 0.5]
        zero.sort(key=lambda t: t[0][1] / sum(t[0]))
        one.sort(key=lambda t: -t[0][0] / sum(t[0]))
        self.probs = [p for p, _ in zero + one]
        if self.auxiliary is not None:
            self.auxiliary = [a for _, a in zero + one]

    def _merged_aux(self, group, count):
        out = [set() for _ in range(count)]
        for i, g in enumerate(group):
            if g >= 0:
                out[g] |= self.auxiliary[i]
        return out

    def mergeEquivalentSymbols(self):
        """Merge letters whose posteriors are math.isclose, sort by LLR, normalise
        (native, bit-identical).  Auxiliary sets are merged by union."""
        merged, group = construction.merge_equivalent(self.probs)
        if self.auxiliary is not None:
            self.auxiliary = self._merged_aux(group, len(merged))
        self.probs = merged.tolist()

    def degrade(self, L):
        """Degraded channel with at most L letters (greedy merge of LLR-adjacent letters
        with the least mutual-information loss).  Merges self's equivalent letters first,
        as the reference does; auxiliary sets are carried as unions."""
        self.mergeEquivalentSymbols()
        letters, group = construction.degrade(self.probs, L)
        out = BinaryMemorylessDistribution()
        out.probs = letters.tolist()
        if self.auxiliary is not None:
            out.auxiliary = self._merged_aux(group, len(letters))
        return out

    def upgrade(self, L):
        """Upgraded channel with at most L letters (each removed letter's mass split onto
        its neighbours).  Merges self's equivalent letters first."""
        if self.auxiliary is not None:
            raise NotImplementedError("upgrade with auxiliary letter sets")
        self.mergeEquivalentSymbols()
        out = BinaryMemorylessDistribution()
        out.probs = construction.upgrade(self.probs, L).tolist()
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


def makeBernoulli(p):
    ber = BinaryMemorylessDistribution()
    ber.append([1.0 - p, p])
    return ber


def calcFrozenSet_degradingUpgrading(n, L, upperBoundOnErrorProbability, xDistribution, xyDistribution, threads=0):
    """Frozen set from the degraded xy tree (Pe) and the upgraded x tree (TV), at most L
    letters per channel (ScalarDistributions/BinaryMemorylessDistribution.py:624-680).
    The reference crashes for a non-None xDistribution (it calls a missing
    totalVariation()); here TV is the upgraded channels' totalVariationDistance."""
    from . import coding
    assert n >= 0
    assert L > 0
    assert upperBoundOnErrorProbability > 0
    assert xyDistribution is not None
    TV, Pe = construction.tv_pe(n, L, None if xDistribution is None else xDistribution.probs, xyDistribution.probs,
                                threads)
    return coding.frozenSetFromTVAndPe(TV.tolist(), Pe.tolist(), upperBoundOnErrorProbability)


def makeBEC(p):
    bec = BinaryMemorylessDistribution()
    bec.append([0.5 * (1.0 - p), 0])
    bec.append([0, 0.5 * (1.0 - p)])
    bec.append([0.5 * p, 0.5 * p])
    return bec
