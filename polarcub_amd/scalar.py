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


use_fast = False  # the reference's switch for its (absent) Cython eta/hxgiveny (:10-14)


# The degrade / upgrade merge-cost helpers (:509-621).  The constructions themselves run in the
# native host library (csrc/host/tv_core.h restates the same arithmetic); these are the
# reference's Python entry points, for callers that use them directly.
def _calcKey_degrade(dataLeft, dataCenter):
    """Cost of merging two adjacent letters (:510-521); data = (probs, ...) tuples as in the
    reference's heap entries."""
    if dataLeft is None:
        return float("inf")
    probLeft, probCenter = dataLeft[0], dataCenter[0]
    assert len(probLeft) == len(probCenter) == 2
    probMerge = [probLeft[0] + probCenter[0], probLeft[1] + probCenter[1]]
    return hxgiveny(probMerge) - hxgiveny(probLeft) - hxgiveny(probCenter)


def _calcKey_upgrade(dataLeft, dataCenter, dataRight):
    """Cost of splitting the centre letter onto its neighbours (:524-537)."""
    if dataLeft is None or dataRight is None:
        return float("inf")
    assert len(dataLeft[0]) == len(dataCenter[0]) == len(dataRight[0]) == 2
    probMergeLeft, probMergeRight = upgradedLeftRightProbs(dataLeft, dataCenter, dataRight)
    return hxgiveny(dataCenter[0]) - hxgiveny(probMergeLeft) - hxgiveny(probMergeRight)


def _listIndexingHelper(l, i):
    return l[i] if (0 <= i < len(l)) else None


def upgradedLeftRightProbs(dataLeft, dataCenter, dataRight):
    """Split of the centre letter's mass pi_c into theta_l * pi_c and theta_r * pi_c along its
    neighbours' posteriors (:544-621), with the reference's case split for numerical stability
    (the smaller theta computed directly, the other as 1 - theta)."""
    probLeft, probCenter, probRight = dataLeft[0], dataCenter[0], dataRight[0]
    piLeft, piCenter, piRight = sum(probLeft), sum(probCenter), sum(probRight)
    nL = [probLeft[b] / piLeft for b in range(2)]
    nC = [probCenter[b] / piCenter for b in range(2)]
    nR = [probRight[b] / piRight for b in range(2)]
    if nL[0] < 0.5 and nR[0] < 0.5:
        dLR = 2.0 * (nL[0] - nR[0])
    elif nL[1] < 0.5 and nR[1] < 0.5:
        dLR = 2.0 * (nR[1] - nL[1])
    else:
        dLR = (nL[0] - nL[1]) - (nR[0] - nR[1])
    assert dLR > 0.0  # equivalent letters are merged before upgrading
    if nL[0] < 0.5 and nR[0] < 0.5:
        if nL[0] - nC[0] < nC[0] - nR[0]:
            thetaRight = 2.0 * (nL[0] - nC[0]) / dLR
            thetaLeft = 1.0 - thetaRight
        else:
            thetaLeft = 2.0 * (nC[0] - nR[0]) / dLR
            thetaRight = 1.0 - thetaLeft
    elif nL[1] < 0.5 and nR[1] < 0.5:
        if nC[1] - nL[1] < nR[1] - nC[1]:
            thetaRight = 2.0 * (nC[1] - nL[1]) / dLR
            thetaLeft = 1.0 - thetaRight
        else:
            thetaLeft = 2.0 * (nR[1] - nC[1]) / dLR
            thetaRight = 1.0 - thetaLeft
    else:
        thetaRight = ((nL[0] - nL[1]) - (nC[0] - nC[1])) / dLR
        thetaLeft = 1.0 - thetaRight
    assert 0.0 <= thetaLeft <= 1.0 and 0.0 <= thetaRight <= 1.0
    return ([thetaLeft * piCenter * nL[b] for b in range(2)], [thetaRight * piCenter * nR[b] for b in range(2)])


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
