"""Scalar q-ary channels, the vector factory feeding the q-ary decoder, and the q-ary
degrading/upgrading code construction.

Counterpart of ScalarDistributions/QaryMemorylessDistribution.py with the reference's names:
probs[y][x], calcXMarginals (:155-165), probXGivenY (:174-175), calcYMarginal (:177-179),
errorProb / conditionalEntropy / totalVariation (:53-96), minusTransform / plusTransform
(:182-212), degrade / upgrade (dynamic, :215-475), removeZeroProbOutput / normalize
(:708-751), calcMFromL (:753-755), makeQaryMemorylessVectorDistribution (:757-776),
makeQSC / makeQEC / makeInputDistribution (:780-811), and the construction
calcFrozenSet_degradingUpgrading / calcTVAndPe_degradingUpgrading with its .npy cache
(:910-991).  degrade / upgrade and the tree run in the native host library
(polarcub_amd.construction, csrc/host/qary_construct.cpp), bit-identical to the reference.
"""
import math
import os
from enum import Enum

import numpy as np

from . import construction, vectors

# constants (ScalarDistributions/QaryMemorylessDistribution.py:15-17): the left / centre / right
# images of an old letter in the dynamic upgrade
lcrLeft = 0
lcrCenter = 1
lcrRight = 2


class Binning(Enum):
    """Cell functions of the static constructions (:20-22)."""
    TalSharovVardy = 1  # standard cell function for static degrade
    PeregTal = 2  # standard cell function for static upgrade


def eta(p):
    """-p log2 p (ScalarDistributions/BinaryMemorylessDistribution.py:451-459)."""
    assert 0.0 <= p <= 1.0 + 10 * 2.220446049250313e-16
    p = min(1.0, p)
    return 0.0 if p == 0.0 else -p * math.log2(p)


def eta_list(probs):
    return sum(0.0 if p == 0 else -p * math.log2(p) for p in probs)


class QaryMemorylessDistribution:
    def __init__(self, q, use_log=False):
        self.q = q
        self.use_log = use_log
        self.probs = []  # probs[yindex][xindex]

    def __str__(self):
        rows = ", ".join("[" + ", ".join(str(p) for p in row) + "]" for row in self.probs)
        return ("Qry memoryless channel with q = " + str(self.q) + " and " + str(len(self.probs))
                + " output symbols. The error probability is " + str(self.errorProb())
                + ". The conditional entropy is " + str(self.conditionalEntropy())
                + ". [p(y,x=0), p(y,x=1), ..., p(y,x=q-1)]: " + rows)

    def append(self, item):
        self.probs.append(item)

    def calcOutputAlphabetSize(self):
        return len(self.probs)

    # -- polar toolbox ---------------------------------------------------------
    def errorProb(self):
        total = 0.0
        for row in self.probs:
            t = sorted(row)
            total += sum(t[:-1])
        return total

    def conditionalEntropy(self):
        s = 0.0
        for row in self.probs:
            for p in row:
                s += eta(p)
            s -= eta(sum(row))
        return s

    def totalVariation(self):
        s = 0.0
        for row in self.probs:
            for p1 in row:
                for p2 in row:
                    s += abs(p1 - p2)
        return s / (2 * (self.q - 1))

    def calcXMarginals(self):
        out = []
        for x in range(self.q):
            s = 0.0
            for row in self.probs:
                s += row[x]
            out.append(s)
        return out

    def calcXMarginal(self, x):
        s = 0.0
        for row in self.probs:
            s += row[x]
        return s

    def probXGivenY(self, x, y):
        return self.probs[y][x] / sum(self.probs[y])

    def calcYMarginal(self, y):
        return sum(self.probs[y])

    def minusTransform(self):
        q = self.q
        new = QaryMemorylessDistribution(q)
        for y1 in self.probs:
            for y2 in self.probs:
                t = [0 for _ in range(q)]
                for x1 in range(q):
                    for x2 in range(q):
                        t[(x1 + x2) % q] += y1[x1] * y2[x2]
                new.append(t)
        return new

    def plusTransform(self):
        q = self.q
        new = QaryMemorylessDistribution(q)
        for y1 in self.probs:
            for y2 in self.probs:
                for u1 in range(q):
                    t = [0 for _ in range(q)]
                    for u2 in range(q):
                        t[u2] += y1[(u1 - u2 + q) % q] * y2[u2]
                    new.append(t)
        return new

    # -- degrading / upgrading (native) ------------------------------------------
    def _from_rows(self, rows):
        new = QaryMemorylessDistribution(self.q)
        new.probs = [list(map(float, r)) for r in rows]
        return new

    def degrade(self, L):
        return self.degrade_dynamic(L)

    def degrade_dynamic(self, L):
        return self._from_rows(construction.qmd_degrade(self.q, self.probs, L))

    def upgrade(self, L):
        return self.upgrade_dynamic(L)

    def upgrade_dynamic(self, L):
        return self._from_rows(construction.qmd_upgrade(self.q, self.probs, L))

    def removeZeroProbOutput(self):
        self.probs = [row for row in self.probs if sum(row) > 0.0]

    def normalize(self):
        flat = sorted(p for row in self.probs for p in row)
        s = 0.0
        for p in flat:
            s += p
        self.probs = [[p / s for p in row] for row in self.probs]

    def calcMFromL(self, L):
        return construction.calc_m(self.q, L)

    def makeQaryMemorylessVectorDistribution(self, length, yvec, use_log=False):
        vd = vectors.QaryMemorylessVectorDistribution(self.q, length, use_log)
        table = np.array(self.probs, dtype=np.float64)
        rows = table[np.asarray(yvec, dtype=np.int64)] if yvec is not None else np.tile(table[0], (length, 1))
        if yvec is not None:
            assert len(yvec) == length
        if use_log:
            with np.errstate(divide="ignore"):
                rows = np.where(rows != 0, np.log(np.where(rows != 0, rows, 1.0)), -math.inf)
        vd.probs[:] = rows
        return vd


def makeQSC(q, p):
    qsc = QaryMemorylessDistribution(q)
    qsc.probs = [[1.0 - p if x == y else p / (q - 1) for x in range(q)] for y in range(q)]
    return qsc


def makeQEC(q, p):
    qec = QaryMemorylessDistribution(q)
    for y in range(q):
        qec.append([(1.0 - p) / q if x == y else 0.0 for x in range(q)])
    qec.append([p / q for _ in range(q)])
    return qec


def makeAWGN(q, snr, rate):
    """The reference's placeholder (:800-804): binary only, and the channel has no output
    letters (probs == []); test3.py's AWGN branch builds nothing usable from it."""
    assert (q == 2)
    awgn = QaryMemorylessDistribution(q)
    awgn.probs = []
    return awgn


def makeQuantizedUniform(q, T):
    """Joint distribution with output (a_0, .., a_{q-1}), a_i >= 0 summing to T, and
    P(x, a) = a_x / (M T), M = binom(T + q - 1, q - 1) output letters (:815-853); letters in the
    reference's lexicographic enumeration order."""
    M = math.comb(T + q - 1, q - 1)
    quantizedUniform = QaryMemorylessDistribution(q)
    recursivlyBuildQuantizedUniform(quantizedUniform, [], q, T, M)
    return quantizedUniform


def recursivlyBuildQuantizedUniform(quantizedUniform, outputLetter, level, T, M):
    """Enumerates the output letters of makeQuantizedUniform (:856-873), appending to
    quantizedUniform.probs; outputLetter is the prefix built so far."""
    if level == 0:
        quantizedUniform.probs.append([(1.0 * outputLetter[x]) / (M * T) for x in range(quantizedUniform.q)])
        return
    if level == 1:
        outputLetter.append(T - sum(outputLetter))
        recursivlyBuildQuantizedUniform(quantizedUniform, outputLetter, level - 1, T, M)
        outputLetter.pop()
        return
    for t in range(0, T + 1 - sum(outputLetter)):
        outputLetter.append(t)
        recursivlyBuildQuantizedUniform(quantizedUniform, outputLetter, level - 1, T, M)
        outputLetter.pop()


def makeInputDistribution(probs):
    dist = QaryMemorylessDistribution(len(probs))
    dist.append(list(probs))
    dist.normalize()
    return dist


def _cache_names(directory_name, L):
    base = directory_name + "DegradingUpgrading_L=" + str(L)
    return base + "_tv.npy", base + "_pe.npy"


def calcTVAndPe_degradingUpgrading(n, L, xDistribution, xyDistribution, directory_name=None, verbosity=False,
                                   threads=0):
    """TV / Pe vectors of the degraded xy tree and upgraded x tree (:934-991).  With a
    directory_name the reference's .npy cache is read if both files exist, else written
    (directory_name + 'DegradingUpgrading_L=<L>_tv.npy' / '_pe.npy').  Without one the
    reference returns None (and calcFrozenSet_degradingUpgrading then fails); here the
    vectors are computed and returned uncached."""
    if directory_name is not None:
        tv_name, pe_name = _cache_names(directory_name, L)
        if verbosity:
            print(tv_name)
            print(pe_name)
        if os.path.isfile(tv_name) and os.path.isfile(pe_name):
            return np.load(tv_name), np.load(pe_name)
        if verbosity:
            print("Calculating TV and Pe vectors...")
    q = xyDistribution.q
    TV, Pe = construction.qary_tv_pe(q, n, L, None if xDistribution is None else xDistribution.probs,
                                     xyDistribution.probs, threads)
    TVvec, Pevec = [float(v) for v in TV], [float(v) for v in Pe]
    if directory_name is None:
        return TVvec, Pevec
    if verbosity:
        print("Done calculating!")
    if not os.path.exists(directory_name):
        os.makedirs(directory_name)
    np.save(tv_name, TVvec)
    np.save(pe_name, Pevec)
    return TVvec, Pevec


def calcFrozenSet_degradingUpgrading(n, L, xDistribution, xyDistribution, directory_name=None,
                                     upperBoundOnErrorProbability=None, numInfoIndices=None, verbosity=False):
    """Frozen set from the degrading/upgrading construction (:910-932) through
    QaryPolarEncoderDecoder.frozenSetFromTVAndPe."""
    from . import coding_qary
    assert n >= 0
    assert L > 0
    assert upperBoundOnErrorProbability is None or upperBoundOnErrorProbability > 0
    assert xyDistribution is not None
    TVvec, Pevec = calcTVAndPe_degradingUpgrading(n, L, xDistribution, xyDistribution, directory_name,
                                                  verbosity=verbosity)
    return coding_qary.frozenSetFromTVAndPe(TVvec, Pevec, upperBoundOnErrorProbability, numInfoIndices,
                                            verbosity=verbosity)


def degrade_dynamic_upper_bound(q, L):
    """Equation (27) of Ordentlich-Tal, in bits (:876-882)."""
    M = construction.calc_m(q, L)
    return (64 * (q - 1) / (M ** 2)) / math.log(2)


def upgrade_dynamic_upper_bound(q, L):
    """Equation (13) of Ordentlich-Tal, in bits (:885-891)."""
    M = construction.calc_m(q, L)
    return (128 * (q - 1) / (M ** 2)) / math.log(2)


def degrade_cost_lower_bound(q, L):
    """Equation (3) of Tal, "On the construction of polar codes for channels with moderate
    input alphabet sizes", in bits (:894-899)."""
    sigma = (math.pi ** ((q - 1) / 2)) / (math.gamma((q - 1) / 2 + 1))
    return (q - 1) / (2 * (q + 1)) * ((1.0 / (sigma * math.factorial(q - 1) * L)) ** (2 / (q - 1))) / math.log(2)


def upgrade_cost_lower_bound(q, L):
    """Equation (43) of Kartowsky-Tal, in bits (:902-907)."""
    kappa = (q - 1) / (2 * math.pi * (q + 1)) * (math.gamma(1 + (q - 1) / 2) / math.factorial(q - 1))
    return kappa * (L ** (-2 / (q - 1))) / math.log(2)
