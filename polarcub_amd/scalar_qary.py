"""Scalar q-ary channels and the vector factory feeding the q-ary decoder.

Counterpart of ScalarDistributions/QaryMemorylessDistribution.py for the hot
path: probs[y][x], calcXMarginals (:155-172),
probXGivenY (:174-175), makeQaryMemorylessVectorDistribution (:757-776),
makeQSC (:780-784), makeQEC (:787-798).  The degrading/upgrading construction
(:400-991) is not part of the decode path.
"""
import math

import numpy as np

from . import vectors


def eta_list(probs):
    return sum(0.0 if p == 0 else -p * math.log2(p) for p in probs)


class QaryMemorylessDistribution:
    def __init__(self, q):
        self.q = q
        self.probs = []  # probs[yindex][xindex]

    def append(self, item):
        self.probs.append(item)

    def calcXMarginals(self):
        out = []
        for x in range(self.q):
            s = 0.0
            for row in self.probs:
                s += row[x]
            out.append(s)
        return out

    def probXGivenY(self, x, y):
        return self.probs[y][x] / sum(self.probs[y])

    def calcYMarginal(self, y):
        return sum(self.probs[y])

    def errorProb(self):
        return sum(sum(row) - max(row) for row in self.probs)

    def normalize(self):
        s = sum(sum(row) for row in self.probs)
        self.probs = [[p / s for p in row] for row in self.probs]

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
