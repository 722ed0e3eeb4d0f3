#!/usr/bin/env python3
"""BSC polar-coding run -- the counterpart of the reference's test2.py (same code,
same printouts): Tal-Vardy construction for BSC(0.11) with n=7, L=100 and error
bound 0.1 on the native host library, then encodeDecodeSimulation over 4000 trials
with the decodes batched onto the GPU kernel.

    python -m polarcub_amd.cli.test2 [--trials 4000] [--seed S]

The reference draws the channel from the unseeded global `random` (test2.py:37);
--seed seeds it, so a run is reproducible and comparable with a seeded reference run.
"""
import argparse
import random

from .. import coding, scalar


def make_xVectorDistribuiton_fromBinaryMemorylessDistribution(xyDistribution, length):
    def make_xVectorDistribuiton():
        xDistribution = scalar.BinaryMemorylessDistribution()
        xDistribution.probs.append([xyDistribution.calcXMarginal(0), xyDistribution.calcXMarginal(1)])
        return xDistribution.makeBinaryMemorylessVectorDistribution(length, None)

    return make_xVectorDistribuiton


def make_codeword_noprocessing(encodedVector):
    return encodedVector


def simulateChannel_fromBinaryMemorylessDistribution(xyDistribution):
    """y ~ P(y | x) by inverse CDF over the output letters, one global random() per bit."""
    def simulateChannel(codeword):
        received = []
        for x in codeword:
            r = random.random()
            acc = 0.0
            for y in range(len(xyDistribution.probs)):
                p = xyDistribution.probXGivenY(x, y)
                if acc + p >= r:
                    received.append(y)
                    break
                acc += p
        return received

    return simulateChannel


def make_xyVectorDistribution_fromBinaryMemorylessDistribution(xyDistribution):
    def make_xyVectrorDistribution(receivedWord):
        return xyDistribution.makeBinaryMemorylessVectorDistribution(len(receivedWord), receivedWord)

    return make_xyVectrorDistribution


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--trials", type=int, default=4000)
    ap.add_argument("--seed", type=int, default=None, help="seed of the global random used by the channel")
    a = ap.parse_args(argv)
    if a.seed is not None:
        random.seed(a.seed)
    p, L, n = 0.11, 100, 7
    N = 2 ** n
    upperBoundOnErrorProbability = 0.1
    xyDistribution = scalar.makeBSC(p)
    frozenSet = scalar.calcFrozenSet_degradingUpgrading(n, L, upperBoundOnErrorProbability, None, xyDistribution)
    coding.encodeDecodeSimulation(N, make_xVectorDistribuiton_fromBinaryMemorylessDistribution(xyDistribution, N),
                                  make_codeword_noprocessing,
                                  simulateChannel_fromBinaryMemorylessDistribution(xyDistribution),
                                  make_xyVectorDistribution_fromBinaryMemorylessDistribution(xyDistribution), a.trials,
                                  frozenSet)


if __name__ == "__main__":
    main()
