#!/usr/bin/env python3
"""q-ary polar-coding runs -- the counterpart of the reference's test3.py (its closures, code
construction and simulation entry points, same printouts), on the GPU decoders:

  make_xVectorDistribution_fromQaryMemorylessDistribution / make_codeword_noprocessing /
  simulateChannel_fromQaryMemorylessDistribution / make_xyVectorDistribution_fromQaryMemoryless-
  Distribution (test3.py:21-70), get_construction_path (:72-93), getFrozenSet (:95-116),
  test (:118-155), test_ir (:157-186), test_ir_per_config (:188-240), write_header /
  write_result (:292-330), calc_theoretic_key_rate / calc_theoretic_key_qrate (:332-348),
  snr_to_qer (:402-405).

    python -m polarcub_amd.cli.test3 [--q 2] [--trials 200] [--seed S] [--list L --check C]

Two reference defects are kept where they are behaviour, and bypassed where they would make
the run useless:
  * test() and test_ir() pass upperBoundOnErrorProbability / numInfoIndices positionally into
    getFrozenSet's snr / rate slots (test3.py:130, :169), so the construction gets no bound and
    frozenSetFromTVAndPe compares a float with None (TypeError).  test() / test_ir() here do
    the same; `body()` (and the command line) runs test()'s body with the bound passed by name.
  * The construction cache lives beside the script (test3.py:79); here it is under
    $POLARCUB_CONSTRUCTIONS (default ~/.cache/polarcub_amd/polar_codes_constructions), in the
    reference's directory layout and .npy format.
The channel draws from the unseeded global `random` (test3.py:43); --seed seeds it.
"""
import argparse
import csv
import math
import os
import random
from collections import Counter
from timeit import default_timer as timer

import numpy as np

from .. import coding_qary as QaryPolarEncoderDecoder
from .. import scalar_qary as QaryMemorylessDistribution


def make_xVectorDistribution_fromQaryMemorylessDistribution(q, xyDistribution, length, use_log=False):
    def make_xVectorDistribution():
        xDistribution = QaryMemorylessDistribution.QaryMemorylessDistribution(q)
        xDistribution.probs = [xyDistribution.calcXMarginals()]
        return xDistribution.makeQaryMemorylessVectorDistribution(length, None, use_log=use_log)

    return make_xVectorDistribution


def make_codeword_noprocessing(encodedVector):
    return encodedVector


def simulateChannel_fromQaryMemorylessDistribution(xyDistribution):
    """y ~ P(y | x) by inverse CDF over the output letters, one global random() per symbol."""
    def simulateChannel(codeword):
        receivedWord = []
        for x in codeword:
            rand = random.random()
            probSum = 0.0
            for y in range(len(xyDistribution.probs)):
                p = xyDistribution.probXGivenY(x, y)
                if probSum + p >= rand:
                    receivedWord.append(y)
                    break
                probSum += p
        return receivedWord

    return simulateChannel


def make_xyVectorDistribution_fromQaryMemorylessDistribution(xyDistribution, use_log=False):
    def make_xyVectorDistribution(receivedWord):
        return xyDistribution.makeQaryMemorylessVectorDistribution(len(receivedWord), receivedWord, use_log)

    return make_xyVectorDistribution


def _constructions_root():
    return os.environ.get("POLARCUB_CONSTRUCTIONS",
                          os.path.join(os.path.expanduser("~"), ".cache", "polarcub_amd", "polar_codes_constructions"))


def get_construction_path(q, N, channel_type="QSC", QER=None, SNR=None, rate=None):
    """Directory of a code's cached TV / Pe vectors, the reference's layout (:72-93)."""
    assert channel_type in ["QSC", "AWGN"]
    path = _constructions_root() + "/q={}/N={}/".format(q, N)
    if channel_type == "QSC":
        assert QER is not None
        path += "QER={}/".format(QER)
    else:
        assert SNR and rate
        path += "SNR={}/rate={}/".format(SNR, rate)
    return path


def getFrozenSet(q, N, n, L, channel_type, xDistribution, xyDistribution, qer, snr=None, rate=None,
                 upperBoundOnErrorProbability=None, numInfoIndices=None, verbosity=False):
    """The code construction through the cached TV / Pe vectors (:95-116)."""
    if channel_type == "QSC":
        construction_path = get_construction_path(q, N, QER=qer)
    elif channel_type == "AWGN":
        construction_path = get_construction_path(q, N, channel_type, SNR=snr, rate=rate)
    else:
        raise TypeError("exceptions must derive from BaseException")  # the reference raises a str
    if channel_type != "QSC":
        raise TypeError("exceptions must derive from BaseException")
    return QaryMemorylessDistribution.calcFrozenSet_degradingUpgrading(n, L, xDistribution, xyDistribution,
                                                                      construction_path, upperBoundOnErrorProbability,
                                                                      numInfoIndices, verbosity)


def body(q, listDecode=False, maxListSize=None, checkSize=None, numInfoIndices=None, verbosity=False,
         numberOfTrials=200):
    """test()'s body (:118-150) with the error bound passed to getFrozenSet by name."""
    p, L, n = 0.99, 100, 8
    N = 2 ** n
    upperBoundOnErrorProbability = 0.1
    xyDistribution = QaryMemorylessDistribution.makeQSC(q, p)
    frozenSet = getFrozenSet(q, N, n, L, "QSC", None, xyDistribution, p,
                             upperBoundOnErrorProbability=upperBoundOnErrorProbability,
                             numInfoIndices=numInfoIndices, verbosity=verbosity)
    args = (make_xVectorDistribution_fromQaryMemorylessDistribution(q, xyDistribution, N), make_codeword_noprocessing,
            simulateChannel_fromQaryMemorylessDistribution(xyDistribution),
            make_xyVectorDistribution_fromQaryMemorylessDistribution(xyDistribution), numberOfTrials, frozenSet)
    if not listDecode:
        QaryPolarEncoderDecoder.encodeDecodeSimulation(q, N, *args, verbosity=verbosity)
    else:
        QaryPolarEncoderDecoder.encodeListDecodeSimulation(q, N, *args, maxListSize, checkSize, verbosity=verbosity)
    return frozenSet


def test(q, listDecode=False, maxListSize=None, checkSize=None, numInfoIndices=None, verbosity=False):
    """test3.test (:118-155) as written: the bound lands in getFrozenSet's snr slot, so the
    construction runs without one and the frozen-set picker raises TypeError, as there."""
    print("q = " + str(q))
    p, L, n = 0.99, 100, 8
    N = 2 ** n
    upperBoundOnErrorProbability = 0.1
    xyDistribution = QaryMemorylessDistribution.makeQSC(q, p)
    frozenSet = getFrozenSet(q, N, n, L, "QSC", None, xyDistribution, p, upperBoundOnErrorProbability, numInfoIndices,
                             verbosity=verbosity)
    return frozenSet  # not reached: the reference's picker fails first


def test_ir(q, channel_type="QSC", maxListSize=None, checkSize=0, numberOfTrials=200, ir_version=1,
            numInfoIndices=None, use_log=False, verbosity=False):
    """test3.test_ir (:157-186), with the same positional getFrozenSet call (and failure) as test()."""
    p, L, n = 0.98, 100, 6
    N = 2 ** n
    upperBoundOnErrorProbability = 0.1
    xyDistribution = QaryMemorylessDistribution.makeQSC(q, p)
    if channel_type != "QSC":
        raise TypeError("exceptions must derive from BaseException")
    frozenSet = getFrozenSet(q, N, n, L, channel_type, None, xyDistribution, p, upperBoundOnErrorProbability,
                             numInfoIndices, verbosity=verbosity)
    if maxListSize is None:
        maxListSize = (max(frozenSet) + 1 - len(frozenSet)) ** q
        print(maxListSize)
    return QaryPolarEncoderDecoder.irSimulation(
        q, N, simulateChannel_fromQaryMemorylessDistribution(xyDistribution),
        make_xyVectorDistribution_fromQaryMemorylessDistribution(xyDistribution, use_log), numberOfTrials, frozenSet,
        maxListSize, checkSize, use_log=use_log, verbosity=verbosity, ir_version=ir_version)


def test_ir_per_config(q, L, n, maxListSize, numTrials, channel_type="QSC", qer=None, snr=None, rate=None,
                       numInfoIndices=None, frozenSet=None, use_log=False, verbosity=False, file_name=None):
    """One IR configuration (:188-240): construction by numInfoIndices, irSimulation, an optional
    CSV row.  Returns (frame_error_prob, symbol_error_prob, key_rate, time_rate, maxListSize,
    prob_result_list)."""
    N = 2 ** n
    assert channel_type in ["QSC", "AWGN"]
    if numInfoIndices is None:
        assert rate is not None
        numInfoIndices = math.floor(rate * N)
    if channel_type == "QSC":
        xyDistribution = QaryMemorylessDistribution.makeQSC(q, qer)
    else:
        xyDistribution = QaryMemorylessDistribution.makeAWGN(q, snr, rate)
    if frozenSet is None:
        frozenSet = getFrozenSet(q, N, n, L, channel_type, None, xyDistribution, qer=qer, snr=snr, rate=rate,
                                 numInfoIndices=numInfoIndices, verbosity=verbosity)
    if maxListSize is None:
        maxListSize = (max(frozenSet) + 1 - len(frozenSet)) ** q
        print(maxListSize)
    if verbosity:
        print("q=" + str(q) + ", channelType=" + str(channel_type) + ", qer=" + str(qer) + ", snr=" + str(snr)
              + ", rate=" + str(rate) + ", n=" + str(n) + ", L=" + str(L) + ", numInfoQudits=" + str(numInfoIndices)
              + ", maxListSize=" + str(maxListSize) + ", numTrials=" + str(numTrials))
    if channel_type == "AWGN":
        raise TypeError("exceptions must derive from BaseException")
    start = timer()
    frame_error_prob, symbol_error_prob, key_rate, prob_result_list = QaryPolarEncoderDecoder.irSimulation(
        q, N, simulateChannel_fromQaryMemorylessDistribution(xyDistribution),
        make_xyVectorDistribution_fromQaryMemorylessDistribution(xyDistribution, use_log), numTrials, frozenSet,
        maxListSize, use_log=use_log, verbosity=verbosity)
    time_rate = (timer() - start) / (numTrials * N)
    if file_name is not None:
        write_header(file_name)
        write_result(file_name, q, qer, snr, calc_theoretic_key_rate(q, channel_type, qer=qer, snr=snr, rate=rate), n,
                     N, L, "degradingUpgrading", numInfoIndices, rate, maxListSize, frame_error_prob,
                     symbol_error_prob, key_rate, time_rate, numTrials, prob_result_list, verbosity=verbosity)
    return frame_error_prob, symbol_error_prob, key_rate, time_rate, maxListSize, prob_result_list


HEADER = ["q", "qer", "snr", "theoreticKeyRate", "n", "N", "L", "frozenBitsAlgorithm", "numInfoQudits", "rate",
          "maxListSize", "frameErrorProb", "symbolErrorProb", "keyRate", "yield", "efficiency", "timeRate", "numTrials"]


def write_header(file_name):
    """The results CSV's header row, checked against an existing file (:292-305)."""
    header = HEADER + [r.name for r in QaryPolarEncoderDecoder.ProbResult]
    try:
        with open(file_name, "r") as f:
            for row in f:
                assert row.rstrip("\n").split(",") == header
                return
    except FileNotFoundError:
        with open(file_name, "a", newline="") as f:
            csv.writer(f).writerow(header)
    except AssertionError:
        raise AssertionError(f"Header of {file_name} is bad.")


def write_result(file_name, q, qer, snr, theoretic_key_rate, n, N, L, frozenBitsAlgorithm, numInfoQudits, rate,
                 maxListSize, frame_error_prob, symbol_error_prob, key_rate, time_rate, numTrials, prob_result_list,
                 verbosity=False):
    """One results row (:307-330); yield and efficiency for q = 2 only."""
    if verbosity:
        print("writing results")
    if q == 2:
        yld = (1 - frame_error_prob) * numInfoQudits * math.log(q, 2)
        efficiency = numInfoQudits * math.log(q, 2) / (-qer * math.log(qer, 2) - (1 - qer) * math.log(1 - qer, 2))
    else:
        yld = efficiency = None
    counter = Counter(prob_result_list)
    if verbosity:
        print(counter)
    stats = [counter[r] / numTrials for r in QaryPolarEncoderDecoder.ProbResult]
    with open(file_name, "a", newline="") as f:
        csv.writer(f).writerow([q, qer, snr, theoretic_key_rate, n, N, L, frozenBitsAlgorithm, numInfoQudits, rate,
                                maxListSize, frame_error_prob, symbol_error_prob, key_rate, yld, efficiency, time_rate,
                                numTrials] + stats)


def calc_theoretic_key_rate(q, channel_type="QSC", qer=None, snr=None, rate=None):
    """QSC key-rate bound in bits (:332-339)."""
    if channel_type != "QSC":
        raise TypeError("exceptions must derive from BaseException")
    if qer == 0.0:
        return math.log(q, 2)
    if qer == 1.0:
        return math.log(q / (q - 1), 2)
    return math.log(q, 2) + (1 - qer) * math.log(1 - qer, 2) + qer * math.log(qer / (q - 1), 2)


def calc_theoretic_key_qrate(q, qer):
    """The same in q-ary units (:341-346)."""
    if qer == 0.0:
        return 1.0
    if qer == 1.0:
        return math.log(q / (q - 1), q)
    return 1.0 + (1 - qer) * math.log(1 - qer, q) + qer * math.log(qer / (q - 1), q)


def snr_to_qer(q, snr, rate):
    """Hard-decision symbol error rate of BPSK at the given SNR (dB) and rate (:402-405)."""
    from scipy.stats import norm
    assert q == 2
    return 1 - norm.cdf(math.sqrt(2 * rate * 10 ** (snr / 10)))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--q", type=int, default=2)
    ap.add_argument("--trials", type=int, default=200)
    ap.add_argument("--seed", type=int, default=None, help="seed of the global random used by the channel")
    ap.add_argument("--list", type=int, default=0, help="list-decode with this maxListSize (0: SC)")
    ap.add_argument("--check", type=int, default=0, help="checkSize of the list run")
    a = ap.parse_args(argv)
    if a.seed is not None:
        random.seed(a.seed)
        np.random.seed(a.seed)
    print("q = " + str(a.q))
    body(a.q, listDecode=a.list > 0, maxListSize=a.list, checkSize=a.check, numberOfTrials=a.trials)


if __name__ == "__main__":
    main()
