#!/usr/bin/env python3
"""Polar coding over the deletion channel -- the counterpart of the reference's
main_deletion.py (flags and printouts of main_deletion.py:62-146), on the MI355X path:
genie construction and encode/decode trials run through the GPU kernels
(pcub_sc_leaf_deletion / pcub_sc_decode_deletion) whenever the shape is supported.

    python -m polarcub_amd.cli.main_deletion -n 8 -g 8000 -e 8000 -f frozen.txt
"""
import argparse
import random

import numpy as np

from .. import coding, deletion, vectors


def make_xVectorDistribuiton_deletion_uniform(length):
    def make_xVectorDistribuiton():
        v = vectors.BinaryMemorylessVectorDistribution(length)
        v.probs[:] = 0.5
        return v

    return make_xVectorDistribuiton


def make_codeword_addDeletionGuardBands(xi, n, n0, ones):
    def make_codeword(encodedVector):
        return deletion.addDeletionGuardBands(encodedVector, n, n0, xi, ones)

    return make_codeword


def make_simulateChannel_deletion(p, seed=None):
    rng = random.Random()
    if seed is not None:
        rng.seed(seed)

    def simulateChannel(codeword):
        return deletion.deletionChannelSimulation(codeword, p, seed=None, randomNumberGenerator=rng)

    return simulateChannel


def make_xyVectorDistribution_deletion(pd, xi, n, n0, ones):
    def make_xyVectorDistribution(receivedWord, verbosity=0):
        return deletion.buildCollectionOfBinaryTrellises_uniformInput_deletion(receivedWord, pd, xi, n, n0, ones,
                                                                               verbosity)

    return make_xyVectorDistribution


def parser():
    ap = argparse.ArgumentParser(description="polar encoder/decoder for the deletion channel")
    ap.add_argument("-pd", "--deletion-probability", type=float, default=0.1,
                    help="The deletion probability of the channel. Default is 0.1.")
    ap.add_argument("-pe", "--error-probability", type=float, default=0.1,
                    help="Upper bound on error probability, when constructing the frozen set. Default is 0.1.")
    ap.add_argument("-n", "--n", type=int, required=True, help="The total number of polarization steps.")
    ap.add_argument("-n0", "--n0", type=int, help="The number of slow (trellis) polarization steps. The default is n//3.")
    ap.add_argument("-g", "--genie-simulations", nargs="?", const=8000, type=int,
                    help="Perform genie encoding/decoding trials to find the frozen set. Default is 8000.")
    ap.add_argument("-e", "--encoding-decoding-simulations", type=int, nargs="?", const=8000,
                    help="Perform encoding/decoding trials to test the code. Default is 8000.")
    ap.add_argument("--xi", type=float, default=0.1,
                    help="The paramter through which the length of the guard bands is defined. Default is 0.1.")
    ap.add_argument("--ones-added-at-end-of-guard-band", type=int, default=0,
                    help="Add a sequence of ones at the start and end of a guard band (and also at the start and end "
                         "of the codeword). Defult is 0 (all-zero guardbands).")
    ap.add_argument("-f", "--frozen-bits-file", help="Read/write the frozen bits from/to a file.")
    ap.add_argument("-cs", "--channel-seed", type=int, default=100, help="Seed for simulating the channel. Default is 100.")
    ap.add_argument("-crs", "--common-randomness-seed", type=int, default=200,
                    help="Seed for common randomness between encoder and decoder. Default is 200.")
    ap.add_argument("-gs", "--genie-seed", type=int, default=300,
                    help="Seed for letting the genie pick a different common randomness for each encoding/decoding "
                         "run. Default is 300.")
    ap.add_argument("-is", "--information-seed", type=int, default=400,
                    help="Seed for picking the random bits to encode. Default is 400.")
    return ap


def main(argv=None):
    args = vars(parser().parse_args(argv))
    pd = args["deletion_probability"]
    G = args["genie_simulations"]
    E = args["encoding_decoding_simulations"]
    n = args["n"]
    N = 2 ** n
    n0 = args["n0"] if args["n0"] is not None else n // 3
    ones = args["ones_added_at_end_of_guard_band"]
    filename = args["frozen_bits_file"]
    xi = args["xi"]
    print("n =", n, ", n0 =", n0, ", xi =", xi, ", deletion probability =", pd)
    if filename is not None:
        print("frozen bits file = ", filename)
    bound = args["error_probability"]
    make_x = make_xVectorDistribuiton_deletion_uniform(N)
    make_codeword = make_codeword_addDeletionGuardBands(xi, n, n0, ones)
    print("codeword length = ", len(make_codeword(np.zeros(2 ** n, dtype=np.int64))))
    channel = make_simulateChannel_deletion(pd, seed=args["channel_seed"])
    make_xy = make_xyVectorDistribution_deletion(pd, xi, n, n0, ones)
    frozenSet = None
    if G is not None:
        print("performing", G, "genie encoding/decoding trials to find a frozen set with WER at most", bound)
        frozenSet = coding.genieEncodeDecodeSimulation(N, make_x, make_codeword, channel, make_xy, G, bound,
                                                       genieSeed=args["genie_seed"], trustXYProbs=(n <= n0),
                                                       filename=filename)
    if E is not None:
        if filename is not None:
            frozenSet = coding.read_frozen_file(filename)
        print("performing", E, "encoding/decoding trials")
        coding.encodeDecodeSimulation(N, make_x, make_codeword, channel, make_xy, E, frozenSet,
                                      commonRandomnessSeed=args["common_randomness_seed"],
                                      randomInformationSeed=args["information_seed"], verbosity=0)
    return frozenSet


if __name__ == "__main__":
    main()
