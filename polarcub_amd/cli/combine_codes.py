#!/usr/bin/env python3
"""Merge genie frozen-set files into one code -- the counterpart of the reference's
combine_codes.py (same arguments, printout and output file).

    python -m polarcub_amd.cli.combine_codes FILE [FILE ...]

Each FILE is a frozen-set file in the genie format (BinaryPolarEncoderDecoder.py:471-489,
written by coding.write_frozen_file): '** number of trials = M' and one
'*** i  (TV+Pe)*trials' line per index.  The per-index sums over all files, divided by the
total number of trials, are sorted ascending; the code keeps the longest prefix whose
cumulative sum stays below 0.1 (combine_codes.py:35-46).  Prints 'N = .., K = .., Rate = ..'
and writes the merged file to ./out in the same format (:49-66).
"""
import sys

import numpy as np

_MAX_N = 1 << 20  # combine_codes.py:27


def read_frozen_file_sums(filename, acc):
    """Adds one file's '*** i v' values into acc[i]; returns (number of trials, 1 + largest i).
    The trials line is '** number of trials = M' (its value starts at column 22)."""
    trials = None
    top = 0
    with open(filename) as f:
        for line in f:
            if line.startswith("** "):
                trials = int(line[22:])
            elif line.startswith("*** "):
                idx, val = line[4:].split()[:2]
                acc[int(idx)] += float(val)
                top = max(top, int(idx))
    return trials, top + 1


def combine(filenames):
    """(printed line, text of ./out) for the given files."""
    acc = [0] * _MAX_N
    total = 0
    N = 0
    for name in filenames:
        M, N = read_frozen_file_sums(name, acc)  # N: the last file's length, as the reference
        total += M
    scores = np.asarray(acc[:N])
    order = np.argsort(scores)
    cumulative = np.cumsum(scores[order] / total)
    K = np.sum(cumulative < 0.1)
    line = " ".join(str(v) for v in ("N = ", N, ", K = ", K, " Rate = ", K / N))
    frozen = set(order[K:])
    out = ["* Combined"]
    out += [str(i) for i in frozen]
    out.append("** number of trials = " + str(total))
    out.append("* (TotalVariation+errorProbability) * (number of trials)")
    out += ["*** " + str(i) + " " + str(scores[i]) for i in range(N)]
    return line, "\n".join(out) + "\n"


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    line, text = combine(argv)
    print(line)
    with open("out", "w") as f:
        f.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
