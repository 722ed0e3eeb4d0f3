"""bench.py with an experimental binary decode kernel selected (pcub_sc_set_experiment; the kernels
linked in by scripts/exp_build.sh).  Diagnostic, not a bench line.

    python scripts/bench_exp.py <experiment> [bench.py arguments]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from polarcub_amd import _lib  # noqa: E402

e = int(sys.argv[1])
L = _lib.lib()
L.pcub_sc_set_experiment(e)
sys.exit(bench.main(sys.argv[2:]))
