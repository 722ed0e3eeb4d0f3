"""Profiling driver: build one bench.py workload (same arguments as bench.py) and run its
decode step --reps times, nothing else on the GPU afterwards (for rocprofv3 passes).

    python scripts/profile_step.py --workload deletion --reps 1 [bench.py args]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    argv = sys.argv[1:]
    reps = 1
    if "--reps" in argv:
        i = argv.index("--reps")
        reps = int(argv[i + 1])
        del argv[i:i + 2]
    a = bench.build_parser().parse_args(argv)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    w = bench.WORKLOADS[a.workload](a, dev, 0)
    torch.cuda.synchronize()
    for _ in range(reps):
        w.step()
    torch.cuda.synchronize()
    print("done: %s x%d, batch %d" % (a.workload, reps, w.B), flush=True)


if __name__ == "__main__":
    main()
