"""In-tree build of the HIP library (gfx950) that backs polarcub_amd.

    python -m polarcub_amd.build [--force]

Produces polarcub_amd/lib/libpolarcub_hip.so with hipcc.  -ffp-contract=off is
part of the arithmetic contract (no a*b+c contraction into FMA); never build
with -ffast-math.
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib", "libpolarcub_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PCUB_ARCH", "gfx950")

SOURCES = ["sc_bin.hip", "sc_qary.hip", "sc_util.hip"]
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
         "-std=c++17", "-Wall", "-Wno-unused-function"]


def _deps():
    out = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".h"))]
    out.append(os.path.join(ROOT, "include", "polarcub_sc.h"))
    return out


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in _deps())


def build(force=False, verbose=False):
    if not force and up_to_date():
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [HIPCC] + FLAGS + ["-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    cmd += [os.path.join(CSRC, s) for s in SOURCES] + ["-o", tmp]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
