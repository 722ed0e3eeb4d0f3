"""In-tree build of the HIP library (gfx950) that backs polarcub_amd.

    python -m polarcub_amd.build [--force]

Compiles every csrc/*.hip translation unit to an object (in parallel, only the
stale ones) and links polarcub_amd/lib/libpolarcub_hip.so with hipcc; builds the
host-only construction library polarcub_amd/lib/libpolarcub_construct.so
(csrc/host/*.cpp) with g++.
-ffp-contract=off is part of the arithmetic contract (no a*b+c contraction into
FMA); never build with -ffast-math.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libpolarcub_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PCUB_ARCH", "gfx950")

SOURCES = ["sc_bin.hip", "sc_bin_k0.hip", "sc_bin_k1.hip", "sc_bin_k2.hip", "sc_bin_k3.hip", "sc_qary.hip",
           "sc_util.hip", "sc_del.hip", "sc_leaf.hip", "sc_mc.hip"]
CFLAGS = ["--offload-arch=" + ARCH, "-O3", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-std=c++17", "-Wall",
          "-Wno-unused-function"]


HOST_LIB = os.path.join(LIBDIR, "libpolarcub_construct.so")
HOST_SOURCES = [os.path.join(CSRC, "host", "tv_construct.cpp")]
CXX = os.environ.get("CXX", "g++")
HOST_CFLAGS = ["-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared", "-std=c++17", "-Wall", "-pthread"]


def build_host(force=False, verbose=False):
    """The construction library: plain C++, IEEE binary64 without contraction, libm log2."""
    deps = HOST_SOURCES + [os.path.join(ROOT, "include", "polarcub_construct.h")]
    if not force and not _stale(HOST_LIB, deps):
        return HOST_LIB
    os.makedirs(LIBDIR, exist_ok=True)
    tmp = HOST_LIB + ".tmp"
    cmd = [CXX] + HOST_CFLAGS + ["-I" + os.path.join(ROOT, "include")] + HOST_SOURCES + ["-o", tmp, "-lm"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, HOST_LIB)
    return HOST_LIB


def _headers():
    out = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    out.append(os.path.join(ROOT, "include", "polarcub_sc.h"))
    return out


def _obj(src):
    return os.path.join(OBJDIR, src.replace(".hip", ".o"))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def up_to_date():
    hdr = _headers()
    objs = [_obj(s) for s in SOURCES]
    if any(_stale(_obj(s), hdr + [os.path.join(CSRC, s)]) for s in SOURCES):
        return False
    return not _stale(LIB, objs)


def _compile(src, verbose):
    obj = _obj(src)
    tmp = obj + ".tmp.o"
    cmd = [HIPCC] + CFLAGS + ["-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "-c", os.path.join(CSRC, src),
                              "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, obj)


def build(force=False, verbose=False):
    build_host(force, verbose)
    if not force and up_to_date():
        return LIB
    os.makedirs(OBJDIR, exist_ok=True)
    hdr = _headers()
    todo = [s for s in SOURCES if force or _stale(_obj(s), hdr + [os.path.join(CSRC, s)])]
    with ThreadPoolExecutor(max(1, min(len(todo), int(os.environ.get("MAX_JOBS", "8"))))) as ex:
        list(ex.map(lambda s: _compile(s, verbose), todo))
    tmp = LIB + ".tmp"
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC"] + [_obj(s) for s in SOURCES] + ["-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
