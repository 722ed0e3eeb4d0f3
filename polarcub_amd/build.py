"""In-tree build of the HIP library (gfx950) that backs polarcub_amd.

    python -m polarcub_amd.build [--force]

Compiles every csrc/*.hip translation unit to an object (in parallel, only the
stale ones: staleness is a sha256 of the source, the headers it includes and the flags, stored
beside each object and the library, never file mtimes) and links polarcub_amd/lib/libpolarcub_hip.so with hipcc; builds the
host-only construction library polarcub_amd/lib/libpolarcub_construct.so
(csrc/host/*.cpp) with g++.
-ffp-contract=off is part of the arithmetic contract (no a*b+c contraction into
FMA); never build with -ffast-math.
"""
import hashlib
import os
import re
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

SOURCES = ["sc_del_w4.hip", "sc_del_dense.hip", "sc_del_n4w.hip", "sc_del_n4.hip", "sc_del_n4o.hip", "sc_del_n4x.hip", "sc_del_n3.hip", "sc_del_n3o.hip", "sc_del_n3x.hip",
           "sc_del_n2.hip", "sc_del_n2o.hip", "sc_del_n2x.hip", "sc_del_n1.hip", "sc_del_n1o.hip", "sc_del_n1x.hip",
           "sc_bin.hip", "sc_bin_k0.hip", "sc_bin_k1.hip", "sc_bin_k2.hip", "sc_bin_k4.hip", "sc_bin_k5.hip", "sc_bin_k6.hip", "sc_bin_k7.hip", "sc_bin_k8.hip", "sc_bin_k9.hip", "sc_qary.hip",
           "sc_qary_q2.hip", "sc_qary_q3.hip", "sc_qary_q4.hip", "sc_qary_q56.hip", "sc_qary_q78.hip",
           "sc_util.hip", "sc_del.hip", "sc_leaf.hip", "sc_qary_log.hip", "scl.hip",
           "sc_mc.hip"]
CFLAGS = ["--offload-arch=" + ARCH, "-O3", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-std=c++17", "-Wall",
          "-Wno-unused-function"]


HOST_LIB = os.path.join(LIBDIR, "libpolarcub_construct.so")
HOST_SOURCES = [os.path.join(CSRC, "host", "tv_construct.cpp"), os.path.join(CSRC, "host", "qary_construct.cpp")]
CXX = os.environ.get("CXX", "g++")
HOST_CFLAGS = ["-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared", "-std=c++17", "-Wall", "-pthread"]


def _digest(paths, extra=()):
    """sha256 over the contents of `paths` (in order) and the strings in `extra` (flags)."""
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    for e in extra:
        h.update(e.encode() + b"\0")
    return h.hexdigest()


def _stamp(target):
    return target + ".sha256"


def _stale(target, digest):
    """A target is stale unless it exists and its stamp records the same content digest
    (never decided by mtimes: a pushed tree can carry any mtimes)."""
    if not os.path.exists(target) or not os.path.exists(_stamp(target)):
        return True
    with open(_stamp(target)) as f:
        return f.read().strip() != digest


def _write_stamp(target, digest):
    with open(_stamp(target), "w") as f:
        f.write(digest + "\n")


def build_host(force=False, verbose=False):
    """The construction library: plain C++, IEEE binary64 without contraction, libm log2."""
    deps = HOST_SOURCES + [os.path.join(ROOT, "include", "polarcub_construct.h"),
                           os.path.join(CSRC, "host", "tv_core.h")]
    dig = _digest(deps, [CXX] + HOST_CFLAGS)
    if not force and not _stale(HOST_LIB, dig):
        return HOST_LIB
    os.makedirs(LIBDIR, exist_ok=True)
    tmp = HOST_LIB + ".tmp"
    cmd = [CXX] + HOST_CFLAGS + ["-I" + os.path.join(ROOT, "include")] + HOST_SOURCES + ["-o", tmp, "-lm"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, HOST_LIB)
    _write_stamp(HOST_LIB, dig)
    return HOST_LIB


_INCLUDE = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)
_INC_DIRS = [CSRC, os.path.join(ROOT, "include")]


def _headers(src):
    """The project headers `src` includes, transitively (quoted includes resolved in
    csrc/ and include/), sorted: a translation unit is rebuilt when one of them changes."""
    seen, todo = set(), [os.path.join(CSRC, src)]
    while todo:
        with open(todo.pop()) as f:
            text = f.read()
        for name in _INCLUDE.findall(text):
            for d in _INC_DIRS:
                path = os.path.join(d, name)
                if os.path.exists(path):
                    if path not in seen:
                        seen.add(path)
                        todo.append(path)
                    break
    return sorted(seen)


def _obj(src):
    return os.path.join(OBJDIR, src.replace(".hip", ".o"))


def _obj_digest(src):
    return _digest([os.path.join(CSRC, src)] + _headers(src), [HIPCC, ARCH] + CFLAGS)


def _lib_digest():
    return hashlib.sha256("".join(_obj_digest(s) for s in SOURCES).encode()).hexdigest()


def lib_current():
    """True when the library's stamp matches the current sources, headers and flags (its objects
    need not be present: they stay on the build host)."""
    return os.path.exists(LIB) and not _stale(LIB, _lib_digest())


def up_to_date():
    """True when every object and the library match the current sources, headers and flags."""
    if any(_stale(_obj(s), _obj_digest(s)) for s in SOURCES):
        return False
    return not _stale(LIB, _lib_digest())


def _compile(src, verbose):
    obj = _obj(src)
    # the stamp records the sources as they were when the compile started: a header edited while
    # the compiler runs leaves the object stale for the next build instead of wrongly current
    dig = _obj_digest(src)
    tmp = obj + ".tmp.o"
    cmd = [HIPCC] + CFLAGS + ["-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "-c", os.path.join(CSRC, src),
                              "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, obj)
    _write_stamp(obj, dig)


class _tree_lock:
    """One build at a time in this tree (fcntl lock on lib/.build.lock)."""

    def __enter__(self):
        import fcntl
        os.makedirs(LIBDIR, exist_ok=True)
        self.f = open(os.path.join(LIBDIR, ".build.lock"), "w")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *a):
        self.f.close()


def build(force=False, verbose=False):
    with _tree_lock():
        return _build_locked(force, verbose)


def torch_ops_current(verbose=False):
    """build_torch_ops under the tree lock: rebuilds when torch_ops.cpp, polarcub_sc.h, the
    compiler or the torch version changed (digest stamp), else returns at once."""
    with _tree_lock():
        return build_torch_ops(False, verbose)


TORCH_LIB = os.path.join(LIBDIR, "libpolarcub_torch.so")
TORCH_SRC = os.path.join(CSRC, "torch", "torch_ops.cpp")


def build_torch_ops(force=False, verbose=False):
    """The PyTorch-ROCm operator library (torch.ops.polarcub.*, csrc/torch/torch_ops.cpp): host-only
    C++ over the C ABI, linked against libpolarcub_hip.so (found beside it through $ORIGIN)."""
    import torch
    tdir = os.path.dirname(torch.__file__)
    flags = ["-O2", "-fPIC", "-shared", "-std=c++17", "-Wall", "-DUSE_ROCM",
             "-D_GLIBCXX_USE_CXX11_ABI=%d" % int(torch._C._GLIBCXX_USE_CXX11_ABI)]
    dig = _digest([TORCH_SRC, os.path.join(ROOT, "include", "polarcub_sc.h")], [HIPCC, torch.__version__] + flags)
    if not force and not _stale(TORCH_LIB, dig):
        return TORCH_LIB
    tmp = TORCH_LIB + ".tmp"
    cmd = ([HIPCC] + flags + ["-I" + os.path.join(tdir, "include"),
                              "-I" + os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
                              "-I" + os.path.join(ROOT, "include"), TORCH_SRC, "-o", tmp,
                              "-L" + os.path.join(tdir, "lib"), "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip",
                              "-L" + LIBDIR, "-lpolarcub_hip", "-Wl,-rpath,$ORIGIN"])
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, TORCH_LIB)
    _write_stamp(TORCH_LIB, dig)
    return TORCH_LIB


def _build_locked(force, verbose):
    build_host(force, verbose)
    lib = _build_hip_locked(force, verbose)
    build_torch_ops(force, verbose)
    return lib


def _build_hip_locked(force, verbose):
    if not force and up_to_date():
        return LIB
    os.makedirs(OBJDIR, exist_ok=True)
    todo = [s for s in SOURCES if force or _stale(_obj(s), _obj_digest(s))]
    with ThreadPoolExecutor(max(1, min(len(todo), int(os.environ.get("MAX_JOBS", "8"))))) as ex:
        list(ex.map(lambda s: _compile(s, verbose), todo))
    lib_dig = _lib_digest()
    tmp = LIB + ".tmp"
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC"] + [_obj(s) for s in SOURCES] + ["-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    _write_stamp(LIB, lib_dig)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
