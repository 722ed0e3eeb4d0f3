"""The C-ABI library builds, loads and exports every symbol the public header
declares (no GPU needed; no compute call is made)."""
import ctypes
import glob
import os
import re

from tests.conftest import ROOT


def _declared(header="*.h"):
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", header)):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names.update(re.findall(r"\b(pcub_\w+)\s*\(", text))
    return names


def test_header_declares_the_boundary():
    d = _declared()
    for must in ("pcub_sc_decode_bin", "pcub_sc_decode_bin_workspace", "pcub_polar_encode_bin",
                 "pcub_sc_decode_qary", "pcub_polar_encode_qary", "pcub_transpose_pairs"):
        assert must in d


def test_library_exports_every_declared_symbol():
    from polarcub_amd import _lib, build
    build.build()
    L = ctypes.CDLL(build.LIB)
    missing = [n for n in sorted(_declared("polarcub_sc.h")) if not hasattr(L, n)]
    assert not missing, missing
    assert set(_lib.EXPORTS) <= _declared("polarcub_sc.h")
    H = ctypes.CDLL(build.HOST_LIB)  # host-only construction library (include/polarcub_construct.h)
    missing = [n for n in sorted(_declared("polarcub_construct.h")) if not hasattr(H, n)]
    assert not missing, missing
    assert _lib.lib().pcub_abi_version() == _lib.ABI_VERSION == 4


def test_built_variants_are_the_launchable_ones():
    """The library builds the binary variants pick_variant can launch and no other (host-only calls)."""
    from polarcub_amd import _lib
    from tests.test_gpu_decode import VARIANTS
    L = _lib.lib()
    built = [v for v in range(L.pcub_sc_num_variants()) if L.pcub_sc_set_variant(v) == 0]
    L.pcub_sc_set_variant(L.pcub_sc_default_variant())
    assert built == VARIANTS
    for n in range(6, 17):
        assert L.pcub_sc_variant_for(n) in VARIANTS


def test_invalid_arguments_are_rejected_without_touching_the_device():
    from polarcub_amd import _lib
    L = _lib.lib()
    # log2N out of range / null frozen tables -> PCUB_EINVAL before any launch
    assert L.pcub_sc_decode_bin(None, 1, 30, None, None, 0, None, None, None, None, 0, None) == _lib.EINVAL
    assert L.pcub_sc_decode_qary(None, 1, 8, 9, None, 0, None, None, None, 0, None) == _lib.EINVAL
    assert L.pcub_polar_encode_bin(None, 1, 40, None, None, 0, None, None) == _lib.EINVAL
    assert L.pcub_transpose_pairs(None, 4, 4, 9, None, None) == _lib.EINVAL
    assert L.pcub_tile_pairs(None, 4, 4, 2, 0, None, None) == _lib.EINVAL
    assert L.pcub_tile_pairs(None, 4, 4, 2, 16, None, None) == _lib.EINVAL
    assert L.pcub_sc_decode_bin_workspace(0, 10) == 0
    # segment-state tables: sizes, argument checks, and the layout query (host-only code paths)
    assert L.pcub_sc_deletion_table_bytes(2) == (8 + 32 * 16) * 8  # header (magic, n0, pd) + rows
    assert L.pcub_sc_deletion_table_bytes(3) == (8 + 512 * 256) * 8
    assert L.pcub_sc_deletion_table_bytes(1) == 0 and L.pcub_sc_deletion_table_bytes(4) == 0
    assert L.pcub_sc_deletion_build_table(1, 0.1, ctypes.c_void_p(4096), None) == _lib.EINVAL
    assert L.pcub_sc_deletion_build_table(3, 0.1, None, None) == _lib.EINVAL
    assert L.pcub_sc_deletion_build_table(3, 0.1, ctypes.c_void_p(4097), None) == _lib.EINVAL  # misaligned
    assert L.pcub_sc_deletion_build_table(3, 1.5, ctypes.c_void_p(4096), None) == _lib.EINVAL
    # n0 = 2 runs the table-driven layout from 16 trellises on (its table can be built per
    # workgroup); n0 = 3 only with a table given (checked on the device: a rejected table sends the
    # batch to the gated fallback); never with ones or n0 = 1, 4
    assert L.pcub_sc_deletion_dense_layout(8, 2, 0, 800, None, 0.1) == 1
    assert L.pcub_sc_deletion_dense_layout(5, 2, 0, 100, None, 0.1) == 0   # 8 trellises
    assert L.pcub_sc_deletion_dense_layout(8, 2, 1, 800, None, 0.1) == 0   # guard-band ones
    assert L.pcub_sc_deletion_dense_layout(10, 3, 0, 3000, None, 0.1) == 0  # no table
    assert L.pcub_sc_deletion_dense_layout(10, 3, 0, 3000, ctypes.c_void_p(4096), 0.1) == 1  # header checked on device
    assert L.pcub_sc_deletion_dense_layout(12, 4, 0, 9000, None, 0.1) == 0
    assert L.pcub_sc_deletion_dense_layout(8, 2, 0, 30000, None, 0.1) == 0  # rows past the LDS budget
    # the compact-root decode: a kernel of its own where the default variant has a twin (N = 1024 ..
    # 16384), else an expansion into pairs (the Monte-Carlo pipeline then generates pairs itself)
    assert L.pcub_sc_decode_bin_compact_direct(10) == 1 and L.pcub_sc_decode_bin_compact_direct(12) == 1
    assert L.pcub_sc_decode_bin_compact_direct(14) == 1
    assert L.pcub_sc_decode_bin_compact_direct(15) == 0 and L.pcub_sc_decode_bin_compact_direct(5) == 0
    assert L.pcub_sc_decode_bin_compact_direct(30) == _lib.EINVAL


def test_oracle_and_emulator_build():
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "emu")], check=True)
    assert os.path.exists(os.path.join(ROOT, "oracle", "build", "liborc.so"))
    assert os.path.exists(os.path.join(ROOT, "tests", "emu", "build", "libemu.so"))


def test_no_long_branch_through_the_return_address():
    """scripts/check_isa.py: no device function of the built code object computes a long
    branch into s[30:31] (LLVM's expansion clobbers the return address; seen as an illegal
    memory access in a round-2 deletion callee), and no out-of-line device function other
    than the allowlisted window decoder exchanges lanes (out-of-line deletion node functions
    gave batch-dependent wrong results on the GPU)."""
    import subprocess
    import sys
    from polarcub_amd import build
    build.build()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_isa.py"), build.LIB],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 hazard(s)" in r.stdout


def test_no_kernel_uses_a_dynamic_stack():
    """Every kernel's code-object metadata says .uses_dynamic_stack: false (the SCL recursion is
    an explicit frame loop since round 3; no launcher sets the device's stack limit)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import check_isa
    from polarcub_amd import build
    build.build()
    meta = check_isa.kernel_metadata(build.LIB)
    assert len(meta) > 50
    assert [k["name"] for k in meta if k.get("uses_dynamic_stack", True)] == []
    scl = [k for k in meta if "k_scl" in k["name"]]
    assert scl and all(k["private_segment_fixed_size"] < 4096 for k in scl)
    src = open(os.path.join(ROOT, "polarcub_amd", "csrc", "scl.hip")).read()
    assert "hipDeviceSetLimit" not in src
