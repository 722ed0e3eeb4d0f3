#!/usr/bin/env python3
"""ISA hazard check of the built HIP library (gfx950 code object).

LLVM's long-branch expansion (s_getpc_b64 / s_add / s_setpc_b64 through s[30:31]) inside
a non-kernel device function clobbers the return address held in s[30:31]; the function
then 'returns' into its own body.  Observed on a >128 KiB deletion-kernel callee (round 2),
where it ended in an illegal memory access.  The library must not contain such a function:
every device function must either be inlined or free of s_setpc_b64 s[30:31] other than
its final return.

    python scripts/check_isa.py [path/to/libpolarcub_hip.so]
Second rule: cross-lane operations (ds_bpermute / ds_permute / ds_swizzle, DPP moves) live
in kernels only, or in an allowlisted leaf function called under a full wave.  Out-of-line
deletion node functions with lane exchanges gave batch-dependent wrong results on the GPU
(round 2: 32-trellis shapes, the host emulation clean under ASan/UBSan); they are
force-inlined, and this rule keeps them so.

Third rule: no kernel uses a dynamic stack.  Its code-object metadata
(`.uses_dynamic_stack`, read with llvm-readelf --notes) must be false: a kernel whose stack
depth the compiler cannot bound (recursion, e.g. round 2's SclNode::run) overruns each wave's
scratch at full occupancy unless the device's per-thread stack limit is raised, a device-wide
side effect a library call must not have.  `--report` prints every kernel's private segment
size and spill counts as JSON.

Exit status 1 lists the offending functions.
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    """The gfx950 code objects of every translation unit: the library's .hip_fatbin section
    is a sequence of clang offload bundles (magic, entry count, then offset/size/triple
    per entry, offsets relative to the bundle)."""
    import struct
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fat, lib,
                        os.path.join(d, "stripped.so")], check=True)
        data = open(fat, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        q = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tl].decode()
            q += 24 + tl
            if "gfx950" in triple and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 24)
    return out


def device_disasm(lib):
    texts = []
    with tempfile.TemporaryDirectory() as d:
        for i, co in enumerate(code_objects(lib)):
            f = os.path.join(d, "co%d.o" % i)
            with open(f, "wb") as fh:
                fh.write(co)
            texts.append(subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", f],
                                        check=True, capture_output=True, text=True).stdout)
    return "\n".join(texts)


def kernel_metadata(lib):
    """[{name, uses_dynamic_stack, private_segment_fixed_size, vgpr_count, sgpr_count,
    vgpr_spill_count, sgpr_spill_count, group_segment_fixed_size}] of every gfx950 kernel (the
    AMDGPU metadata note of each code object)."""
    keys = ("uses_dynamic_stack", "private_segment_fixed_size", "vgpr_count", "sgpr_count", "vgpr_spill_count",
            "sgpr_spill_count", "group_segment_fixed_size")
    out = []
    with tempfile.TemporaryDirectory() as d:
        for i, co in enumerate(code_objects(lib)):
            f = os.path.join(d, "co%d.o" % i)
            with open(f, "wb") as fh:
                fh.write(co)
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f], check=True,
                                   capture_output=True, text=True).stdout
            for block in re.split(r"\n\s*- \.agpr_count:", notes)[1:]:
                m = re.search(r"^\s*\.name:\s+(\S+)", block, re.M)
                if not m:
                    continue
                k = {"name": m.group(1)}
                for key in keys:
                    v = re.search(r"^\s*\.%s:\s+(\S+)" % key, block, re.M)
                    if v:
                        k[key] = v.group(1) == "true" if key == "uses_dynamic_stack" else int(v.group(1))
                out.append(k)
    return out


# device functions allowed to exchange lanes: called by wave 0 of the deletion kernel with all
# lanes active (the T > 64 window decoder, kept out of line for the branch range above)
CROSS_LANE_OK = ("del_window",)
CROSS_LANE = re.compile(r"ds_bpermute|ds_permute|ds_swizzle|quad_perm|row_ror|row_shl|row_shr|row_mirror|row_bcast|wave_")


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else os.path.join(ROOT, "polarcub_amd", "lib", "libpolarcub_hip.so")
    meta = kernel_metadata(lib)
    if "--report" in sys.argv:
        import json
        print(json.dumps(meta, indent=1))
    text = device_disasm(lib)
    bad = []
    for k in meta:
        if k.get("uses_dynamic_stack", True):
            bad.append((k["name"], 1, "dynamic stack (.uses_dynamic_stack, private segment %s B)"
                        % k.get("private_segment_fixed_size")))
    if not meta:
        bad.append(("<library>", 1, "no kernel metadata found"))
    for m in re.finditer(r"^[0-9a-f]+ <([^>]+)>:\n(.*?)(?=^[0-9a-f]+ <|\Z)", text, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if ".kd" in name:
            continue
        if "s_endpgm" in body:
            continue
        # a return is a bare s_setpc_b64 s[30:31] (tail duplication gives a function several);
        # a long branch computes the target into the pair first (s_getpc_b64 + s_add/s_addc)
        lines = body.splitlines()
        n = 0
        for i, line in enumerate(lines):
            if "s_setpc_b64 s[30:31]" in line:
                prev = " ".join(lines[max(0, i - 4):i])
                if re.search(r"s_getpc_b64 s\[30:31\]|s_add_u32 s30|s_addc_u32 s31|s_sub_u32 s30", prev):
                    n += 1
        if n:
            bad.append((name, n, "long branch through the return address (%d long branch(es) via s[30:31])" % n))
        x = len(CROSS_LANE.findall(body))
        if x and not any(a in name for a in CROSS_LANE_OK):
            bad.append((name, x, "cross-lane operations in an out-of-line device function (%d)" % x))
    for name, n, what in bad:
        print("%s in %s" % (what, name))
    print("%d function(s), %d kernel(s) checked, %d hazard(s)" % (len(re.findall(r"^[0-9a-f]+ <", text, re.M)),
                                                                  len(meta), len(bad)))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
