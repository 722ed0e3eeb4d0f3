"""ctypes binding of the HIP C-ABI library (include/polarcub_sc.h).

There is no CPU fallback: if the library is missing or a call fails, this
module raises.  Device pointers come from torch CUDA (HIP) tensors.
"""
import ctypes
import os

from . import build as _build

_c_void_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32

_lib = None

EINVAL = -1
ABI_VERSION = 4  # include/polarcub_sc.h (2: guard-band ones in the deletion entry points; 3: table headers, tile_pairs; 4: pcub_scl_set_wave removed)


class HipError(RuntimeError):
    pass


def lib():
    """Load libpolarcub_hip.so, (re)building it in-tree first when it is absent or does not
    match the current sources (content-hash stamps, polarcub_amd/build.py)."""
    global _lib
    if _lib is not None:
        return _lib
    path = _build.LIB
    if not _build.lib_current():
        _build.build()
    L = ctypes.CDLL(path)
    L.pcub_abi_version.restype = ctypes.c_int
    L.pcub_abi_version.argtypes = []
    L.pcub_sc_set_variant.restype = ctypes.c_int
    L.pcub_sc_default_variant.restype = ctypes.c_int
    L.pcub_sc_default_variant.argtypes = []
    L.pcub_sc_variant_for.restype = ctypes.c_int
    L.pcub_sc_variant_for.argtypes = [ctypes.c_int32]
    L.pcub_sc_set_variant.argtypes = [ctypes.c_int]
    L.pcub_sc_set_max_blocks_per_cu.restype = ctypes.c_int
    L.pcub_sc_set_max_blocks_per_cu.argtypes = [ctypes.c_int]
    L.pcub_sc_set_qary_lanes.restype = ctypes.c_int
    L.pcub_sc_set_qary_lanes.argtypes = [ctypes.c_int]
    L.pcub_sc_set_qary_regs.restype = ctypes.c_int
    L.pcub_sc_set_qary_regs.argtypes = [ctypes.c_int]
    L.pcub_sc_set_qary_lds.restype = ctypes.c_int
    L.pcub_sc_set_qary_lds.argtypes = [ctypes.c_int]
    L.pcub_sc_set_qary_hl.restype = ctypes.c_int
    L.pcub_sc_set_qary_hl.argtypes = [ctypes.c_int]
    L.pcub_sc_num_variants.restype = ctypes.c_int
    L.pcub_sc_num_variants.argtypes = []
    L.pcub_sc_variant_info.restype = ctypes.c_int
    L.pcub_sc_variant_info.argtypes = [ctypes.c_int] + [ctypes.POINTER(ctypes.c_int)] * 3
    L.pcub_sc_decode_bin_workspace.restype = ctypes.c_size_t
    L.pcub_sc_decode_bin_workspace.argtypes = [_i64, _i32]
    L.pcub_sc_decode_bin.restype = ctypes.c_int
    L.pcub_sc_decode_bin.argtypes = [_c_void_p, _i64, _i32, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p,
                                     _c_void_p, _c_void_p, ctypes.c_size_t, _c_void_p]
    L.pcub_sc_decode_qary_workspace.restype = ctypes.c_size_t
    L.pcub_sc_decode_qary_workspace.argtypes = [_i64, _i32, _i32]
    L.pcub_sc_decode_qary.restype = ctypes.c_int
    L.pcub_sc_decode_qary.argtypes = [_c_void_p, _i64, _i32, _i32, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p,
                                      ctypes.c_size_t, _c_void_p]
    L.pcub_polar_encode_qary.restype = ctypes.c_int
    L.pcub_polar_encode_qary.argtypes = [_c_void_p, _i64, _i32, _i32, _c_void_p, _i32, _c_void_p, _c_void_p]
    L.pcub_polar_encode_bin.restype = ctypes.c_int
    L.pcub_polar_encode_bin.argtypes = [_c_void_p, _i64, _i32, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p]
    L.pcub_pack_bits.restype = ctypes.c_int
    L.pcub_pack_bits.argtypes = [_c_void_p, _i64, _i32, _c_void_p, _c_void_p]
    L.pcub_unpack_bits.restype = ctypes.c_int
    L.pcub_unpack_bits.argtypes = [_c_void_p, _i64, _i32, _c_void_p, _c_void_p]
    L.pcub_transpose_pairs.restype = ctypes.c_int
    L.pcub_transpose_pairs.argtypes = [_c_void_p, _i64, _i32, _i32, _c_void_p, _c_void_p]
    L.pcub_tile_pairs.restype = ctypes.c_int
    L.pcub_tile_pairs.argtypes = [_c_void_p, _i64, _i32, _i32, _i32, _c_void_p, _c_void_p]
    L.pcub_sc_deletion_supported.restype = ctypes.c_int
    L.pcub_sc_deletion_supported.argtypes = [_i32, _i32, _i32]
    L.pcub_sc_leaf_deletion_supported.restype = ctypes.c_int
    L.pcub_sc_leaf_deletion_supported.argtypes = [_i32, _i32, _i32]
    L.pcub_sc_decode_deletion.restype = ctypes.c_int
    L.pcub_sc_decode_deletion.argtypes = [_c_void_p, _c_void_p, _i64, _i32, _i32, _i32, _i32, ctypes.c_double, _c_void_p,
                                          _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p]
    L.pcub_sc_leaf_bin_workspace.restype = ctypes.c_size_t
    L.pcub_sc_leaf_bin_workspace.argtypes = [_i64, _i32]
    L.pcub_sc_leaf_bin.restype = ctypes.c_int
    L.pcub_sc_leaf_bin.argtypes = [_c_void_p, _i64, _i32, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p,
                                   _c_void_p, _c_void_p, ctypes.c_size_t, _c_void_p]
    L.pcub_sc_leaf_deletion.restype = ctypes.c_int
    L.pcub_sc_leaf_deletion.argtypes = [_c_void_p, _c_void_p, _i64, _i32, _i32, _i32, _i32, ctypes.c_double, _c_void_p,
                                        _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p]
    L.pcub_sc_deletion_table_bytes.restype = _i64
    L.pcub_sc_deletion_table_bytes.argtypes = [_i32]
    L.pcub_sc_set_deletion_dense.restype = ctypes.c_int
    L.pcub_sc_set_deletion_dense.argtypes = [_i32]
    L.pcub_sc_set_deletion_lanes.restype = ctypes.c_int
    L.pcub_sc_set_deletion_lanes.argtypes = [_i32]
    L.pcub_sc_deletion_dense_layout.restype = ctypes.c_int
    L.pcub_sc_deletion_dense_layout.argtypes = [_i32, _i32, _i32, _i32, _c_void_p, ctypes.c_double]
    L.pcub_sc_deletion_build_table.restype = ctypes.c_int
    L.pcub_sc_deletion_build_table.argtypes = [_i32, ctypes.c_double, _c_void_p, _c_void_p]
    L.pcub_sc_decode_deletion_tab.restype = ctypes.c_int
    L.pcub_sc_decode_deletion_tab.argtypes = L.pcub_sc_decode_deletion.argtypes[:-1] + [_c_void_p, _c_void_p]
    L.pcub_sc_leaf_deletion_tab.restype = ctypes.c_int
    L.pcub_sc_leaf_deletion_tab.argtypes = L.pcub_sc_leaf_deletion.argtypes[:-1] + [_c_void_p, _c_void_p]
    L.pcub_scl_qary_workspace.restype = ctypes.c_size_t
    L.pcub_scl_qary_workspace.argtypes = [_i64, _i32, _i32, _i32, _i32]
    L.pcub_scl_qary.restype = ctypes.c_int
    L.pcub_scl_qary.argtypes = [_c_void_p, _i64, _i32, _i32, _i32, _c_void_p, _c_void_p, _i32, _c_void_p, _i32,
                                _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, ctypes.c_size_t, _c_void_p]
    L.pcub_scl_qary_log.restype = ctypes.c_int
    L.pcub_scl_qary_log.argtypes = L.pcub_scl_qary.argtypes
    L.pcub_sc_decode_qary_log_workspace.restype = ctypes.c_size_t
    L.pcub_sc_decode_qary_log_workspace.argtypes = [_i64, _i32, _i32]
    L.pcub_sc_decode_qary_log.restype = ctypes.c_int
    L.pcub_sc_decode_qary_log.argtypes = [_c_void_p, _i64, _i32, _i32, _c_void_p, _i32, _c_void_p, _c_void_p,
                                          _c_void_p, _c_void_p, ctypes.c_size_t, _c_void_p]
    L.pcub_sc_prior_bin_workspace.restype = ctypes.c_size_t
    L.pcub_sc_prior_bin_workspace.argtypes = [_i64, _i32]
    L.pcub_sc_prior_bin.restype = ctypes.c_int
    L.pcub_sc_prior_bin.argtypes = [_c_void_p, _c_void_p, _i64, _i64, _i32, _c_void_p, _c_void_p, _i32, _c_void_p,
                                    _c_void_p, _c_void_p, _c_void_p, ctypes.c_size_t, _c_void_p]
    L.pcub_leaf_marginals.restype = ctypes.c_int
    L.pcub_leaf_marginals.argtypes = [_c_void_p, _i64, _c_void_p, _c_void_p]
    _u64 = ctypes.c_uint64
    L.pcub_mc_info.restype = ctypes.c_int
    L.pcub_mc_info.argtypes = [_u64, _i64, _i64, _i32, _c_void_p, _c_void_p]
    L.pcub_mc_channel.restype = ctypes.c_int
    L.pcub_mc_channel.argtypes = [_u64, _i64, _i64, _i32, _i32, ctypes.c_double, _c_void_p, _c_void_p, _c_void_p]
    L.pcub_mc_count_errors.restype = ctypes.c_int
    L.pcub_mc_count_errors.argtypes = [_c_void_p, _c_void_p, _i64, _i32, _c_void_p, _c_void_p]
    L.pcub_sc_bin_tile.restype = ctypes.c_int
    L.pcub_sc_bin_tile.argtypes = [_i32]
    L.pcub_sc_decode_bin_tiled.restype = ctypes.c_int
    L.pcub_sc_decode_bin_tiled.argtypes = [_c_void_p, _i64, _i32, _i32, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p,
                                           _c_void_p, _c_void_p, ctypes.c_size_t, _c_void_p]
    L.pcub_sc_decode_bin_compact_tiled.restype = ctypes.c_int
    L.pcub_sc_decode_bin_compact_tiled.argtypes = [_c_void_p, _i64, _i32, _i32, _c_void_p, _c_void_p, _i32, _c_void_p,
                                                   _c_void_p, _c_void_p, _c_void_p, ctypes.c_size_t, _c_void_p]
    L.pcub_sc_decode_bin_compact_direct.restype = ctypes.c_int
    L.pcub_sc_decode_bin_compact_direct.argtypes = [_i32]
    L.pcub_sc_decode_bin_compact_workspace.restype = ctypes.c_size_t
    L.pcub_sc_decode_bin_compact_workspace.argtypes = [_i64, _i32]
    L.pcub_sc_decode_bin_compact.restype = ctypes.c_int
    L.pcub_sc_decode_bin_compact.argtypes = [_c_void_p, _i64, _i32, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p,
                                             _c_void_p, _c_void_p, ctypes.c_size_t, _c_void_p]
    L.pcub_mc_channel_tiled.restype = ctypes.c_int
    L.pcub_mc_channel_tiled.argtypes = [_u64, _i64, _i64, _i32, _i32, ctypes.c_double, _c_void_p, _c_void_p, _i32,
                                        _c_void_p]
    L.pcub_mc_channel_norm_tiled.restype = ctypes.c_int
    L.pcub_mc_channel_norm_tiled.argtypes = [_u64, _i64, _i64, _i32, _i32, ctypes.c_double, _c_void_p, _c_void_p,
                                             _i32, _i32, _c_void_p]
    L.pcub_mc_channel_norm.restype = ctypes.c_int
    L.pcub_mc_channel_norm.argtypes = [_u64, _i64, _i64, _i32, _i32, ctypes.c_double, _c_void_p, _c_void_p, _i32,
                                       _c_void_p]
    L.pcub_mc_info_qary.restype = ctypes.c_int
    L.pcub_mc_info_qary.argtypes = [_u64, _i64, _i64, _i32, _i32, _c_void_p, _c_void_p]
    L.pcub_mc_channel_qsc_tiled.restype = ctypes.c_int
    L.pcub_mc_channel_qsc_tiled.argtypes = [_u64, _i64, _i64, _i32, _i32, ctypes.c_double, _c_void_p, _c_void_p, _i32,
                                            _c_void_p]
    L.pcub_sc_qary_tile.restype = ctypes.c_int
    L.pcub_sc_qary_tile.argtypes = [_i32, _i32]
    L.pcub_sc_decode_qary_tiled.restype = ctypes.c_int
    L.pcub_sc_decode_qary_tiled.argtypes = [_c_void_p, _i64, _i32, _i32, _i32, _c_void_p, _i32, _c_void_p, _c_void_p,
                                            _c_void_p, ctypes.c_size_t, _c_void_p]
    L.pcub_mc_channel_qsc.restype = ctypes.c_int
    L.pcub_mc_channel_qsc.argtypes = [_u64, _i64, _i64, _i32, _i32, ctypes.c_double, _c_void_p, _c_void_p, _c_void_p]
    L.pcub_mc_deletion.restype = ctypes.c_int
    L.pcub_mc_deletion.argtypes = [_u64, _i64, _i64, _i32, _c_void_p, _i32, ctypes.c_double, _c_void_p, _c_void_p,
                                   _c_void_p, _c_void_p]
    L.pcub_mc_run_bin_workspace.restype = ctypes.c_size_t
    L.pcub_mc_run_bin_workspace.argtypes = [_i64, _i32, _i32]
    L.pcub_mc_run_bin.restype = ctypes.c_int
    L.pcub_mc_run_bin.argtypes = [_u64, _i64, _i64, _i32, _i32, ctypes.c_double, _c_void_p, _c_void_p, _i32, _i64,
                                  _c_void_p, _c_void_p, ctypes.c_size_t, _c_void_p]
    L.pcub_mc_run_qary_workspace.restype = ctypes.c_size_t
    L.pcub_mc_run_qary_workspace.argtypes = [_i64, _i32, _i32, _i32]
    L.pcub_mc_run_qary.restype = ctypes.c_int
    L.pcub_mc_run_qary.argtypes = [_u64, _i64, _i64, _i32, _i32, ctypes.c_double, _c_void_p, _i32, _i64, _c_void_p,
                                   _c_void_p, ctypes.c_size_t, _c_void_p]
    L.pcub_mc_run_deletion_workspace.restype = ctypes.c_size_t
    L.pcub_mc_run_deletion_workspace.argtypes = [_i64, _i32, _i32, _i32]
    L.pcub_mc_run_deletion.restype = ctypes.c_int
    L.pcub_mc_run_deletion.argtypes = [_u64, _i64, _i64, _i32, _i32, _c_void_p, _i32, _i32, ctypes.c_double,
                                       _c_void_p, _c_void_p, _i32, _c_void_p, _i64, _c_void_p, _c_void_p,
                                       ctypes.c_size_t, _c_void_p]
    if L.pcub_abi_version() != ABI_VERSION:
        raise ImportError("libpolarcub_hip.so ABI mismatch; rebuild with python -m polarcub_amd.build --force")
    _lib = L
    return L


# every exported symbol declared in include/polarcub_sc.h
EXPORTS = ["pcub_abi_version", "pcub_sc_decode_bin_workspace", "pcub_sc_decode_bin", "pcub_polar_encode_bin",
           "pcub_sc_decode_qary_workspace", "pcub_sc_decode_qary", "pcub_polar_encode_qary",
           "pcub_pack_bits", "pcub_unpack_bits", "pcub_transpose_pairs", "pcub_tile_pairs", "pcub_sc_deletion_supported",
           "pcub_sc_leaf_deletion_supported", "pcub_sc_decode_deletion", "pcub_sc_leaf_bin_workspace", "pcub_sc_leaf_bin", "pcub_sc_leaf_deletion",
           "pcub_sc_prior_bin_workspace", "pcub_sc_prior_bin",
           "pcub_sc_decode_qary_log_workspace", "pcub_sc_decode_qary_log",
           "pcub_scl_qary_workspace", "pcub_scl_qary", "pcub_scl_qary_log", "pcub_leaf_marginals", "pcub_mc_info", "pcub_mc_channel", "pcub_mc_count_errors", "pcub_mc_channel_norm", "pcub_sc_decode_bin_compact_direct", "pcub_sc_decode_bin_compact_workspace",
           "pcub_sc_decode_bin_compact", "pcub_mc_info_qary", "pcub_mc_channel_qsc", "pcub_mc_deletion",
           "pcub_mc_run_bin_workspace", "pcub_mc_run_bin", "pcub_sc_deletion_table_bytes",
           "pcub_sc_deletion_build_table", "pcub_sc_decode_deletion_tab", "pcub_sc_leaf_deletion_tab",
           "pcub_sc_set_deletion_dense", "pcub_sc_set_deletion_lanes", "pcub_sc_deletion_dense_layout", "pcub_sc_bin_tile", "pcub_sc_decode_bin_tiled",
           "pcub_sc_decode_bin_compact_tiled", "pcub_mc_channel_tiled", "pcub_mc_channel_norm_tiled",
           "pcub_mc_channel_qsc_tiled", "pcub_sc_qary_tile", "pcub_sc_decode_qary_tiled",
           "pcub_mc_run_qary_workspace", "pcub_mc_run_qary", "pcub_mc_run_deletion_workspace", "pcub_mc_run_deletion"]


def check(rc, what):
    if rc != 0:
        if rc == EINVAL:
            raise ValueError("%s: invalid arguments (PCUB_EINVAL)" % what)
        raise HipError("%s failed: hipError_t %d" % (what, rc))
