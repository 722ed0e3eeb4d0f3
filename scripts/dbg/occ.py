"""Debug: resident workgroups the binary / q-ary launchers choose (inferred from workspace sizes)."""
import ctypes, sys
sys.path.insert(0, ".")
import torch
from polarcub_amd import _lib
L = _lib.lib()
torch.cuda.init()
cus = torch.cuda.get_device_properties(0).multi_processor_count
L.pcub_sc_decode_bin_workspace.restype = ctypes.c_size_t
L.pcub_sc_decode_bin_workspace.argtypes = [ctypes.c_int64, ctypes.c_int32]
for n in (10, 12):
    ws = L.pcub_sc_decode_bin_workspace(1 << 20, n)
    Nv = (1 << n) // 4
    slot = (Nv // 2 - 32) * 16
    ef = ((1 << (n - 2 - 5)) + 255) & ~255
    g = (ws - ef) / (256 * slot)
    print("bin n=%d workspace %d -> grid %.1f workgroups = %.2f per CU (%d CUs)" % (n, ws, g, g / cus, cus))
