"""Diagnostic: the device stack limit, then one SCL list decode at q=4, N=256, L=8 (the bench's
shape) for batch B (argv[1]); prints the limit before/after and the decode's status."""
import ctypes, sys
sys.path.insert(0, ".")
import numpy as np
import torch
from polarcub_amd import _lib, sc
L = _lib.lib()
L.pcub_scl_stack_limit.restype = ctypes.c_longlong
torch.cuda.init()
B = int(sys.argv[1])
print("stack limit before", L.pcub_scl_stack_limit(), flush=True)
rng = np.random.default_rng(1)
N, q, Ls = 256, 4, 8
frozen = (rng.random(N) < 0.5).astype(np.uint8)
dec = sc.QaryListDecoder(q, N, frozen, Ls)
xy = torch.rand((N, B, q), dtype=torch.float64, device="cuda")
fv = torch.zeros((int(frozen.sum()), B), dtype=torch.uint8, device="cuda")
info, prob, size, _ = dec.decode_native(xy, fv)
torch.cuda.synchronize()
print("stack limit after", L.pcub_scl_stack_limit(), "B", B, "ok, mean list size %.2f" % size.float().mean().item(), flush=True)
