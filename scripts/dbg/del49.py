"""Debug: the (n0=4, n=9) random case on the GPU, whole batch vs one word at a time vs the oracle."""
import random, sys
sys.path.insert(0, ".")
import numpy as np
import torch
from oracle import trellis_oracle as tro
from polarcub_amd import sc
n0, n, ones = 4, 9, 0
N = 1 << n
rng = np.random.default_rng(1000 * n0 + 10 * n + ones)
prng = random.Random(n + 100 * ones)
frozen = (rng.random(N) < 0.5).astype(np.uint8)
frozen[: N // 4] = 1
frozen[-(N // 8) or -1:] = 0
fval = (rng.random(N) < 0.5).astype(np.uint8)
pd = [0.05, 0.1, 0.3][n % 3]
words = []
for t in range(10):
    x = [int(b) for b in rng.integers(0, 2, N)]
    cw = tro.add_guard_bands(x, n, n0, 0.1, ones)
    words.append(tro.deletion_channel(cw, pd if t < 8 else 0.6, prng))
words += [[], [1], [0] * 9, [int(b) for b in rng.integers(0, 2, 3 * N)]]
def dec(ws):
    W = max(1, max(len(w) for w in ws))
    rx = np.zeros((len(ws), W), np.uint8)
    for i, w in enumerate(ws):
        rx[i, :len(w)] = w
    code = sc.CodeSpec(N, frozen, fval, device="cuda")
    d = sc.DeletionDecoder(code, n0, pd, ones)
    info, xh = d.decode(torch.from_numpy(rx).cuda(), torch.from_numpy(np.array([len(w) for w in ws], np.int32)).cuda())
    torch.cuda.synchronize()
    return info.cpu().numpy(), xh.cpu().numpy()
info, xh = dec(words)
for i, w in enumerate(words):
    xr, ir = tro.decode_deletion(w, n, n0, pd, frozen, fval, ones=ones)
    i1, x1 = dec([w])
    bi = [k for k in range(len(ir)) if info[i][k] != ir[k]]
    bx = [k for k in range(N) if xh[i][k] != xr[k]]
    b1 = [k for k in range(len(ir)) if i1[0][k] != ir[k]]
    print(i, len(w), "batch info diff", bi[:10], len(bi), "xhat diff", bx[:10], len(bx), "single info diff", b1[:10], len(b1), flush=True)
