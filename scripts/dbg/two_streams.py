"""Experiment: one decode launch over B codewords vs two concurrent launches of B/2 on two
streams (tail / ramp overlap), same inputs, N = 1024 and 4096."""
import sys, time
sys.path.insert(0, ".")
import numpy as np
import torch
from polarcub_amd import sc, construction

def run(n, B, reps=10):
    N = 1 << n
    K = N // 2
    s2 = construction.awgn_sigma2(2.0, 0.5)
    frozen = construction.bhattacharyya_frozen(n, K, s2)
    code = sc.CodeSpec.from_frozen_set(N, set(np.nonzero(frozen)[0].tolist()), 1, device=torch.device("cuda"))
    g = torch.Generator(device="cuda").manual_seed(1)
    xy = torch.rand((N, B, 2), dtype=torch.float64, device="cuda", generator=g)
    xa = xy[:, : B // 2].contiguous()
    xb = xy[:, B // 2:].contiguous()
    d1, da, db = sc.BinaryDecoder(code), sc.BinaryDecoder(code), sc.BinaryDecoder(code)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    def one():
        d1.decode_native(xy, want_xhat=True)
    def two():
        cur = torch.cuda.current_stream()
        sa.wait_stream(cur); sb.wait_stream(cur)
        with torch.cuda.stream(sa):
            ra = da.decode_native(xa, want_xhat=True)
        with torch.cuda.stream(sb):
            rb = db.decode_native(xb, want_xhat=True)
        cur.wait_stream(sa); cur.wait_stream(sb)
        return ra, rb
    # parity: the halves decode exactly as the full batch
    i1, x1, _ = d1.decode_native(xy)
    (ia, xa_, _), (ib, xb_, _) = two()
    torch.cuda.synchronize()
    assert torch.equal(i1, torch.cat([ia, ib], 1)) and torch.equal(x1, torch.cat([xa_, xb_], 1))
    for name, f in (("one", one), ("two", two), ("one", one), ("two", two)):
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / reps
        print("n=%d %s: %.2f ms per %d codewords, %.2f M cw/s" % (n, name, dt * 1e3, B, B / dt / 1e6), flush=True)

run(10, 1 << 20)
run(12, 1 << 18)
