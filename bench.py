#!/usr/bin/env python3
"""Throughput benchmark: decoded codewords/s, binary SC, N=1024 rate-1/2 BI-AWGN.

BASELINE.json metric: "decoded codewords/sec at N=1024 BI-AWGN, batch=1M; FER
match vs reference".  Workload = BASELINE.json configs[1]: N=1024, K=512,
Eb/N0 = 2 dB, batch 2^20 codewords per GPU (weak scaling), synthetic data
generated on the device (Philox via torch.randn) and resident in HBM before the
timed region.  One step = one pcub_sc_decode_bin launch over the whole batch
(joint-probability pairs in -> packed info bits + packed x_hat out).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 10] [--batch 1048576]

Multi-GPU: launched by torch.distributed.run, one rank per GPU; each rank
decodes its own batch (no data-path collective); one RCCL all_reduce of the
error counters and a max-reduce of the elapsed time at the end.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from polarcub_amd import channel, construction, sc  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_inputs(code, B, sigma2, seed, device, chunk=1 << 18):
    """Random info bits -> GPU encoder -> BI-AWGN joint pairs in native [N, B, 2] layout."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    xy = torch.empty((code.N, B, 2), dtype=torch.float64, device=device)
    info = torch.empty((B, code.K), dtype=torch.uint8, device=device)
    for b0 in range(0, B, chunk):
        b1 = min(B, b0 + chunk)
        inf = torch.randint(0, 2, (b1 - b0, code.K), dtype=torch.uint8, device=device, generator=gen)
        info[b0:b1] = inf
        xw = sc.encode_native(code, sc.pack(inf))
        x_nb = channel.bits_from_words(xw, code.N)
        channel.awgn_pairs_native(x_nb, sigma2, generator=gen, out=xy[:, b0:b1, :])
        del xw, x_nb
    return xy, info


def measured_traffic(variant, n, batch):
    """Per-launch HBM bytes of this exact decode configuration from the committed
    rocprofv3 PMC passes (profiles/<round>/bin_v<variant>_n<n>/summary.json, written by
    scripts/collect_profiles.py; FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "bin_v%d_n%d" % (variant, n), "summary.json")),
                       reverse=True):
        with open(path) as f:
            s = json.load(f)
        if s.get("batch") == batch and "traffic_bytes" in s:
            return s["traffic_bytes"], os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(code, xy_native, seconds_target=12.0):
    """The C oracle (oracle/sc_oracle.c, -O2 -ffp-contract=off) on the host cores, on a
    bounded sample of the same synthetic codewords (rank 0 only)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import orc
    orc.lib()
    ncw = 4096
    sample = xy_native[:, :ncw, :].permute(1, 0, 2).contiguous().cpu().numpy()  # [ncw, N, 2]
    t0 = time.perf_counter()
    orc.decode_bin(sample[:64], code.frozen_mask, code.frozen_values)
    per_cw = (time.perf_counter() - t0) / 64
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    reps = max(1, int(round(seconds_target / (per_cw * ncw))))

    def work(i):
        part = sample[(i * ncw) // cores:((i + 1) * ncw) // cores]
        for _ in range(reps):
            orc.decode_bin(part, code.frozen_mask, code.frozen_values)
        return part.shape[0] * reps

    t0 = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:
        total = sum(ex.map(work, range(cores)))
    dt = time.perf_counter() - t0
    return {"value": total / dt, "unit": "codewords/s", "cores": cores, "kind": "port",
            "sample": "%d codewords x %d passes of the bench's own synthetic N=%d inputs, "
                      "oracle/sc_oracle.c on %d threads (%.1f CPU-s)" % (ncw, reps, code.N, cores, dt * cores)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=10, help="log2 code length")
    ap.add_argument("--rate", type=float, default=0.5)
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--batch", type=int, default=1 << 20, help="codewords per GPU")
    ap.add_argument("--variant", type=int, default=None, help="decode kernel variant (default: the library's)")
    ap.add_argument("--max-blocks", type=int, default=0, help="cap decode workgroups per CU (0 = occupancy)")
    ap.add_argument("--seed", type=int, default=20250204)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-xhat", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(device)

    n, N = args.n, 1 << args.n
    K = int(round(N * args.rate))
    sigma2 = construction.awgn_sigma2(args.ebn0, K / N)
    frozen = construction.bhattacharyya_frozen(n, K, sigma2)
    code = sc.CodeSpec.from_frozen_set(N, set(np.nonzero(frozen)[0].tolist()), 1, device=device)
    sc.set_variant(args.variant)
    variant = sc.default_variant() if args.variant is None else args.variant
    sc.set_max_blocks_per_cu(args.max_blocks)
    dec = sc.BinaryDecoder(code)
    B = args.batch

    t0 = time.time()
    xy, info_tx = make_inputs(code, B, sigma2, args.seed + 7919 * rank, device)
    torch.cuda.synchronize()
    log("rank %d: inputs %.1f GB generated in %.1f s" % (rank, xy.numel() * 8 / 1e9, time.time() - t0))
    outs = (torch.empty((code.info_words, B), dtype=torch.int32, device=device),
            None if args.no_xhat else torch.empty((code.n_words, B), dtype=torch.int32, device=device), None)
    dec.workspace(B)

    for _ in range(args.warmup):
        dec.decode_native(xy, out=outs)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t_start = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        dec.decode_native(xy, out=outs)
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    kern_ms = [a.elapsed_time(b) for a, b in evs]

    # frame errors of the last decode (identical each step)
    info_dec = sc.unpack(outs[0], K)
    errs = (info_dec != info_tx).any(dim=1)
    counters = torch.tensor([B, int(errs.sum().item()), int((info_dec != info_tx).sum().item()), 0],
                            dtype=torch.int64, device=device)
    el = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(counters, op=dist.ReduceOp.SUM)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    total_cw = int(counters[0].item()) * args.steps
    value = total_cw / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    if rank == 0:
        avg_kern_s = float(np.mean(kern_ms)) / 1e3
        b_alg = 16 * N + N // 8 + K // 8  # f64 pairs in + packed x_hat + packed info, per codeword
        achieved = b_alg * B / avg_kern_s / 1e9
        traffic, traffic_src = measured_traffic(variant, n, B)
        rec = {
            "metric": "decoded codewords/sec at N=%d BI-AWGN, batch=%d per GPU; FER match vs reference" % (N, B),
            "value": value,
            "unit": "codewords/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: uniform info bits, GPU polar encoder, BI-AWGN Eb/N0=%.1f dB pairs generated on device" % args.ebn0,
            "config": {"workload": "binary SC decode N=%d K=%d BI-AWGN %.1f dB (BASELINE configs[1])" % (N, K, args.ebn0),
                       "N": N, "K": K, "batch_per_gpu": B, "ebn0_db": args.ebn0, "kernel_variant": variant, "max_blocks_per_cu": args.max_blocks,
                       "parallelism": "dp%d (codeword sharding, RCCL all_reduce of counters)" % world},
            "fer": float(counters[1].item()) / int(counters[0].item()),
            "frame_errors": int(counters[1].item()),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "k_sc_bin", "kernel_ms": float(np.mean(kern_ms)),
                         "bytes_alg_per_cw": b_alg},
        }
        if world == 1 and not args.no_cpu:
            rec["cpu_baseline"] = cpu_baseline(code, xy)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
