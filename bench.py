#!/usr/bin/env python3
"""Throughput benchmark: decoded codewords/s of the SC decoder on MI355X.

BASELINE.json metric: "decoded codewords/sec at N=1024 BI-AWGN, batch=1M; FER match
vs reference".  Default workload = BASELINE.json configs[1]: binary SC, N=1024,
K=512, Eb/N0 = 2 dB, 2^20 codewords per GPU (weak scaling).  Other configs as
--workload (reported beside it, not the headline):

  awgn      configs[1] (N=1024) / configs[2] with --n 12 (N=4096)
  deletion  configs[4]: main_deletion.py defaults, n=8, n0=2, pd=0.1, xi=0.1
  qary      configs[3]: q=4, N=256, QSC(0.11)

Synthetic data is generated on the device (torch Philox), resident in HBM before the
timed region.  One step = one decode launch over the whole per-GPU batch.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload awgn|deletion|qary] [--batch B]

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) this
process is one rank; started directly with --gpus N > 1 it launches the N ranks itself
(torch.distributed.run as a child process, before anything touches the GPU) and exits
with their status.  Rank r decodes global codewords [r*B, (r+1)*B) (no data-path
collective); one RCCL all_reduce of the error counters, a max-reduce of the elapsed
time and an all_gather of the per-rank times at the end.

--workload stub is the same rank logic on the CPU (gloo, oracle decode of N=64 BSC
codewords keyed by global codeword index): the multi-rank test of the launcher.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from polarcub_amd import channel, construction, mc, sc  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cores():
    """(threads to use, description): every core in this process's affinity mask, capped by
    the cgroup CPU quota when one is set (more threads than the quota only time-slice)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    used = aff if quota is None else min(aff, quota)
    desc = "%d host threads (sched_getaffinity %d cores, cgroup cpu quota %s)" % (
        used, aff, "none" if quota is None else "%d CPUs" % quota)
    return max(1, used), desc


def measured_traffic(tag, batch):
    """Per-launch HBM bytes of this exact configuration from the committed rocprofv3 PMC
    passes (profiles/<round>/<tag>/summary.json, written by scripts/collect_profiles.py:
    FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), or (None, None)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", tag, "summary.json")), reverse=True):
        with open(path) as f:
            s = json.load(f)
        if s.get("batch") == batch and "traffic_bytes" in s:
            return s["traffic_bytes"], os.path.relpath(path, ROOT)
    return None, None


# ----------------------------------------------------------------------------- workloads

class Awgn:
    """Binary SC over BI-AWGN (configs[1], configs[2] with --n 12)."""
    kernel = "k_sc_bin"

    def __init__(self, a, device, rank):
        self.a = a
        n = a.n if a.n is not None else 10
        N = 1 << n
        K = int(round(N * a.rate))
        self.n, self.N, self.K, self.B = n, N, K, a.batch
        self.sigma2 = construction.awgn_sigma2(a.ebn0, K / N)
        frozen = construction.bhattacharyya_frozen(n, K, self.sigma2)
        self.code = sc.CodeSpec.from_frozen_set(N, set(np.nonzero(frozen)[0].tolist()), 1, device=device)
        sc.set_variant(a.variant)
        self.variant = sc.variant_for(self.n)  # the kernel that runs (fallback included)
        sc.set_max_blocks_per_cu(a.max_blocks)
        self.dec = sc.BinaryDecoder(self.code)
        # global codewords [rank*B, (rank+1)*B), Philox keyed by (seed, codeword index)
        self.offset = mc.rank_offset(rank, self.B)
        # the root rows in the kernel's tiles (a wave's codewords contiguous, pcub_sc_decode_bin_tiled) unless
        # --no-tile ([N][B][2] rows, pcub_sc_decode_bin)
        self.tile = 0 if a.no_tile else sc.bin_tile(n)
        self.info_w, self.xy = mc.philox_batch(self.code, a.seed, self.offset, self.B, mc.CHANNEL_AWGN, self.sigma2,
                                               tile=self.tile)
        self.rank = rank
        self.outs = (torch.empty((self.code.info_words, self.B), dtype=torch.int32, device=device),
                     None if a.no_xhat else torch.empty((self.code.n_words, self.B), dtype=torch.int32, device=device),
                     None)
        self.dec.workspace(self.B)

    def step(self):
        if self.tile:
            self.dec.decode_tiled_native(self.xy, self.B, out=self.outs)
        else:
            self.dec.decode_native(self.xy, out=self.outs)

    def rows(self, ncw):
        """The first ncw codewords' rows, [ncw, N, 2] (the reference's layout)."""
        if not self.tile:
            return self.xy[:, :ncw, :].permute(1, 0, 2).contiguous()
        T = self.tile
        nt = (ncw + T - 1) // T
        return self.xy[:nt].permute(0, 2, 1, 3).reshape(nt * T, self.N, 2)[:ncw].contiguous()

    def errors(self):
        d = sc.unpack(self.outs[0], self.K)
        return mc.error_counts(d, sc.unpack(self.info_w, self.K))

    def end_to_end(self, reps=5):
        """The whole Monte-Carlo pipeline on the device (pcub_mc_run_bin: information bits ->
        encoder -> BI-AWGN -> decode -> counters) over this rank's codewords, in chunks of 2^18
        codewords back to back on one stream: seconds of the median of `reps` warm runs (the spread
        goes into the bench line)."""
        chunk = min(self.B, self.a.e2e_chunk)
        mc.run_bin(self.code, self.a.seed, self.offset, self.B, mc.CHANNEL_AWGN, self.sigma2, chunk=chunk)
        times = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mc.run_bin(self.code, self.a.seed, self.offset, self.B, mc.CHANNEL_AWGN, self.sigma2, chunk=chunk)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        self.e2e_times = times
        return float(np.median(times))

    def bytes_alg(self):
        return 16 * self.N + self.N // 8 + self.K // 8  # f64 pairs in + packed x_hat + packed info

    def tag(self):
        return "bin_v%d_n%d" % (self.variant, self.n)

    def describe(self, world):
        a = self.a
        return dict(
            metric="decoded codewords/sec at N=%d BI-AWGN, batch=%d per GPU; FER match vs reference" % (self.N, self.B),
            dtype="f64",
            data="synthetic: uniform info bits, GPU polar encoder, BI-AWGN Eb/N0=%.1f dB pairs generated on device "
                 "(Philox keyed by global codeword index)%s" % (
                     a.ebn0, ", rows in %d-codeword tiles [B/%d][N][%d][2]" % (self.tile, self.tile, self.tile)
                     if self.tile else ", rows [N][B][2]"),
            config={"workload": "binary SC decode N=%d K=%d BI-AWGN %.1f dB (BASELINE configs[%d])"
                                % (self.N, self.K, a.ebn0, 1 if self.n == 10 else 2),
                    "N": self.N, "K": self.K, "batch_per_gpu": self.B, "ebn0_db": a.ebn0,
                    "kernel_variant": self.variant, "max_blocks_per_cu": a.max_blocks, "root_tile": self.tile,
                    "parallelism": "dp%d (codeword sharding, RCCL all_reduce of counters)" % world})

    def cpu_baseline(self, seconds=12.0):
        """oracle/sc_oracle.c (-O2 -ffp-contract=off) on the host cores, threads over a bounded
        sample of the bench's own codewords."""
        from concurrent.futures import ThreadPoolExecutor

        from oracle import orc
        orc.lib()
        code, ncw = self.code, 4096
        sample = self.rows(ncw).cpu().numpy()
        t0 = time.perf_counter()
        orc.decode_bin(sample[:64], code.frozen_mask, code.frozen_values)
        per_cw = (time.perf_counter() - t0) / 64
        cores, cdesc = host_cores()
        reps = max(1, int(round(seconds / (per_cw * ncw))))

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
                "sample": "%d codewords x %d passes of the bench's own synthetic N=%d inputs, oracle/sc_oracle.c "
                          "on %s (%.1f CPU-s)" % (ncw, reps, code.N, cdesc, dt * cores)}


def _genie_file_scores(path):
    """Per-index genie counts (TV + Pe summed over the trials) of a frozen-set file in the
    format of BinaryPolarEncoderDecoder.py:471-489 ('*** i count' lines), and the frozen set
    (index lines)."""
    scores, frozen = {}, set()
    with open(path) as f:
        for line in f:
            if line.startswith("***"):
                _, i, c = line.split()
                scores[int(i)] = float(c)
            elif not line.startswith("*") and line.strip():
                frozen.add(int(line))
    return scores, frozen


class Deletion:
    """Deletion channel, configs[4] = main_deletion.py's configuration: n=8, n0=n//3=2,
    pd=0.1, xi=0.1, no guard-band ones; the frozen set of its default construction (genie,
    -g 8000, -pe 0.1: K=3, tests/golden/frozen_deletion_n8_g8000.txt written by this
    framework's main_deletion counterpart), or with --del-k K the K indices of smallest genie
    TV+Pe (a heavier decode).  Other n: n0 = n//3 unless --n0, frozen set = the N/4 most
    reliable indices of a Bhattacharyya ranking (stand-in; no genie fixture at that size)."""
    kernel = "k_sc_del"

    def __init__(self, a, device, rank):
        self.a = a
        self.n = a.n if a.n is not None else 8
        self.n0 = a.n0 if a.n0 is not None else self.n // 3
        self.pd, self.xi, self.ones = a.pd, a.xi, a.ones
        self.N = 1 << self.n
        self.B = a.batch
        if self.n == 8 and self.n0 == 2 and abs(self.pd - 0.1) < 1e-12 and abs(self.xi - 0.1) < 1e-12:
            scores, frozen = _genie_file_scores(os.path.join(ROOT, "tests", "golden", "frozen_deletion_n8_g8000.txt"))
            if a.del_k:
                order = sorted(range(self.N), key=lambda i: (scores[i], i))
                frozen = set(order[a.del_k:])
                self.construction = "genie (8000 trials) ranking, K=%d" % a.del_k
            else:
                self.construction = "main_deletion.py default construction: genie 8000 trials, Pe bound 0.1"
        else:
            K = a.del_k or self.N // 4
            frozen = set(np.nonzero(construction.bhattacharyya_frozen(self.n, K, 0.5))[0].tolist())
            self.construction = "Bhattacharyya ranking stand-in, K=%d" % K
        self.code = sc.CodeSpec.from_frozen_set(self.N, frozen, 200, device=device)
        self.K = self.code.K
        if a.del_lanes:
            sc.set_deletion_lanes(a.del_lanes)
        if a.del_rate1 >= 0:
            sc.set_deletion_rate1(a.del_rate1)
        if a.del_wave >= 0:
            sc.set_deletion_wave(a.del_wave)
        self.dec = sc.DeletionDecoder(self.code, self.n0, self.pd, self.ones)
        # Philox keyed by the global codeword index: rank r's shard is codewords [r*B, (r+1)*B) of
        # the one-GPU run, so sharded counters sum to the single run's
        info_w, self.rx, self.rx_len = mc.philox_deletion_batch(self.code, a.seed, mc.rank_offset(rank, self.B),
                                                                self.B, self.n0, self.xi, self.pd, self.ones)
        self.info_tx = sc.unpack(info_w, self.K)
        self.outs = None
        self.dense = self.dec.dense_layout(self.rx.shape[1], self.rx.device)
        self.kernel = "k_sc_del_dense" if self.dense else "k_sc_del"
        # n0 = 4, 64 .. 1024 trellises, no ones: the wave-per-task kernel (sc_del.hip's dispatch)
        if (self.n0 == 4 and self.ones == 0 and 6 <= self.n - self.n0 <= 10 and a.del_wave != 0
                and (self.rx.shape[1] + 31) // 32 * 4 <= 32768):
            self.kernel = "k_sc_del_w4"

    def step(self):
        self.outs = self.dec.decode_native(self.rx, self.rx_len)

    def errors(self):
        return mc.error_counts(sc.unpack(self.outs[0], self.K), self.info_tx)

    def bytes_alg(self):
        return float(self.rx_len.float().mean().item()) + 4 + self.N // 8 + self.K // 8

    def tag(self):
        return "del_n%d_n0%d%s%s" % (self.n, self.n0, "_k%d" % self.K if self.K != 3 else "",
                                     "_dense" if self.dense else "")

    def describe(self, world):
        return dict(
            metric="decoded codewords/sec, deletion channel N=%d n0=%d pd=%.2f (main_deletion.py), batch=%d per GPU"
                   % (self.N, self.n0, self.pd, self.B),
            dtype="f64",
            data="synthetic: uniform info bits, GPU polar encoder, guard bands (xi=%.2f), deletions drawn on device "
                 "(Philox keyed by global codeword index)" % self.xi,
            config={"workload": "deletion SC decode N=%d n0=%d K=%d pd=%.2f ones=%d%s"
                                % (self.N, self.n0, self.K, self.pd, self.ones,
                                   " (BASELINE configs[4])" if self.n == 8 else ""),
                    "N": self.N, "K": self.K, "n0": self.n0, "pd": self.pd, "xi": self.xi, "ones": self.ones,
                    "frozen_set": self.construction, "batch_per_gpu": self.B,
                    "received_len_mean": float(self.rx_len.float().mean().item()),
                    "parallelism": "dp%d (codeword sharding, RCCL all_reduce of counters)" % world})

    def cpu_baseline(self, seconds=10.0):
        """oracle/trellis_oracle.c (the C restatement of the reference's trellis SC; ctypes releases the
        GIL) on the host threads, each on its own slice of a bounded sample of the bench's own
        received words, repeated to about `seconds` of wall time."""
        from concurrent.futures import ThreadPoolExecutor

        from oracle import orc
        orc.lib()
        cores, cdesc = host_cores()
        ncw = min(self.B, 64 * cores)
        rx = self.rx[:ncw].cpu().numpy()
        ln = self.rx_len[:ncw].cpu().numpy()
        fm, fv = self.code.frozen_mask, self.code.frozen_values
        t0 = time.perf_counter()
        orc.decode_deletion(rx[:8], ln[:8], self.n, self.n0, self.pd, fm, fv, self.ones)
        per_cw = max((time.perf_counter() - t0) / 8, 1e-7)
        reps = max(1, int(round(seconds * cores / (per_cw * ncw))))

        def work(i):
            sl = slice((i * ncw) // cores, ((i + 1) * ncw) // cores)
            for _ in range(reps):
                orc.decode_deletion(rx[sl], ln[sl], self.n, self.n0, self.pd, fm, fv, self.ones)
            return (sl.stop - sl.start) * reps

        t0 = time.perf_counter()
        with ThreadPoolExecutor(cores) as ex:
            done = sum(ex.map(work, range(cores)))
        dt = time.perf_counter() - t0
        return {"value": done / dt, "unit": "codewords/s", "cores": cores, "kind": "port",
                "sample": "%d of the bench's own received words x %d passes, oracle/trellis_oracle.c (C restatement) "
                          "on %s (%.1f CPU-s)" % (ncw, reps, cdesc, dt * cores)}


class Qary:
    """q-ary SC (configs[3]): q=4, N=256, K=128, QSC(p)."""
    kernel = "k_sc_qary"

    def __init__(self, a, device, rank):
        self.a = a
        self.q, self.n = a.q, (a.n if a.n is not None else 8)
        self.N = 1 << self.n
        self.K = self.N // 2
        self.B = a.batch
        if self.q == 4 and self.n == 8 and abs(a.qsc_p - 0.11) < 1e-12:
            # the reference's own q-ary degrading construction (n=8, L=64, QSC(0.11),
            # numInfoIndices=127 -> K=128), a fixture made by running it (oracle/make_golden.py)
            g = np.load(os.path.join(ROOT, "tests", "golden", "construct_qary.npz"), allow_pickle=False)
            mask = g["qsc4_n8_L64_frozen"].astype(np.uint8)
            self.construction = "reference QaryMemorylessDistribution degrading construction, L=64, numInfoIndices=127"
        else:
            z = construction.bhattacharyya_z(self.n, 0.5)
            order = sorted(range(self.N), key=lambda i: (z[i], i))
            mask = np.ones(self.N, np.uint8)
            mask[order[:self.K]] = 0
            self.construction = "binary Bhattacharyya ranking (stand-in)"
        self.K = int(self.N - mask.sum())
        self.code = sc.QaryCode(self.q, self.N, mask, device=device)
        if a.qlanes:
            sc.set_qary_lanes(a.qlanes)
        if a.qregs:
            sc.set_qary_regs(a.qregs)
        if a.qlds is not None:
            sc.set_qary_lds(bool(a.qlds))

        self.dec = sc.QaryDecoder(self.code)
        self.tile = 0 if (a.no_tile or type(self) is not Qary) else self.dec.tile()
        info, self.xy = mc.philox_qsc_batch(self.code, a.seed, mc.rank_offset(rank, self.B), self.B, a.qsc_p,
                                            tile=self.tile)
        self.info_tx = info.t()
        self.dec.workspace(self.B)
        self.outs = None

    def step(self):
        if self.tile:
            self.outs = self.dec.decode_tiled_native(self.xy, self.B)
        else:
            self.outs = self.dec.decode_native(self.xy)

    def rows(self, ncw):
        """The first ncw codewords' rows, [ncw, N, q] (the reference's layout)."""
        if not self.tile:
            return self.xy[:, :ncw, :].permute(1, 0, 2).contiguous()
        T = self.tile
        nt = (ncw + T - 1) // T
        return self.xy[:nt].permute(0, 2, 1, 3).reshape(nt * T, self.N, self.q)[:ncw].contiguous()

    def errors(self):
        return mc.error_counts(self.outs[0].t(), self.info_tx)

    def bytes_alg(self):
        bits = max(1, (self.q - 1).bit_length())
        return 8 * self.q * self.N + (self.N * bits) // 8 + (self.K * bits) // 8

    def tag(self):
        return "qary_q%d_n%d" % (self.q, self.n)

    def describe(self, world):
        return dict(
            metric="decoded codewords/sec, q=%d SC N=%d QSC(%.2f), batch=%d per GPU" % (self.q, self.N, self.a.qsc_p,
                                                                                     self.B),
            dtype="f64",
            data="synthetic: uniform info symbols, GPU q-ary encoder, QSC(%.2f) on device (Philox keyed by global "
                 "codeword index)%s" % (self.a.qsc_p, ", rows in %d-codeword tiles" % self.tile if self.tile else ""),
            config={"workload": "q-ary SC decode q=%d N=%d K=%d QSC(%.2f) (BASELINE configs[3])"
                                % (self.q, self.N, self.K, self.a.qsc_p),
                    "N": self.N, "K": self.K, "q": self.q, "batch_per_gpu": self.B, "frozen_set": self.construction,
                    "root_tile": self.tile,
                    "parallelism": "dp%d (codeword sharding, RCCL all_reduce of counters)" % world})

    def cpu_baseline(self, seconds=10.0):
        """oracle/sc_oracle.c q-ary recursion on the host threads (ctypes releases the GIL)."""
        from concurrent.futures import ThreadPoolExecutor

        from oracle import orc
        orc.lib()
        cores, cdesc = host_cores()
        ncw = 4096
        sample = self.rows(ncw).cpu().numpy()
        t0 = time.perf_counter()
        orc.decode_qary(self.q, sample[:64], self.code.frozen_mask)
        per_cw = (time.perf_counter() - t0) / 64
        reps = max(1, int(round(seconds * cores / (per_cw * ncw))))

        def work(i):
            part = sample[(i * ncw) // cores:((i + 1) * ncw) // cores]
            for _ in range(reps):
                orc.decode_qary(self.q, part, self.code.frozen_mask)
            return part.shape[0] * reps

        t0 = time.perf_counter()
        with ThreadPoolExecutor(cores) as ex:
            total = sum(ex.map(work, range(cores)))
        dt = time.perf_counter() - t0
        return {"value": total / dt, "unit": "codewords/s", "cores": cores, "kind": "port",
                "sample": "%d codewords x %d passes of the bench's own inputs, oracle/sc_oracle.c q-ary on %s"
                          % (ncw, reps, cdesc)}


class Scl(Qary):
    """q-ary list decoding (QaryPolarEncoderDecoder.listDecode, pcub_scl_qary) of the q-ary
    workload's inputs: the same code (C4 frozen set at q=4, N=256) and QSC batch, frozen values 0
    (the encoder's), list size --list-size; the decoded word is the path of largest metric."""
    kernel = "k_scl"

    def __init__(self, a, device, rank):
        super().__init__(a, device, rank)
        self.L = a.list_size
        self.ldec = sc.QaryListDecoder(self.q, self.N, self.code.frozen_mask, self.L, device=device)
        self.fv = torch.zeros((self.N - self.K, self.B), dtype=torch.uint8, device=device)
        self.outs = None

    def step(self):
        self.outs = self.ldec.decode_native(self.xy, self.fv)

    def errors(self):
        info, prob, size, _ = self.outs
        best = torch.argmax(prob, dim=0)  # [B]
        sel = info.gather(0, best.view(1, 1, -1).expand(1, info.shape[1], -1))[0]  # [K, B]
        return mc.error_counts(sel.t(), self.info_tx)

    def tag(self):
        return "scl_q%d_n%d_L%d" % (self.q, self.n, self.L)

    def describe(self, world):
        d = super().describe(world)
        d["metric"] = "list-decoded codewords/sec, q=%d SCL L=%d N=%d QSC(%.2f), batch=%d per GPU" % (
            self.q, self.L, self.N, self.a.qsc_p, self.B)
        d["config"]["workload"] = "q-ary SCL / Fast-SSC list decode q=%d N=%d K=%d L=%d QSC(%.2f)" % (
            self.q, self.N, self.K, self.L, self.a.qsc_p)
        d["config"]["list_size"] = self.L
        return d

    def cpu_baseline(self, seconds=10.0):
        """oracle/scl_oracle.py (pure Python restatement, one core) on a bounded sample."""
        from oracle import scl_oracle
        ncw = 16
        xy = self.xy[:, :ncw, :].permute(1, 0, 2).contiguous().cpu().numpy()
        fv = [0] * (self.N - self.K)
        t0 = time.perf_counter()
        done = 0
        while done < ncw and time.perf_counter() - t0 < seconds:
            scl_oracle.list_decode(self.q, self.code.frozen_mask, self.L, xy[done], fv)
            done += 1
        dt = time.perf_counter() - t0
        return {"value": done / dt, "unit": "codewords/s", "cores": 1, "kind": "port",
                "sample": "%d codewords of the bench's own inputs, oracle/scl_oracle.py (Python) on 1 core" % done}


class Stub:
    """The multi-rank logic of this script on the CPU (gloo): N=64 binary SC over BSC(0.11)
    decoded by the CPU oracle; codeword g's information bits and channel flips are drawn
    from a generator keyed by (seed, g), and rank r owns global codewords
    [rank_offset(r, B), rank_offset(r, B) + B) exactly as the GPU workloads do.  Used by
    tests/test_bench_launch.py; never a bench line."""
    kernel = "oracle"

    def __init__(self, a, device, rank):
        from oracle import orc
        self.a, self.orc = a, orc
        self.n, self.N, self.B = 6, 64, a.batch
        self.K = self.N // 2
        self.frozen = construction.bhattacharyya_frozen(self.n, self.K, 0.5)
        self.fval = np.zeros(self.N, np.uint8)
        off = mc.rank_offset(rank, self.B)
        p = 0.11
        table = np.array([[0.5 * (1 - p), 0.5 * p], [0.5 * p, 0.5 * (1 - p)]])
        self.info = np.zeros((self.B, self.K), np.uint8)
        self.xy = np.zeros((self.B, self.N, 2))
        for b in range(self.B):
            g = np.random.default_rng([a.seed, off + b])
            self.info[b] = g.integers(0, 2, self.K)
            x = orc.encode_bin(self.info[b], self.frozen, fval=self.fval)
            y = x ^ (g.random(self.N) < p).astype(np.uint8)
            self.xy[b] = table[y]
        self.out = None

    def step(self):
        self.out = self.orc.decode_bin(self.xy, self.frozen, self.fval)[0]

    def errors(self):
        d = self.out != self.info
        return int(d.any(axis=1).sum()), int(d.sum())

    def bytes_alg(self):
        return 16 * self.N + self.N // 8 + self.K // 8

    def tag(self):
        return "stub"

    def describe(self, world):
        return dict(metric="stub: decoded codewords/sec of the CPU oracle (launcher test, not a bench line)",
                    dtype="f64", data="synthetic BSC(0.11), generator keyed by global codeword index",
                    config={"workload": "stub N=64 K=32 BSC(0.11) on the CPU oracle", "N": self.N, "K": self.K,
                            "batch_per_gpu": self.B, "parallelism": "dp%d over gloo" % world})


WORKLOADS = {"awgn": Awgn, "deletion": Deletion, "qary": Qary, "scl": Scl, "stub": Stub}


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(a, argv):
    """--gpus N > 1 outside torch.distributed.run: start the N ranks as one child
    torch.distributed.run process (this process has not touched the GPU and never does),
    pass its output through, return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(a.master_port or _free_port()),
           os.path.abspath(__file__)] + argv
    log("bench: launching %d ranks: %s" % (a.gpus, " ".join(cmd)))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def build_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="awgn")
    ap.add_argument("--n", type=int, default=None, help="log2 code length (default: awgn 10, deletion / qary 8)")
    ap.add_argument("--rate", type=float, default=0.5)
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--n0", type=int, default=None, help="deletion: log2 inputs per trellis (default n // 3)")
    ap.add_argument("--ones", type=int, default=0, help="deletion: guard-band ones (numberOfOnesToAddAtBothEndsOfGuardbands)")
    ap.add_argument("--del-k", type=int, default=0, help="deletion: information bits (0 = the configuration's frozen set)")
    ap.add_argument("--del-lanes", type=int, default=0, help="deletion: lanes a codeword of the table-driven layout (0 = the library's)")
    ap.add_argument("--del-rate1", type=int, default=-1,
                    help="deletion: 0 = the 8-lane subtrees without the rate-1 shortcut (diagnostic A/B; -1 = the library's)")
    ap.add_argument("--del-wave", type=int, default=-1,
                    help="deletion n0 = 4: 0 = the lane-per-trellis kernel instead of the wave-per-task one (A/B; -1 = the library's)")
    ap.add_argument("--pd", type=float, default=0.1, help="deletion probability")
    ap.add_argument("--xi", type=float, default=0.1, help="guard-band parameter")
    ap.add_argument("--q", type=int, default=4)
    ap.add_argument("--list-size", type=int, default=8, help="scl: maxListSize")
    ap.add_argument("--qsc-p", type=float, default=0.11)
    ap.add_argument("--qlanes", type=int, default=0, help="q-ary: lanes per codeword (0 = the library's)")
    ap.add_argument("--qregs", type=int, default=0, help="q-ary: cap on register positions per lane (0 = the library's)")
    ap.add_argument("--qlds", type=int, default=None, help="q-ary: re-encoded symbols in LDS (1) or in the workspace (0)")
    ap.add_argument("--batch", type=int, default=1 << 20, help="codewords per GPU")
    ap.add_argument("--variant", type=int, default=None, help="binary decode kernel variant (default: the library's)")
    ap.add_argument("--max-blocks", type=int, default=0, help="cap decode workgroups per CU (0 = occupancy)")
    ap.add_argument("--seed", type=int, default=20250204)
    ap.add_argument("--master-port", type=int, default=0, help="rendezvous port when launching ranks (0 = free port)")
    ap.add_argument("--static-tiles", action="store_true",
                    help="decode kernels stride over their tiles statically instead of taking them from a counter (A/B)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-xhat", action="store_true")
    ap.add_argument("--no-tile", action="store_true", help="awgn: root rows [N][B][2] instead of the kernel's tiles")
    ap.add_argument("--e2e-chunk", type=int, default=1 << 18,
                    help="codewords per chunk of the end-to-end Monte-Carlo line")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end Monte-Carlo leg (profiling: only the timed decode launches)")
    return ap


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = build_parser()
    a = ap.parse_args(argv)

    world, rank, local = mc.dist_env()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(a, argv)
    if world != a.gpus and world > 1:
        log("bench: WORLD_SIZE=%d differs from --gpus %d; reporting the launched world" % (world, a.gpus))
    on_gpu = a.workload != "stub"
    shared = False
    if on_gpu:
        ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
        # more ranks than GPUs (a rehearsal of the multi-rank path on a smaller box): ranks share
        # devices round-robin and the counters go over gloo (RCCL wants one GPU per rank)
        shared = world > 1 and int(os.environ.get("LOCAL_WORLD_SIZE", world)) > ndev  # same on every rank
        device = torch.device("cuda", (local % max(1, ndev)) if world > 1 else 0)
        torch.cuda.set_device(device)
        if a.static_tiles:
            sc.set_dynamic_tiles(0)
        if world > 1 and not shared:
            dist.init_process_group("nccl", device_id=device)
        elif world > 1:
            dist.init_process_group("gloo")
            log("rank %d: %d ranks on %d GPU(s): device cuda:%d shared, counters over gloo" % (rank, world, ndev,
                                                                                         device.index))
        sync = torch.cuda.synchronize
    else:
        device = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")

        def sync():
            pass
    coll_dev = device if (on_gpu and world > 1 and not shared) else None

    t0 = time.time()
    w = WORKLOADS[a.workload](a, device, rank)
    sync()
    log("rank %d: %s inputs for %d codewords generated in %.1f s" % (rank, a.workload, w.B, time.time() - t0))

    # a slow step (deletion at n >= 12) logs progress per step, so a long run is visibly alive;
    # the per-step sync this adds is microseconds against tens of seconds
    slow = False
    for i in range(a.warmup):
        tw = time.perf_counter()
        w.step()
        sync()
        dt = time.perf_counter() - tw
        slow = slow or dt > 20.0
        if slow:
            log("rank %d: warmup step %d/%d %.1f s" % (rank, i + 1, a.warmup, dt))
    if world > 1:
        dist.barrier()
    sync()

    evs = None
    if on_gpu:
        stream = torch.cuda.current_stream()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t_start = time.perf_counter()
    for i in range(a.steps):
        if evs:
            evs[i][0].record(stream)
        w.step()
        if evs:
            evs[i][1].record(stream)
        if slow:
            sync()
            log("rank %d: step %d/%d done at %.1f s" % (rank, i + 1, a.steps, time.perf_counter() - t_start))
    sync()
    t_local = time.perf_counter() - t_start  # this rank's own decode time
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t_start
    kern_ms = [x.elapsed_time(y) for x, y in evs] if evs else [t_local * 1e3 / max(1, a.steps)]

    fe, be = w.errors()  # of the last decode (identical every step)
    counters, elapsed = mc.reduce_counters([w.B, fe, be, 0], elapsed, coll_dev)
    per_rank = mc.gather_floats([t_local, float(np.mean(kern_ms)), w.B], coll_dev)
    total_cw = counters[0] * a.steps
    value = total_cw / elapsed
    e2e = None
    if hasattr(w, "end_to_end") and not a.no_e2e:
        if world > 1:
            dist.barrier()
        _, e2e_s = mc.reduce_counters([0], w.end_to_end(), coll_dev)
        e2e = counters[0] / e2e_s
        # spread of the runs (rank 0's own times at N > 1)
        e2e_spread = [counters[0] / max(w.e2e_times) * (e2e_s / float(np.median(w.e2e_times))),
                      counters[0] / min(w.e2e_times) * (e2e_s / float(np.median(w.e2e_times)))]

    if rank == 0:
        avg_kern_s = float(np.mean(kern_ms)) / 1e3
        b_alg = w.bytes_alg()
        achieved = b_alg * w.B / avg_kern_s / 1e9
        traffic, traffic_src = measured_traffic(w.tag(), w.B)
        d = w.describe(world)
        rec = {
            "metric": d["metric"],
            "value": value,
            "unit": "codewords/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": d["dtype"],
            "data": d["data"],
            "config": d["config"],
            "fer": counters[1] / counters[0],
            "frame_errors": counters[1],
            "bit_errors": counters[2],
            "codewords_per_step": counters[0],
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": w.kernel, "kernel_ms": float(np.mean(kern_ms)), "bytes_alg_per_cw": b_alg},
            "per_rank": [{"rank": r, "codewords": int(v[2]), "value": v[2] * a.steps / v[0],
                          "kernel_ms": v[1], "hbm_frac": b_alg * v[2] / (v[1] / 1e3) / 1e9 / HBM_PEAK_GBS}
                         for r, v in enumerate(per_rank)],
        }
        if e2e is not None:
            rec["mc_end_to_end"] = {"value": e2e, "unit": "codewords/s",
                                    "what": "pcub_mc_run_bin: info bits + encode + channel + decode + counters, "
                                            "all on device, same codewords; chunks of %d back to back, median of "
                                            "%d warm runs" % (min(w.B, a.e2e_chunk), len(w.e2e_times)),
                                    "min": e2e_spread[0], "max": e2e_spread[1]}
        if world == 1 and not a.no_cpu and hasattr(w, "cpu_baseline"):
            rec["cpu_baseline"] = w.cpu_baseline()
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
