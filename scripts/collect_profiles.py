#!/usr/bin/env python3
"""Copy one profiling run's rocprofv3 outputs into profiles/<round>/<tag>/ and summarise the
named kernel per launch.

    python scripts/collect_profiles.py --round r2 --tag bin_n10 --kernel k_sc_bin --batch 1048576
          [--src gpurun_out/<tag>] [--grid G] [--bench gpurun_out/bench.json]

Layout read (scripts/prof_passes.sh): <src>/trace/run_kernel_trace.csv (+ _stats.csv) and
<src>/pmc*/pmc_counter_collection.csv (older runs: <src>/prof/, <src>/pmc_*/).

Only launches of the profiled configuration count: rows of the named kernel whose
Grid_Size equals --grid, or, by default, the grid size of the kernel's most frequent
launch shape in the trace (the bench/profile step repeats one launch; other launches of
the same kernel at other batch sizes -- input generation, tails -- are excluded, so
`trace_avg_ms` is the per-launch duration at the stated batch).

Traffic (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half of the bytes of a wide (16 B/lane) coalesced read, so it is doubled;
WRITE_SIZE is exact for 16 B/lane stores.  The summary keeps raw and corrected figures.
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil


def read_csv(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def grid_of(r):
    """Grid size in work-items (kernel trace: Grid_Size_X*Y*Z; PMC rows: Grid_Size)."""
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)


def wg_of(r):
    if "Workgroup_Size" in r:
        return int(r["Workgroup_Size"])
    return int(r["Workgroup_Size_X"]) * int(r.get("Workgroup_Size_Y", 1) or 1) * int(r.get("Workgroup_Size_Z", 1) or 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r2")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--src", default=None)
    ap.add_argument("--kernel", default="k_sc_bin")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--bench", default=None, help="bench JSON line to keep beside the profile")
    ap.add_argument("--note", default=None)
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, a.src or os.path.join("gpurun_out", a.tag))
    dst = os.path.join(root, "profiles", a.round, a.tag)
    os.makedirs(dst, exist_ok=True)
    summ = {"kernel": a.kernel, "batch": a.batch}
    if a.note:
        summ["note"] = a.note

    traces = glob.glob(os.path.join(src, "trace", "*kernel_trace.csv")) + glob.glob(
        os.path.join(src, "prof", "*kernel_trace.csv"))
    grid = a.grid
    if traces:
        rows = [r for r in read_csv(traces[0]) if a.kernel in r["Kernel_Name"]]
        if grid is None and rows:
            grid = collections.Counter(grid_of(r) for r in rows).most_common(1)[0][0]
        sel = [r for r in rows if grid_of(r) == grid]
        with open(os.path.join(dst, "kernel_trace.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()) if rows else ["none"])
            w.writeheader()
            w.writerows(rows)
        if sel:
            durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in sel]
            summ.update(trace_calls=len(sel), trace_avg_ms=sum(durs) / len(durs), trace_min_ms=min(durs),
                        trace_max_ms=max(durs), trace_kernel_name=sel[0]["Kernel_Name"], grid_size=grid,
                        workgroup_size=wg_of(sel[0]), vgpr=int(sel[0].get("VGPR_Count", 0) or 0),
                        sgpr=int(sel[0].get("SGPR_Count", 0) or 0),
                        scratch_bytes_per_lane=int(sel[0].get("Scratch_Size", 0) or 0),
                        lds_bytes=int(sel[0].get("LDS_Block_Size", 0) or 0),
                        other_launches_excluded=len(rows) - len(sel))
    for st in glob.glob(os.path.join(src, "trace", "*kernel_stats.csv")) + glob.glob(
            os.path.join(src, "prof", "*kernel_stats.csv")):
        shutil.copy(st, os.path.join(dst, "kernel_stats.csv"))
    counters = {}
    pmc_dirs = sorted(glob.glob(os.path.join(src, "pmc*")))
    for d in pmc_dirs:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            rs = [r for r in read_csv(p) if a.kernel in r["Kernel_Name"]]
            if not rs:
                continue
            g = grid if grid is not None else collections.Counter(grid_of(r) for r in rs).most_common(1)[0][0]
            rs = [r for r in rs if grid_of(r) == g]
            with open(os.path.join(dst, os.path.basename(d) + ".csv"), "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=list(rs[0].keys()))
                w.writeheader()
                w.writerows(rs)
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in rs:  # one row per (dispatch, counter) after rocprofv3's per-dispatch aggregation
                per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            for k, v in per.items():
                counters.setdefault(k, []).extend(v.values())
    avg = {k: sum(v) / len(v) for k, v in counters.items()}
    summ["counters_per_launch"] = avg
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        fetch = avg["FETCH_SIZE"] * 1024 * 2  # KiB, x2 gfx950 wide-read correction
        write = avg["WRITE_SIZE"] * 1024
        summ["hbm_read_bytes"] = fetch
        summ["hbm_write_bytes"] = write
        summ["traffic_bytes"] = fetch + write
        summ["traffic_bytes_per_cw"] = (fetch + write) / a.batch
        summ["traffic_note"] = "FETCH_SIZE KiB x1024 x2 (gfx950 16B/lane read correction) + WRITE_SIZE KiB x1024, per launch"
        if "trace_avg_ms" in summ:
            summ["traffic_gbs"] = (fetch + write) / (summ["trace_avg_ms"] / 1e3) / 1e9
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        summ["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if "SQ_WAVE_CYCLES" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        summ["valu_active_per_wave_cycle"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        summ["valu_insts_per_wave"] = avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]
    summ["counters_per_codeword"] = {k: v / a.batch for k, v in avg.items()
                                     if k.startswith("SQ_INSTS") or k in ("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES")}
    if "GRBM_GUI_ACTIVE" in avg and "SQ_BUSY_CYCLES" not in avg:
        summ["gpu_active_cycles"] = avg["GRBM_GUI_ACTIVE"]
    if a.bench and os.path.exists(os.path.join(root, a.bench)):
        shutil.copy(os.path.join(root, a.bench), os.path.join(dst, "bench.json"))
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(summ, f, indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
