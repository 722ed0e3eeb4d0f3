#!/usr/bin/env python3
"""Copy one gpu_check.sh run's rocprofv3 outputs into profiles/<round>/<tag>/ and
summarise the decode kernel's per-launch HBM traffic.

    python scripts/collect_profiles.py --round r1 --tag bin_v17_n10 [--src gpurun_out]
          [--kernel k_sc_bin] [--batch 1048576] [--n 10] [--variant 17]

Traffic (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half of the bytes of a wide (16 B/lane) coalesced read,
so it is doubled; WRITE_SIZE is exact for 16 B/lane stores.  The summary keeps both
the raw and the corrected figures.  Only rows of the named kernel are kept.
"""
import argparse
import csv
import json
import os
import shutil


def rows(path, kernel):
    with open(path) as f:
        return [r for r in csv.DictReader(f) if kernel in r["Kernel_Name"]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r1")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--src", default="gpurun_out")
    ap.add_argument("--kernel", default="k_sc_bin")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--variant", type=int, default=None)
    ap.add_argument("--bench", default=None, help="bench JSON line to keep beside the profile")
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, a.src)
    dst = os.path.join(root, "profiles", a.round, a.tag)
    os.makedirs(dst, exist_ok=True)
    summ = {"kernel": a.kernel, "batch": a.batch, "n": a.n, "variant": a.variant}

    stats = os.path.join(src, "prof", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
        with open(stats) as f:
            for r in csv.DictReader(f):
                if a.kernel in r["Name"]:
                    summ["trace_calls"] = int(r["Calls"])
                    summ["trace_avg_ms"] = float(r["AverageNs"]) / 1e6
                    summ["trace_kernel_name"] = r["Name"]
    counters = {}
    for d in sorted(os.listdir(src)):
        p = os.path.join(src, d, "pmc_counter_collection.csv")
        if not d.startswith("pmc_") or not os.path.exists(p):
            continue
        rs = rows(p, a.kernel)
        if not rs:
            continue
        with open(os.path.join(dst, d + ".csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rs[0].keys()))
            w.writeheader()
            w.writerows(rs)
        for r in rs:
            counters.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
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
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        summ["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if a.bench and os.path.exists(os.path.join(root, a.bench)):
        shutil.copy(os.path.join(root, a.bench), os.path.join(dst, "bench.json"))
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(summ, f, indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
