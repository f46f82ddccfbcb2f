#!/usr/bin/env python
"""Summarise a tools/profile.sh run into profiles/ (kernel stats + PMC HBM traffic per launch).

HBM bytes per launch of the dominant kernel (name contains KERNEL, default "k_wsum"):
    read  = 2 * FETCH_SIZE * 1024   (gfx950 FETCH_SIZE reports half the bytes of a wide coalesced
                                     streaming read: MI355X_MICROARCH.md §HBM)
    write = WRITE_SIZE * 1024       (exact for 16-B-per-lane streaming stores)
FETCH_SIZE and WRITE_SIZE come from separate --pmc passes (TCC counter slots).
"""
from __future__ import annotations

import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = os.environ.get("KERNEL", "k_wsum")


def find(d, pattern):
    return sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))


def counter_values(d, counter, name):
    """Counter values of every dispatch of the kernel `name` (exact match)."""
    vals = []
    for f in find(d, "*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Kernel_Name", "") == name and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main(out_dir, tag, dest=None):
    prof = dest or os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    summary = {"tag": tag, "kernel_filter": KERNEL}
    stats = find(os.path.join(out_dir, "trace"), "*kernel_stats.csv")
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
        with open(stats[0]) as fh:
            rows = [r for r in csv.DictReader(fh) if KERNEL in r["Name"]]
        if rows:  # the dominant kernel = largest total duration among the engine's kernels
            row = max(rows, key=lambda r: float(r["TotalDurationNs"]))
            summary["kernel"] = row["Name"]
            summary["calls"] = int(row["Calls"])
            summary["avg_ns"] = float(row["AverageNs"])
            summary["min_ns"] = float(row["MinNs"])
            summary["max_ns"] = float(row["MaxNs"])
    try:
        with open(os.path.join(out_dir, "trace_bench.json")) as fh:
            bench = json.loads(fh.read().strip().splitlines()[-1])
        summary["bench_line"] = bench
        workload = bench["config"]["workload"]
        algo = bench["roofline"]["algorithmic_bytes_per_launch"]
    except Exception as e:  # noqa: BLE001
        print("no bench line:", e)
        workload, algo = "unknown", None
    name = summary.get("kernel", "")
    fetch = counter_values(os.path.join(out_dir, "fetch"), "FETCH_SIZE", name)
    write = counter_values(os.path.join(out_dir, "write"), "WRITE_SIZE", name)
    if fetch:
        summary["fetch_size_kb_median"] = statistics.median(fetch)
        summary["fetch_dispatches"] = len(fetch)
    if write:
        summary["write_size_kb_median"] = statistics.median(write)
        summary["write_dispatches"] = len(write)
    if fetch and write:
        rd = 2.0 * statistics.median(fetch) * 1024
        wr = statistics.median(write) * 1024
        summary["hbm_read_bytes_per_launch"] = rd
        summary["hbm_write_bytes_per_launch"] = wr
        summary["hbm_bytes_per_launch"] = rd + wr
        if algo:
            summary["traffic_over_algorithmic"] = (rd + wr) / algo
        if summary.get("avg_ns"):
            summary["hbm_gbs_from_counters"] = (rd + wr) / summary["avg_ns"]
    with open(os.path.join(prof, f"{tag}_pmc_summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    tp = os.path.join(prof, "pmc_traffic.json")
    try:
        with open(tp) as fh:
            allw = json.load(fh)
    except (OSError, ValueError):
        allw = {}
    if "hbm_bytes_per_launch" in summary:
        allw[workload] = {"hbm_bytes_per_launch": int(summary["hbm_bytes_per_launch"]),
                          "source": f"profiles/{tag}_pmc_summary.json",
                          "avg_kernel_ns": summary.get("avg_ns"),
                          "traffic_over_algorithmic": summary.get("traffic_over_algorithmic")}
        with open(tp, "w") as fh:
            json.dump(allw, fh, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "bench_line"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "r01", sys.argv[3] if len(sys.argv) > 3 else None)
