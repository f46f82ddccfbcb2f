#!/usr/bin/env python
"""Summarise the r05b / r05c address-translation counter passes (rocprofv3 --pmc CSVs) of the metric
kernel per input layout: UTCL1 misses / hits per request, the share of the kernel the UTCL2 was busy,
kernel durations.  python tools/translation_summary.py > profiles/r05b/translation_summary.json"""
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(paths):
    med, dur = {}, collections.defaultdict(float)
    for p in paths:
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(p)):
            per[r["Counter_Name"]][r["Dispatch_Id"]] = float(r["Counter_Value"])
            dur[(p, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            kern = r["Kernel_Name"]
        for c, d in per.items():
            v = sorted(d.values())
            med[c] = v[len(v) // 2]
    ds = sorted(dur.values())
    out = {"kernel": kern[:70], "kernel_ms_median": round(ds[len(ds) // 2], 4)}
    req = med.get("TCP_UTCL1_REQUEST_sum")
    if req:
        out["utcl1_requests"] = req
        for c, k in (("TCP_UTCL1_TRANSLATION_MISS_sum", "utcl1_miss_per_request"),
                     ("TCP_UTCL1_TRANSLATION_HIT_sum", "utcl1_hit_per_request"),
                     ("TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum", "utcl1_miss_under_miss_per_request")):
            if c in med:
                out[k] = round(med[c] / req, 5)
        out["utcl1_misses"] = med.get("TCP_UTCL1_TRANSLATION_MISS_sum")
    if med.get("GRBM_GUI_ACTIVE"):
        out["utcl2_busy_frac"] = round(med["GRBM_UTCL2_BUSY"] / med["GRBM_GUI_ACTIVE"], 4)
    for c in ("TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum"):
        if c in med:
            out[c] = med[c]
    return out


res = {}
for lay in ("tiled", "arena", "tensors"):
    res[f"{lay} (r05b, default kernel U8 S1)"] = load(sorted(glob.glob(os.path.join(ROOT, "profiles/r05b/pmc", f"{lay}_pass*_counters.csv"))))
for v, what in ((5, "U8 S2"), (6, "U4 S4")):
    res[f"tensors (r05c, variant {v}: {what})"] = load([os.path.join(ROOT, "profiles/r05c/pmc", f"tensors_v{v}_counters.csv")])
res["tensors (r05e, XCD-contiguous tiles, U8 S1)"] = load([os.path.join(ROOT, "profiles/r05e/pmc", "tensors_xcd_counters.csv")])
print(json.dumps(res, indent=1))
