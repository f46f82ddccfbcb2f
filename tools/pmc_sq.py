"""Summarise a rocprofv3 --pmc CSV of SQ counters: per-dispatch sums averaged over dispatches of
the kernels matching a name filter, as fractions of SQ_WAVE_CYCLES."""
import collections
import csv
import sys


def summary(path, name_filter="k_pairdist"):  # every kernel whose name contains the filter
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if name_filter in r["Kernel_Name"]:
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    m = {c: sum(d.values()) / len(d) for c, d in per.items()}
    out = {c: round(v, 1) for c, v in m.items()}
    w = m.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if c in m:
                out[c + "_frac"] = round(m[c] / w, 3)
    if m.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_conflict_frac"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"], 3)
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p, summary(p))
