#!/usr/bin/env python
"""r05: host-side cost per call of the bench's small-step workloads.  For each: N calls issued back
to back with no synchronisation (host time per call = the issue loop's wall time / N), then the
same N calls' GPU time per call (events around the loop after a sync).  Host > GPU means the
workload is host-bound at that step size.  One JSON line per workload."""
from __future__ import annotations

import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from fedml_amd.arena import ArenaLayout, ClientArena
    from fedml_amd.engine import get_engine
    from fedml_amd.ml.aggregator.state_dict_agg import MUL_W, aggregate
    eng = get_engine(0)
    layout = bench.load_layout("resnet18_gn")
    K = 32
    counts = bench.client_counts(K)
    w = [c / sum(counts) for c in counts]
    dicts = bench.make_layout_clients(list(range(K)), layout)
    arena = ClientArena(ArenaLayout([(n, tuple(s), getattr(torch, dt)) for n, s, dt in layout]), capacity=K, tiled=True)
    for j, d in enumerate(dicts):
        arena.write(j, d)
    xs = bench._robust_inputs(32, bench.RESNET18_P)
    forms = {"krum_K32": lambda: eng.pairwise_sqdist([xs]),
             "median_K32": lambda: eng.coord_median([xs]) if hasattr(eng, "coord_median") else None,
             "cfg2_tensors": lambda: aggregate(dicts, MUL_W, w), "cfg2_tiled": lambda: arena.aggregate(MUL_W, w)}
    n = int(os.environ.get("N", "40"))
    for name, fn in forms.items():
        try:
            for _ in range(5):
                fn()
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"workload": name, "error": str(e)[:200]}), flush=True)
            continue
        res = {"workload": name, "calls": n}
        for rep in range(3):
            torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            t1 = time.perf_counter()
            b.record()
            torch.cuda.synchronize()
            res.setdefault("host_us_per_call", []).append(round((t1 - t0) / n * 1e6, 1))
            res.setdefault("gpu_us_per_call", []).append(round(a.elapsed_time(b) / n * 1e3, 1))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
