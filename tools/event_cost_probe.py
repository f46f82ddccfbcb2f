#!/usr/bin/env python
"""r05: what the bench's per-step timing events cost.  cfg2 (ResNet-18-GN state_dict, K = 32) on
separate tensors and on the tiled arena, and the Krum K = 32 pairwise pass: N steps back to back
timed (a) by one event pair around all N (no event between steps) and (b) with an event pair around
every step as bench.py's Timed does.  Prints one JSON line per workload: ms per step both ways."""
from __future__ import annotations

import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, n, per_step):
    ev = []
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        if per_step:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        fn()
        if per_step:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            ev.append((e0, e1))
    b.record()
    torch.cuda.synchronize()
    inner = sum(x.elapsed_time(y) for x, y in ev) / n if ev else None
    return a.elapsed_time(b) / n, inner


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
    forms = {"cfg2_tensors": lambda: aggregate(dicts, MUL_W, w), "cfg2_tiled": lambda: arena.aggregate(MUL_W, w),
             "krum_K32": lambda: eng.pairwise_sqdist([xs])}
    n = int(os.environ.get("N", "50"))
    for name, fn in forms.items():
        for _ in range(5):
            fn()
        res = {"workload": name, "steps": n}
        for rep in range(3):
            whole, _ = timed(fn, n, False)
            outer, inner = timed(fn, n, True)
            res.setdefault("no_step_events_ms", []).append(round(whole, 4))
            res.setdefault("step_events_outer_ms", []).append(round(outer, 4))
            res.setdefault("step_events_inner_ms", []).append(round(inner, 4))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
