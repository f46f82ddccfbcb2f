#!/usr/bin/env python
"""r06: can a slow arena placement be told at allocation time?  For each of ARENAS contiguous
metric-size arenas (allocated one after another, all kept): right after the allocation, 3 x (read
probe, metric kernel) interleaved, the ratio of their medians; then, after every arena exists, the
steady metric kernel time of each (median of 3 x 5, interleaved).  Prints one JSON line."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from fedml_amd.engine import MUL_W, get_engine
    eng = get_engine(0)
    K, P, E = 128, 125_000_000, 1024
    nt = -(-P // E)
    n = int(os.environ.get("ARENAS", "3"))
    rng = np.random.RandomState(7)
    counts = [int(v) for v in rng.randint(50, 601, size=K)]
    w = [c / sum(counts) for c in counts]
    out = torch.empty(P, device="cuda")
    st = torch.cuda.current_stream()

    def ev_ms(fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        b.synchronize()
        return a.elapsed_time(b)

    arenas, res = [], []
    for i in range(n):
        raw = eng.alloc_contiguous(nt * K * E * 4)
        buf = raw.view(torch.float32).view(nt, K, E)
        buf.fill_(1.0)
        torch.cuda.synchronize()
        kern = lambda b=buf: eng.weighted_sum_tiled(b, list(range(K)), MUL_W, w, n=P, out=out)  # noqa: E731
        probe = lambda b=buf: eng.read_probe(b, K)  # noqa: E731
        pm, km = [], []
        for _ in range(3):
            pm.append(ev_ms(probe))
            km.append(ev_ms(kern))
        arenas.append((buf, kern))
        res.append({"quick_probe_ms": round(float(np.median(pm)), 3), "quick_kernel_ms": round(float(np.median(km)), 3),
                    "quick_ratio": round(float(np.median(km) / np.median(pm)), 4)})
    t = time.perf_counter()
    while time.perf_counter() - t < 1.0:
        arenas[0][1]()
    torch.cuda.synchronize()
    steady = [[] for _ in arenas]
    for _ in range(3):
        for i, (_, kern) in enumerate(arenas):
            steady[i] += [ev_ms(kern) for _ in range(5)]
    for i in range(n):
        res[i]["steady_kernel_ms"] = round(float(np.median(steady[i])), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
