#!/usr/bin/env python
"""r06: the headline's two modes (9.39 vs 10.03 ms per step on one box with one
binary, each mode lasting a whole process).  In ONE process: tiled arenas A and B of the metric's
size (K = 128 x P = 125 M fp32, 64.5 GB each) allocated one after the other; for each, the metric
kernel (fa_weighted_sum_tiled, HIP-event timed, 10 launches) and the read probe over the same pages
(fa_read_probe, K rows per workgroup) -- then A again.  If the two arenas of one process differ, the
mode lives in the physical placement of the allocation (translation / channel interleave); if both
match and only processes differ, it lives in process-wide state.  Prints one JSON line.
"""
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
    K = int(os.environ.get("K", "128"))
    P = int(os.environ.get("P", "125000000"))
    narenas = int(os.environ.get("ARENAS", "2"))
    E = 1024
    nt = -(-P // E)
    rng = np.random.RandomState(7)
    counts = [int(v) for v in rng.randint(50, 601, size=K)]
    w = [c / sum(counts) for c in counts]
    out = torch.empty(P, device="cuda")
    nbytes = K * P * 4 + P * 4
    st = torch.cuda.current_stream()

    def timed(fn, reps):
        ms = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            fn()
            b.record(st)
            b.synchronize()
            ms.append(a.elapsed_time(b))
        return ms

    arenas, res = [], {}

    def measure(tag, buf):
        kern = lambda: eng.weighted_sum_tiled(buf, list(range(K)), MUL_W, w, n=P, out=out)  # noqa: E731
        probe = lambda: eng.read_probe(buf, K)  # noqa: E731
        for _ in range(3):
            kern()
        torch.cuda.synchronize()
        # warm the clock for ~0.3 s, then interleave kernel and probe
        t = time.perf_counter()
        while time.perf_counter() - t < 0.3:
            kern()
            torch.cuda.synchronize()
        km, pm = [], []
        for _ in range(3):
            km += timed(kern, 4)
            pm += timed(probe, 2)
        res[tag] = {"kernel_ms_min": round(min(km), 4), "kernel_ms_med": round(float(np.median(km)), 4),
                    "kernel_GBs_med": round(nbytes / (np.median(km) * 1e-3) / 1e9, 1),
                    "probe_ms_min": round(min(pm), 4), "probe_GBs_best": round(K * nt * 4096 / (min(pm) * 1e-3) / 1e9, 1),
                    "base_hex": hex(buf.data_ptr())}
        print(tag, res[tag], file=sys.stderr, flush=True)

    for a in range(narenas):
        buf = torch.empty((nt, K, E), device="cuda")
        buf.fill_(1.0)
        torch.cuda.synchronize()
        arenas.append(buf)
        measure(f"arena{a}", buf)
    measure("arena0_again", arenas[0])
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
