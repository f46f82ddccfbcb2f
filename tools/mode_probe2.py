#!/usr/bin/env python
"""r06: the metric's process-level modes (r06k: 9.54 vs 9.70 ms per step in fresh processes on one box,
the gfx clock (2.31-2.32 GHz), memory clock and the read probe over the same pages all equal).  In ONE
process: one tiled arena of the metric's size, the read probe over it, and the metric kernel writing
into each of NOUT output buffers allocated at different points (right after the arena, behind a
spacer allocation, ...: each its own hipMalloc, so its own physical pages), interleaved over 4 rounds.
If the outputs differ within a process as much as processes differ, the mode is the output's
placement; if not, it is process-wide.  Prints one JSON line."""
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
    nout = int(os.environ.get("NOUT", "4"))
    nt = -(-P // E)
    rng = np.random.RandomState(7)
    counts = [int(v) for v in rng.randint(50, 601, size=K)]
    w = [c / sum(counts) for c in counts]
    buf = torch.empty((nt, K, E), device="cuda")
    buf.fill_(1.0)
    outs, spacers = [], []
    for i in range(nout):
        outs.append(torch.empty(P, device="cuda"))
        spacers.append(torch.empty((i + 1) * (257 << 20), dtype=torch.uint8, device="cuda"))
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    nbytes = K * P * 4 + P * 4

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

    kern = lambda o: eng.weighted_sum_tiled(buf, list(range(K)), MUL_W, w, n=P, out=o)  # noqa: E731
    t = time.perf_counter()
    while time.perf_counter() - t < 1.0:
        kern(outs[0])
    torch.cuda.synchronize()
    km = {i: [] for i in range(nout)}
    pm = []
    for _ in range(4):
        for i in range(nout):
            km[i] += timed(lambda: kern(outs[i]), 5)
        pm += timed(lambda: eng.read_probe(buf, K), 2)
    res = {"outs": {i: {"ms_med": round(float(np.median(v)), 4), "ms_min": round(min(v), 4),
                        "GBs_med": round(nbytes / (np.median(v) * 1e-3) / 1e9, 1), "ptr": hex(outs[i].data_ptr())}
                    for i, v in km.items()},
           "probe_GBs_best": round(K * nt * 4096 / (min(pm) * 1e-3) / 1e9, 1), "arena_ptr": hex(buf.data_ptr())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
