#!/usr/bin/env python
"""r06: is the metric's slow mode (9.80 vs 9.42 ms) a property of the arena, of the output, or of
the pair?  One process, two tiled arenas A and B of the metric's size and NOUT outputs (each behind a
spacer allocation), every (arena, output) pair timed, interleaved over 4 rounds (median of 4 x 5
HIP-event-timed launches).  Prints one JSON line: {arena: {output: ms}}."""
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
    arenas = {}
    for a in "AB":
        arenas[a] = torch.empty((nt, K, E), device="cuda")
        arenas[a].fill_(1.0)
    outs, spacers = {}, []
    for i in range(nout):
        outs[f"o{i}"] = torch.empty(P, device="cuda")
        spacers.append(torch.empty((i + 1) * (257 << 20), dtype=torch.uint8, device="cuda"))
    torch.cuda.synchronize()
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

    kern = lambda b, o: eng.weighted_sum_tiled(b, list(range(K)), MUL_W, w, n=P, out=o)  # noqa: E731
    t = time.perf_counter()
    while time.perf_counter() - t < 1.0:
        kern(arenas["A"], outs["o0"])
    torch.cuda.synchronize()
    km = {(a, o): [] for a in arenas for o in outs}
    for _ in range(4):
        for (a, o) in km:
            km[(a, o)] += timed(lambda: kern(arenas[a], outs[o]), 5)
    res = {a: {o: round(float(np.median(km[(a, o)])), 3) for o in outs} for a in arenas}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
