#!/usr/bin/env python
"""r06: the counters of the metric's slow arena (r06n: of two arenas in one process, one runs 9.7-9.8
ms and the other 9.38-9.42, alternating between processes).  Two tiled arenas A, B and one output;
~0.5 s of warm launches on A, then A x 6, B x 6, A x 6, B x 6 (HIP-event timed), for a rocprofv3 --pmc
pass to split by dispatch.  Prints one JSON line: the 24 launches' arena and ms, in dispatch order."""
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
    rng = np.random.RandomState(7)
    counts = [int(v) for v in rng.randint(50, 601, size=K)]
    w = [c / sum(counts) for c in counts]
    arenas = {}
    for a in "AB":
        arenas[a] = torch.empty((nt, K, E), device="cuda")
        arenas[a].fill_(1.0)
    out = torch.empty(P, device="cuda")
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    kern = lambda b: eng.weighted_sum_tiled(b, list(range(K)), MUL_W, w, n=P, out=out)  # noqa: E731
    nwarm = 0
    t = time.perf_counter()
    while time.perf_counter() - t < 0.5:
        kern(arenas["A"])
        torch.cuda.synchronize()
        nwarm += 1
    seq = []
    for a in "ABAB":
        for _ in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            kern(arenas[a])
            e1.record(st)
            e1.synchronize()
            seq.append((a, round(e0.elapsed_time(e1), 3)))
    print(json.dumps({"warm": nwarm, "seq": seq,
                      "median": {a: float(np.median([m for x, m in seq if x == a])) for a in "AB"}}), flush=True)


if __name__ == "__main__":
    main()
