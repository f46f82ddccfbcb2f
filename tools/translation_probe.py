#!/usr/bin/env python
"""r05: the literal-input metric (128 separately allocated fp32[125 M] client buffers) is address-
translation bound (profiles/r05b: UTCL2 busy 96 % of the kernel vs 4 % on the tiled arena; S = 4
slots per client cut UTCL1 misses 8x but left UTCL2 busy at 74 % and the time at -2 %, profiles/r05c).
Hypothesis: the concurrent translation working set (every client's current window) exceeds what the
UTCL2 holds.  Test: the same ordered FedAvg in client passes -- pass 1 clients [0, K/p), pass j adds
the next K/p clients to the running partial (the partial re-enters as client 0 with coefficient 1.0,
exact: fp32(p) * 1.0 = p and -0 + p = p) -- halving / quartering the clients in flight for one extra
read + write of the model per extra pass.  Prints one JSON line: per-form best/median ms over
interleaved reps, bit-equality of every form with the one-pass result.
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
    layout = os.environ.get("LAYOUT", "tensors")
    rng = np.random.RandomState(7)
    counts = [int(v) for v in rng.randint(50, 601, size=K)]
    N = sum(counts)
    w = [c / N for c in counts]
    if layout == "tensors":
        xs = []
        for i in range(K):
            g = torch.Generator(device="cuda").manual_seed(1000 + i)
            xs.append(torch.randn(P, generator=g, device="cuda"))
    else:  # client-major rows of one allocation
        big = torch.empty(K, P, device="cuda")
        for i in range(K):
            g = torch.Generator(device="cuda").manual_seed(1000 + i)
            big[i].copy_(torch.randn(P, generator=g, device="cuda"))
        xs = list(big)
    out = torch.empty(P, device="cuda")
    part = torch.empty(P, device="cuda")
    part2 = torch.empty(P, device="cuda")

    def passes(p):
        per = K // p
        def run():
            eng.weighted_sum(xs[:per], MUL_W, w[:per], out=part if p > 1 else out)
            src, dst = part, part2
            for j in range(1, p):
                tgt = out if j == p - 1 else dst
                eng.weighted_sum([src] + xs[j * per:(j + 1) * per], MUL_W, [1.0] + w[j * per:(j + 1) * per], out=tgt)
                src, dst = tgt, src
        return run

    forms = {f"{p}pass": passes(p) for p in (1, 2, 4)}
    res = {k: [] for k in forms}
    ref = None
    for rep in range(int(os.environ.get("REPS", "4"))):
        for name, fn in forms.items():
            fn()
            torch.cuda.synchronize()
            if rep == 0:
                if name == "1pass":
                    ref = out.clone()
                else:
                    res.setdefault(name + "_bitexact", torch.equal(out.view(torch.int32), ref.view(torch.int32)))
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                fn()
            b.record()
            torch.cuda.synchronize()
            res[name].append(a.elapsed_time(b) / 5)
    line = {"probe": "translation passes", "layout": layout, "K": K, "P": P}
    for name in forms:
        v = res[name]
        line[name] = {"best_ms": round(min(v), 4), "median_ms": round(float(np.median(v)), 4),
                      "all_ms": [round(x, 4) for x in v]}
    line.update({k: v for k, v in res.items() if k.endswith("_bitexact")})
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
