#!/usr/bin/env python
"""Tool: weighted-sum kernel variants on one rank's N = 8 local step (K = 16 x 125 M, tiled)."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_tiled_arena  # noqa: E402
from fedml_amd.engine import MUL_W, get_engine  # noqa: E402
eng = get_engine(0)
K, P = int(os.environ.get("K", 16)), 125_000_000
arena = make_tiled_arena(range(K), P)
buf, rows, w = arena.bufs[torch.float32], list(range(K)), [1.0 / K] * K
out = torch.empty(P, device="cuda")
res = {}
for rep in range(2):
    for v in (0, 1, 2, 4, 5, 6, 7, 8):
        eng.set_variant(v)
        for _ in range(2): eng.weighted_sum_tiled(buf, rows, MUL_W, w, n=P, out=out)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10): eng.weighted_sum_tiled(buf, rows, MUL_W, w, n=P, out=out)
        b.record(); b.synchronize()
        res.setdefault(f"v{v}", []).append(round(a.elapsed_time(b) / 10, 3))
eng.set_variant(0)
print(json.dumps(res))
