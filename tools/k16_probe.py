#!/usr/bin/env python
"""Tool: GPU time of one rank's N = 8 local step (K = 16 x 125 M, tiled) -- one launch vs chunked,
default vs CU-masked stream."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_tiled_arena  # noqa: E402
from fedml_amd.engine import MUL_W, get_engine  # noqa: E402
eng = get_engine(0)
K, P, E = 16, 125_000_000, 1024
arena = make_tiled_arena(range(K), P)
buf, rows, w = arena.bufs[torch.float32], list(range(K)), [1.0 / K] * K
out = torch.empty(P, device="cuda")
def bounds(c):
    units = -(-P // E)
    return [(min(P, units * i // c * E), min(P, units * (i + 1) // c * E)) for i in range(c)]
def run(c, st):
    for a, b in bounds(c):
        eng.weighted_sum_tiled(buf, rows, MUL_W, w, n=b - a, t0=a // E, out=out[a:b], stream=st)
res = {}
for name, st in (("default", torch.cuda.current_stream()), ("cu192", eng.cu_masked_stream(192)),
                 ("cu224", eng.cu_masked_stream(224))):
    st.wait_stream(torch.cuda.current_stream())
    for c in (1, 4, 8, 16):
        for _ in range(2): run(c, st)
        a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a_.record(st)
        for _ in range(10): run(c, st)
        b_.record(st); b_.synchronize()
        ms = a_.elapsed_time(b_) / 10
        res[f"{name}_chunks{c}_ms"] = round(ms, 3)
res["gbs_ideal_8.5GB_at_6.6TBs_ms"] = round((K + 1) * P * 4 / 6.6e12 * 1e3, 3)
print(json.dumps(res))
