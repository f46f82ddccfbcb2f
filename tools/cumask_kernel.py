#!/usr/bin/env python
"""Tool: the metric kernel (tiled arena, K=128 x 125M fp32) on CU-masked streams vs the default stream."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_tiled_arena, client_counts  # noqa: E402
from fedml_amd.engine import MUL_W, get_engine  # noqa: E402
eng = get_engine(0)
K, P = 128, 125_000_000
arena = make_tiled_arena(range(K), P)
buf, rows = arena.bufs[torch.float32], list(range(K))
c = client_counts(K); w = [x / sum(c) for x in c]
out = torch.empty(P, device="cuda")
res = {}
for ncu in (0, 224, 192, 160, 128, 0):
    st = eng.cu_masked_stream(ncu) if ncu else torch.cuda.current_stream()
    st.wait_stream(torch.cuda.current_stream())
    ts = []
    with torch.cuda.stream(st):
        for _ in range(6):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st); eng.weighted_sum_tiled(buf, rows, MUL_W, w, n=P, out=out); b.record(st)
            b.synchronize(); ts.append(a.elapsed_time(b))
    ms = sorted(ts[1:])[len(ts[1:]) // 2]
    res.setdefault(f"cu{ncu or 'all'}_ms", []).append(round(ms, 3))
print(json.dumps(res))
