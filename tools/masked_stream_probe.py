#!/usr/bin/env python
"""Tool: per-operation cost on a CU-masked stream vs torch's default stream: tiny engine launches
(each = a small pinned->device table copy + a kernel), bare small H2D copies, bare tiny kernels."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.engine import MUL_W, get_engine  # noqa: E402
eng = get_engine(0)
K, E = 16, 1024
buf = torch.zeros(64, K, E, device="cuda")
rows, w = list(range(K)), [1.0 / K] * K
out = torch.empty(64 * E, device="cuda")
h = torch.zeros(512, dtype=torch.float32).pin_memory()
d = torch.empty(512, device="cuda")
x = torch.zeros(1024, device="cuda")
res = {}
for name, st in (("default", torch.cuda.current_stream()), ("cu192", eng.cu_masked_stream(192)),
                 ("cu256", eng.cu_masked_stream(256)), ("plain", torch.cuda.Stream())):
    st.wait_stream(torch.cuda.current_stream())
    ops = {"engine_launch": lambda: eng.weighted_sum_tiled(buf, rows, MUL_W, w, n=8 * E, out=out[:8 * E], stream=st),
           "h2d_2KB": lambda: d.copy_(h, non_blocking=True),
           "tiny_kernel": lambda: x.add_(1.0)}
    for op, fn in ops.items():
        with torch.cuda.stream(st):
            for _ in range(5): fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(100): fn()
            b.record(st)
        b.synchronize()
        res[f"{name}_{op}_us"] = round(a.elapsed_time(b) * 10, 1)
print(json.dumps(res))
