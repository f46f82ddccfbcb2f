#!/usr/bin/env python
"""Tool: tiled metric read pattern on CU-masked streams (how many CUs saturate HBM?)."""
import ctypes, json, os
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "liblayoutprobe.so"))
L.lp_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
L.lp_masked_stream.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
K, P = 128, 125_000_000
p16 = P * 4 // 16 // 16384 * 16384
big = torch.empty(K * P, dtype=torch.float32, device="cuda").normal_()
out = torch.empty(p16 * 4, dtype=torch.float32, device="cuda")
res = {}
for ncu in (256, 248, 240, 224, 192, 160, 128):
    h = ctypes.c_void_p()
    total = L.lp_masked_stream(ncu, ctypes.byref(h))
    assert total > 0, total
    st = torch.cuda.ExternalStream(h.value)
    ts = []
    with torch.cuda.stream(st):
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st); L.lp_run(1, big.data_ptr(), p16, K, 256, out.data_ptr(), h); b.record(st)
            b.synchronize(); ts.append(a.elapsed_time(b))
    ms = sorted(ts[1:])[len(ts[1:]) // 2]
    res[f"cu{ncu}_of_{total}"] = round((K + 1) * p16 * 16 / ms / 1e6, 1)
print(json.dumps(res))
