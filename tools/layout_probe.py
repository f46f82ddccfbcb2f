#!/usr/bin/env python
"""Tool: client-major vs tile-interleaved arena read rate at the metric's size (K=128, 500 MB/client)."""
import ctypes, json, os, subprocess
import torch
HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "liblayoutprobe.so")
L = ctypes.CDLL(SO)
L.lp_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
K, P = 128, 125_000_000
p16 = P * 4 // 16 // 16384 * 16384  # every tile size below divides it: no read past the arena
s = torch.cuda.current_stream().cuda_stream
res = {}
for rep in range(3):
    big = torch.empty(K * P, dtype=torch.float32, device="cuda").normal_()
    out = torch.empty(p16 * 4, dtype=torch.float32, device="cuda")
    for name, mode, t16 in [("rows", 0, 0), ("tiled_4K", 1, 256), ("tiled_4K_xcd", 2, 256), ("tiled_4K_b", 1, 256),
                            ("tiled_4K_xcd_b", 2, 256)]:
        ts = []
        for _ in range(6):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); L.lp_run(mode, big.data_ptr(), p16, K, t16, out.data_ptr(), s); b.record()
            torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
        ms = sorted(ts[1:])[len(ts[1:]) // 2]
        res.setdefault(name, []).append(round((K + 1) * p16 * 16 / ms / 1e6, 1))
    del big, out
    torch.cuda.empty_cache()
print(json.dumps(res))
