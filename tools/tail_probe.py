#!/usr/bin/env python
"""Launch-shape probe for the weighted-sum access pattern at cfg2 / cfg3 / metric sizes
(tools/tail_probe.hip): one tile per workgroup at 64-512 threads vs a persistent grid.
Prints one JSON object of GB/s (K streams read + one output written, per launch)."""
import ctypes, json, os, subprocess, sys
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libtailprobe.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", SO,
                    os.path.join(HERE, "tail_probe.hip")], check=True)
L = ctypes.CDLL(SO)
L.tail_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                         ctypes.c_int, ctypes.c_void_p]


def timeit(fn, reps=20):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        a.record()
        for _ in range(reps):
            fn()
        b.record(); torch.cuda.synchronize()
        t = a.elapsed_time(b) / reps * 1e-3
        best = t if best is None else min(best, t)
    return best


s = torch.cuda.current_stream().cuda_stream
res = {}
shapes = [("cfg2", 32, 11_699_132 * 4), ("cfg3", 128, 86_415_592 * 2)]
if os.environ.get("PROBE_BIG", "0") == "1":
    shapes.append(("metric", 128, 125_000_000 * 4))
for name, k, per in shapes:
    per = per // 8192 * 8192
    buf = torch.empty(k * per // 4, dtype=torch.float32, device="cuda").normal_()
    ptrs = torch.tensor([buf.data_ptr() + i * per for i in range(k)], dtype=torch.int64, device="cuda")
    out = torch.empty(per // 4, dtype=torch.float32, device="cuda")
    tot = (k + 1) * per
    for blk in (64, 128, 256, 512):
        t = timeit(lambda: L.tail_probe(ptrs.data_ptr(), k, per, out.data_ptr(), blk, 0, 0, s))
        res[f"{name}_tiles_b{blk}_GBs"] = round(tot / t / 1e9, 1)
    for blk in (64, 256):
        for g in (256, 512, 1024, 2048, 4096):
            t = timeit(lambda: L.tail_probe(ptrs.data_ptr(), k, per, out.data_ptr(), blk, 1, g, s))
            res[f"{name}_persist_b{blk}_g{g}_GBs"] = round(tot / t / 1e9, 1)
    del buf, out, ptrs
    torch.cuda.empty_cache()
    print(json.dumps({kk: v for kk, v in res.items() if kk.startswith(name)}), file=sys.stderr, flush=True)
print(json.dumps(res))
