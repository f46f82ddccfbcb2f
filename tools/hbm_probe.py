#!/usr/bin/env python
"""Practical HBM ceilings on this MI355X (read-only stream, copy), for DESIGN.md's roofline table."""
import ctypes, json, os, subprocess, sys
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libhbmprobe.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", SO,
                    os.path.join(HERE, "hbm_probe.hip")], check=True)
L = ctypes.CDLL(SO)
L.hbm_probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
L.hbm_probe_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]

def timeit(fn, reps=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3

GB = int(float(sys.argv[1]) * 2**30) if len(sys.argv) > 1 else 16 * 2**30
src = torch.empty(GB // 4, dtype=torch.float32, device="cuda").normal_()
s = torch.cuda.current_stream().cuda_stream
res = {"bytes": GB}
for blocks in (2048, 4096, 8192, 16384):
    out = torch.empty(blocks * 256, dtype=torch.int32, device="cuda")
    for u in (4, 8, 16):
        t = timeit(lambda: L.hbm_probe_read(src.data_ptr(), GB, out.data_ptr(), blocks, u, s))
        res[f"read_b{blocks}_u{u}_GBs"] = round(GB / t / 1e9, 1)
L.hbm_probe_multi.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
for k in (8, 32, 128):
    per = (GB // k) // 4096 * 4096
    views = [src[i * per // 4:(i + 1) * per // 4] for i in range(k)]
    ptrs = torch.tensor([v.data_ptr() for v in views], dtype=torch.int64, device="cuda")
    out = torch.empty(per // 16, dtype=torch.int32, device="cuda")
    for u in (8, 16):
        t = timeit(lambda: L.hbm_probe_multi(ptrs.data_ptr(), k, per, out.data_ptr(), u, s))
        res[f"multi_k{k}_u{u}_GBs"] = round(k * per / t / 1e9, 1)
    # with the aggregation kernel's output: one 16-byte vector per lane (bytes counted: k reads + 1 write)
    outw = torch.empty(per // 4, dtype=torch.float32, device="cuda")
    t = timeit(lambda: L.hbm_probe_multi(ptrs.data_ptr(), k, per, outw.data_ptr(), -8, s))
    res[f"multi_k{k}_wide_out_incl_write_GBs"] = round((k + 1) * per / t / 1e9, 1)
    del outw
# the metric's shape: 128 streams x 500 MB in ONE 64 GB allocation, with and without a 16-B/lane output
if os.environ.get("PROBE_BIG", "1") == "1":
    del src
    torch.cuda.empty_cache()
    kb, pb = 128, 125_000_000 * 4
    big = torch.empty(kb * pb // 4, dtype=torch.float32, device="cuda").normal_()
    ptrs = torch.tensor([big.data_ptr() + i * pb for i in range(kb)], dtype=torch.int64, device="cuda")
    outw = torch.empty(pb // 4, dtype=torch.float32, device="cuda")
    for u, tag in ((8, "xor"), (-8, "wide_out")):
        t = timeit(lambda: L.hbm_probe_multi(ptrs.data_ptr(), kb, pb, outw.data_ptr(), u, s), reps=5)
        res[f"metric_shape_k128_500MB_{tag}_GBs"] = round(kb * pb / t / 1e9, 1)
        if u < 0:
            res[f"metric_shape_k128_500MB_{tag}_incl_write_GBs"] = round((kb + 1) * pb / t / 1e9, 1)
    del big, outw
    torch.cuda.empty_cache()
    src = torch.empty(GB // 4, dtype=torch.float32, device="cuda").normal_()
# 128 SEPARATE allocations (how bench.py lays out the clients)
k, per = 128, (GB // 2 // 128) // 4096 * 4096
sep = [torch.empty(per // 4, dtype=torch.float32, device="cuda").normal_() for _ in range(k)]
ptrs = torch.tensor([v.data_ptr() for v in sep], dtype=torch.int64, device="cuda")
out = torch.empty(per // 16, dtype=torch.int32, device="cuda")
t = timeit(lambda: L.hbm_probe_multi(ptrs.data_ptr(), k, per, out.data_ptr(), 8, s))
res["multi_sep_k128_u8_GBs"] = round(k * per / t / 1e9, 1)
del sep
half = GB // 2
dst = torch.empty(half // 4, dtype=torch.float32, device="cuda")
for blocks in (2048, 8192):
    t = timeit(lambda: L.hbm_probe_copy(src.data_ptr(), dst.data_ptr(), half, blocks, s))
    res[f"copy_b{blocks}_GBs"] = round(2 * half / t / 1e9, 1)
res["read_best_GBs"] = max(v for k, v in res.items() if k.startswith("read_"))
res["copy_best_GBs"] = max(v for k, v in res.items() if k.startswith("copy_"))
print(json.dumps(res))
