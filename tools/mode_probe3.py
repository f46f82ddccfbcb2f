#!/usr/bin/env python
"""r06: which output placements are slow (r06l: in one process the metric kernel ran 9.42 or 9.80 ms
by output buffer alone).  One tiled arena; output buffers made four ways, interleaved over 4 rounds:
  early   -- torch.empty(P) before the arena (the process's first large allocation)
  torch   -- torch.empty(P) after the arena (what bench.py's metric line does), x3
  contig  -- hipExtMallocWithFlags(hipDeviceMallocContiguous) (physically contiguous VRAM), x2
  slice   -- a P-element view at offset 0 of a 2 GiB torch allocation
For each: the metric kernel (median of 5 x 4 launches) and out.fill_() (the write stream alone).
Prints one JSON line."""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Contig:
    def __init__(self, nbytes):
        self.hip = ctypes.CDLL("libamdhip64.so")
        p = ctypes.c_void_p()
        rc = self.hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(0x4))
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags contiguous rc={rc}")
        self.ptr, self.n = p.value, nbytes // 4
        self.__cuda_array_interface__ = {"shape": (self.n,), "typestr": "<f4", "data": (self.ptr, False),
                                         "version": 3, "strides": None}


def main():
    from fedml_amd.engine import MUL_W, get_engine
    eng = get_engine(0)
    K, P, E = 128, 125_000_000, 1024
    nt = -(-P // E)
    rng = np.random.RandomState(7)
    counts = [int(v) for v in rng.randint(50, 601, size=K)]
    w = [c / sum(counts) for c in counts]
    outs = {"early": torch.empty(P, device="cuda")}
    buf = torch.empty((nt, K, E), device="cuda")
    buf.fill_(1.0)
    for i in range(3):
        outs[f"torch{i}"] = torch.empty(P, device="cuda")
    keep = []
    for i in range(2):
        try:
            c = Contig(P * 4)
            keep.append(c)
            outs[f"contig{i}"] = torch.as_tensor(c, device="cuda")
        except Exception as e:
            print("contig failed:", e, file=sys.stderr)
    big = torch.empty(512 << 20, device="cuda")
    outs["slice"] = big[:P]
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    nbytes = K * P * 4 + P * 4

    def timed(fn, reps):
        ms = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            fn()
            b.record(st)
            b.synchronize()
            ms.append(a.elapsed_time(b))
        return ms

    kern = lambda o: eng.weighted_sum_tiled(buf, list(range(K)), MUL_W, w, n=P, out=o)  # noqa: E731
    t = time.perf_counter()
    while time.perf_counter() - t < 1.0:
        kern(outs["torch0"])
    torch.cuda.synchronize()
    km = {k: [] for k in outs}
    fm = {k: [] for k in outs}
    for _ in range(4):
        for k, o in outs.items():
            km[k] += timed(lambda: kern(o), 5)
            fm[k] += timed(lambda: o.fill_(0.5), 3)
    ref = outs["torch0"].clone()
    same = all(torch.equal(o, ref) for o in outs.values()) if False else None
    res = {k: {"ms_med": round(float(np.median(km[k])), 4), "ms_min": round(min(km[k]), 4),
               "fill_GBs": round(P * 4 / (np.median(fm[k]) * 1e-3) / 1e9, 1), "ptr": hex(outs[k].data_ptr())}
           for k in outs}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
