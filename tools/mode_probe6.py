#!/usr/bin/env python
"""r06: does a physically contiguous arena (hipExtMallocWithFlags(hipDeviceMallocContiguous)) escape
the metric's slow placement (r06n / r06o: one of two torch-allocated arenas of a process runs
9.7-10.2 ms, the other 9.4-9.6, with identical translation, L2 and request counters)?  Arenas: T0
(torch), C0, C1 (contiguous), T1 (torch, allocated last); each timed (median of 4 x 5 launches,
interleaved).  Prints one JSON line."""
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
HIP = ctypes.CDLL("libamdhip64.so")


class Raw:
    def __init__(self, shape, flags):
        n = int(np.prod(shape))
        p = ctypes.c_void_p()
        rc = HIP.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(4 * n), ctypes.c_uint(flags))
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags({flags}) rc={rc}")
        self.ptr = p.value
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": "<f4", "data": (self.ptr, False),
                                         "version": 3, "strides": None}


def main():
    from fedml_amd.engine import MUL_W, get_engine
    eng = get_engine(0)
    K, P, E = 128, 125_000_000, 1024
    nt = -(-P // E)
    rng = np.random.RandomState(7)
    counts = [int(v) for v in rng.randint(50, 601, size=K)]
    w = [c / sum(counts) for c in counts]
    arenas, keep = {}, []
    order = os.environ.get("ORDER", "T0,C0,C1").split(",")
    for name in order:
        try:
            if name.startswith("C"):
                r = Raw((nt, K, E), 0x4)
                keep.append(r)
                t = torch.as_tensor(r, device="cuda")
            else:
                t = torch.empty((nt, K, E), device="cuda")
            t.fill_(1.0)
            arenas[name] = t
        except Exception as e:
            print(name, "failed:", e, file=sys.stderr)
    out = torch.empty(P, device="cuda")
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()

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

    kern = lambda b: eng.weighted_sum_tiled(b, list(range(K)), MUL_W, w, n=P, out=out)  # noqa: E731
    first = next(iter(arenas.values()))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        kern(first)
    torch.cuda.synchronize()
    km = {a: [] for a in arenas}
    for _ in range(4):
        for a in arenas:
            km[a] += timed(lambda: kern(arenas[a]), 5)
    print(json.dumps({a: round(float(np.median(v)), 3) for a, v in km.items()}), flush=True)


if __name__ == "__main__":
    main()
