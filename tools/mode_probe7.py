#!/usr/bin/env python
"""r06: within ONE physically contiguous allocation, does the arena's start offset decide the
metric's placement mode (r06p: contiguous arenas ran anywhere from 9.28 to 9.99 ms)?  One contiguous
allocation of the arena plus 64 MiB; views of the arena's shape at offsets 0, 4 KiB, 64 KiB, 256 KiB,
1 MiB and 2..62 MiB in 2 MiB steps, each timed (median of 2 x 5 launches, interleaved).  Prints one
JSON line {offset_bytes: ms}."""
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
    def __init__(self, n, flags):
        p = ctypes.c_void_p()
        rc = HIP.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(4 * n), ctypes.c_uint(flags))
        if rc != 0:
            raise RuntimeError(f"hipExtMallocWithFlags({flags}) rc={rc}")
        self.ptr = p.value
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (self.ptr, False),
                                         "version": 3, "strides": None}


def main():
    from fedml_amd.engine import MUL_W, get_engine
    eng = get_engine(0)
    K, P, E = 128, 125_000_000, 1024
    nt = -(-P // E)
    n = nt * K * E
    rng = np.random.RandomState(7)
    counts = [int(v) for v in rng.randint(50, 601, size=K)]
    w = [c / sum(counts) for c in counts]
    flags = int(os.environ.get("FLAGS", "4"))
    if flags >= 0:
        r = Raw(n + (64 << 20) // 4, flags)
        flat = torch.as_tensor(r, device="cuda")
    else:
        flat = torch.empty(n + (64 << 20) // 4, device="cuda")
    flat.fill_(1.0)
    offs = [0, 4 << 10, 64 << 10, 256 << 10, 1 << 20] + [m << 20 for m in range(2, 64, 2)]
    views = {o: flat[o // 4: o // 4 + n].view(nt, K, E) for o in offs}
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
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        kern(views[0])
    torch.cuda.synchronize()
    km = {o: [] for o in offs}
    for _ in range(2):
        for o in offs:
            km[o] += timed(lambda: kern(views[o]), 5)
    print(json.dumps({"base": hex(flat.data_ptr()), "ms": {o: round(float(np.median(v)), 3) for o, v in km.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
