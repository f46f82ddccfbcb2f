"""Where the host time of aggregate() over separately allocated device state_dicts goes when calls are
issued back to back (cfg2 ResNet-18-GN, K = 32): cProfile of 100 calls, plus per-call host time with
and without dropping the previous result first."""
import cProfile
import io
import json
import os
import pstats
import sys
import time
from collections import OrderedDict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.ml.aggregator import state_dict_agg as S  # noqa: E402

K = 32
layout = [(n, tuple(s), getattr(torch, dt)) for n, s, dt in
          json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "layouts.json")))["resnet18_gn"]]
dicts = [OrderedDict((n, torch.zeros(s, dtype=dt, device="cuda")) for n, s, dt in layout) for _ in range(K)]
w = [1.0 / K] * K
res = {}
for _ in range(10):
    res["o"] = S.aggregate(dicts, 0, w)
torch.cuda.synchronize()


def b2b(n=100, keep=True):
    per = []
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    t0 = time.perf_counter()
    for _ in range(n):
        t1 = time.perf_counter()
        if keep:
            res["o"] = S.aggregate(dicts, 0, w)
        else:
            S.aggregate(dicts, 0, w)
        per.append(time.perf_counter() - t1)
    th = time.perf_counter() - t0
    b.record()
    torch.cuda.synchronize()
    return {"host_us": round(th / n * 1e6, 1), "host_median_us": round(float(np.median(per)) * 1e6, 1),
            "gpu_us": round(a.elapsed_time(b) / n * 1e3, 1)}


out = {"b2b_keep": b2b(), "b2b_drop": b2b(keep=False)}
pr = cProfile.Profile()
pr.enable()
for _ in range(100):
    res["o"] = S.aggregate(dicts, 0, w)
pr.disable()
torch.cuda.synchronize()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
out["profile_top"] = s.getvalue().splitlines()[:40]
print(json.dumps(out, indent=1))
