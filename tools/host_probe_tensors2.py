"""Host time of FedMLAggOperator.agg over SEPARATELY allocated device state_dicts (cfg2 ResNet-18-GN,
K = 32; cfg3 ViT-B/16 bf16, K = 128), piece by piece (GPU work async; host only)."""
import json
import os
import sys
import time
from collections import OrderedDict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd import _host  # noqa: E402
from fedml_amd.ml.aggregator import state_dict_agg as S  # noqa: E402
from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator  # noqa: E402

out = {}
for name, K in (("resnet18_gn", 32), ("vit_b16_bf16", 128)):
    layout = [(n, tuple(s), getattr(torch, dt)) for n, s, dt in
              json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "layouts.json")))[name]]
    dicts = [OrderedDict((n, torch.zeros(s, dtype=dt, device="cuda")) for n, s, dt in layout) for _ in range(K)]
    keys = list(dicts[0].keys())
    A = type("A", (), {"federated_optimizer": "FedAvg"})()
    raw = [(100 + i, d) for i, d in enumerate(dicts)]

    def t(fn, n=30):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
            torch.cuda.synchronize()  # host-only timing: no queueing behind the GPU
        return round(float(np.median(ts)) * 1e6, 1)
    ptrs, numel, codes, shapes, dev = _host.gather(dicts, keys)
    r = {"agg_us": t(lambda: FedMLAggOperator.agg(A, raw)),
         "gather_us": t(lambda: _host.gather(dicts, keys)),
         "alloc_outputs_us": t(lambda: _host.alloc_outputs(shapes, [torch.float32 if c == 4 else S._CODE_DTYPE[c] for c in codes.tolist()], dev)),
         "aggregate_device_us": t(lambda: S._aggregate_device(keys, ptrs, numel, codes, shapes, dev, K, 0, [1.0 / K] * K, 1.0, None))}
    out[name] = r
print(json.dumps(out))

# back-to-back (no per-call sync), as the bench issues steps: host time per call vs GPU time per call
for name, K in (("resnet18_gn", 32),):
    layout = [(n, tuple(s), getattr(torch, dt)) for n, s, dt in
              json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "layouts.json")))[name]]
    dicts = [OrderedDict((n, torch.zeros(s, dtype=dt, device="cuda")) for n, s, dt in layout) for _ in range(K)]
    w = [1.0 / K] * K
    res = {}
    for _ in range(5):
        res["o"] = S.aggregate(dicts, 0, w)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    t0 = time.perf_counter()
    per = []
    for _ in range(50):
        t1 = time.perf_counter()
        res["o"] = S.aggregate(dicts, 0, w)
        per.append(time.perf_counter() - t1)
    t_host = time.perf_counter() - t0
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"b2b_host_us_per_call": round(t_host / 50 * 1e6, 1), "b2b_host_median_us": round(float(np.median(per)) * 1e6, 1),
                      "b2b_host_max_us": round(max(per) * 1e6, 1), "b2b_gpu_us_per_call": round(a.elapsed_time(b) / 50 * 1e3, 1)}))
