"""cfg2 (ResNet-18-GN, K = 32) through FedMLAggOperator.agg's state_dict path on SEPARATELY allocated
device tensors: where a call's time goes, on the box it runs on.

Phases (host wall time, GPU work asynchronous): _host.gather (the 3,904-tensor walk), plan_outputs
(outputs + per-dtype tables), the launch call (descriptor staging + k_wsum_pair launch), and the whole
aggregate().  Then back-to-back calls as the bench issues them: host time per call vs GPU time per call
(HIP events on the stream).  Run under `rocprofv3 --kernel-trace --stats` for the kernel's own time:
if host per call >= the kernel's time, the step is host-bound and box CPU speed sets the rate.

  python tools/cfg2_host_probe.py [--calls 200] [--out file.json]
"""
import argparse
import json
import os
import sys
import time
from collections import OrderedDict

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fedml_amd import _host  # noqa: E402
from fedml_amd.engine import get_engine  # noqa: E402
from fedml_amd.ml.aggregator import state_dict_agg as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    layout = [(n, tuple(s), getattr(torch, dt)) for n, s, dt in
              json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))["resnet18_gn"]]
    K = 32
    g = torch.Generator(device="cuda").manual_seed(1)
    dicts = [OrderedDict((n, (torch.randn(s, generator=g, device="cuda").to(dt) if dt != torch.int64 else
                              torch.randint(0, 100, s, generator=g, device="cuda"))) for n, s, dt in layout)
             for _ in range(K)]
    keys = list(dicts[0].keys())
    w = [1.0 / K] * K
    eng = get_engine(0)

    def host_t(fn, n=50):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
        return round(float(np.median(ts)) * 1e6, 1)

    ptrs, numel, codes, shapes, dev = _host.gather(dicts, keys)
    phases = {
        "gather_us": host_t(lambda: _host.gather(dicts, keys)),
        "plan_outputs_us": host_t(lambda: _host.plan_outputs(shapes, codes, True, dev, ptrs, K)),
        "launch_only_us": None,
        "aggregate_us": host_t(lambda: S.aggregate(dicts, 0, w)),
    }
    _, views, groups = _host.plan_outputs(shapes, codes, True, dev, ptrs, K)
    if len(groups) == 2 and groups[1][0] == 4:
        (fc, n0, i0, o0), (_, n1, i1, o1) = groups
        phases["launch_only_us"] = host_t(lambda: eng.weighted_sum_table_pair(fc, 0, n0, i0, o0, n1, i1, o1, k=K, coef=w))

    # back to back, as the bench's timed loop
    res = {}
    for _ in range(10):
        res["o"] = S.aggregate(dicts, 0, w)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    per = []
    ev0.record()
    t0 = time.perf_counter()
    for _ in range(a.calls):
        t1 = time.perf_counter()
        res["o"] = S.aggregate(dicts, 0, w)
        per.append(time.perf_counter() - t1)
    t_host = time.perf_counter() - t0
    ev1.record()
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    out = {"phases_synced": phases,
           "b2b": {"calls": a.calls, "host_us_per_call": round(t_host / a.calls * 1e6, 1),
                   "host_median_us": round(float(np.median(per)) * 1e6, 1),
                   "wall_us_per_call": round(t_all / a.calls * 1e6, 1),
                   "gpu_event_us_per_call": round(ev0.elapsed_time(ev1) / a.calls * 1e3, 1)},
           "cpu_model": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": ")
           if os.path.exists("/proc/cpuinfo") else None}
    print(json.dumps(out))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
