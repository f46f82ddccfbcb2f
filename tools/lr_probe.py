"""cfg1 (LR-MNIST, K = 2) latency breakdown on the box: where an agg() call's ~30-50 us go.
Prints medians (us) of: the reference op sequence on CPU dicts and on DEVICE dicts (+ sync), the
launch+sync floor of one tiny HIP kernel, and our pieces (gather, alloc_outputs, the raw
fa_weighted_sum_host call, whole agg() on CPU / device dicts)."""
import json
import os
import sys
import time
from collections import OrderedDict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle.torch_port as tp  # noqa: E402
from fedml_amd import _host  # noqa: E402
from fedml_amd.engine import MUL_W, get_engine  # noqa: E402
from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator  # noqa: E402

eng = get_engine(0)
g = torch.Generator().manual_seed(3)
host = [OrderedDict((n, torch.randn(s, generator=g)) for n, s in [("linear.weight", (10, 784)), ("linear.bias", (10,))])
        for _ in range(2)]
dev = [OrderedDict((k, v.cuda()) for k, v in d.items()) for d in host]
counts = [120, 300]
A = type("A", (), {"federated_optimizer": "FedAvg"})()
keys = list(host[0].keys())


def med(fn, n=3000):
    for _ in range(200):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e6, 2)


def sync():
    torch.cuda.current_stream().synchronize()


ptrs, numel, codes, shapes, _ = _host.gather(host, keys)
_, views, optrs = _host.alloc_outputs(shapes, [torch.float32] * 2, "cpu")
x = torch.zeros(1, device="cuda")
res = {
    "ref_loop_cpu_dicts": med(lambda: tp.agg("FedAvg", [(n, OrderedDict(d)) for n, d in zip(counts, host)])),
    "ref_loop_device_dicts_sync": med(lambda: (tp.agg("FedAvg", [(n, OrderedDict(d)) for n, d in zip(counts, dev)]), sync())),
    "tiny_torch_kernel_sync_floor": med(lambda: (x.add_(1), sync())),
    "sync_only": med(sync),
    "gather": med(lambda: _host.gather(host, keys)),
    "alloc_outputs_cpu": med(lambda: _host.alloc_outputs(shapes, [torch.float32] * 2, "cpu")),
    "fa_weighted_sum_host_raw": med(lambda: eng.weighted_sum_host_table(0, MUL_W, numel, 2, ptrs, optrs, [0.3, 0.7])),
    "agg_cpu_dicts": med(lambda: FedMLAggOperator.agg(A, list(zip(counts, host)))),
    "agg_device_dicts_nosync": med(lambda: FedMLAggOperator.agg(A, list(zip(counts, dev)))),
    "agg_device_dicts_sync": med(lambda: (FedMLAggOperator.agg(A, list(zip(counts, dev))), sync())),
    "engine_weighted_sum_2x2_sync": med(lambda: (eng.weighted_sum_multi([[d[k].view(-1) for d in dev] for k in keys], MUL_W, [0.3, 0.7]), sync())),
}
print(json.dumps(res))
