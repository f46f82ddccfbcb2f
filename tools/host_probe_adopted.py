"""Host time of the drop-in path over arena-adopted ResNet-18-GN dicts (K = 32), piece by piece:
FedMLAggOperator.agg as a whole, resident_rows (C++ match_rows), ClientArena.aggregate, carve.
GPU work is asynchronous; this measures the host side only (the GPU-bound limit is ~0.26 ms)."""
import json
import os
import sys
import time
from collections import OrderedDict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.arena import ArenaLayout, ClientArena, resident_rows  # noqa: E402
from fedml_amd.engine import MUL_W  # noqa: E402
from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator  # noqa: E402
from fedml_amd import _host  # noqa: E402

layout = [(n, tuple(s), getattr(torch, dt)) for n, s, dt in
          json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "layouts.json")))["resnet18_gn"]]
K = 32
arena = ClientArena(ArenaLayout(layout), K)
dicts = []
for i in range(K):
    d = OrderedDict((n, torch.randn(s, device="cuda").to(dt) if dt != torch.int64 else torch.zeros(s, dtype=dt, device="cuda"))
                    for n, s, dt in layout)
    arena.adopt(i, d)
    dicts.append(d)
torch.cuda.synchronize()
A = type("A", (), {"federated_optimizer": "FedAvg"})()
raw = [(100 + i, d) for i, d in enumerate(dicts)]
w = [1.0 / K] * K


def t(fn, n=50):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    return round(dt * 1e6, 1)


res = {
    "agg_us": t(lambda: FedMLAggOperator.agg(A, raw)),
    "resident_rows_us": t(lambda: resident_rows(dicts)),
    "arena_aggregate_us": t(lambda: arena.aggregate(MUL_W, w)),
    "gather_us": t(lambda: _host.gather(dicts, list(dicts[0].keys()))),
}
o = {torch.float32: torch.empty(arena.layout.group_numel[torch.float32], device="cuda"),
     torch.int64: torch.empty(arena.layout.group_numel[torch.int64], device="cuda")}
res["carve_us"] = t(lambda: arena.layout.carve(o))
a = torch.cuda.Event(enable_timing=True)
b = torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
a.record()
for _ in range(50):
    FedMLAggOperator.agg(A, raw)
b.record()
torch.cuda.synchronize()
res["agg_wall_per_call_us_gpu"] = round(a.elapsed_time(b) / 50 * 1e3, 1)
print(json.dumps(res))
