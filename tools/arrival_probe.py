#!/usr/bin/env python
"""Where the arrival config's last-arrival latency goes (bench.py --config arrival): K = 32 ResNet-18-GN
CPU state_dicts ingested on arrival; after the last one, time each phase with a device sync between
phases (so the phases do not overlap as they do in the real path):
  add   -- FedMLAggregator.add_local_trained_result of the last client (pinned pack + H2D issue)
  h2d   -- until the copy stream has drained
  agg   -- FedMLAggregator's ServerAggregator.aggregate (one launch over the arena rows)
  d2h   -- ArrivalIngest.to_host (result into pinned send buffers)
plus the unsynchronised end-to-end latency as the bench measures it.  Prints one JSON object (ms)."""
import json
import os
import statistics
import sys
import time
from collections import OrderedDict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from fedml_amd.core.alg_frame.server_aggregator import ServerAggregator  # noqa: E402
from fedml_amd.cross_silo.server.fedml_aggregator import FedMLAggregator  # noqa: E402

K = 32
layout, pristine = bench._resnet_host_dicts(K)
counts = bench.client_counts(K)


class SA(ServerAggregator):
    def get_model_params(self):
        return self.params

    def set_model_params(self, p):
        self.params = p

    def test(self, *a):
        return None


A = type("Args", (), {"federated_optimizer": "FedAvg"})()
sa = SA(None, A)
agg = FedMLAggregator(K, torch.device("cuda", 0), A, sa)


def arrive_all_but_last():
    dicts = [OrderedDict(d) for d in pristine]
    for i in range(K - 1):
        agg.add_local_trained_result(i, dicts[i], counts[i])
        t = time.perf_counter() + 0.002
        while time.perf_counter() < t:
            pass
    torch.cuda.synchronize()
    return dicts


def phased():
    dicts = arrive_all_but_last()
    s = torch.cuda.synchronize
    t0 = time.perf_counter()
    agg.add_local_trained_result(K - 1, dicts[K - 1], counts[K - 1])
    t1 = time.perf_counter()
    s()
    t2 = time.perf_counter()
    agg.check_whether_all_receive()
    model_list = [(agg.sample_num_dict[i], agg.model_dict[i]) for i in range(K)]
    averaged = sa.aggregate(model_list)
    s()
    t3 = time.perf_counter()
    agg.ingest.to_host(averaged)
    t4 = time.perf_counter()
    agg.ingest.round_done()
    return {"add": t1 - t0, "h2d": t2 - t1, "agg": t3 - t2, "d2h": t4 - t3}


def e2e():
    dicts = arrive_all_but_last()
    t0 = time.perf_counter()
    agg.add_local_trained_result(K - 1, dicts[K - 1], counts[K - 1])
    agg.check_whether_all_receive()
    agg.aggregate()
    agg.get_global_model_params_host()
    return time.perf_counter() - t0


for _ in range(3):
    phased()
ph = [phased() for _ in range(10)]
res = {k: round(statistics.median(p[k] for p in ph) * 1e3, 3) for k in ph[0]}
res["sum_phases"] = round(sum(res.values()), 3)
for _ in range(2):
    e2e()
res["e2e_median"] = round(statistics.median(e2e() for _ in range(10)) * 1e3, 3)
print(json.dumps(res))

if os.environ.get("PROBE_PROFILE"):  # cProfile of the aggregate phase (host side)
    import cProfile
    import io
    import pstats
    prof = cProfile.Profile()
    for _ in range(5):
        dicts = arrive_all_but_last()
        agg.add_local_trained_result(K - 1, dicts[K - 1], counts[K - 1])
        torch.cuda.synchronize()
        agg.check_whether_all_receive()
        model_list = [(agg.sample_num_dict[i], agg.model_dict[i]) for i in range(K)]
        prof.enable()
        averaged = sa.aggregate(model_list)
        torch.cuda.synchronize()
        prof.disable()
        agg.ingest.to_host(averaged)
        agg.ingest.round_done()
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(25)
    print(s.getvalue(), file=sys.stderr)

if os.environ.get("PROBE_SPLIT"):  # host time of the aggregate phase's pieces (no profiler)
    from fedml_amd.arena import resident_rows
    from fedml_amd.engine import MUL_W
    out = {"resident_rows": [], "launch": [], "kernel_wait": []}
    for _ in range(8):
        dicts = arrive_all_but_last()
        agg.add_local_trained_result(K - 1, dicts[K - 1], counts[K - 1])
        torch.cuda.synchronize()
        agg.check_whether_all_receive()
        ds = [agg.model_dict[i] for i in range(K)]
        N = sum(counts)
        t0 = time.perf_counter()
        arena, rows = resident_rows(ds)
        t1 = time.perf_counter()
        averaged = arena.aggregate(MUL_W, [c / N for c in counts], clients=rows)
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        agg.ingest.to_host(averaged)
        agg.ingest.round_done()
        out["resident_rows"].append(t1 - t0)
        out["launch"].append(t2 - t1)
        out["kernel_wait"].append(t3 - t2)
    print(json.dumps({k: round(statistics.median(v) * 1e3, 4) for k, v in out.items()}), file=sys.stderr)
