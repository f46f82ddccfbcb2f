#!/usr/bin/env python
"""Benchmark: device-resident FedAvg aggregation GB/s (BASELINE.json metric) on MI355X.

Default workload (the metric's configuration): K = 128 synthetic client updates x P = 125,000,000
fp32 parameters, all resident in HBM; one step = one FedAvg aggregation (ordered weighted sum over
the 128 clients, reference formula of python/fedml/ml/aggregator/agg_operator.py:35-44).

  python bench.py [--gpus N --steps K --warmup W] [--config metric|resnet18|vit_bf16]

N > 1 (launched by torch.distributed.run, one rank per GPU, RCCL): the SAME total problem is
split by client groups -- rank r holds clients [r*K/N, (r+1)*K/N) -- each rank forms its ordered
local partial with the global weights (the group step), then the partials are SUM-reduced over
xGMI to rank 0 (the global step; the reference's pattern in simulation/nccl/base_framework/
params.py:98-105 + common.py:196-210).  The reduce is pipelined in chunks behind the local
kernels.  That is strong scaling of a fixed workload.

Output: ONE JSON line on rank 0 (see DESIGN.md for the roofline / traffic definitions).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "device-resident aggregate GB/s, K=128 × 125M fp32 params; 1/2/4/8 GPU"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="metric", choices=["metric", "resnet18", "vit_bf16"])
    p.add_argument("--clients", type=int, default=128)
    p.add_argument("--params", type=int, default=125_000_000)
    p.add_argument("--variant", type=int, default=0, help="kernel variant (fa_ctx_set_variant)")
    p.add_argument("--chunks", type=int, default=8, help="pipeline chunks of the cross-GPU reduce")
    p.add_argument("--collective", default="reduce", choices=["reduce", "reduce_scatter", "all_reduce"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline time budget")
    p.add_argument("--check-samples", type=int, default=65536)
    return p.parse_args()


# ----------------------------------------------------------------------------- distributed setup
def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ----------------------------------------------------------------------------- workloads
def client_counts(K):
    rng = np.random.RandomState(7)  # n_i ~ U{50..600}, seed 7
    return [int(v) for v in rng.randint(50, 601, size=K)]


def make_flat_clients(idx, P, dtype=torch.float32):
    out = []
    for i in idx:
        g = torch.Generator(device="cuda").manual_seed(1000 + i)
        out.append(torch.randn(P, generator=g, device="cuda", dtype=torch.float32).to(dtype))
    return out


def load_layout(name):
    with open(os.path.join(ROOT, "tests", "golden", "layouts.json")) as f:
        return json.load(f)[name]


def make_layout_clients(idx, layout):
    dicts = []
    for i in idx:
        g = torch.Generator(device="cuda").manual_seed(1000 + i)
        d = {}
        for name, shape, dt in layout:
            dt = getattr(torch, dt)
            if dt == torch.int64:
                d[name] = torch.randint(0, 100, tuple(shape), generator=g, device="cuda", dtype=dt)
            else:
                d[name] = torch.randn(tuple(shape), generator=g, device="cuda").to(dt)
        dicts.append(d)
    return dicts


# ----------------------------------------------------------------------------- CPU baseline
def cpu_baseline(K, budget_s):
    """The reference's CPU cost: oracle/torch_port.py (op-for-op restatement of agg_operator.py's
    FedAvg loop) on host-resident tensors, K clients x a bounded P, best of several runs."""
    from oracle import torch_port
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    torch.set_num_threads(threads)
    P = 4_000_000
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(P, generator=g) for _ in range(K)]
    counts = client_counts(K)
    raw = [(counts[i], {"w": xs[i]}) for i in range(K)]
    best = float("inf")
    t_end = time.perf_counter() + budget_s
    runs = 0
    while runs < 3 or (time.perf_counter() < t_end and runs < 50):
        t0 = time.perf_counter()
        torch_port.agg("FedAvg", raw)
        best = min(best, time.perf_counter() - t0)
        runs += 1
    gbs = (K * P * 4 + P * 4) / best / 1e9
    return {"value": round(gbs, 2), "unit": "GB/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"K={K} x P={P} fp32 host-resident, best of {runs} runs of oracle/torch_port.agg('FedAvg')"}


def pmc_traffic(workload):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py), if any."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(workload, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


# ----------------------------------------------------------------------------- main
def main():
    args = parse()
    rank, world, local = init_dist(args)
    from fedml_amd.engine import MUL_W, get_engine
    eng = get_engine(local)
    if args.variant:
        eng.set_variant(args.variant)

    K, P = args.clients, args.params
    counts = client_counts(K)
    N_tot = sum(counts)
    w_all = [c / N_tot for c in counts]
    per = K // world
    mine = list(range(rank * per, (rank + 1) * per if rank < world - 1 else K))
    w_mine = [w_all[i] for i in mine]

    if args.config == "metric":
        workload = f"fedavg_flat_K{K}_P{P}_fp32"
        xs = make_flat_clients(mine, P)
        out = torch.empty(P, device="cuda")
        bytes_total = K * P * 4 + P * 4
        dtype = "fp32"
        segs = None
    else:
        layout = load_layout("resnet18_gn" if args.config == "resnet18" else "vit_b16_bf16")
        if args.config == "resnet18":
            K = args.clients if args.clients != 128 else 32
        counts = client_counts(K)
        N_tot = sum(counts)
        w_all = [c / N_tot for c in counts]
        per = K // world
        mine = list(range(rank * per, (rank + 1) * per if rank < world - 1 else K))
        w_mine = [w_all[i] for i in mine]
        dicts = make_layout_clients(mine, layout)
        P = sum(int(np.prod(s)) for _, s, _ in layout)
        in_b = sum(int(np.prod(s)) * (8 if dt == "int64" else (2 if dt == "bfloat16" else 4)) for _, s, dt in layout)
        out_b = sum(int(np.prod(s)) * (2 if dt == "bfloat16" else 4) for _, s, dt in layout)
        bytes_total = K * in_b + out_b
        workload = f"fedavg_{args.config}_K{K}_P{P}"
        dtype = "bf16" if args.config == "vit_bf16" else "fp32"
        from fedml_amd.ml.aggregator.state_dict_agg import aggregate
        segs = (dicts, aggregate)

    stream = torch.cuda.current_stream()
    kernel_ms = []

    def local_step(record):
        if segs is None:
            if world == 1:
                ev0 = torch.cuda.Event(enable_timing=True) if record else None
                if record:
                    ev0.record(stream)
                eng.weighted_sum(xs, MUL_W, w_mine, out=out)
                if record:
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev1.record(stream)
                    kernel_ms.append((ev0, ev1))
                return out
            # pipelined group -> global: local partial per chunk, then the collective on that chunk
            import torch.distributed as dist
            C = max(1, args.chunks)
            bounds = [(P * c // C, P * (c + 1) // C) for c in range(C)]
            works = []
            for (a, b) in bounds:
                ev0 = torch.cuda.Event(enable_timing=True) if record else None
                if record:
                    ev0.record(stream)
                eng.weighted_sum([x[a:b] for x in xs], MUL_W, w_mine, out=out[a:b])
                if record:
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev1.record(stream)
                    kernel_ms.append((ev0, ev1))
                if args.collective == "reduce":
                    works.append(dist.reduce(out[a:b], dst=0, op=dist.ReduceOp.SUM, async_op=True))
                elif args.collective == "all_reduce":
                    works.append(dist.all_reduce(out[a:b], op=dist.ReduceOp.SUM, async_op=True))
                else:
                    n = b - a
                    sh = n // world
                    works.append(dist.reduce_scatter_tensor(shard[a // world:a // world + sh], out[a:a + sh * world],
                                                            op=dist.ReduceOp.SUM, async_op=True))
            for wk in works:
                wk.wait()
            return out
        dicts_, agg = segs
        ev0 = torch.cuda.Event(enable_timing=True) if record else None
        if record:
            ev0.record(stream)
        r = agg(dicts_, MUL_W, w_mine)
        if record:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record(stream)
            kernel_ms.append((ev0, ev1))
        if world > 1:
            import torch.distributed as dist
            for t in r.values():
                dist.reduce(t, dst=0)
        return r

    shard = torch.empty(P // world + 1, device="cuda") if world > 1 else None
    for _ in range(args.warmup):
        local_step(False)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        local_step(True)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    ms_per_step = elapsed / args.steps * 1e3
    value = bytes_total * args.steps / elapsed / 1e9

    # dominant kernel: average launch duration (HIP events on the launch stream)
    durs = [a.elapsed_time(b) for a, b in kernel_ms]
    launches_per_step = len(durs) // max(1, args.steps)
    kernel_avg_ms = float(np.mean(durs)) if durs else None
    if segs is None:
        per_launch_bytes = (len(mine) * P * 4 + P * 4) / max(1, launches_per_step)
    else:
        per_launch_bytes = bytes_total * len(mine) / K
    achieved = per_launch_bytes / (kernel_avg_ms * 1e-3) / 1e9 if kernel_avg_ms else None

    # parity spot-check at full size: sampled elements vs the C oracle (exact for N = 1)
    parity = None
    if segs is None and world == 1 and args.check_samples > 0:
        from oracle import orc
        torch.cuda.synchronize()
        gi = torch.Generator(device="cuda").manual_seed(99)
        idx = torch.randint(0, P, (args.check_samples,), generator=gi, device="cuda")
        sample = [x.index_select(0, idx).cpu() for x in xs]
        exp = orc.weighted_sum(sample, MUL_W, w_mine)
        got = out.index_select(0, idx).cpu()
        ok = torch.equal(got.view(torch.int32), exp.view(torch.int32))
        parity = f"{'bit-exact' if ok else 'MISMATCH'} vs oracle on {args.check_samples} sampled elements"

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(K if segs is None else K, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC if args.config == "metric" else f"device-resident aggregate GB/s, {workload}",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (N(0,1) client updates, seeds 1000+i; n_i ~ U{50..600}, seed 7), resident in HBM",
            "config": {"workload": workload, "clients": K, "params_per_client": P,
                       "parallelism": f"client-groups x{world}" + (f" + {args.collective} over RCCL, {args.chunks} chunks" if world > 1 else ""),
                       "kernel_variant": args.variant},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                         "traffic": pmc_traffic(workload),
                         "kernel_avg_ms": round(kernel_avg_ms, 4) if kernel_avg_ms else None,
                         "algorithmic_bytes_per_launch": int(per_launch_bytes)},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
