#!/usr/bin/env python
"""Benchmark: device-resident FedAvg aggregation GB/s (BASELINE.json metric) on MI355X.

Default workload (the metric's configuration, BASELINE.json configs / SURVEY.md §8(d)):
K = 128 synthetic client updates x P = 125,000,000 fp32 parameters, all resident in HBM; one
step = one FedAvg aggregation (ordered weighted sum over the 128 clients, the reference formula
of python/fedml/ml/aggregator/agg_operator.py:35-44), value = algorithmic bytes / step time with
B = K*P*4 (reads) + P*4 (write) = 64.5 GB.

  python bench.py [--gpus N --steps K --warmup W] [--config metric|resnet18|vit_bf16|hier|gossip]

N > 1 (one rank per GPU, RCCL over xGMI): ``python bench.py --gpus N`` starts its N ranks itself
(torch.distributed.run as a child process, before anything touches the GPU); under an outer
torch.distributed.run (WORLD_SIZE set) it runs as one rank.  The SAME total problem is split by
client group -- rank r holds clients [r*K/N, (r+1)*K/N) -- each rank forms its ordered local
partial with the global weights (group step, HIP kernel), and the partials are summed across the
GPUs (global step): by default the "ordered" exchange, which delivers the WHOLE global model to
rank 0 summed in rank order (bit-exact; the reference NCCL simulator's reduce to rank 0,
simulation/nccl/base_framework/common.py:196-210), pipelined in chunks behind the local kernels
(fedml_amd/distributed/group_reduce.py; --collective picks reduce / all_reduce / reduce_scatter /
ordered_all).  Total work is fixed, so scaling is "strong"; roofline.frac at N > 1 is the whole
step's aggregate GB/s over N x 8 TB/s.  Every collective has a process-group
timeout (--pg-timeout) and every rank a stage watchdog (--stage-timeout), so a hang exits non-zero.

Other configs (one JSON line each, same fields): resnet18 = cfg2 (ResNet-18-GN state_dict, 122
tensors incl. 20 int64, K=32); vit_bf16 = cfg3 (ViT-B/16 layout, bf16, K=128); hier = cfg4 (8
groups x 64 clients of ResNet-18 size, group FedAvg then the cloud step); gossip = cfg5 (256 ranks,
ring W, one DSGD step over ResNet-18-size models).
"""
from __future__ import annotations

import argparse
import json
from collections import OrderedDict
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
MFMA_F32_PEAK_TFS = 157.3  # dense f32-input MFMA (v_mfma_f32_{32x32x2,16x16x4}_f32), MI355X_MICROARCH.md
# FEDML_AMD_BENCH_REHEARSAL=cpu (tests only): the N-rank metric / hier / gossip code paths -- launcher,
# gloo process group, GroupReducer / DistributedGossip, per-rank parity -- on the CPU, with the local
# reductions of an engine the TEST injects (FEDML_AMD_BENCH_ENGINE=module:factory, e.g.
# tests/rehearsal_engine.py).  The product has no CPU path: without an injected engine this mode
# refuses to run, and its lines are rehearsals, not measurements.
CPU_REHEARSAL = os.environ.get("FEDML_AMD_BENCH_REHEARSAL") == "cpu"
DEV = "cpu" if CPU_REHEARSAL else "cuda"


def sync():
    if not CPU_REHEARSAL:
        torch.cuda.synchronize()
METRIC = "device-resident aggregate GB/s, K=128 × 125M fp32 params; 1/2/4/8 GPU"
RESNET18_P = 11_699_132


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=None,
                   help="untimed warmup steps (default: 3, and on one GPU as many more as make ~1 s of the "
                        "workload's own steps -- short steps otherwise run on the clock ramp, DESIGN A.2 3b)")
    p.add_argument("--config", default="metric",
                   choices=["metric", "fragmented", "resnet18", "vit_bf16", "hier", "gossip", "host", "secagg", "fedopt",
                            "dropin_cpu", "median",
                            "krum", "arrival", "lr", "samask"])
    p.add_argument("--clients", type=int, default=None)
    p.add_argument("--params", type=int, default=None)
    p.add_argument("--variant", type=int, default=0, help="kernel variant (fa_ctx_set_variant)")
    p.add_argument("--chunks", type=int, default=8, help="pipeline chunks of the cross-GPU reduce")
    p.add_argument("--cu-mask", type=int, default=192,
                   help="N > 1: run the local partials on a stream restricted to this many CUs (0 = off), "
                        "leaving the rest to RCCL's kernels (fa_stream_create_cu_masked)")
    p.add_argument("--collective", default="ordered",
                   choices=["ordered", "ordered_all", "reduce", "reduce_scatter", "all_reduce"],
                   help="group -> global exchange for N > 1 (fedml_amd/distributed/group_reduce.py): ordered = the "
                        "full global model on rank 0, summed in rank order by the other ranks (bit-exact); "
                        "ordered_all = the same on every rank; reduce = RCCL's reduce to rank 0 (the reference "
                        "NCCL simulator's call); reduce_scatter = the global model left SHARDED over the GPUs "
                        "(no rank holds all of it); all_reduce = RCCL all-reduce")
    p.add_argument("--pg-timeout", type=float, default=180.0,
                   help="N > 1: process-group timeout (s) of every collective (a hung RCCL op fails the rank)")
    p.add_argument("--stage-timeout", type=float, default=300.0,
                   help="a rank making no progress for this long in one stage exits 124, naming the stage")
    p.add_argument("--launch-timeout", type=float, default=1500.0,
                   help="--gpus N > 1 without an outer launcher: wall-clock limit (s) of the whole N-rank run")
    p.add_argument("--exchange-impl", default="native", choices=["native", "torch"],
                   help="N > 1 over RCCL: native = the whole step in one fa_group_reduce call of libfedagg "
                        "(include/fedagg_comm.h, its own RCCL communicators); torch = the same algorithm issued "
                        "per chunk through torch.distributed (group_reduce.py; always used over gloo)")
    p.add_argument("--self-launch", action="store_true",
                   help="start the ranks through torch.distributed.run even at --gpus 1 (the chain the multi-GPU "
                        "driver runs: parent -> launcher -> rank -> RCCL init -> native exchange)")
    p.add_argument("--loopback", action="store_true",
                   help="metric / hier: run the group -> global exchange even at one rank, native ordered exchanges "
                        "with FA_XCHG_LOOPBACK (every rank owns a piece, its own piece goes through RCCL as a self "
                        "send / receive) -- at --gpus 1 it executes the whole N > 1 exchange body on one GPU")
    p.add_argument("--soak-seconds", type=float, default=5.0,
                   help="one GPU: after the timed steps, keep stepping (untimed by the line's value) for this long and "
                        "report the sustained rate beside it (clock / thermal steadiness; 0 = off)")
    p.add_argument("--cold-reps", type=int, default=5,
                   help="one GPU: after the soak, this many single calls each after --cold-idle seconds of idle; "
                        "their median wall time is the line's `cold.ms` (the reference's per-round AggregationTime "
                        "pays one call after waiting for the clients; 0 = off)")
    p.add_argument("--cold-idle", type=float, default=1.0, help="idle seconds before each cold call")
    p.add_argument("--no-read-probe", action="store_true",
                   help="skip the in-process read-stream probe (measured_read_ceiling)")
    p.add_argument("--no-clock", action="store_true",
                   help="skip the amdsmi clock / power / temperature sampler (the line's `clock`)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline time budget")
    p.add_argument("--check-samples", type=int, default=65536)
    p.add_argument("--arrival-gap-ms", type=float, default=2.0,
                   help="arrival config: time between two clients' updates arriving")
    p.add_argument("--pinned", action="store_true", help="host config: client updates already in pinned memory")
    p.add_argument("--dtype", default="fp32", choices=["fp32", "bf16", "fp16"],
                   help="median config: element type of the client vectors")
    p.add_argument("--layout", default=None, choices=["arena", "tiled", "tensors", "adopted"],
                   help="arena: client updates as rows of one ClientArena allocation (fedml_amd/arena.py); "
                        "tiled: tile-interleaved ClientArena (4-KiB tiles of all clients contiguous); "
                        "tensors: one allocation per client tensor; adopted: state_dicts adopted into client-major "
                        "arena rows on arrival (ClientArena.adopt, what the round drivers do) and aggregated through "
                        "FedMLAggOperator.agg.  Default: tiled, except gossip (arena: its "
                        "row-sequential sliding window measured 5.12 ms client-major vs 5.52 ms tiled)")
    a = p.parse_args()
    if a.layout is None:
        a.layout = "arena" if a.config == "gossip" else "tiled"
    return a


# ----------------------------------------------------------------------------- distributed setup
def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_count():
    """GPUs this process may use, counted WITHOUT initialising HIP -- the launcher parent must not touch
    the GPU before its ranks start (torch.cuda.device_count() may fall back to hipGetDeviceCount when
    amdsmi discovery fails).  KFD topology nodes with SIMDs whose render node this process can open;
    if none can be read, the render nodes this process can open; capped by ROCR_VISIBLE_DEVICES /
    HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES when set (an explicitly EMPTY mask = 0 devices).
    None = could not tell (neither the topology nor a render node readable, no mask)."""
    import glob
    n = 0
    for prop in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(prop) as f:
                kv = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
        except OSError:
            continue  # a node this container may not see
        if int(kv.get("simd_count", "0")) <= 0:
            continue  # a CPU node
        minor = kv.get("drm_render_minor")
        dev = f"/dev/dri/renderD{minor}" if minor is not None else None
        if dev is None or not os.path.exists(dev) or os.access(dev, os.R_OK | os.W_OK):
            n += 1
    if n == 0:
        n = sum(1 for d in glob.glob("/dev/dri/renderD*") if os.access(d, os.R_OK | os.W_OK))
    known = n > 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        m = len([x for x in v.split(",") if x.strip() != ""])
        if m == 0:
            return 0  # set and empty: no device is visible, whatever the topology says
        if known:
            n = min(n, m)
    return n if known else None


def launch_cmd(n, argv, port, script=None):
    """The torch.distributed.run command that starts ``n`` ranks of this script on one node
    (rendezvous on 127.0.0.1), each with the caller's own arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            script or os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, argv, timeout_s, script=None):
    """``python bench.py --gpus N`` without an outer launcher: start the N ranks as CHILD processes
    (torch.distributed.run, one rank per GPU) -- nothing here has touched the GPU, and the parent
    never execs -- relay their output (rank 0's JSON line to stdout, any other line the ranks print
    to stderr), and return the worst rc.  A run that outlives ``timeout_s`` is killed as a process
    group and returns 124."""
    import signal
    import subprocess
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")  # a collective timeout tears the rank down
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")      # dmabuf IPC (the host driver's only mode)
    import threading
    p = subprocess.Popen(launch_cmd(n, argv, _free_port(), script), env=env, start_new_session=True,
                         stdout=subprocess.PIPE, text=True, bufsize=1)

    def relay():  # the JSON line (rank 0) to stdout; whatever else a rank prints (gloo banners) to stderr
        for line in p.stdout:
            (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
            (sys.stdout if line.lstrip().startswith("{") else sys.stderr).flush()
    pump = threading.Thread(target=relay, daemon=True)
    pump.start()
    try:
        rc = p.wait(timeout=timeout_s)
        pump.join(timeout=10)
    except subprocess.TimeoutExpired:
        print(f"bench.py: the {n}-rank run exceeded {timeout_s:.0f} s; killing its process group",
              file=sys.stderr, flush=True)
        try:
            os.killpg(p.pid, signal.SIGTERM)
            p.wait(timeout=20)
        except (subprocess.TimeoutExpired, ProcessLookupError):
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()
        return 124
    return rc if rc >= 0 else 128 - rc


class Stage:
    """Names what every rank is doing, and ends a rank that stays in one stage longer than
    ``limit_s`` with a message naming the stage (and, inside the exchange, the chunk) and exit 124 --
    so a hung collective fails the run promptly instead of spending the launcher's whole budget."""

    def __init__(self, rank, limit_s):
        import threading
        self.rank, self.limit, self.name, self.t0 = rank, limit_s, "start", time.monotonic()
        self._lock = threading.Lock()
        if limit_s and limit_s > 0:
            threading.Thread(target=self._watch, daemon=True).start()

    def __call__(self, name):
        with self._lock:
            self.name, self.t0 = name, time.monotonic()

    def done(self):
        self.limit = float("inf")

    def _watch(self):
        while True:
            time.sleep(1.0)
            with self._lock:
                name, dt = self.name, time.monotonic() - self.t0
            if dt > self.limit:
                try:
                    from fedml_amd.distributed.group_reduce import last_issued
                    where = last_issued()
                except Exception:  # noqa: BLE001 -- diagnostics only
                    where = None
                print(f"bench.py rank {self.rank}: no progress for {dt:.0f} s in stage '{name}'"
                      + (f" (last exchange op issued: {where})" if where else "") + "; exiting 124",
                      file=sys.stderr, flush=True)
                os._exit(124)


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and args.gpus > 1:
        raise SystemExit("--gpus N > 1: WORLD_SIZE is 1 (launch through bench.py itself, or torch.distributed.run "
                         "with --nproc-per-node N)")
    if world > 1 and args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.loopback and args.config not in ("metric", "hier"):
        raise SystemExit("--loopback: the metric and hier configs run the group -> global exchange")
    # FEDML_AMD_BENCH_REHEARSAL=1: rehearse the N > 1 code path with every rank on device 0 over gloo
    # (RCCL refuses two ranks on one GPU); numbers from such a run are not measurements
    rehearsal = os.environ.get("FEDML_AMD_BENCH_REHEARSAL") in ("1", "cpu")
    if CPU_REHEARSAL and args.config not in ("metric", "hier", "gossip"):
        raise SystemExit("FEDML_AMD_BENCH_REHEARSAL=cpu: the metric, hier and gossip configs only")
    if rehearsal:
        local = 0
    if not CPU_REHEARSAL:
        torch.cuda.set_device(local)
    if world > 1 or args.loopback:
        import datetime

        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        tmo = datetime.timedelta(seconds=args.pg_timeout)
        if rehearsal:
            dist.init_process_group("gloo", timeout=tmo)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
    return rank, world, local


def masked_stream(eng, args):
    """N > 1: make a CU-masked stream torch's CURRENT stream for the whole run (the local partials,
    the collectives' dependencies and the HIP-event timing all live on it), so no per-step
    cross-stream synchronisation is added (measured: +0.14 ms per step when the reducer switched
    streams every step).  Returns None: the GroupReducer then uses the current stream.  Only ONE
    such stream per process -- HIP multiplexes streams onto 4 hardware queues per process, and
    extra CU-masked queues serialised launches (tools/host_overhead.py)."""
    if not args.cu_mask or CPU_REHEARSAL:
        return None
    total = torch.cuda.get_device_properties(eng.device).multi_processor_count
    if args.cu_mask >= total:
        return None
    ms = eng.cu_masked_stream(args.cu_mask)
    sync()
    torch.cuda.set_stream(ms)
    return None


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=DEV)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ----------------------------------------------------------------------------- synthetic inputs
def client_counts(K):
    rng = np.random.RandomState(7)  # n_i ~ U{50..600}, seed 7
    return [int(v) for v in rng.randint(50, 601, size=K)]


def make_flat_clients(idx, P, dtype=torch.float32):
    out = []
    for i in idx:
        g = torch.Generator(device=DEV).manual_seed(1000 + i)
        out.append(torch.randn(P, generator=g, device=DEV, dtype=torch.float32).to(dtype))
    return out


def make_arena_rows(idx, P, dtype=torch.float32):
    """Client updates as rows of ONE ClientArena allocation (same values as make_flat_clients)."""
    if CPU_REHEARSAL:  # rows of one host allocation (a ClientArena is device memory)
        rows = torch.empty(len(idx), P, dtype=dtype)
        for j, i in enumerate(idx):
            g = torch.Generator(device=DEV).manual_seed(1000 + i)
            rows[j].copy_(torch.randn(P, generator=g, device=DEV, dtype=torch.float32).to(dtype))
        return list(rows)
    from fedml_amd.arena import ArenaLayout, ClientArena
    arena = ClientArena(ArenaLayout([("w", (P,), dtype)]), capacity=len(idx), zero=False)
    rows = []
    for j, i in enumerate(idx):
        g = torch.Generator(device=DEV).manual_seed(1000 + i)
        row = arena.bufs[dtype][j][:P]
        row.copy_(torch.randn(P, generator=g, device=DEV, dtype=torch.float32).to(dtype))
        rows.append(row)
    return rows


ARENA_ALLOC = set()  # how the tiled arenas of this run were allocated (ClientArena.alloc_kind)
ARENA_PLACEMENT = []  # their placement checks (ClientArena.placement)


def make_tiled_arena(idx, P, dtype=torch.float32):
    """Client updates in a TILE-INTERLEAVED ClientArena (same values as make_flat_clients)."""
    if CPU_REHEARSAL:  # the same [tiles, capacity, E] group layout in host memory (E: 4 KiB of fp32)
        import types
        E = 1024
        nt = -(-P // E)
        buf = torch.zeros(nt, len(idx), E, dtype=dtype)
        for j, i in enumerate(idx):
            g = torch.Generator(device=DEV).manual_seed(1000 + i)
            f = torch.zeros(nt * E, dtype=dtype)
            f[:P] = torch.randn(P, generator=g, device=DEV, dtype=torch.float32).to(dtype)
            buf[:, j, :] = f.view(nt, E)
        return types.SimpleNamespace(bufs={dtype: buf})
    from fedml_amd.arena import ArenaLayout, ClientArena
    arena = ClientArena(ArenaLayout([("w", (P,), dtype)]), capacity=len(idx), zero=False, tiled=True)
    ARENA_ALLOC.add(arena.alloc_kind[dtype])
    if dtype in arena.placement:
        ARENA_PLACEMENT.append(arena.placement[dtype])
    for j, i in enumerate(idx):
        g = torch.Generator(device=DEV).manual_seed(1000 + i)
        arena.write(j, {"w": torch.randn(P, generator=g, device=DEV, dtype=torch.float32).to(dtype)})
    sync()
    arena._scratch.clear()
    return arena


def sample_tiles(P, count, seed, E=1024):
    """``count`` distinct 4-KiB tiles (E fp32 elements) of a P-element vector, sorted: the parity
    sample.  Whole tiles are taken by slicing -- torch's index_select/gather kernels fault on
    tensors of more than 2^31 elements on this ROCm build (tools/diag_large.py), and a tiled
    arena group at the metric size holds 16 * 10^9."""
    nt = -(-P // E)
    g = torch.Generator().manual_seed(seed)
    return sorted(torch.randperm(nt, generator=g)[:min(count, nt)].tolist())


def flat_pick(x, tiles, P, E=1024):
    """Elements of the sampled tiles of a flat (or tile-row) device vector, as one CPU tensor."""
    return torch.cat([x[t * E:min((t + 1) * E, P)] for t in tiles]).cpu()


def tiled_pick(buf, tiles, P):
    """The sampled tiles of EVERY client row of a tiled arena group [tiles, capacity, E]:
    returns a CPU tensor [capacity, m] (m = sampled elements), row r = flat_pick of client r."""
    E = buf.shape[2]
    blk = torch.stack([buf[t] for t in tiles]).cpu()  # [nt, cap, E], each buf[t] one contiguous run
    cols = [blk[j, :, :min(E, P - t * E)] for j, t in enumerate(tiles)]
    return torch.cat(cols, dim=1)


def load_layout(name):
    with open(os.path.join(ROOT, "tests", "golden", "layouts.json")) as f:
        return json.load(f)[name]


def make_layout_clients(idx, layout):
    dicts = []
    for i in idx:
        g = torch.Generator(device=DEV).manual_seed(1000 + i)
        d = {}
        for name, shape, dt in layout:
            dt = getattr(torch, dt)
            if dt == torch.int64:
                d[name] = torch.randint(0, 100, tuple(shape), generator=g, device=DEV, dtype=dt)
            else:
                d[name] = torch.randn(tuple(shape), generator=g, device=DEV).to(dt)
        dicts.append(d)
    return dicts


def split(K, rank, world):
    per = K // world
    return list(range(rank * per, (rank + 1) * per if rank < world - 1 else K))


class _HostEvent:
    """CPU rehearsal stand-in for a timing event (wall clock)."""

    def record(self, _stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class Timed:
    """HIP-event timing of the dominant kernel launches, on the stream they are issued on.

    Per-launch mode (default): an event pair around every timed launch.  Loop mode (``loop``, set
    for one-GPU workloads whose step IS the timed call -- ``loop_timing`` in the workload): one event
    pair around the whole timed region and a count of the timed launches inside it, so the average
    launch duration includes the gaps between launches and the measured loop carries no per-step
    event records (r05: they cost 6-8 us a step, tools/event_cost_probe.py)."""

    def __init__(self):
        self.pairs = []
        self.on = False
        self.loop = False
        self.launches = 0
        self.loop_events = None
        self.natives = []  # native GroupReducers: their local-step kernels are timed inside libfedagg
        self.native_ms, self.native_launches = 0.0, 0

    def _event(self):
        e = _HostEvent() if CPU_REHEARSAL else torch.cuda.Event(enable_timing=True)
        e.record(None if CPU_REHEARSAL else torch.cuda.current_stream())
        return e

    def __enter__(self):
        if self.on and not self.loop:
            self.a = self._event()
        return self

    def __exit__(self, *exc):
        if self.on:
            if self.loop:
                self.launches += 1
            else:
                self.pairs.append((self.a, self._event()))

    def start(self):
        for r in self.natives:  # drop the warmup steps' native local-step timings
            r.local_time(reset=True)
        self.on = True
        if self.loop:
            self.launches = 0
            self.loop_events = [self._event(), None]

    def end(self):
        """After the last timed step is issued (before the synchronisation): loop mode's end event."""
        if self.on and self.loop:
            self.loop_events[1] = self._event()

    def stop(self):
        self.on = False
        self.native_ms, self.native_launches = 0.0, 0
        for r in self.natives:
            ms, cnt = r.local_time(reset=True)
            self.native_ms += ms
            self.native_launches += cnt

    def _loop_ms(self):
        a, b = self.loop_events or (None, None)
        return a.elapsed_time(b) if a is not None and b is not None else None

    def avg_ms(self):
        if self.native_launches:
            return self.native_ms / self.native_launches
        if self.loop:
            t = self._loop_ms()
            return t / self.launches if t is not None and self.launches else None
        d = [a.elapsed_time(b) for a, b in self.pairs]
        return float(np.mean(d)) if d else None

    def per_step_ms(self, steps):
        """Summed kernel time per step (several timed launches per step)."""
        if self.native_launches:
            return self.native_ms / steps
        if self.loop:
            t = self._loop_ms()
            return t / steps if t is not None else None
        d = [a.elapsed_time(b) for a, b in self.pairs]
        return float(np.sum(d)) / steps if d else None


# ----------------------------------------------------------------------------- workloads
def reducer(args, eng, timer, **kw):
    """The N > 1 group -> global exchange (fedml_amd/distributed/group_reduce.py) with the bench's
    HIP-event timing on the local partials (the owners' rank-ordered sum of the "ordered"
    exchange is left out of that average: it is not the dominant kernel)."""
    from fedml_amd.distributed.group_reduce import GroupReducer

    import torch.distributed as dist
    if args.exchange_impl == "native" and dist.get_backend() == "nccl":
        # the product path: one fa_group_reduce call per step (include/fedagg_comm.h), its local-step
        # kernels HIP-event timed inside the library
        red = GroupReducer(collective=args.collective, chunks=args.chunks, stream=masked_stream(eng, args),
                           native=True, timing=True, loopback=args.loopback)
        timer.natives.append(red)
        return red
    if args.loopback:
        raise SystemExit("--loopback: the native exchange over RCCL only (--exchange-impl native, nccl backend)")

    def untimed_sum(xs_, mode, coef, div, o):
        return eng.weighted_sum(xs_, mode, coef, div, out=o)
    return GroupReducer(collective=args.collective, chunks=args.chunks, stream=masked_stream(eng, args),
                        combine_sum=untimed_sum, native=False, **kw)


def count_bad(got, exp):
    """Mismatching elements (bitwise; NaN payloads compared as bits)."""
    ib = {4: torch.int32, 2: torch.int16, 8: torch.int64}[got.element_size()]
    return int((got.view(ib) != exp.view(ib)).sum())


def sum_over_ranks(v, world):
    if world == 1:
        return v
    import torch.distributed as dist
    t = torch.tensor([float(v)], dtype=torch.float64, device=DEV)
    dist.all_reduce(t)
    return float(t.item())


def collective_note(args, world):
    if world == 1 and not args.loopback:
        return ""
    return {"ordered": "the whole global model on rank 0, rank-ordered sum (bit-exact)",
            "ordered_all": "the whole global model on every rank, rank-ordered sum (bit-exact)",
            "reduce": "the whole global model on rank 0 (RCCL reduce order)",
            "all_reduce": "the whole global model on every rank (RCCL order)",
            "reduce_scatter": "the global model SHARDED over the ranks, every shard checked"}[args.collective]


def wl_metric(args, eng, rank, world, timer):
    """Flat FedAvg K x P fp32 (the metric).  Returns a workload dict."""
    from fedml_amd.engine import MUL_W
    K = args.clients or 128
    P = args.params or 125_000_000
    counts = client_counts(K)
    N = sum(counts)
    mine = split(K, rank, world)
    w = [counts[i] / N for i in mine]
    tiled = args.layout == "tiled"
    if tiled:
        arena = make_tiled_arena(mine, P)
        buf, rows = arena.bufs[torch.float32], list(range(len(mine)))
        xs = None
    else:
        xs = make_arena_rows(mine, P) if args.layout == "arena" else make_flat_clients(mine, P)
    out = torch.empty(P, device=DEV)
    res = {}
    if world > 1 or args.loopback:
        def timed_sum(xs_, mode, coef, div, o):
            with timer:
                return eng.weighted_sum(xs_, mode, coef, div, out=o)

        class TimedEngine:  # the tiled local step, HIP-event timed like timed_sum
            def weighted_sum_tiled(self, *a, **kw):
                with timer:
                    return eng.weighted_sum_tiled(*a, **kw)

            def weighted_sum_tiled_multi(self, *a, **kw):
                with timer:
                    return eng.weighted_sum_tiled_multi(*a, **kw)
        red = reducer(args, eng, timer, local_sum=timed_sum)

        def step():
            if tiled:
                res["g"] = red.fedavg_tiled(TimedEngine(), buf, rows, w, P, out=out)
            else:
                res["g"] = red.fedavg(xs, w, out=out)
        launches = args.chunks
    else:
        def step():
            with timer:
                if tiled:
                    eng.weighted_sum_tiled(buf, rows, MUL_W, w, n=P, out=out)
                else:
                    eng.weighted_sum(xs, MUL_W, w, out=out)
            res["g"] = out
        launches = 1

    def parity():
        """The oracle's ordered FedAvg on 64 sampled 4-KiB tiles of the model.  N > 1: the oracle's
        ordered partial of every rank's clients (regenerated from their seeds), summed in rank
        order, vs the global model -- on rank 0 (ordered / reduce / all_reduce), or on every rank
        for its shard (reduce_scatter); RCCL's own summation order (reduce, all_reduce,
        reduce_scatter) is held to 1e-6 normwise, the rank-ordered exchanges to bit-exactness."""
        if args.check_samples <= 0:
            return None
        from oracle import orc
        tiles = sample_tiles(P, max(1, args.check_samples // 1024), 99)
        if world == 1 and not args.loopback:
            sampled = list(tiled_pick(buf, tiles, P)[rows]) if tiled else [flat_pick(x, tiles, P) for x in xs]
            exp = orc.weighted_sum(sampled, MUL_W, w)
            bad = count_bad(flat_pick(out, tiles, P), exp)
            return f"{'bit-exact' if bad == 0 else f'{bad} MISMATCHES'} vs oracle on {exp.numel()} sampled elements"
        return parity_multi(tiles)

    def parity_multi(tiles):
        if args.collective == "reduce_scatter":  # rank r's shard [r*S, min((r+1)*S, P))
            S = -(-P // (world * 1024)) * 1024
            lo, hi = rank * S, min(P, (rank + 1) * S)
            tiles = [t for t in tiles if lo <= t * 1024 < hi]
        elif rank != 0 and args.collective != "ordered_all" and args.collective != "all_reduce":
            tiles = []
        bad = cnt = 0
        rel = 0.0
        if tiles:
            from oracle import orc
            parts = []
            for r in range(world):
                ids = split(K, r, world)
                cols = []
                for i in ids:
                    g = torch.Generator(device=DEV).manual_seed(1000 + i)
                    cols.append(flat_pick(torch.randn(P, generator=g, device=DEV), tiles, P))
                parts.append(orc.weighted_sum(cols, MUL_W, [counts[i] / N for i in ids]))
            exp = orc.weighted_sum(parts, 2)
            g_ = res["g"]
            got = flat_pick(g_, [t - (rank * S // 1024) for t in tiles], g_.numel()) \
                if args.collective == "reduce_scatter" else flat_pick(g_, tiles, P)
            bad, cnt = count_bad(got, exp), exp.numel()
            rel = float((got.double() - exp.double()).norm() / exp.double().norm())
        bad, cnt = sum_over_ranks(bad, world), sum_over_ranks(cnt, world)
        rel = max_over_ranks(rel, world)
        where = collective_note(args, world)
        if bad == 0:
            return f"bit-exact vs oracle (rank-ordered partials) on {int(cnt)} sampled elements of {where}"
        return (f"{'within' if rel <= 1e-6 else 'OUTSIDE'} 1e-6 normwise vs oracle (rel {rel:.2e}, {int(bad)} "
                f"elements differ in the last bits) on {int(cnt)} sampled elements of {where}")

    suffix = {"arena": "", "tiled": "_tiled", "tensors": "_tensors"}[args.layout]
    return dict(loop_timing=True, name=f"fedavg_flat_K{K}_P{P}_fp32" + suffix,
                dtype="fp32", step=step, parity=parity,
                bytes_total=K * P * 4 + P * 4, launch_bytes=(len(mine) * P * 4 + P * 4) / launches,
                clients=K, params=P, cpu_K=K,
                probe=(buf, buf.shape[1], f"this workload's tiled arena group ({buf.shape[1]} consecutive 4-KiB rows "
                       "per workgroup: the pages and the row runs the kernel reads)") if tiled and not CPU_REHEARSAL
                else None)


def wl_layout(args, eng, rank, world, timer):
    """cfg2 / cfg3: a real state_dict layout, all keys of one dtype in one launch.  N > 1: each
    rank aggregates its clients' arena (one launch per dtype group), and every dtype group's flat
    partial goes through the pipelined group -> global exchange."""
    from fedml_amd.ml.aggregator.state_dict_agg import MUL_W, aggregate
    resnet = args.config == "resnet18"
    layout = load_layout("resnet18_gn" if resnet else "vit_b16_bf16")
    K = args.clients or (32 if resnet else 128)
    counts = client_counts(K)
    N = sum(counts)
    mine = split(K, rank, world)
    w = [counts[i] / N for i in mine]
    dicts = make_layout_clients(mine, layout)
    arena = None
    adopted = args.layout == "adopted" and world == 1
    if adopted:  # the round drivers' form: updates adopted into arena rows, aggregated by the drop-in
        from fedml_amd.arena import ArenaLayout, ClientArena
        from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator
        keep = ClientArena(ArenaLayout([(n, tuple(s), getattr(torch, dt)) for n, s, dt in layout]), capacity=len(mine))
        for j, d in enumerate(dicts):
            keep.adopt(j, d)
        sync()
        A = type("Args", (), {"federated_optimizer": "FedAvg"})()
        raw = [(counts[i], d) for i, d in zip(mine, dicts)]
        res_keep = keep  # the arena stays alive (its rows back the dicts; residency needs the object)
    elif args.layout in ("arena", "tiled") or world > 1:
        from fedml_amd.arena import ArenaLayout, ClientArena
        arena = ClientArena(ArenaLayout([(n, tuple(s), getattr(torch, dt)) for n, s, dt in layout]),
                            capacity=len(mine), tiled=args.layout == "tiled" or world > 1)
        for j, d in enumerate(dicts):
            arena.write(j, d)
        if not arena.tiled:
            dicts = [arena.slot(j) for j in range(len(mine))]
        sync()
    P = sum(int(np.prod(s)) for _, s, _ in layout)
    size = {"int64": 8, "bfloat16": 2, "float32": 4}
    in_b = sum(int(np.prod(s)) * size[dt] for _, s, dt in layout)
    out_b = sum(int(np.prod(s)) * (2 if dt == "bfloat16" else 4) for _, s, dt in layout)
    res = {"arena": res_keep} if adopted else {}
    if world > 1:
        class TimedEngine:
            def weighted_sum_tiled(self, *a, **kw):
                with timer:
                    return eng.weighted_sum_tiled(*a, **kw)

            def weighted_sum_tiled_multi(self, *a, **kw):
                with timer:
                    return eng.weighted_sum_tiled_multi(*a, **kw)
        red = reducer(args, eng, timer)
        te = TimedEngine()
        rows = list(range(len(mine)))
        outs = {dt: torch.empty(n, dtype=torch.float32 if dt == torch.int64 else dt, device=DEV)
                for dt, n in arena.layout.group_numel.items()}

    def step():
        if world > 1:
            flat = {dt: red.fedavg_tiled(te, arena.bufs[dt], rows, w, n, out=outs[dt])
                    for dt, n in arena.layout.group_numel.items()}
            res["out"] = arena.layout.carve(flat) if args.collective != "reduce_scatter" else None
            return
        with timer:
            if adopted:
                res["out"] = FedMLAggOperator.agg(A, raw)
            else:
                res["out"] = arena.aggregate(MUL_W, w) if arena is not None else aggregate(dicts, MUL_W, w)

    def parity():
        from oracle import orc
        if world > 1:
            if args.collective == "reduce_scatter" or (rank != 0 and args.collective not in ("ordered_all", "all_reduce")):
                bad = cnt = 0
            else:  # every client's dict regenerated from its seed, oracle partial per rank, rank-ordered sum
                bad = cnt = 0
                keys = layout[:: max(1, len(layout) // 24)]
                idxs = {name: torch.arange(0, int(np.prod(shape)), max(1, int(np.prod(shape)) // 512), device=DEV)
                        for name, shape, _ in keys}
                cols = {}  # (key, client) -> sampled elements
                for i in range(K):
                    d = make_layout_clients([i], layout)[0]
                    for name, _, _ in keys:
                        cols[name, i] = d[name].reshape(-1).index_select(0, idxs[name]).cpu()
                    del d
                for name, _, _ in keys:
                    parts = [orc.weighted_sum([cols[name, i] for i in split(K, r, world)], MUL_W,
                                              [counts[i] / N for i in split(K, r, world)]) for r in range(world)]
                    exp = orc.weighted_sum(parts, 2)
                    bad += count_bad(res["out"][name].reshape(-1).index_select(0, idxs[name]).cpu(), exp)
                    cnt += exp.numel()
            bad, cnt = sum_over_ranks(bad, world), sum_over_ranks(cnt, world)
            if args.collective == "reduce_scatter":
                return "not checked (reduce_scatter leaves the state_dict sharded)"
            return (f"{'bit-exact' if bad == 0 else f'{int(bad)} elements differ (RCCL order)'} vs oracle "
                    f"(rank-ordered partials) on a strided sample of 24 keys ({int(cnt)} elements) of "
                    f"{collective_note(args, world)}")
        bad = 0
        for name, shape, dt in layout:
            n = int(np.prod(shape))
            idx = torch.arange(0, n, max(1, n // 512), device=DEV)
            exp = orc.weighted_sum([d[name].reshape(-1).index_select(0, idx).cpu() for d in dicts], MUL_W, w)
            got = res["out"][name].reshape(-1).index_select(0, idx).cpu()
            bad += count_bad(got, exp)
        return f"{'bit-exact' if bad == 0 else f'{bad} MISMATCHES'} vs oracle on a strided sample of every key"

    tag = ("resnet18gn" if resnet else "vitb16_bf16") + {"arena": "", "tiled": "_tiled", "tensors": "_tensors",
                                                         "adopted": "_adopted_agg"}[args.layout]
    return dict(loop_timing=True, name=f"fedavg_{tag}_K{K}_P{P}", dtype="fp32" if resnet else "bf16", step=step, parity=parity,
                bytes_total=K * in_b + out_b, launch_bytes=None, clients=K, params=P, cpu_K=None,
                step_bytes=len(mine) * in_b + out_b if world > 1 else None)


def wl_dropin_cpu(args, eng, rank, world, timer):
    """The drop-in boundary as the reference's callers use it: FedMLAggOperator.agg(args,
    [(n_i, state_dict_i)]) on CPU state_dicts (as unpickled from MPI / socket receive buffers),
    ResNet-18-GN layout, K = 32; result returned as CPU tensors.  Step = pack to pinned + H2D +
    aggregation + D2H (fedml_amd/ml/aggregator/state_dict_agg.py:_aggregate_host).  CPU baseline: the
    reference's op sequence (oracle/torch_port.agg) on the same CPU dicts, 16 threads."""
    if world > 1:
        raise SystemExit("--config dropin_cpu is a single-GPU configuration")
    from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator
    layout = load_layout("resnet18_gn")
    K = args.clients or 32
    counts = client_counts(K)
    dicts = []
    g = torch.Generator().manual_seed(1)
    for i in range(K):
        d = OrderedDict()
        for name, shape, dt in layout:
            dt = getattr(torch, dt)
            d[name] = (torch.randint(0, 100, tuple(shape), generator=g, dtype=dt) if dt == torch.int64
                       else torch.randn(tuple(shape), generator=g).to(dt))
        dicts.append(d)

    class A:
        federated_optimizer = "FedAvg"
    res = {}

    def step():
        with timer:
            res["out"] = FedMLAggOperator.agg(A(), list(zip(counts, dicts)))

    P = sum(int(np.prod(s)) for _, s, _ in layout)
    size = {"int64": 8, "bfloat16": 2, "float32": 4}
    in_b = sum(int(np.prod(s)) * size[dt] for _, s, dt in layout)
    out_b = sum(int(np.prod(s)) * 4 for _, s, dt in layout)

    def parity():
        import oracle.torch_port as tp
        exp = tp.agg("FedAvg", [(n, OrderedDict((k, v.clone()) for k, v in d.items())) for n, d in zip(counts, dicts)])
        bad = sum(int((res["out"][k].view(-1).view(torch.int32) != exp[k].view(-1).view(torch.int32)).sum())
                  for k in exp)
        return f"{'bit-exact' if bad == 0 else f'{bad} MISMATCHES'} vs the reference op sequence on every element"

    def cpu(budget_s):
        import oracle.torch_port as tp
        lists = []

        def run():  # agg() rebinds client 0's dict: fresh shallow copies, made outside the timed call
            tp.agg("FedAvg", lists.pop())

        def one():
            lists.append([(n, OrderedDict((k, v.clone()) for k, v in d.items())) for n, d in zip(counts, dicts)])
            t0 = time.perf_counter()
            run()
            return time.perf_counter() - t0
        legs = {}
        for th in cpu_thread_legs():
            if th > cpu_quota():  # oversubscribed: minutes per run (see cpu_thread_legs)
                continue
            torch.set_num_threads(th)
            ts = [one() for _ in range(5)]
            legs[th] = (min(ts), len(ts), 1.0)
        return legs_record(legs, K * in_b + out_b,
                           f"the same K={K} ResNet-18-GN CPU state_dicts, oracle/torch_port.agg('FedAvg') "
                           "(agg_operator.py:35-44)")

    return dict(name=f"dropin_agg_cpu_resnet18gn_K{K}_P{P}", dtype="fp32", step=step, parity=parity, cpu=cpu,
                bytes_total=K * in_b + out_b, launch_bytes=None, clients=K, params=P, cpu_K=K,
                data="synthetic CPU state_dicts (ResNet-18-GN layout), host-resident: the step includes H2D and D2H",
                roofline_note="kernel time = the whole agg() call incl. PCIe transfers (host-resident inputs)")


def _resnet_host_dicts(K, seed=1):
    """K ResNet-18-GN state_dicts of CPU tensors (as unpickled from MPI / socket receive buffers)."""
    layout = load_layout("resnet18_gn")
    g = torch.Generator().manual_seed(seed)
    dicts = []
    for _ in range(K):
        d = OrderedDict()
        for name, shape, dt in layout:
            dt = getattr(torch, dt)
            d[name] = (torch.randint(0, 100, tuple(shape), generator=g, dtype=dt) if dt == torch.int64
                       else torch.randn(tuple(shape), generator=g).to(dt))
        dicts.append(d)
    return layout, dicts


def wl_arrival(args, eng, rank, world, timer):
    """SURVEY.md §8(f) #1 / the reference's cross-silo round (cross_silo/server/fedml_aggregator.py:
    57-104): K = 32 ResNet-18-GN updates arrive one at a time as CPU state_dicts; each is ingested
    into HBM on arrival (FedMLAggregator.add_local_trained_result -> ArrivalIngest: pinned staging +
    H2D on a copy stream, fedml_amd/ml/aggregator/ingest.py) while the next one is awaited
    (``--arrival-gap-ms`` between arrivals, a network receive of 47 MB at ~25 GB/s takes ~2 ms);
    after the last arrival: FedMLAggregator.aggregate (the user's ServerAggregator ->
    FedMLAggOperator.agg, recognised as arena-resident: one launch) and the D2H of the global model
    into pinned send buffers.  Value = latency from the last arrival to the host-resident global
    model (ms, lower is better); the reference CPU loop can only start at that instant too."""
    if world > 1:
        raise SystemExit("--config arrival is a single-GPU configuration")
    from fedml_amd.core.alg_frame.server_aggregator import ServerAggregator
    from fedml_amd.cross_silo.server.fedml_aggregator import FedMLAggregator
    K = args.clients or 32
    layout, pristine = _resnet_host_dicts(K)
    counts = client_counts(K)
    gap = args.arrival_gap_ms * 1e-3

    class BenchServerAggregator(ServerAggregator):
        def get_model_params(self):
            return self.params

        def set_model_params(self, p):
            self.params = p

        def test(self, *a):
            return None

    A = type("Args", (), {"federated_optimizer": "FedAvg"})()
    sagg = BenchServerAggregator(None, A)
    agg = FedMLAggregator(K, torch.device("cuda", 0), A, sagg)
    res = {}

    def round_(gap_s):
        dicts = [OrderedDict(d) for d in pristine]  # fresh containers; tensors are the received ones
        for i in range(K - 1):
            agg.add_local_trained_result(i, dicts[i], counts[i])
            t_next = time.perf_counter() + gap_s
            while time.perf_counter() < t_next:
                pass
        t0 = time.perf_counter()  # the last client's message has arrived
        agg.add_local_trained_result(K - 1, dicts[K - 1], counts[K - 1])
        agg.check_whether_all_receive()
        agg.aggregate()
        host = agg.get_global_model_params_host()
        lat = time.perf_counter() - t0
        res["host"] = host
        return lat

    def step():
        return round_(gap)

    P = sum(int(np.prod(s)) for _, s, _ in layout)

    def parity():
        import oracle.torch_port as tp
        exp = tp.agg("FedAvg", [(n, OrderedDict(d)) for n, d in zip(counts, pristine)])
        bad = sum(count_bad(res["host"][k].reshape(-1), exp[k].reshape(-1)) for k in exp)
        back = [round_(0.0) * 1e3 for _ in range(3)]
        res["b2b_ms"] = round(min(back), 3)
        return (f"{'bit-exact' if bad == 0 else f'{bad} MISMATCHES'} vs the reference op sequence on every element "
                f"of the host-resident global model")

    def cpu(budget_s):
        import oracle.torch_port as tp

        def run():
            tp.agg("FedAvg", [(n, OrderedDict(d)) for n, d in zip(counts, pristine)])
        legs = timed_legs(run, budget_s, min_runs=3, max_runs=20)
        best = min(legs, key=lambda th: legs[th][0])
        return {"value": round(legs[best][0] * 1e3, 3), "unit": "ms", "cores": best, "kind": "port",
                "value_by_threads": {str(th): round(b * 1e3, 3) for th, (b, _, _) in sorted(legs.items())},
                "os_cpu_count": os.cpu_count(), "cpu_quota": cpu_quota(),
                "sample": f"the reference loop oracle/torch_port.agg('FedAvg') (agg_operator.py:35-44) over the same "
                          f"K={K} CPU state_dicts, started once all have arrived; best of runs per thread count"}

    return dict(name=f"arrival_fedavg_resnet18gn_K{K}_P{P}", dtype="fp32", step=step, parity=parity, cpu=cpu,
                latency=True, extra=res, clients=K, params=P, cpu_K=K, bytes_total=None, launch_bytes=None,
                data=f"synthetic CPU state_dicts (ResNet-18-GN layout) arriving {args.arrival_gap_ms} ms apart; "
                     "ingested to HBM on arrival; result D2H to pinned host memory",
                metric_name=f"last-arrival -> host-resident global model latency, cross-silo FedAvg round, "
                            f"ResNet-18-GN K={K}")


def wl_lr(args, eng, rank, world, timer):
    """cfg1 (BASELINE configs[0], the reference's quick_start): FedAvg of K = 2 logistic-regression
    updates (784 -> 10 weight + bias, 62.8 KB per client) through the drop-in
    FedMLAggOperator.agg.  A round this small is launch/latency-bound, so the value is the latency
    of one agg() call (ms, lower is better) until the result is usable: ``--layout host`` (default
    here): CPU state_dicts in, CPU tensors out, as the reference's MPI/CPU quick_start holds them;
    ``tensors``: device dicts, device result (synchronised); ``adopted``: arena-resident updates.
    CPU baseline: the reference's loop (oracle/torch_port.agg) on the same CPU dicts."""
    if world > 1:
        raise SystemExit("--config lr is a single-GPU configuration")
    from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator
    K = args.clients or 2
    layout = [("linear.weight", (10, 784), "float32"), ("linear.bias", (10,), "float32")]
    counts = client_counts(K)
    g = torch.Generator().manual_seed(3)
    host = [OrderedDict((n, torch.randn(s, generator=g)) for n, s, _ in layout) for _ in range(K)]
    mode = args.layout if args.layout in ("tensors", "adopted") else "host"
    if mode == "host":
        dicts = host
    else:
        dicts = [OrderedDict((k, v.cuda()) for k, v in d.items()) for d in host]
        if mode == "adopted":
            from fedml_amd.arena import ClientArena
            keep = ClientArena.for_model(dicts[0], K)
            for j, d in enumerate(dicts):
                keep.adopt(j, d)
    A = type("Args", (), {"federated_optimizer": "FedAvg"})()
    raw = list(zip(counts, dicts))
    res = {"arena": keep} if mode == "adopted" else {}  # the adopting arena must stay alive

    def step():
        t0 = time.perf_counter()
        out = FedMLAggOperator.agg(A, raw)
        if mode != "host":
            torch.cuda.current_stream().synchronize()
        res["out"] = out
        return time.perf_counter() - t0

    def parity():
        import oracle.torch_port as tp
        exp = tp.agg("FedAvg", [(n, OrderedDict(d)) for n, d in zip(counts, host)])
        bad = sum(count_bad(res["out"][k].cpu().reshape(-1), exp[k].reshape(-1)) for k in exp)
        return f"{'bit-exact' if bad == 0 else f'{bad} MISMATCHES'} vs the reference op sequence on every element"

    def cpu(budget_s):
        import oracle.torch_port as tp
        lat = {}
        for th in sorted({1, min(16, cpu_quota())}):
            torch.set_num_threads(th)
            ts = []
            for _ in range(2000):
                lst = [(n, OrderedDict(d)) for n, d in zip(counts, host)]
                t0 = time.perf_counter()
                tp.agg("FedAvg", lst)
                ts.append(time.perf_counter() - t0)
            lat[th] = float(np.median(ts))
        best = min(lat, key=lambda th: lat[th])
        return {"value": round(lat[best] * 1e3, 4), "unit": "ms", "cores": best, "kind": "port",
                "value_by_threads": {str(th): round(v * 1e3, 4) for th, v in sorted(lat.items())},
                "sample": f"median of 2000 calls of oracle/torch_port.agg('FedAvg') (agg_operator.py:35-44) on the "
                          f"same K={K} CPU state_dicts"}

    extra = {}

    def host_breakeven():
        """Host-resident rounds: agg() latency with the round summed on the host (host_sum.h) vs sent
        to the device (FEDML_AMD_HOST_CPU_BYTES=0: the zero-copy kernel), over round sizes -- the
        measurement behind state_dict_agg._HOST_CPU_BYTES.  Both results compared bit for bit."""
        from fedml_amd.ml.aggregator import state_dict_agg as sda
        rows = []
        old = os.environ.get("FEDML_AMD_HOST_CPU_BYTES")
        try:
            for kk, pp in ((2, 7850), (2, 32768), (8, 16384), (8, 32768), (8, 65536), (8, 131072), (16, 131072)):
                gg = torch.Generator().manual_seed(kk * 7 + pp)
                ds = [OrderedDict([("w", torch.randn(pp - 10, generator=gg)), ("b", torch.randn(10, generator=gg))])
                      for _ in range(kk)]
                rr = list(zip(client_counts(kk), ds))
                lat, outs = {}, {}
                for path, thr in (("host", str(1 << 40)), ("device", "0")):
                    os.environ["FEDML_AMD_HOST_CPU_BYTES"] = thr
                    ts = []
                    for it in range(400):
                        t0 = time.perf_counter()
                        o = FedMLAggOperator.agg(A, rr)
                        ts.append(time.perf_counter() - t0)
                    lat[path] = float(np.median(ts[50:])) * 1e6
                    outs[path] = o
                bad = sum(count_bad(outs["host"][k].reshape(-1), outs["device"][k].reshape(-1)) for k in outs["host"])
                rows.append({"K": kk, "params": pp, "bytes": kk * pp * 4, "host_us": round(lat["host"], 2),
                             "device_us": round(lat["device"], 2), "host_vs_device_mismatches": bad})
        finally:
            if old is None:
                os.environ.pop("FEDML_AMD_HOST_CPU_BYTES", None)
            else:
                os.environ["FEDML_AMD_HOST_CPU_BYTES"] = old
        extra["host_breakeven"] = {"threshold_bytes": sda._host_cpu_bytes(), "rows": rows,
                                   "note": "median agg() latency (us) of CPU dicts -> CPU result; host = "
                                           "summed where the data is (fedml_amd/csrc/host_sum.h), device = "
                                           "the zero-copy kernel k_wsum_host1"}

    def parity_and_sweep():
        p = parity()
        if mode == "host":
            from fedml_amd.ml.aggregator import state_dict_agg as sda
            extra["host_path"] = ("host sum (fedml_amd/csrc/host_sum.h)" if K * P * 4 <= sda._host_cpu_bytes()
                                  else "device (k_wsum_host1, zero-copy)")
            if os.environ.get("FEDML_AMD_BENCH_LR_SWEEP", "1") == "1":
                host_breakeven()
        return p

    P = sum(int(np.prod(s)) for _, s, _ in layout)
    return dict(name=f"fedavg_lr_mnist_K{K}_P{P}_{mode}", dtype="fp32", step=step, parity=parity_and_sweep, cpu=cpu,
                extra_line=extra,
                latency=True, stat="median", clients=K, params=P, cpu_K=K, bytes_total=None, launch_bytes=None,
                data=f"synthetic LR-MNIST updates (784x10 + 10 fp32), {'CPU' if mode == 'host' else 'device'} "
                     f"state_dicts{' adopted into arena rows' if mode == 'adopted' else ''}",
                metric_name=f"FedMLAggOperator.agg latency per call, cfg1 LR-MNIST K={K} ({mode})")


def fragmented_layout(P, n_tensors=200):
    """The metric's P split ViT-style (SURVEY.md §8(d) "fragmented" variant): a repeating pattern of
    transformer-block tensor shapes, ~n_tensors tensors summing to exactly P fp32 elements."""
    D, M = 768, 3072
    block = [[D], [D], [3 * D, D], [3 * D], [D, D], [D], [D], [D], [M, D], [M], [D, M], [D]]
    per = sum(int(np.prod(s)) for s in block)
    reps = max(1, P // per)
    shapes = [s for _ in range(reps) for s in block]
    # scale the large matrices so that the whole layout holds exactly P elements
    total = sum(int(np.prod(s)) for s in shapes)
    while len(shapes) > n_tensors or total > P:
        total -= int(np.prod(shapes.pop()))
    rest = P - total
    while rest > 0:
        take = min(rest, D * M)
        shapes.append([take])
        rest -= take
    return [(f"t{i}", s, "float32") for i, s in enumerate(shapes)]


def wl_fragmented(args, eng, rank, world, timer):
    """The metric shape (K=128 x P=125 M fp32) with every client update split ViT-style into ~200
    separately allocated tensors, aggregated through the state_dict API (fedml_amd/ml/aggregator/
    state_dict_agg.aggregate: host pointer tables via fedml_amd._host, one launch per dtype group)."""
    if world > 1:
        raise SystemExit("fragmented config: single GPU")
    from fedml_amd.ml.aggregator.state_dict_agg import MUL_W, aggregate
    K = args.clients or 128
    P = args.params or 125_000_000
    layout = fragmented_layout(P)
    counts = client_counts(K)
    N = sum(counts)
    w = [c / N for c in counts]
    dicts = make_layout_clients(range(K), layout)
    res = {}

    def step():
        with timer:
            res["out"] = aggregate(dicts, MUL_W, w)

    def parity():
        if args.check_samples <= 0:
            return None
        from oracle import orc
        bad = 0
        for name, shape, _ in layout[:: max(1, len(layout) // 16)]:
            n = int(np.prod(shape))
            idx = torch.arange(0, n, max(1, n // 256), device=DEV)
            exp = orc.weighted_sum([d[name].reshape(-1).index_select(0, idx).cpu() for d in dicts], MUL_W, w)
            got = res["out"][name].reshape(-1).index_select(0, idx).cpu()
            bad += int((got.view(torch.int32) != exp.view(torch.int32)).sum())
        return f"{'bit-exact' if bad == 0 else f'{bad} MISMATCHES'} vs oracle on a strided sample of 16 keys"

    return dict(loop_timing=True, name=f"fedavg_fragmented{len(layout)}_K{K}_P{P}_fp32", dtype="fp32", step=step, parity=parity,
                bytes_total=K * P * 4 + P * 4, launch_bytes=None, clients=K, params=P, cpu_K=None,
                roofline_note="kernel time = the whole aggregate() call (host pointer tables + launch + kernel)")


def wl_hier(args, eng, rank, world, timer):
    """cfg4: G groups x M clients (ResNet-18 size, flat fp32): group FedAvg (weights n_i/N_g), cloud
    term (G_g * N_g) / N (HierFedAvgCloudAggregator.py:140-157), ordered global sum over groups --
    one fused two-level kernel pass over this rank's clients (fa_weighted_sum_grouped); across
    ranks (one or more groups each) the partials go through the group -> global exchange."""
    from fedml_amd.engine import MUL_N_DIV_N, MUL_W
    G, M = 8, (args.clients or 512) // 8
    P = args.params or RESNET18_P
    counts = client_counts(G * M)
    N = sum(counts)
    my_groups = split(G, rank, world)
    clients = [i for g in my_groups for i in range(g * M, (g + 1) * M)]
    # multi-rank hierarchical: flat rows (GroupReducer slices)
    tiled = args.layout == "tiled" and world == 1 and not args.loopback
    if tiled:
        arena = make_tiled_arena(clients, P)
        buf, rows, xs = arena.bufs[torch.float32], list(range(len(clients))), None
    else:
        xs = (make_arena_rows if args.layout in ("arena", "tiled") else make_flat_clients)(clients, P)
    gcounts = [counts[g * M:(g + 1) * M] for g in my_groups]
    gn = [sum(c) for c in gcounts]
    w = [c / gn[j] for j, cs in enumerate(gcounts) for c in cs]
    gptr = [j * M for j in range(len(my_groups) + 1)]
    out = torch.empty(P, device=DEV)
    res = {}

    def timed_grouped(xs_, mode, coef, div, gp, gm, gc, gd, o):
        with timer:
            return eng.weighted_sum_grouped(xs_, mode, coef, div, gp, gm, gc, gd, out=o)

    if world > 1 or args.loopback:
        red = reducer(args, eng, timer, local_grouped=timed_grouped)

        def step():
            res["g"] = red.hierarchical_groups(xs, gcounts, N, out=out)
        launches = args.chunks
    else:
        def step():
            if tiled:
                with timer:
                    eng.weighted_sum_grouped_tiled(buf, rows, MUL_W, w, 1.0, gptr, MUL_N_DIV_N, gn,
                                                   [float(N)] * len(gn), n=P, out=out)
            else:
                timed_grouped(xs, MUL_W, w, 1.0, gptr, MUL_N_DIV_N, gn, [float(N)] * len(gn), out)
            res["g"] = out
        launches = 1

    def rank_partial(r, tiles):
        """The oracle's local step of rank r: per group FedAvg, cloud term, ordered sum over its groups."""
        from oracle import orc
        terms = []
        for g in split(G, r, world):
            cols = []
            for i in range(g * M, (g + 1) * M):
                gen = torch.Generator(device=DEV).manual_seed(1000 + i)
                cols.append(flat_pick(torch.randn(P, generator=gen, device=DEV), tiles, P))
            cg = counts[g * M:(g + 1) * M]
            Gj = orc.weighted_sum(cols, 0, [c / sum(cg) for c in cg])
            terms.append(orc.weighted_sum([Gj], 1, [sum(cg)], float(N)))
        return orc.weighted_sum(terms, 2) if len(terms) > 1 else terms[0]

    def parity():
        if args.check_samples <= 0:
            return None
        from oracle import orc
        tiles = sample_tiles(P, max(1, min(args.check_samples, 8192) // 1024), 98)
        if world > 1 and (args.collective == "reduce_scatter" or
                          (rank != 0 and args.collective not in ("ordered_all", "all_reduce"))):
            tiles = []
        bad = cnt = 0
        if tiles:
            if world == 1 and tiled:  # the arena's own rows (same values as regenerating them)
                sample = list(tiled_pick(buf, tiles, P)[rows])
                terms = []
                for j in range(len(my_groups)):
                    Gj = orc.weighted_sum(sample[gptr[j]:gptr[j + 1]], 0, w[gptr[j]:gptr[j + 1]])
                    terms.append(orc.weighted_sum([Gj], 1, [gn[j]], float(N)))
                exp = orc.weighted_sum(terms, 2)
            else:
                parts = [rank_partial(r, tiles) for r in range(world)]
                exp = orc.weighted_sum(parts, 2) if world > 1 else parts[0]
            bad, cnt = count_bad(flat_pick(res["g"], tiles, P), exp), exp.numel()
        bad, cnt = sum_over_ranks(bad, world), sum_over_ranks(cnt, world)
        if world > 1 and args.collective == "reduce_scatter":
            return "not checked (reduce_scatter leaves the model sharded)"
        return (f"{'bit-exact' if bad == 0 else f'{int(bad)} elements differ'} vs oracle (group FedAvg -> cloud "
                f"term -> ordered sum{' per rank -> rank-ordered sum' if world > 1 else ''}) on {int(cnt)} sampled "
                f"elements" + (f" of {collective_note(args, world)}" if world > 1 else ""))

    return dict(loop_timing=True, name=f"hier_fedavg_G{G}x{M}_P{P}_fp32" + ("_tiled" if tiled else ""), dtype="fp32", step=step, parity=parity,
                bytes_total=G * M * P * 4 + P * 4, launch_bytes=(len(clients) * P * 4 + P * 4) / launches,
                clients=G * M, params=P, cpu_K=None)


def wl_gossip(args, eng, rank, world, timer):
    """cfg5: n = 256 nodes on a ring (W = 1/3), one synchronous DSGD step, models of ResNet-18 size.
    Value = compulsory bytes (every model read once, every mixed model written once: 2 n P s) per
    second; the survey's 4 n P s accounting counts a ring row's three reads
    separately and would exceed the HBM peak."""
    from fedml_amd.core.distributed.topology.topology_manager import SymmetricTopologyManager, gossip_rows
    n = args.clients or 256
    P = args.params or RESNET18_P
    m = SymmetricTopologyManager(n, 2)
    m.generate_topology()
    W = m.topology
    rp, cs, vs = gossip_rows(W)
    tiled = False
    res = {}
    if world > 1:
        from fedml_amd.distributed.gossip import DistributedGossip

        def timed_mix(xs_, rp_, cs_, vs_, ps, outs, outs2):
            with timer:
                return eng.mix(xs_, rp_, cs_, vs_, ps, outs, outs2)
        dg = DistributedGossip(W, local_mix=timed_mix)
        masked_stream(eng, args)
        xs = (make_arena_rows if args.layout in ("arena", "tiled") else make_flat_clients)(dg.mine, P)
        nodes = dg.mine

        def step():
            res["outs"], _ = dg.step(xs)
        rows = len(dg.mine)
    else:
        tiled = args.layout == "tiled"
        nodes = list(range(n))
        if tiled:  # both the models and the mixed models in tile-interleaved arenas (fa_mix_tiled)
            arena = make_tiled_arena(range(n), P)
            buf = arena.bufs[torch.float32]
            obuf = torch.empty_like(buf)

            def step():
                with timer:
                    eng.mix_tiled(buf, nodes, rp, cs, vs, obuf, nodes, n=P)
        else:
            xs = (make_arena_rows if args.layout == "arena" else make_flat_clients)(range(n), P)
            outs = [torch.empty(P, device=DEV) for _ in range(n)]

            def step():
                with timer:
                    eng.mix(xs, rp, cs, vs, outs=outs)
                res["outs"] = outs
        rows = n

    def parity():
        """Every node of this rank (all n at N = 1) vs the oracle's DSGD rows on sampled tiles; the
        input models are regenerated from their seeds (the in-neighbours of a rank's boundary
        nodes live on the neighbouring ranks); mismatches summed over the ranks."""
        if args.check_samples <= 0:
            return None
        from oracle import orc
        tiles = sample_tiles(P, max(1, min(args.check_samples, 16384) // 1024), 97)
        if tiled:
            sin = list(tiled_pick(buf, tiles, P)[:n])
            sout = list(tiled_pick(obuf, tiles, P)[:n])
        else:
            need = sorted({cs[j] for i in nodes for j in range(rp[i], rp[i + 1])})
            sin = {}
            for i in need:
                gen = torch.Generator(device=DEV).manual_seed(1000 + i)
                sin[i] = flat_pick(torch.randn(P, generator=gen, device=DEV), tiles, P)
            hole = torch.zeros_like(next(iter(sin.values())))  # nodes no row of this rank reads
            sin = [sin.get(i, hole) for i in range(n)]
            sout = {i: flat_pick(o, tiles, P) for i, o in zip(nodes, res["outs"])}
        # the oracle's rows of this rank's nodes only
        prp, pcs, pvs = [0], [], []
        for i in nodes:
            pcs += cs[rp[i]:rp[i + 1]]
            pvs += vs[rp[i]:rp[i + 1]]
            prp.append(len(pcs))
        exp, _ = orc.mix(sin, prp, pcs, pvs)
        bad = sum(count_bad(sout[i], e) for i, e in zip(nodes, exp))
        cnt = sum(e.numel() for e in exp)
        bad, cnt = sum_over_ranks(bad, world), sum_over_ranks(cnt, world)
        return (f"{'bit-exact' if bad == 0 else f'{int(bad)} MISMATCHES'} vs oracle (DSGD rows) on {int(cnt)} "
                f"sampled elements over all {n} nodes" + (f" ({world} ranks, halo exchange)" if world > 1 else ""))

    return dict(name=f"gossip_ring_n{n}_P{P}_fp32" + ("_tiled" if tiled else ""), dtype="fp32", step=step,
                parity=parity, bytes_total=2 * n * P * 4, launch_bytes=2 * rows * P * 4, clients=n, params=P,
                cpu_K=None, step_bytes=2 * rows * P * 4 if world > 1 else None,
                roofline_note="compulsory bytes 2*n*P*4 (each model read once, each mixed model written once); "
                              "the survey's 4*n*P*4 accounting would be 2x these figures")


def pcie_probe(nbytes=1 << 30, reps=5):
    """Pinned H2D and D2H copy rates (GB/s, best of ``reps``) of one ``nbytes`` buffer: the PCIe
    ceiling the host-path line is read against."""
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    out = {}
    for name, (dst, src) in {"h2d": (d, h), "d2h": (h, d)}.items():
        best = float("inf")
        for _ in range(reps):
            sync()
            t0 = time.perf_counter()
            dst.copy_(src, non_blocking=True)
            sync()
            best = min(best, time.perf_counter() - t0)
        out[f"pinned_{name}_GBs"] = round(nbytes / best / 1e9, 2)
    return out


def wl_host(args, eng, rank, world, timer):
    """Host path (SURVEY.md §8(d) 'Host path'; the reference receives updates into MPI / socket
    buffers, core/distributed/communication/mpi/mpi_receive_thread.py:25): client updates start in
    host memory -- pageable (as unpickled from receive buffers) or, with --pinned, already in pinned
    receive buffers -- are copied H2D into the ClientArena (pageable: packed into pinned staging on the
    way, overlapped with the next client's copy), aggregated, and the averaged model is copied back
    D2H for broadcast.  Step = ingest K clients + FedAvg + D2H; value = the aggregate's algorithmic
    bytes / that step time (the PCIe-inclusive rate, never the device-resident metric)."""
    from fedml_amd.arena import ArenaLayout, ClientArena
    from fedml_amd.engine import MUL_W
    K = args.clients or 128
    P = args.params or 16_000_000
    counts = client_counts(K)
    N = sum(counts)
    w = [c / N for c in counts]
    g = torch.Generator().manual_seed(0)
    base = torch.randn(P + K, generator=g)
    # distinct clients without K full randn passes (a metric-size run holds 64 GB of updates)
    host = [{"w": (base[i:i + P].pin_memory() if args.pinned else base[i:i + P].clone())} for i in range(K)]
    del base
    arena = ClientArena(ArenaLayout([("w", (P,), torch.float32)]), capacity=K)
    result = torch.empty(P, pin_memory=True)
    pcie = pcie_probe()

    def step():
        for i in range(K):
            arena.write(i, host[i])
        with timer:
            avg = arena.aggregate(MUL_W, w)
        result.copy_(avg["w"], non_blocking=True)
        torch.cuda.current_stream().synchronize()  # the model is on the host for broadcast

    def parity():
        """The oracle's ordered FedAvg of the HOST updates on 64 sampled 4-KiB tiles vs the host result."""
        if args.check_samples <= 0:
            return None
        from oracle import orc
        tiles = sample_tiles(P, max(1, args.check_samples // 1024), 97)
        cols = [torch.cat([h["w"][t * 1024:min((t + 1) * 1024, P)] for t in tiles]) for h in host]
        exp = orc.weighted_sum(cols, MUL_W, w)
        got = torch.cat([result[t * 1024:min((t + 1) * 1024, P)] for t in tiles])
        bad = count_bad(got, exp)
        return f"{'bit-exact' if bad == 0 else f'{bad} MISMATCHES'} vs oracle on {exp.numel()} sampled elements"

    pcie_floor_ms = ((K * P * 4) / (pcie["pinned_h2d_GBs"] * 1e9) + P * 4 / (pcie["pinned_d2h_GBs"] * 1e9)) * 1e3
    return dict(name=f"fedavg_host_ingest_{'pinned' if args.pinned else 'pageable'}_K{K}_P{P}_fp32", dtype="fp32",
                step=step, parity=parity, bytes_total=K * P * 4 + P * 4, launch_bytes=K * P * 4 + P * 4, clients=K,
                params=P, cpu_K=None,
                data=f"synthetic N(0,1) client updates in {'pinned' if args.pinned else 'pageable'} HOST memory "
                     "(client i = window i of one random vector), n_i ~ U{50..600} (seed 7)",
                extra_line={"pcie": dict(pcie, floor_ms_per_step=round(pcie_floor_ms, 2),
                                         note="K*P*4 B H2D + P*4 B D2H at the pinned copy rates")},
                roofline_note="value includes the H2D of every update (pageable: packed through pinned staging), "
                              "the aggregation and the D2H of the result; `pcie` holds this box's pinned copy rates")


def wl_fedopt(args, eng, rank, world, timer):
    """FedOpt server round (simulation/mpi/fedopt/FedOptAggregator.py:81-131, server_optimizer sgd,
    momentum 0.9): FedAvg of K client updates + pseudo-gradient g = p - avg + torch.optim.SGD step of
    the global model and its momentum buffer, fused in one pass (fa_fedavg_sgd).  Flat fp32 model,
    client-major arena rows.  Bytes per step: K*P*4 read + param r/w + momentum r/w = (K + 4)*P*4."""
    if world > 1:
        raise SystemExit("--config fedopt is a single-GPU configuration")
    K = args.clients or 128
    P = args.params or 125_000_000
    lr, mom = 1.0, 0.9
    counts = client_counts(K)
    w = [c / sum(counts) for c in counts]
    tiled = args.layout == "tiled"
    if tiled:
        arena = make_tiled_arena(range(K), P)
        buf, rows, xs = arena.bufs[torch.float32], list(range(K)), None
    else:
        xs = make_arena_rows(range(K), P)
    g = torch.Generator(device=DEV).manual_seed(5)
    param = torch.randn(P, generator=g, device=DEV)
    mbuf = torch.zeros(P, device=DEV)
    state = {"first": True}

    def run(p_, b_, first, n=None):
        if tiled:
            eng.fedavg_sgd_tiled(buf if n is None else buf[:n // buf.shape[2]], rows, w, p_, b_, lr, mom,
                                 first_step=first)
        else:
            eng.fedavg_sgd([xs if n is None else [x[:n] for x in xs]], w, [p_], [b_], lr, mom, first_step=first)

    def step():
        with timer:
            run(param, mbuf, state["first"])
        state["first"] = False

    def parity():
        if args.check_samples <= 0:
            return None
        from oracle import orc
        n = min(P, 1 << 20) // 1024 * 1024  # a fresh server state over the first n coordinates, two rounds
        p_dev = torch.randn(n, generator=torch.Generator(device=DEV).manual_seed(6), device=DEV)
        b_dev = torch.zeros(n, device=DEV)
        p_cpu, b_cpu = p_dev.cpu(), b_dev.cpu()
        cols = list(buf[:n // buf.shape[2]].cpu().permute(1, 0, 2).reshape(buf.shape[1], -1)[rows]) if tiled \
            else [x[:n].cpu() for x in xs]
        avg = orc.weighted_sum(cols, 0, w)
        for first in (True, False):
            run(p_dev, b_dev, first, n)
            orc.sgd_apply(avg, p_cpu, b_cpu, lr, mom, first_step=first)
        sync()
        ok = torch.equal(p_dev.cpu().view(torch.int32), p_cpu.view(torch.int32)) and \
            torch.equal(b_dev.cpu().view(torch.int32), b_cpu.view(torch.int32))
        return f"{'bit-exact' if ok else 'MISMATCH'} vs oracle (FedAvg + SGD momentum, 2 rounds) on {n} coordinates"

    def cpu(budget_s):
        import oracle.torch_port as tp
        Kc, Pc = K, 2_000_000
        gc = torch.Generator().manual_seed(0)
        cl = [(counts[i], {"w": torch.randn(Pc, generator=gc)}) for i in range(Kc)]
        model = torch.nn.Linear(1, 1, bias=False)
        model.weight = torch.nn.Parameter(torch.randn(Pc, generator=gc))
        opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=mom)

        def run():
            lst = [(n_, {"w": d["w"]}) for n_, d in cl]  # fresh dicts: agg() rebinds client 0's entry
            avg = tp.agg("FedAvg", lst)["w"]
            opt.zero_grad()
            model.weight.grad = model.weight.data - avg       # set_model_global_grads (:118-131)
            opt.step()
        return legs_record(timed_legs(run, budget_s), (Kc + 4) * Pc * 4,
                           f"K={Kc} x P={Pc} fp32 host-resident: oracle/torch_port.agg('FedAvg') + pseudo-gradient "
                           f"+ torch.optim.SGD(momentum={mom}) step")

    return dict(name=f"fedopt_sgd_K{K}_P{P}_fp32" + ("_tiled" if tiled else ""), dtype="fp32", step=step, parity=parity, cpu=cpu,
                bytes_total=(K + 4) * P * 4, launch_bytes=(K + 4) * P * 4, clients=K, params=P, cpu_K=K)


def wl_secagg(args, eng, rank, world, timer):
    """§8(f) #4: the LightSecAgg server reconstruction (lsa_fedml_aggregator.py:101-175) for N = K
    clients (U = N, T = N/2, the reference's setting) with ResNet-18-size models: LCC-decode the
    aggregate mask from the clients' (U x d/(U-T)) encoded-mask buffer, then sum the K masked int64
    models, cancel the mask, reduce mod p, dequantize and average -> float32.  The U x U Lagrange
    coefficients (host, O(U^2) scalars, computed once per active set) are outside the step."""
    if world > 1:
        raise SystemExit("secagg config: single GPU (the driver's multi-GPU runs use the metric config)")
    from fedml_amd.core.mpc.lightsecagg import MOD_END, gen_Lagrange_coeffs
    K = args.clients or 128
    P = args.params or RESNET18_P
    p, q = 2 ** 15 - 19, 10
    U, T = K, K // 2
    m = -(-P // (U - T))
    g = torch.Generator(device=DEV).manual_seed(11)
    tiled = args.layout == "tiled"
    if tiled:  # tile-interleaved arena [tiles, K, 512] (fedml_amd/arena.py, fa_finite_sum_tiled)
        nt = -(-P // 512)
        tbuf = torch.randint(0, p, (nt, K, 512), generator=g, dtype=torch.int64, device=DEV)
        rows = list(range(K))
        xs = None
    else:
        Ppad = -(-P // 64) * 64  # rows 512-byte aligned, as ClientArena lays them out (fedml_amd/arena.py)
        arena = torch.randint(0, p, (K, Ppad), generator=g, dtype=torch.int64, device=DEV)
        xs = [arena[i, :P] for i in range(K)]
    F = torch.randint(0, p, (U, m), generator=g, dtype=torch.int64, device=DEV)
    coef = gen_Lagrange_coeffs(np.arange(U) + K + 1, np.arange(K) + 1, p).tolist()
    state = {}

    def step():
        mask = eng.lcc_decode(coef, F, p, P)
        with timer:
            if tiled:
                _, real = eng.finite_sum_tiled(tbuf, rows, p, MOD_END, mask=mask, finite=False, q_bits=q,
                                               scale=1 / K, n=P)
            else:
                _, real = eng.finite_sum([xs], p, MOD_END, masks=[mask], finite=False, q_bits=q, scale=1 / K)
                real = real[0]
        state["mask"], state["real"] = mask, real

    def parity():
        if args.check_samples <= 0:
            return None
        from oracle import orc
        gi = torch.Generator(device=DEV).manual_seed(99)
        idx = torch.randint(0, P, (args.check_samples,), generator=gi, device=DEV)
        cols_in = ([tbuf[:, r, :].reshape(-1)[:P].index_select(0, idx).cpu() for r in rows] if tiled else
                   [x.index_select(0, idx).cpu() for x in xs])  # 1.5e9-element arena: one row at a time
        _, exp = orc.finite_sum(cols_in, p, MOD_END,
                                mask=state["mask"].index_select(0, idx).cpu(), q_bits=q, scale=1 / K)
        ok = torch.equal(state["real"].index_select(0, idx).cpu().view(torch.int32), exp.view(torch.int32))
        # the decoded mask: every column of a row block is independent -> check a sampled slice
        cols = torch.arange(0, min(m, 4096), device=DEV)
        dec = orc.lcc_decode(torch.tensor(coef, dtype=torch.int64)[: U - T], F[:, cols].cpu(), p, (U - T) * cols.numel())
        got = state["mask"].reshape(-1)
        rows_ok = all(torch.equal(got[j * m: j * m + cols.numel()].cpu(), dec[j * cols.numel():(j + 1) * cols.numel()])
                      for j in range(U - T) if j * m + cols.numel() <= P)
        return (f"{'bit-exact' if ok else 'MISMATCH'} vs oracle on {args.check_samples} sampled elements; "
                f"LCC mask {'bit-exact' if rows_ok else 'MISMATCH'} on {cols.numel()} columns x {U - T} rows")

    def cpu(budget_s):
        from oracle import secagg_port
        Kc, Pc = K, 1_000_000
        rng = np.random.RandomState(0)
        models = [{"w": rng.randint(0, p, size=Pc).astype(np.int64)} for _ in range(Kc)]
        mask = rng.randint(0, p, size=Pc).astype(np.int64)
        best, runs, t_end = float("inf"), 0, time.perf_counter() + budget_s
        while runs < 3 or (time.perf_counter() < t_end and runs < 30):
            t0 = time.perf_counter()
            secagg_port.lsa_reconstruct(models, mask, [Pc], p, q)
            best = min(best, time.perf_counter() - t0)
            runs += 1
        return {"value": round((Kc * Pc * 8 + Pc * 8 + Pc * 4) / best / 1e9, 2), "unit": "GB/s", "cores": 1,
                "kind": "port", "sample": f"K={Kc} x P={Pc} int64 masked models + mask, best of {runs} runs of "
                                          "oracle/secagg_port.lsa_reconstruct (numpy restatement of "
                                          "lsa_fedml_aggregator.py:140-166); mask decoding not included"}

    recon = K * P * 8 + P * 8 + P * 4
    return dict(name=f"lightsecagg_reconstruct_N{K}_P{P}_int64" + ("_tiled" if tiled else ""), dtype="int64", step=step, parity=parity,
                data="synthetic masked finite models uniform in Z_p (p = 2^15-19, q = 10 bits), resident in HBM",
                bytes_total=recon + U * m * 8 + P * 8, launch_bytes=recon, clients=K, params=P, cpu_K=K, cpu=cpu,
                roofline_note="dominant kernel = fa_finite_sum (K masked models + mask in, fp32 out); value also "
                              "counts the LCC mask decoding (U x m int64 in, P int64 out)")


def wl_samask(args, eng, rank, world, timer):
    """§8(f) #4, r03: SecAgg's server mask re-expansion (cross_silo/secagg/sa_fedml_aggregator.py:92-136)
    for N = K clients of ResNet-18 size: every surviving client's numpy MT19937 stream
    (np.random.seed(b_u); randint(0, p, d)) and, for each dropped client, its N - 1 pairwise streams,
    summed mod p -- fa_mt_randint_sum (jump-ahead chunks of every stream in parallel; FA_MT_JUMP=0: one
    wave per stream).  BGW decoding (a few scalars per client) is
    host work outside the step.  ``--variant`` = dropped clients (default 0).  value = latency (ms)."""
    if world > 1:
        raise SystemExit("samask config: single GPU")
    K = args.clients or 32
    P = args.params or RESNET18_P
    p = 2 ** 31 - 1
    dropped = max(0, min(K, args.variant))
    rng = np.random.RandomState(5)
    seeds, signs = [], []
    for i in range(K):
        if i >= dropped:  # model arrived: its own mask stream
            seeds.append(int(rng.randint(0, 2 ** 31 - 1)))
            signs.append(1)
        else:  # dropped: its pairwise streams, sign by index order
            for j in range(K):
                if j != i:
                    seeds.append(int(rng.randint(0, 2 ** 31 - 1)))
                    signs.append(-1 if j < i else 1)
    out = torch.empty(P, dtype=torch.int64, device=DEV)
    state = {}

    def step():
        t0 = time.perf_counter()
        with timer:
            eng.mt_randint_sum(seeds, signs, p, P, out=out)
        torch.cuda.current_stream().synchronize()
        state["out"] = out
        return time.perf_counter() - t0

    def parity():
        # every element (the jump-ahead chunks cover the whole vector): |sum| < len(seeds) * p < 2^63
        acc = np.zeros(P, dtype=np.int64)
        for s_, g_ in zip(seeds, signs):
            np.random.seed(s_)
            acc += g_ * np.random.randint(0, p, size=P).astype(np.int64)
        exp = np.mod(acc, p)
        ok = np.array_equal(out.cpu().numpy(), exp)
        return (f"{'bit-exact' if ok else 'MISMATCH'} vs numpy's own legacy streams (np.random.seed + randint, "
                f"the reference's calls) summed mod p, on all {P} elements of all {len(seeds)} streams")

    def cpu(budget_s):
        """The reference's loop body for surviving clients (seed, randint, +=, mod) on a sample of
        streams, scaled to all streams (each stream is sequential, numpy runs one at a time)."""
        ns = max(1, min(len(seeds), 4))
        t0 = time.perf_counter()
        agg = 0
        for s_ in seeds[:ns]:
            np.random.seed(s_)
            agg = np.mod(agg + np.random.randint(0, p, size=P).astype(int), p)
        dt = (time.perf_counter() - t0) / ns
        return {"value": round(dt * len(seeds) * 1e3, 2), "unit": "ms", "cores": 1, "kind": "reference",
                "sample": f"{ns} of {len(seeds)} streams of np.random.seed + np.random.randint(0, p, size={P}) + "
                          "np.mod accumulate (numpy, the reference's own calls, sa_fedml_aggregator.py:104-107), "
                          "timed and scaled to all streams"}

    return dict(name=f"secagg_mask_expand_N{K}_dropped{dropped}_P{P}_int64", dtype="u32 (MT19937) -> int64", step=step,
                parity=parity, cpu=cpu, latency=True, stat="median", clients=K, params=P, cpu_K=K, bytes_total=None,
                launch_bytes=None, metric_name=f"SecAgg mask re-expansion latency, {len(seeds)} streams x {P} draws",
                data=f"{len(seeds)} MT19937 streams (seeds from RandomState(5)), p = 2^31 - 1")


def _robust_inputs(K, P):
    Ppad = -(-P // 64) * 64  # ClientArena row alignment
    g = torch.Generator(device=DEV).manual_seed(21)
    arena = torch.randn((K, Ppad), generator=g, device=DEV)
    return [arena[i, :P] for i in range(K)]


def _robust_cpu(fn, K, Pc, budget_s, nbytes, what, digits=2):
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(Pc, generator=g) for _ in range(K)]
    return legs_record(timed_legs(lambda: fn(xs), budget_s, min_runs=2, max_runs=20), nbytes,
                       f"K={K} x P={Pc} fp32 host-resident, {what}", digits=digits)


def wl_median(args, eng, rank, world, timer):
    """§8(f) #3: coordinate-wise median (coordinate_wise_median_defense.py:18-44) of K client
    weight vectors of ResNet-18 size: one fa_coord_median launch (a selection per coordinate).
    --layout tiled (default): the clients in a tile-interleaved ClientArena (fa_coord_median_tiled,
    the layout the FedAvg kernels read at the metric's rate); arena / tensors: K rows of one
    allocation (client-major, fa_coord_median)."""
    if world > 1:
        raise SystemExit("median config: single GPU")
    K = args.clients or 32
    P = args.params or RESNET18_P
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[args.dtype]
    xs = _robust_inputs(K, P)
    if dt != torch.float32:
        Ppad = -(-P // 64) * 64
        arena = torch.empty((K, Ppad), dtype=dt, device=DEV)
        for i, x in enumerate(xs):
            arena[i, :P].copy_(x)
        xs = [arena[i, :P] for i in range(K)]
    tiled = args.layout == "tiled"
    if tiled:
        from fedml_amd.arena import ArenaLayout, ClientArena
        ta = ClientArena(ArenaLayout([("w", (P,), dt)]), capacity=K, zero=False, tiled=True)
        for i, x in enumerate(xs):
            ta.write(i, {"w": x})
        sync()
        ta._scratch.clear()
        buf, rows = ta.bufs[dt], list(range(K))
    es = xs[0].element_size()
    ibits = {4: torch.int32, 2: torch.int16}[es]
    out = torch.empty(P, dtype=dt, device=DEV)

    def step():
        with timer:
            if tiled:
                eng.coord_median_tiled(buf, rows, n=P, out=out)
            else:
                eng.coord_median([xs], outs=[out])

    def parity():
        if args.check_samples <= 0:
            return None
        from oracle import orc
        gi = torch.Generator(device=DEV).manual_seed(99)
        idx = torch.randint(0, P, (args.check_samples,), generator=gi, device=DEV)
        exp = orc.coord_median([x.index_select(0, idx).cpu() for x in xs])
        ok = torch.equal(out.index_select(0, idx).cpu().view(ibits), exp.view(ibits))
        return f"{'bit-exact' if ok else 'MISMATCH'} vs oracle on {args.check_samples} sampled coordinates"

    def cpu(budget_s):
        from oracle import robust_port
        Pc = 1_000_000
        return _robust_cpu(robust_port.median_port, K, Pc, budget_s, K * Pc * 4 + Pc * 4,
                           "oracle/robust_port.median_port (cat + torch.median, coordinate_wise_median_defense.py:26-31)")

    return dict(loop_timing=True, name=f"coord_median_K{K}_P{P}_{args.dtype}" + ("_tiled" if tiled else ""), dtype=args.dtype,
                probe=(buf, buf.shape[1], f"this workload's tiled arena group ({buf.shape[1]} consecutive 4-KiB rows "
                       "per workgroup)") if tiled else None,
                step=step, parity=parity,
                bytes_total=(K * P + P) * es, launch_bytes=(K * P + P) * es, clients=K, params=P, cpu_K=K, cpu=cpu,
                data="synthetic N(0,1) client weight vectors, resident in HBM (" +
                     ("tile-interleaved ClientArena rows)" if tiled else "rows 256-byte aligned)"))


def wl_krum(args, eng, rank, world, timer):
    """§8(f) #3: Krum's pairwise squared distances (krum_defense.py:52-66) of K client weight
    vectors of ResNet-18 size: one fa_pairwise_sqdist pass (each client read once)."""
    if world > 1:
        raise SystemExit("krum config: single GPU")
    K = args.clients or 32
    P = args.params or RESNET18_P
    xs = _robust_inputs(K, P)
    state = {}

    def step():
        with timer:
            state["D"] = eng.pairwise_sqdist([xs])

    def parity():
        if args.check_samples <= 0:
            return None
        from oracle import orc
        # the last timed step's distances over the WHOLE model vs the exact oracle (every pair)
        D = state["D"].cpu()
        ref = orc.pairwise_sqdist([x.cpu() for x in xs])
        off = ~torch.eye(K, dtype=torch.bool)
        err = float(((D - ref).abs()[off] / ref[off].clamp_min(1e-300)).max())
        return (f"max relative error {err:.2e} vs the exact float64 oracle over every pair and all {P} coordinates "
                f"(tolerance 1e-6)")

    def cpu(budget_s):
        from oracle import robust_port
        Pc = 1_000_000
        Kc = min(K, 16)
        return _robust_cpu(robust_port.krum_distances_port, Kc, Pc, budget_s, Kc * Pc * 4,
                           "oracle/robust_port.krum_distances_port (one (v_i - v_j).norm() per ordered pair, "
                           "krum_defense.py:52-66)", digits=3)

    pairs = K * (K - 1) // 2
    extra = {}

    def parity_and_form():
        p = parity()
        extra["pair_form"] = getattr(eng, "last_pair_form", None)
        extra["kappa_max"] = getattr(eng, "last_kappa_max", None)
        extra["pair_form_note"] = ("gram: D = A_i + A_j - 2 G_ij on the matrix cores (fa_pairwise_sqdist_gram), kept "
                                   "when kappa_max <= 16; direct: the VALU difference kernel")
        return p
    return dict(loop_timing=True, name=f"krum_pairdist_K{K}_P{P}_fp32", dtype="fp32", step=step, parity=parity_and_form,
                extra_line=extra,
                bytes_total=K * P * 4, launch_bytes=K * P * 4, clients=K, params=P, cpu_K=K, cpu=cpu,
                data="synthetic N(0,1) client weight vectors, resident in HBM (rows 256-byte aligned)",
                mfma_flops_per_launch=K * (K + 1) * P, mfma_bound=K > 32,
                roofline_note=(f"Gram form (float32 default): G = Y Y^T on the f32 MFMA, K (K + 1) P = "
                               f"{K * (K + 1) * P / 1e9:.1f} GFLOP per launch (the upper triangle incl. the "
                               "diagonal); K <= 32 the read bounds it (each client read once), K > 32 the "
                               f"matrix cores; the direct form: {pairs} pairs x 3 flop per coordinate"))


# ----------------------------------------------------------------------------- CPU baseline
def cpu_quota():
    """CPUs this process may actually use: the affinity mask and the cgroup CFS quota (cpu.max);
    on a one-GPU box os.cpu_count() shows the whole machine while the quota is the box's share."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_thread_legs():
    """SURVEY.md §8(d) asks for the CPU baseline on ALL the host's cores (torch.set_num_threads(
    os.cpu_count()), overriding the box's OMP_NUM_THREADS=16).  That leg is run and recorded; so are
    the CPU quota the process really has (cgroup cpu.max / affinity) and 16 threads.  A one-GPU box
    shows all 256 cores but grants a 16-CPU share, where 256 threads collapse (0.07 GB/s measured,
    profiles/r02a_bench.json): the reported value is the best leg, with its thread count."""
    return sorted({os.cpu_count() or 1, cpu_quota(), min(16, os.cpu_count() or 1)}, reverse=True)


def timed_legs(fn, budget_s, min_runs=3, max_runs=50, small=None):
    """Best-of wall time per thread leg: {threads: (best_s, runs, scale)}.  Legs with more threads
    than the CPU quota run ONCE, on ``small()`` = (fn, scale) when given (a scaled-down sample: an
    oversubscribed run of the full sample takes ~30 s)."""
    out = {}
    quota = cpu_quota()
    legs = sorted(cpu_thread_legs())
    for th in legs:
        torch.set_num_threads(th)
        f, scale, lo, hi = fn, 1.0, min_runs, max_runs
        if th > quota:
            if small is None:  # an oversubscribed full-size run takes minutes (138 s measured, r02b)
                continue
            lo = hi = 1
            f, scale = small()
        best, runs, t_end = float("inf"), 0, time.perf_counter() + budget_s / len(legs)
        while runs < lo or (time.perf_counter() < t_end and runs < hi):
            t0 = time.perf_counter()
            f()
            best = min(best, time.perf_counter() - t0)
            runs += 1
        out[th] = (best, runs, scale)
    torch.set_num_threads(min(16, quota))
    return out


def legs_record(legs, nbytes, sample, kind="port", digits=2):
    """The best thread-count leg is the reported value (``cores`` = its threads); every leg's rate
    is kept, the all-core one included (see cpu_thread_legs)."""
    rates = {th: nbytes * sc / b / 1e9 for th, (b, _, sc) in legs.items()}
    rates = {th: round(r, digits if r >= 1 else 5) for th, r in rates.items()}
    best = max(rates, key=lambda th: rates[th])
    byth = {str(th): r for th, r in sorted(rates.items())}
    for th in cpu_thread_legs():
        byth.setdefault(str(th), "not run: oversubscribed past the CPU quota (the metric line records it)")
    return {"value": rates[best], "unit": "GB/s", "cores": best, "kind": kind,
            "value_by_threads": byth,
            "os_cpu_count": os.cpu_count(), "cpu_quota": cpu_quota(),
            "sample": sample + f", best of {legs[best][1]} runs per thread count"}


def cpu_baseline(K, budget_s):
    """The reference's CPU cost: oracle/torch_port.py (op-for-op restatement of agg_operator.py's
    FedAvg loop) on host-resident tensors, K clients x a bounded P, best of several runs, on all
    cores and on 16 threads."""
    from oracle import torch_port
    P = 4_000_000
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(P, generator=g) for _ in range(K)]
    counts = client_counts(K)
    raw = [(counts[i], {"w": xs[i]}) for i in range(K)]

    def small():  # 1/16 of the sample for the oversubscribed all-core leg
        r = [(c, {"w": x[:P // 16]}) for c, x in zip(counts, xs)]
        return (lambda: torch_port.agg("FedAvg", r)), 1 / 16
    legs = timed_legs(lambda: torch_port.agg("FedAvg", raw), budget_s, small=small)
    rec = legs_record(legs, K * P * 4 + P * 4,
                      f"K={K} x P={P} fp32 host-resident, oracle/torch_port.agg('FedAvg') "
                      f"(op-for-op restatement of agg_operator.py:35-44)")
    rec.update(cpu_model=cpu_model(), os_cpu_count=os.cpu_count())
    return rec


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def read_ceiling(eng, wl, reps=5):
    """THIS box's read ceiling, measured in this process before the timed region (never inside it):
    fa_read_probe streams the workload's own tiled arena group -- the same pages, in the same
    per-workgroup row runs (K consecutive 4-KiB rows) as the aggregation kernel reads them, with no
    arithmetic and no output stream -- or, for workloads without a tiled arena, a 8 GiB scratch
    allocation in runs of 128 rows.  Best and median of ``reps`` HIP-event-timed passes (one untimed
    pass first) on the stream the probe is launched on."""
    spec = wl.get("probe")
    scratch = None
    if spec is None:
        scratch = torch.empty(8 << 30, dtype=torch.uint8, device=DEV)
        spec = (scratch, 128, "8 GiB scratch allocation, runs of 128 rows")
    buf, rows, what = spec
    nbytes = (buf.numel() * buf.element_size()) // 4096 * 4096
    st = torch.cuda.current_stream()
    eng.read_probe(buf, rows)
    ms = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        eng.read_probe(buf, rows)
        b.record(st)
        b.synchronize()
        ms.append(a.elapsed_time(b))
    del scratch
    best, med = min(ms), float(np.median(ms))
    return {"value": round(nbytes / (best * 1e-3) / 1e9, 1), "median": round(nbytes / (med * 1e-3) / 1e9, 1),
            "unit": "GB/s", "bytes": int(nbytes), "reps": reps, "buffer": what,
            "probe": "fa_read_probe (include/fedagg.h): the weighted-sum kernel's tiled read pattern, no arithmetic, "
                     "no output stream; run in this process after the warmup, before the timed steps"}


def cold_calls(wl, reps, idle_s):
    """The per-round latency the reference pays (python/fedml/cross_silo/server/
    fedml_server_manager.py:184-195 times ONE aggregation after the server has waited for every
    client): ``reps`` single calls, each after ``idle_s`` of idle, wall time from the call to its
    completion (median reported), and the HIP-event time of the call's GPU work beside it."""
    wall, ev = [], []
    for _ in range(reps):
        sync()
        time.sleep(idle_s)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        wl["step"]()
        b.record()
        sync()
        wall.append((time.perf_counter() - t0) * 1e3)
        ev.append(a.elapsed_time(b))
    return {"ms": round(float(np.median(wall)), 4), "event_ms": round(float(np.median(ev)), 4),
            "all_ms": [round(x, 4) for x in wall], "idle_s": idle_s, "reps": reps,
            "note": "one call after idle (median of reps; wall time incl. launch and completion) -- the reference's "
                    "per-round AggregationTime case; `ms_per_step` is the back-to-back rate at the sustained clock"}


class ClockSampler:
    """The clocks, power and temperature this process's GPU ran at, sampled by a thread every
    ``period`` s from the SMU's gpu_metrics table through amdsmi (sysfs reads: no HIP call) while a
    region runs -- so that a slow line can be told apart as a slower clock (DVFS, power or thermal
    limits) or a slower memory path at the same clock.  Never raises: a box where amdsmi cannot read
    the table gets {"error": ...} in the line."""

    def __init__(self, device_index: int, period: float = 0.01):
        self.period, self.h, self.err, self.amdsmi = period, None, None, None
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self.amdsmi = amdsmi
            p = torch.cuda.get_device_properties(device_index)
            want = (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
            for h in amdsmi.amdsmi_get_processor_handles():
                dom, bus, rest = amdsmi.amdsmi_get_gpu_device_bdf(h).split(":")
                if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
                    self.h = h
            if self.h is None:
                self.err = f"no amdsmi handle with PCI {want}"
        except Exception as e:  # no library, no permission, no table
            self.err = f"{type(e).__name__}: {e}"[:200]

    def _one(self):
        m = self.amdsmi.amdsmi_get_gpu_metrics_info(self.h)

        def num(v):
            return float(v) if isinstance(v, (int, float)) else None
        xcd = [float(v) for v in (m.get("current_gfxclks") or []) if isinstance(v, (int, float)) and v > 0] \
            if isinstance(m.get("current_gfxclks"), list) else []
        return {"gfx_mhz": sum(xcd) / len(xcd) if xcd else num(m.get("current_gfxclk")) or
                num(m.get("average_gfxclk_frequency")),
                "mem_mhz": num(m.get("current_uclk")), "power_w": num(m.get("current_socket_power")),
                "hotspot_c": num(m.get("temperature_hotspot")), "hbm_c": num(m.get("temperature_mem")),
                "throttle": m.get("indep_throttle_status") if m.get("indep_throttle_status") not in (None, "N/A")
                else m.get("throttle_status")}

    def __enter__(self):
        import threading
        self.samples, self.stop_ev = [], threading.Event()
        if self.h is None:
            return self

        def run():
            while not self.stop_ev.is_set():
                try:
                    self.samples.append(self._one())
                except Exception as e:
                    self.err = f"{type(e).__name__}: {e}"[:200]
                    return
                self.stop_ev.wait(self.period)
        self.th = threading.Thread(target=run, daemon=True)
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop_ev.set()
        if self.h is not None:
            self.th.join(1.0)
        return False

    def sample_now(self) -> dict:
        """One reading, synchronously (outside any timed region)."""
        if self.h is None:
            return {"error": self.err or "no handle"}
        try:
            r = self._one()
        except Exception as e:
            return {"error": f"{type(e).__name__}: {e}"[:200]}
        return {k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items() if v is not None}

    @staticmethod
    def maybe(s):
        """``s`` as a context manager, or a no-op one yielding None."""
        import contextlib
        return s if s is not None else contextlib.nullcontext()

    def summary(self):
        if not self.samples:
            return {"error": self.err or "no samples"}
        out = {"samples": len(self.samples), "period_s": self.period, "source": "amdsmi gpu_metrics"}
        for k in ("gfx_mhz", "mem_mhz", "power_w", "hotspot_c", "hbm_c"):
            v = [s[k] for s in self.samples if s[k] is not None]
            if v:
                out[k] = {"median": round(float(np.median(v)), 1), "min": round(min(v), 1), "max": round(max(v), 1)}
        th = [s["throttle"] for s in self.samples if s["throttle"] not in (None, "N/A")]
        if th:
            out["throttle_frac"] = round(sum(1 for t in th if t) / len(th), 3)
        return out


def pmc_traffic(workload):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py), if any."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            return json.load(f).get(workload, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def roofline_block(wl, world, value, unit, achieved, kernel_ms, launch_bytes):
    """The line's ``roofline`` object.  N = 1: the dominant kernel's algorithmic bytes per launch over
    its HIP-event-timed average duration, against one GPU's 8 TB/s.  N > 1: the
    WHOLE step -- local partials plus the cross-GPU exchange -- as aggregate GB/s (``value``) against
    N x 8 TB/s; the per-rank local-kernel rate is kept beside it under ``local_kernel``.  ``traffic``
    is the HBM bytes per launch of the committed rocprofv3 PMC run of this workload (not measured in
    this run; ``traffic_source`` names the file), or null."""
    traffic = pmc_traffic(wl["name"])
    local = {"achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
             "kernel_avg_ms": round(kernel_ms, 4) if kernel_ms else None,
             "algorithmic_bytes_per_launch": int(launch_bytes) if launch_bytes else None}
    block = {"bound": "hbm"}
    if world == 1:
        block.update(local)
    else:
        peak = world * HBM_PEAK_GBS
        block.update({"achieved": round(value, 1) if unit == "GB/s" else None, "peak": peak, "unit": "GB/s",
                      "frac": round(value / peak, 4) if unit == "GB/s" else None,
                      "definition": "whole step (local partials + exchange): aggregate GB/s / (N x 8 TB/s), "
                                    "SURVEY.md 8(d)",
                      "local_kernel": dict(local, definition="one rank's local-partial kernels: its algorithmic "
                                                             "bytes / their summed HIP-event time / 8 TB/s")})
    block["traffic"] = traffic
    block["traffic_source"] = ("profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE/WRITE_SIZE of a separate "
                               "profiling run of this workload, not measured in this run)" if traffic else None)
    return block


# ----------------------------------------------------------------------------- main
def cpu_probe(args):
    """FEDML_AMD_BENCH_CPU_PROBE=1 (tests only, no GPU): each launched rank joins a gloo group,
    sums its rank over the group and rank 0 prints one JSON line -- exercises the self-launch path
    (launch_ranks) end to end on a CPU container."""
    import datetime

    import torch.distributed as dist
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=args.pg_timeout))
    t = torch.tensor([float(rank)])
    dist.all_reduce(t)
    if os.environ.get("FEDML_AMD_BENCH_CPU_PROBE_FAIL_RANK") == str(rank):
        raise SystemExit(3)
    if os.environ.get("FEDML_AMD_BENCH_CPU_PROBE_HANG_RANK") == str(rank):
        stage = Stage(rank, args.stage_timeout)
        stage("probe hang")
        time.sleep(3600)
    if rank == 0:
        print(json.dumps({"metric": "cpu probe", "n_gpus": world, "rank_sum": float(t.item())}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    if (args.gpus > 1 or args.self_launch) and "WORLD_SIZE" not in os.environ:
        # no outer launcher: start the N ranks as child processes before anything touches the GPU
        if os.environ.get("FEDML_AMD_BENCH_REHEARSAL") not in ("1", "cpu") and not os.environ.get("FEDML_AMD_BENCH_CPU_PROBE"):
            have = visible_gpu_count()  # sysfs / device nodes only: no HIP call in the parent
            if have is not None and have < args.gpus:  # None: could not tell -- the ranks then report
                raise SystemExit(f"--gpus {args.gpus}: only {have} HIP device(s) visible "
                                 "(FEDML_AMD_BENCH_REHEARSAL=1 rehearses the N-rank path on one device over gloo)")
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout))
    if os.environ.get("FEDML_AMD_BENCH_CPU_PROBE"):
        return cpu_probe(args)
    rank, world, local = init_dist(args)
    stage = Stage(rank, args.stage_timeout)
    stage("setup")
    if CPU_REHEARSAL:
        spec = os.environ.get("FEDML_AMD_BENCH_ENGINE")
        if not spec:
            raise SystemExit("FEDML_AMD_BENCH_REHEARSAL=cpu needs FEDML_AMD_BENCH_ENGINE=module:factory (a test's "
                             "local-reduction stand-in); the product engine is HIP-only")
        import importlib
        mod, fn = spec.split(":")
        eng = getattr(importlib.import_module(mod), fn)()
    else:
        from fedml_amd.engine import get_engine
        eng = get_engine(local)
    if args.variant:
        eng.set_variant(args.variant)
    timer = Timed()
    wl = {"metric": wl_metric, "fragmented": wl_fragmented, "resnet18": wl_layout, "vit_bf16": wl_layout, "hier": wl_hier,
          "gossip": wl_gossip, "host": wl_host, "secagg": wl_secagg, "fedopt": wl_fedopt, "dropin_cpu": wl_dropin_cpu, "median": wl_median,
          "krum": wl_krum, "arrival": wl_arrival, "lr": wl_lr, "samask": wl_samask}[args.config](args, eng, rank, world,
                                                                                               timer)

    timer.loop = bool(wl.get("loop_timing")) and world == 1 and not args.loopback
    # amdsmi's init takes ~0.1 s: before the warmup, so that it never leaves the GPU idle (and its
    # clocks and power down) right before the timed steps (r06af)
    clk = None if CPU_REHEARSAL or args.no_clock or rank != 0 or wl.get("latency") else ClockSampler(local)
    auto_warmup = args.warmup is None
    if auto_warmup:
        args.warmup = 3
    for i in range(args.warmup):
        stage(f"warmup step {i}")
        wl["step"]()
    sync()
    if auto_warmup and world == 1 and not wl.get("latency"):
        # the chip raises its clock over the first part of sustained work (r05t): keep warming up until
        # ~1 s of this workload's own steps have run (r06c: median K = 128 still ran 1.18 ms per step
        # after 0.2 s of them, 0.98 ms over a 3 s soak)
        t_w = time.perf_counter()
        wl["step"]()
        sync()
        one = max(time.perf_counter() - t_w, 1e-6)
        extra = min(5000, int(1.0 / one))
        for i in range(extra):
            stage(f"warmup step {args.warmup + 1 + i}")
            wl["step"]()
        sync()
        args.warmup += 1 + extra
    ceiling = None
    if world == 1 and not CPU_REHEARSAL and not args.no_read_probe and not wl.get("latency"):
        stage("read probe")
        with ClockSampler.maybe(clk) as cs:
            ceiling = read_ceiling(eng, wl)
        if cs is not None:
            ceiling["clock"] = cs.summary()
    # one clock sample on each side of the timed steps, none inside them: a sampler thread's Python
    # work holds the GIL for ~1-2 ms per sample and slowed host-bound short lines (r06ah), and a sample
    # takes ~1-5 ms -- this one goes before the re-warm, the other after the wall clock stops (r06aj)
    clk_edges = [clk.sample_now()] if clk is not None else None
    if auto_warmup and world == 1 and not wl.get("latency"):
        # ~0.2 s of the workload's own steps, each waited for, right before the timed ones: the timed
        # steps then start on a busy GPU (r06ae / r06af / r06ag: after the probe or any idle gap,
        # Krum K = 64 ran 0.74-1.29 ms per timed step against 0.65-0.68 sustained; with this, 0.69-0.71)
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < 0.2:
            wl["step"]()
            sync()
            args.warmup += 1
    stage("barrier before the timed steps")
    barrier(world)
    sync()
    timer.start()
    stage("timed steps")
    t0 = time.perf_counter()
    lat = []
    for _ in range(args.steps):
        lat.append(wl["step"]())
    timer.end()
    sync()
    barrier(world)
    sync()
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    if clk_edges is not None:  # (after the clock stops: a sample takes ~1-5 ms, r06aj)
        clk_edges.append(clk.sample_now())
    timer.stop()
    sustained = None
    if args.soak_seconds > 0 and world == 1 and not wl.get("latency") and wl.get("bytes_total"):
        stage("soak")
        n_soak = 0
        sync()
        t_s = time.perf_counter()
        while time.perf_counter() - t_s < args.soak_seconds:
            for _ in range(max(1, args.steps)):
                wl["step"]()
            sync()
            n_soak += max(1, args.steps)
        dt_s = time.perf_counter() - t_s
        sustained = {"seconds": round(dt_s, 2), "steps": n_soak,
                     "value": round(wl["bytes_total"] * n_soak / dt_s / 1e9, 2), "unit": "GB/s",
                     "ms_per_step": round(dt_s / n_soak * 1e3, 4),
                     "note": "the same step repeated after the timed region (not part of `value`)"}
    cold = None
    if args.cold_reps > 0 and world == 1 and not CPU_REHEARSAL:
        stage("cold calls")
        cold = cold_calls(wl, args.cold_reps, args.cold_idle)
    stage("parity check")
    ms_per_step = elapsed / args.steps * 1e3
    if wl.get("latency"):  # the step returns its own latency (s); value = mean (or median) latency in ms
        value = float(np.median(lat) if wl.get("stat") == "median" else np.mean(lat)) * 1e3
        unit, hib = "ms", False
    else:
        value, unit, hib = wl["bytes_total"] * args.steps / elapsed / 1e9, "GB/s", True

    kernel_ms = timer.avg_ms()
    launch_bytes = wl["launch_bytes"]
    if wl.get("step_bytes"):  # several launches per step: this rank's bytes over the summed kernel time
        kernel_ms, launch_bytes = timer.per_step_ms(args.steps), wl["step_bytes"]
    elif launch_bytes is None and kernel_ms and wl.get("bytes_total"):  # layout configs: the whole call per step
        launch_bytes = wl["bytes_total"] / world
    achieved = launch_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms and launch_bytes else None
    parity = wl["parity"]()
    cpu = None
    stage("cpu baseline")
    if rank == 0 and world == 1 and not args.no_cpu_baseline and wl.get("cpu_K"):
        cpu = wl["cpu"](args.cpu_seconds) if wl.get("cpu") else cpu_baseline(wl["cpu_K"], args.cpu_seconds)
        cpu.setdefault("cpu_model", cpu_model())
        cpu.setdefault("os_cpu_count", os.cpu_count())

    if rank == 0:
        line = {
            "metric": METRIC if args.config == "metric" else wl.get("metric_name",
                                                                     f"device-resident aggregate GB/s, {wl['name']}"),
            "value": round(value, 4 if unit == "ms" else 2),
            "unit": unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": hib,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": wl["dtype"],
            "data": wl.get("data", "synthetic N(0,1) client updates (seeds 1000+i), n_i ~ U{50..600} (seed 7); "
                                   "resident in HBM"),
            "config": {"workload": wl["name"], "clients": wl["clients"], "params_per_client": wl["params"],
                       "parallelism": f"client-groups x{world}" +
                                      (f", {args.collective} over "
                                       f"{'gloo (CPU rehearsal, injected local reductions)' if CPU_REHEARSAL else 'gloo (one-GPU rehearsal)' if os.environ.get('FEDML_AMD_BENCH_REHEARSAL') else 'RCCL'}"
                                       + (" (native fa_group_reduce)" if timer.natives else " (torch.distributed)")
                                       + f" in {args.chunks} chunks"
                                       + (f", local partials on {args.cu_mask} CUs" if args.cu_mask and not CPU_REHEARSAL else "")
                                       + (", loopback (own pieces through RCCL self send/recv)" if args.loopback
                                          else "")
                                       if world > 1 or args.loopback else ""),
                       "kernel_variant": args.variant, "layout": args.layout,
                       "arena_alloc": "/".join(sorted(ARENA_ALLOC)) or None,
                       "arena_placement": ARENA_PLACEMENT or None},
            "roofline": roofline_block(wl, world, value, unit, achieved, kernel_ms, launch_bytes),
            "cpu_baseline": cpu,
            "parity": parity,
        }
        if wl.get("roofline_note"):
            line["roofline"]["note"] = wl["roofline_note"]
        if ceiling is not None:
            rl = line["roofline"]
            rl["measured_read_ceiling"] = ceiling
            if rl.get("unit") == "GB/s" and rl.get("achieved"):
                rl["frac_of_ceiling"] = round(rl["achieved"] / ceiling["value"], 4)
        if cold is not None:
            line["cold"] = cold
        if clk_edges is not None:
            line["clock"] = {"before_timed_steps": clk_edges[0], "after_timed_steps": clk_edges[1],
                             "note": "before: ahead of the 0.2 s re-warm; after: once the wall clock stopped",
                             "source": "amdsmi gpu_metrics (rank 0's GPU); the read probe's own samples are "
                                       "under roofline.measured_read_ceiling.clock"}
        line.update(wl.get("extra_line", {}))
        mf = wl.get("mfma_flops_per_launch")
        if mf and world == 1 and kernel_ms and line.get("pair_form") == "gram" and wl.get("mfma_bound"):
            # Krum's Gram form past K = 32 is matrix-core work: the bound is the f32 MFMA peak, the HBM
            # figures stay beside it
            rl = line["roofline"]
            hbm = {k: rl.get(k) for k in ("achieved", "peak", "unit", "frac", "frac_of_ceiling")}
            rl.pop("frac_of_ceiling", None)
            tfs = mf / (kernel_ms * 1e-3) / 1e12
            rl.update({"bound": "mfma", "achieved": round(tfs, 2), "peak": MFMA_F32_PEAK_TFS, "unit": "TFLOP/s",
                       "frac": round(tfs / MFMA_F32_PEAK_TFS, 4), "algorithmic_flops_per_launch": int(mf),
                       "hbm": hbm})
        if CPU_REHEARSAL:
            line["rehearsal"] = ("CPU: bench.py's N-rank code path over gloo with a test's injected local reductions "
                                 "(tests/rehearsal_engine.py) -- checks the exchange, not a measurement")
            line["data"] = "synthetic N(0,1) client updates (CPU generator, seeds 1000+i), host memory"
        if sustained is not None:
            line["sustained"] = sustained
        if wl.get("latency"):
            line["latency_ms"] = {"mean": round(float(np.mean(lat)) * 1e3, 4),
                                  "median": round(float(np.median(lat)) * 1e3, 4),
                                  "min": round(min(lat) * 1e3, 4), "max": round(max(lat) * 1e3, 4)}
            line["roofline"] = None  # a latency, not one kernel's rate
            if wl.get("extra", {}).get("b2b_ms") is not None:  # all K updates arriving at once
                line["latency_ms"]["all_arrive_at_once"] = wl["extra"]["b2b_ms"]
        print(json.dumps(line), flush=True)
    stage("teardown")
    if world > 1 or args.loopback:
        import torch.distributed as dist
        barrier(world)  # nobody closes its connections while a peer still finishes its last operation
        from fedml_amd.distributed import group_reduce
        group_reduce.release_groups()  # our extra communicators go before the default group, not at exit
        dist.destroy_process_group()
    stage.done()


if __name__ == "__main__":
    main()
