#!/usr/bin/env python
"""Tool: one rank's N = 8 step (GroupReducer.fedavg_tiled over K = 16 x 125 M, world 1 over RCCL so
the collectives are skipped): wall time per step vs GPU time (events on the reducer's stream) vs
the bare kernels -- where do the extra microseconds go?"""
import json, os, socket, sys, time
import torch, torch.distributed as dist
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_tiled_arena  # noqa: E402
from fedml_amd.distributed.group_reduce import GroupReducer  # noqa: E402
from fedml_amd.engine import get_engine  # noqa: E402
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
eng = get_engine(0)
K, P = 16, 125_000_000
arena = make_tiled_arena(range(K), P)
buf, rows, w = arena.bufs[torch.float32], list(range(K)), [1.0 / K] * K
res = {}
masked = eng.cu_masked_stream(192)  # ONE masked stream, as in bench.py (HIP multiplexes streams on 4 HW queues)
for coll in ("reduce_scatter", "reduce"):
    for chunks in (1, 8):
        for mask in (0, 192):
            st = masked if mask else None
            red = GroupReducer(collective=coll, chunks=chunks, stream=st)
            out = torch.empty(P + 8 * 1024, device="cuda")
            for _ in range(3):
                red.fedavg_tiled(eng, buf, rows, w, P, out=out)
            torch.cuda.synchronize()
            R = 20
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            a.record()
            for _ in range(R):
                red.fedavg_tiled(eng, buf, rows, w, P, out=out)
            b.record()
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / R * 1e3
            res[f"{coll}_c{chunks}_cu{mask}"] = {"wall_ms": round(wall, 3), "gpu_ms": round(a.elapsed_time(b) / R, 3)}
# the bench's N > 1 arrangement: the masked stream is torch's current stream for the whole run
torch.cuda.synchronize()
torch.cuda.set_stream(masked)
for coll in ("reduce_scatter", "reduce"):
    red = GroupReducer(collective=coll, chunks=8)
    out = torch.empty(P + 8 * 1024, device="cuda")
    for _ in range(3):
        red.fedavg_tiled(eng, buf, rows, w, P, out=out)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for _ in range(20):
        red.fedavg_tiled(eng, buf, rows, w, P, out=out)
    b.record()
    torch.cuda.synchronize()
    res[f"{coll}_c8_current_masked"] = {"wall_ms": round((time.perf_counter() - t0) / 20 * 1e3, 3),
                                        "gpu_ms": round(a.elapsed_time(b) / 20, 3)}
print(json.dumps(res))
dist.destroy_process_group()
