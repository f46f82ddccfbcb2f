#!/usr/bin/env python
"""Tool: pure host cost per launch (tiny n, so the GPU never throttles the host)."""
import json, os, socket, sys, time
import torch, torch.distributed as dist
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.distributed.group_reduce import GroupReducer  # noqa: E402
from fedml_amd.engine import MUL_W, get_engine  # noqa: E402
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
eng = get_engine(0)
K, E = 16, 1024
buf = torch.zeros(64, K, E, device="cuda")
rows, w = list(range(K)), [1.0 / K] * K
out = torch.empty(64 * E, device="cuda")
res = {}
def t(fn, R=200):
    for _ in range(10): fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(R): fn()
    dt = (time.perf_counter() - t0) / R
    torch.cuda.synchronize()
    return round(dt * 1e6, 1)
res["weighted_sum_tiled_us"] = t(lambda: eng.weighted_sum_tiled(buf, rows, MUL_W, w, n=8 * E, out=out[:8 * E]))
res["weighted_sum_tiled_multi8_us"] = t(lambda: eng.weighted_sum_tiled_multi(buf, rows, MUL_W, w, 1.0,
    [(i * 8 * E, (i + 1) * 8 * E) for i in range(8)], [out[i * 8 * E:(i + 1) * 8 * E] for i in range(8)]))
ev = lambda: torch.cuda.Event(enable_timing=True).record()
res["event_record_us"] = t(ev)
ms = eng.cu_masked_stream(192)
def ctx():
    with torch.cuda.stream(ms):
        pass
res["stream_ctx_us"] = t(ctx)
for coll in ("reduce_scatter", "reduce"):
    red = GroupReducer(collective=coll, chunks=8, stream=ms)
    res[f"step_{coll}_8chunks_us"] = t(lambda: red.fedavg_tiled(eng, buf, rows, w, 64 * E, out=out), R=50)
x = torch.zeros(1024, device="cuda")
res["dist_reduce_async_us"] = t(lambda: dist.reduce(x, 0, async_op=True).wait())
print(json.dumps(res))
dist.destroy_process_group()
