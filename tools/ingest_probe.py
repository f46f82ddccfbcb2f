"""Cost of ingesting DEVICE-produced client updates into the arenas: ClientArena.write of
K flat fp32 updates of P elements, tiled vs client-major, HIP-event timed; bytes moved per client
= 2 P s (read the update, write the row) for both after the direct tile scatter."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from fedml_amd.arena import ArenaLayout, ClientArena  # noqa: E402

K, P = 16, 125_000_000
x = torch.randn(P, device="cuda")
res = {}
for tiled in (False, True):
    a = ClientArena(ArenaLayout([("w", (P,), torch.float32)]), K, zero=False, tiled=tiled)
    a.write(0, {"w": x})
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(K):
        a.write(i, {"w": x})
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / K
    res["tiled" if tiled else "client_major"] = {"ms_per_client": round(ms, 4),
                                                  "GBs_2Ps": round(2 * P * 4 / ms / 1e6, 1)}
    del a
    torch.cuda.empty_cache()
print(json.dumps(res))
