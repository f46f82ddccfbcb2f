import sys, time, torch, json
sys.path.insert(0, '.')
import bench
from fedml_amd import _host
from collections import OrderedDict
lay = bench.load_layout('resnet18_gn')
ds = [OrderedDict((n, torch.zeros(s, dtype=getattr(torch, dt), device='cuda')) for n, s, dt in lay) for _ in range(32)]
keys = list(ds[0].keys())
res = {}
for _ in range(3):
    t = time.perf_counter()
    for _ in range(50): r = _host.gather(ds, keys)
    res['gather_us'] = (time.perf_counter() - t) / 50 * 1e6
    ptrs, numel, codes, shapes, dev = r
    t = time.perf_counter()
    for _ in range(50): _host.alloc_outputs(shapes, [torch.float32] * len(keys), dev)
    res['alloc_us'] = (time.perf_counter() - t) / 50 * 1e6
    from fedml_amd.ml.aggregator.state_dict_agg import aggregate, MUL_W
    w = [1 / 32] * 32
    aggregate(ds, MUL_W, w); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(50): aggregate(ds, MUL_W, w)
    res['aggregate_call_us'] = (time.perf_counter() - t) / 50 * 1e6
    torch.cuda.synchronize()
    res['aggregate_wall_us'] = (time.perf_counter() - t) / 50 * 1e6
print(json.dumps(res))
# one call at a time (no back-pressure from the descriptor ring): host part vs GPU part
hs, ws = [], []
for _ in range(30):
    torch.cuda.synchronize()
    t0 = time.perf_counter(); aggregate(ds, MUL_W, w); t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
    hs.append((t1 - t0) * 1e6); ws.append((t2 - t0) * 1e6)
hs.sort(); ws.sort()
print(json.dumps({"isolated_host_us_median": hs[15], "isolated_wall_us_median": ws[15]}))
