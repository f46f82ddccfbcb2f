"""state_dict-level aggregation on the HIP engine.

`aggregate(dicts, mode, coef, divisor)` reproduces, for every key of client 0's dict (in that
key order), the reference's per-key client loop -- e.g. python/fedml/ml/aggregator/
agg_operator.py:37-44 -- with the dtype semantics of the PyTorch ops it issues:

* float32 / bfloat16 / float16 / float64 keys aggregate in their own type (per-op rounding);
* integer keys: weighted modes promote to float32 (``int_tensor * python_float``); SUM keeps the
  integer type with wrap-around (``int_tensor += int_tensor``); bool SUM is a logical OR;
* every key of one dtype goes to the device in ONE launch (fa_weighted_sum_multi).

Device placement: tensors already on a HIP device are aggregated in place on that device; CPU
tensors (what the reference's transports deliver) are staged to the engine's device, aggregated
there, and the result is returned on the CPU, matching the reference's output placement.  The CPU
path (`_aggregate_host`) packs every client's tensors of one dtype into a client-major staging
matrix with a multi-threaded C++ copy (`_host.pack_range`, GIL released) through a ring of pinned
slots, each slot's H2D overlapping the packing of the next, then aggregates the device matrix in
one launch per dtype and returns the result through one pinned D2H per dtype.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import torch

from ... import _host
from ...arena import resident_rows
from ...engine import MUL_N_DIV_N, MUL_W, SUM, AggEngine, get_engine, out_dtype

_NATIVE = (torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64)
_SMALL_INT = (torch.int32, torch.int16, torch.int8, torch.uint8)


def _engine_for(tensors) -> AggEngine:
    for t in tensors:
        if t.is_cuda:
            return get_engine(t.device.index)
    return get_engine(None)


def _to_engine(t: torch.Tensor, eng: AggEngine) -> torch.Tensor:
    if t.device != eng.device:
        t = t.to(eng.device, non_blocking=False)
    return t if t.is_contiguous() else t.contiguous()


_CODE_DTYPE = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16, 3: torch.float64, 4: torch.int64}


def aggregate(dicts: Sequence[Dict[str, torch.Tensor]], mode: int, coef: Optional[Sequence[float]] = None,
              divisor: float = 1.0, engine: Optional[AggEngine] = None) -> "OrderedDict[str, torch.Tensor]":
    """Ordered per-key reduction over client state_dicts (see module docstring)."""
    if len(dicts) == 0:
        raise IndexError("list index out of range")  # the reference indexes raw_grad_list[0]
    keys = list(dicts[0].keys())
    if not keys:
        return OrderedDict()
    if _host_small() and not getattr(dicts[0][keys[0]], "is_cuda", True):
        # small CPU round (cfg1): the whole call in C++ (None: not small / not uniform / not native)
        eng = engine or get_engine(None)
        fn, err, ctx = eng.host_round_abi()
        with eng.lock:
            out = _host.small_host_round(dicts if isinstance(dicts, list) else list(dicts), keys, mode, coef,
                                         divisor, fn, err, ctx, 0, _SMALL_HOST_BYTES, _host_cpu_bytes())
        if out is not None:
            return out
    hit = resident_rows(dicts)
    if hit is not None:  # updates adopted into arena rows on arrival: one launch per dtype group
        arena, rows = hit
        return arena.aggregate(mode, coef, divisor, clients=rows)
    try:
        ptrs, numel, codes, shapes, dev = _host.gather(list(dicts), keys)
    except (ValueError, TypeError):  # mixed devices or dtypes / non-contiguous: the staging path handles them
        ptrs = None
    if ptrs is not None and int(codes.min()) >= 0:
        if dev.startswith("cuda"):
            return _aggregate_device(keys, ptrs, numel, codes, shapes, dev, len(dicts), mode, coef, divisor, engine)
        if dev == "cpu" and _host_small():
            nbytes = sum(n * _ELEM[c] for n, c in zip(numel.tolist(), codes.tolist())) * len(dicts)
            # the zero-copy kernel takes at most _HOST_MAX_TABLE keys and clients (fa_weighted_sum_host)
            if nbytes <= _SMALL_HOST_BYTES and len(keys) <= _HOST_MAX_TABLE and len(dicts) <= _HOST_MAX_TABLE:
                return _aggregate_host_small(keys, ptrs, numel, codes, shapes, len(dicts), mode, coef, divisor,
                                             engine)
            return _aggregate_host(keys, ptrs, numel, codes, shapes, len(dicts), mode, coef, divisor, engine)
    return _aggregate_staged(dicts, keys, mode, coef, divisor, engine)


def _aggregate_device(keys, ptrs, numel, codes, shapes, dev, k, mode, coef, divisor, engine):
    """Fast path: every tensor already on one HIP device, native dtypes; one launch per dtype.  The
    outputs and the per-dtype launch tables come from one C++ call (_host.plan_outputs)."""
    eng = engine or get_engine(torch.device(dev).index)
    _, views, groups = _host.plan_outputs(shapes, codes, mode != SUM, dev, ptrs, k)
    if len(groups) == 2 and groups[1][0] == 4:
        # a float group + the int64 BatchNorm counters: one launch (fa_weighted_sum_pair_multi)
        (fc, n0, i0, o0), (_, n1, i1, o1) = groups
        eng.weighted_sum_table_pair(fc, mode, n0, i0, o0, n1, i1, o1, k=k, coef=coef, divisor=divisor)
    else:
        for c, nm, it, ot in groups:
            eng.weighted_sum_table(c, mode, nm, k, it, ot, coef, divisor)
    return OrderedDict(zip(keys, views))


_ELEM = {0: 4, 1: 2, 2: 2, 3: 8, 4: 8}  # bytes per element of each dtype code


def _host_small() -> bool:
    """FEDML_AMD_HOST_PATH=packed (default): small CPU rounds take the zero-copy kernel.  Read per call,
    so every check of it agrees with the variable's current value."""
    return os.environ.get("FEDML_AMD_HOST_PATH", "packed") == "packed"


_SMALL_HOST_BYTES = 4 << 20             # CPU rounds up to this size: zero-copy kernel (fa_weighted_sum_host)


def _host_cpu_bytes() -> int:
    """Host-resident rounds of at most this many input bytes are summed on the host that holds them
    (_host.small_host_round's host branch, fedml_amd/csrc/host_sum.h), larger ones go to the device:
    the break-even measured on the GPU box -- a device round trip costs at
    least the 13.7 us PCIe doorbell floor, more than the reference's whole 10.9 us CPU loop for
    cfg1.  FEDML_AMD_HOST_CPU_BYTES overrides it (0: every host round on the device)."""
    v = os.environ.get("FEDML_AMD_HOST_CPU_BYTES")
    return int(v) if v not in (None, "") else _HOST_CPU_BYTES


_HOST_CPU_BYTES = 1 << 20  # profiles/r05c/lr.json: host 2.6-2.8x faster than the device path up to 1 MiB
_HOST_MAX_TABLE = 4096                  # fa_weighted_sum_host's limit on num_segments and on k


def _aggregate_host_small(keys, ptrs, numel, codes, shapes, k, mode, coef, divisor, engine):
    """Small CPU state_dicts (cfg1's LR-MNIST: 63 KB a client): one synchronous zero-copy launch
    per dtype group -- inputs packed into mapped pinned memory, read and the result written in
    place by the kernel over PCIe, copied into fresh CPU tensors (fa_weighted_sum_host)."""
    eng = engine or get_engine(None)
    code_list = codes.tolist()
    out_dt = [out_dtype(_CODE_DTYPE[c], mode) for c in code_list]
    _, views, optrs = _host.alloc_outputs(shapes, out_dt, "cpu")
    groups: Dict[int, List[int]] = {}
    for t, c in enumerate(code_list):
        groups.setdefault(c, []).append(t)
    with eng.lock:
        if len(groups) == 1:
            c = code_list[0]
            eng.weighted_sum_host_table(c, mode, numel, k, ptrs, optrs, coef, divisor)
        else:
            table = ptrs.view(len(keys), k)
            for c, idx in groups.items():
                sel = torch.tensor(idx, dtype=torch.int64)
                eng.weighted_sum_host_table(c, mode, numel.index_select(0, sel).contiguous(), k,
                                            table.index_select(0, sel).reshape(-1).contiguous(),
                                            optrs.index_select(0, sel).contiguous(), coef, divisor)
    return OrderedDict(zip(keys, views))
_SLOT_BYTES = 64 << 20                  # pinned staging slot (two of them, ping-pong)


class _HostStaging:
    """Pinned slots + a device matrix per dtype group, reused across rounds of the same shape."""

    def __init__(self, eng: AggEngine):
        self.eng = eng
        self.stream = torch.cuda.Stream(eng.device)
        self.slots = [torch.empty(_SLOT_BYTES, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        self.events: List[Optional[torch.cuda.Event]] = [None, None]
        self.dev: Dict[tuple, torch.Tensor] = {}
        self.next = 0

    def matrix(self, key: tuple, nbytes: int) -> torch.Tensor:
        t = self.dev.get(key)
        if t is None or t.numel() < nbytes:
            t = self.dev[key] = torch.zeros(nbytes, dtype=torch.uint8, device=self.eng.device)
        return t


_STAGING: Dict[int, _HostStaging] = {}


def _pack_threads() -> int:
    env = os.environ.get("FEDML_AMD_PACK_THREADS")
    return int(env) if env else max(1, min(16, os.cpu_count() or 1))


def _aggregate_host(keys, ptrs, numel, codes, shapes, k, mode, coef, divisor, engine):
    """CPU state_dicts: pack -> pinned -> H2D (overlapped) -> one launch per dtype -> D2H.
    The pinned slots and device matrices are per-device state shared by every caller: the
    engine's lock serialises concurrent rounds (e.g. two receive threads)."""
    eng = engine or get_engine(None)
    with eng.lock:
        return _aggregate_host_locked(eng, keys, ptrs, numel, codes, shapes, k, mode, coef, divisor)


def _aggregate_host_locked(eng, keys, ptrs, numel, codes, shapes, k, mode, coef, divisor):
    st = _STAGING.get(eng.device_index)
    if st is None:
        st = _STAGING[eng.device_index] = _HostStaging(eng)
    code_list = codes.tolist()
    numel_list = numel.tolist()
    groups: Dict[int, List[int]] = {}
    for t, c in enumerate(code_list):
        groups.setdefault(c, []).append(t)
    table = ptrs.view(len(keys), k)
    nthreads = _pack_threads()
    cur = torch.cuda.current_stream(eng.device)
    st.stream.wait_stream(cur)  # the device matrices may still be read by the previous round's launch
    results: Dict[int, tuple] = {}
    for c, idx in groups.items():
        es = _ELEM[c]
        offs, row = [], 0
        for t in idx:
            offs.append(row)
            row += -(-max(numel_list[t], 1) * es // 256) * 256  # 256-byte aligned keys
        total = row * k
        mat = st.matrix((c,), total)
        # job table, sorted by destination: client-major, keys in order inside a row
        src = table.index_select(0, torch.tensor(idx, dtype=torch.int64)).t().contiguous().view(-1)
        dst = (torch.arange(k, dtype=torch.int64).view(k, 1) * row + torch.tensor(offs, dtype=torch.int64)).view(-1)
        nb = (torch.tensor([numel_list[t] for t in idx], dtype=torch.int64) * es).repeat(k)
        for lo in range(0, total, _SLOT_BYTES):
            hi = min(total, lo + _SLOT_BYTES)
            j = st.next % 2
            st.next += 1
            if st.events[j] is not None:
                st.events[j].synchronize()  # the H2D that last read this slot is done
            _host.pack_range(src, dst, nb, lo, hi, st.slots[j].data_ptr(), nthreads)
            with torch.cuda.stream(st.stream):
                mat[lo:hi].copy_(st.slots[j][:hi - lo], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st.stream)
            st.events[j] = ev
        results[c] = (idx, offs, row, mat)
    cur.wait_stream(st.stream)
    out = OrderedDict()
    views: Dict[int, torch.Tensor] = {}
    for c, (idx, offs, row, mat) in results.items():
        dt = _CODE_DTYPE[c]
        buf = mat[:row * k].view(dt).view(k, row // _ELEM[c])
        o = eng.weighted_sum_rows(buf, list(range(k)), mode, coef, divisor)
        host = torch.empty(o.numel(), dtype=o.dtype, pin_memory=True)
        host.copy_(o, non_blocking=True)
        views[c] = host
    cur.synchronize()  # the reference returns materialised CPU tensors
    for c, (idx, offs, row, mat) in results.items():
        host = views[c]
        for t, off in zip(idx, offs):
            e0 = off // _ELEM[c]
            out[keys[t]] = host[e0:e0 + numel_list[t]].view(shapes[t])
    return OrderedDict((kk, out[kk]) for kk in keys)


def _aggregate_staged(dicts, keys, mode, coef, divisor, engine):
    """General path: host (CPU) tensors are staged to the engine's device; narrow integer types are
    widened exactly to int64 first.  Arithmetic is still the HIP kernels'."""
    first = [dicts[0][k] for k in keys]
    eng = engine or _engine_for(first)
    on_cpu = not any(t.is_cuda for t in first)
    out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    groups: Dict[torch.dtype, List[str]] = {}
    post: Dict[str, torch.dtype] = {}
    staged: Dict[str, List[torch.Tensor]] = {}
    mixed: Dict[str, List[torch.Tensor]] = {}
    for k in keys:
        col = [d[k] for d in dicts]  # KeyError on a missing key, like the reference
        dt = col[0].dtype
        for i, t in enumerate(col):
            if t.shape != col[0].shape:
                raise RuntimeError(f"key {k!r}: client {i} shape {tuple(t.shape)} != {tuple(col[0].shape)}")
        col = [_to_engine(t, eng) for t in col]
        if any(t.dtype != dt for t in col):  # clients disagree on this key's dtype: promotion
            mixed[k] = col
            continue
        if dt in _SMALL_INT or dt == torch.bool:
            # exact widening: int64 arithmetic gives the same low bits (SUM) and the same fp32
            # conversion (weighted modes) as the narrower integer type
            col = [t.to(torch.int64) for t in col]
            if mode == SUM:
                post[k] = dt
        elif dt not in _NATIVE:
            raise TypeError(f"key {k!r}: dtype {dt} is not supported")
        staged[k] = col
        groups.setdefault(col[0].dtype, []).append(k)
    results: Dict[str, torch.Tensor] = {}
    for dt, ks in groups.items():
        outs = eng.weighted_sum_multi([staged[k] for k in ks], mode, coef, divisor)
        for k, o in zip(ks, outs):
            results[k] = o
    for k, col in mixed.items():
        results[k] = _aggregate_mixed(k, col, mode, coef, divisor, eng)
        if mode == SUM and col[0].dtype in _SMALL_INT:
            post[k] = col[0].dtype
    for k in keys:
        r = results[k]
        if k in post:
            tgt = post[k]
            r = (r != 0) if tgt == torch.bool else r.to(tgt)
        if on_cpu:
            r = r.cpu()
        out[k] = r
    return out


def _aggregate_mixed(k, col, mode, coef, divisor, eng):
    """One key whose clients disagree on its dtype, with the reference's in-place semantics
    (agg_operator.py:37-44, 55-63): avg = t_0; avg += t_i, each += computed in
    promote_types(avg, t_i) and rounded to avg's dtype (fa_promote_add).  t_i = x_i * w_i in x_i's
    own dtype (a K = 1 launch of the ordinary kernel: the reference's ``x * w``), or x_i for the
    plain-sum branch; integer sums stay in int64 (wrap-around), narrow integer types widened
    exactly first.  Pinned by tests/golden/g19_* (generated from the reference)."""
    def widen(t):
        if t.dtype in _SMALL_INT:
            return t.to(torch.int64)  # exact
        if t.dtype == torch.bool or t.dtype not in _NATIVE:
            raise TypeError(f"key {k!r}: dtype {t.dtype} cannot take part in a mixed-dtype aggregation")
        return t
    terms = []
    for i, x in enumerate(col):
        x = widen(x).reshape(-1)
        if mode == SUM:
            terms.append(x)
        else:
            terms.append(eng.weighted_sum([x], mode, [coef[i]], divisor))
    acc = terms[0].clone() if mode == SUM else terms[0]
    for i, t in enumerate(terms[1:], 1):
        if acc.dtype == t.dtype:
            acc = eng.weighted_sum([acc, t], SUM)
        elif acc.dtype == torch.int64:  # the reference's `int_tensor += float_tensor`
            raise RuntimeError(f"result type {t.dtype} can't be cast to the desired output type Long "
                               f"(key {k!r}, client {i})")
        else:
            acc = eng.promote_add(acc, t, out=acc)
    return acc.view(col[0].shape)


def fedavg(dicts, counts, engine=None):
    """avg[k] = sum_i x_i[k] * (n_i / N), client order (agg_operator.py:35-44)."""
    N = sum(counts)
    return aggregate(dicts, MUL_W, [n / N for n in counts], engine=engine)


def fedavg_xn_div_n(dicts, counts, engine=None):
    """avg[k] = sum_i (x_i[k] * n_i) / N (simulation/mpi/fedavg/FedAVGAggregator.py:99-116)."""
    return aggregate(dicts, MUL_N_DIV_N, list(counts), float(sum(counts)), engine=engine)


def plain_sum(dicts, engine=None):
    """avg[k] = sum_i x_i[k] (agg_operator.py:55-63 FedAvg_seq, :68-77 FedDyn)."""
    return aggregate(dicts, SUM, engine=engine)


def mix(dicts: Sequence[Dict[str, torch.Tensor]], row_ptr, cols, vals, post_scale=None,
        engine: Optional[AggEngine] = None):
    """Per-key CSR mixing of model dicts (fa_mix): returns (rows, rows2) lists of OrderedDicts.

    rows[r][k] = ordered sum over the row's entries j of dicts[cols[j]][k] * vals[j]
    (HierFedAvgCloudAggregator.py:174-195 with a dense row; client_dsgd.py:104-122 with a gossip
    row); rows2[r][k] = rows[r][k] * post_scale[r] when post_scale is given (client_pushsum.py:150-156).
    """
    keys = list(dicts[0].keys())
    eng = engine or _engine_for([dicts[0][k] for k in keys])
    on_cpu = not any(dicts[0][k].is_cuda for k in keys)
    nrows = len(row_ptr) - 1
    rows = [OrderedDict() for _ in range(nrows)]
    rows2 = [OrderedDict() for _ in range(nrows)] if post_scale is not None else None
    for k in keys:
        col = [_to_engine(d[k], eng) for d in dicts]
        dt = col[0].dtype
        if dt in _SMALL_INT or dt in (torch.int64, torch.bool):
            # int tensor * float32 weight -> float32 (PyTorch promotion): exact int -> fp32 cast first
            col = [t.to(torch.float32) for t in col]
        elif dt not in (torch.float32, torch.bfloat16, torch.float16):
            raise TypeError(f"mix: key {k!r} has dtype {dt} (float32/bfloat16/float16/integer only)")
        shape = col[0].shape
        outs, outs2 = eng.mix([t.reshape(-1) for t in col], row_ptr, cols, vals, post_scale)
        for r in range(nrows):
            o = outs[r].reshape(shape)
            rows[r][k] = o.cpu() if on_cpu else o
            if rows2 is not None:
                o2 = outs2[r].reshape(shape)
                rows2[r][k] = o2.cpu() if on_cpu else o2
    return rows, rows2
