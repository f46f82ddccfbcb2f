"""On-arrival ingest of client updates into HBM.

The reference server moves each client update to its device as it arrives
(python/fedml/cross_silo/server/fedml_aggregator.py:57-66 -> ml/engine/ml_engine_adapter.py:234-254,
one ``.to(device)`` per tensor, in place on the update's dict) and aggregates once every client
has reported.  ``ArrivalIngest`` does the same move into a ClientArena row (fedml_amd/arena.py):
the update is packed into pinned staging and copied H2D on a copy stream while the server waits
for the next client, and the dict's entries are rebound to the row's device views.  The round's
aggregation over those dicts is then recognised as arena-resident (arena.resident_rows) and runs
as one launch per dtype group over the rows; only the LAST client's ingest, the kernel and the
result's D2H remain after the last arrival.

Rows are double-buffered by round parity, so round r+1's updates can be ingested while round r's
result is still being read.  ``to_host`` copies the aggregated model into pinned buffers (also
double-buffered) that a send path can pickle or post directly (fedml_server_manager.py:217-231).

Ownership: a returned result (or an adopted update) stays valid for as long as the caller holds
it.  Buffers are recycled two rounds later only when nothing outside still references the tensors
handed out from them; otherwise the ingest takes fresh pinned buffers (to_host) or moves the held
row views to private copies before the row is overwritten (ClientArena._detach).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Optional

import torch

from ... import _host
from ...arena import ArenaLayout, ClientArena


class ArrivalIngest:
    def __init__(self, capacity: int, device=None):
        self.capacity = int(capacity)
        self.device = device
        self.arena: Optional[ClientArena] = None
        self.parity = 0
        self._host: Dict[int, "OrderedDict[str, torch.Tensor]"] = {}
        self._flat_host: Dict[int, list] = {}  # per round parity: pinned flat buffers, one per dtype group

    @staticmethod
    def wants(device) -> bool:
        """The server device is a HIP device (the reference moves updates there on arrival)."""
        return device is not None and torch.device(device).type == "cuda"

    def add(self, index: int, state_dict) -> bool:
        """Adopt client ``index``'s update into this round's row.  False if it cannot be adopted
        (empty, unsupported dtype, or a layout other than the round's first update) -- the
        caller then keeps the reference's per-tensor move."""
        if not 0 <= index < self.capacity or len(state_dict) == 0:
            return False
        if self.arena is None:
            try:
                layout = ArenaLayout.from_state_dict(state_dict)
            except TypeError:
                return False
            dev = torch.device(self.device) if self.device is not None else None
            self.arena = ClientArena(layout, 2 * self.capacity, device=dev)
        try:
            self.arena.adopt(index + self.parity * self.capacity, state_dict)
        except (TypeError, KeyError):
            return False
        return True

    def round_done(self) -> None:
        """The round's aggregation has been issued: the next round fills the other rows."""
        self.parity ^= 1

    def to_host(self, averaged) -> "OrderedDict[str, torch.Tensor]":
        """The aggregated model in pinned host memory: the broadcast's send buffer.  The engine's
        outputs are views of one device allocation per dtype group, so each group goes D2H as ONE
        copy into a pinned flat buffer whose per-key views (built in C++, _host.carve) are returned
        (r02: 122 per-key copies of a ResNet-18-GN model cost 1.47 ms, mostly per-copy overhead).
        Other dicts: one D2H per tensor.  Buffers alternate between two rounds."""
        if not any(v.is_cuda for v in averaged.values()):
            return averaged
        flat = self._to_host_flat(averaged)
        if flat is not None:
            return flat
        bufs = self._host.get(self.parity)
        if bufs is None or list(bufs.keys()) != list(averaged.keys()) or any(
                bufs[k].shape != v.shape or bufs[k].dtype != v.dtype for k, v in averaged.items()) or \
                _storage_held(bufs.values()):
            bufs = self._host[self.parity] = OrderedDict(
                (k, torch.empty(v.shape, dtype=v.dtype, pin_memory=True)) for k, v in averaged.items())
        for k, v in averaged.items():
            bufs[k].copy_(v, non_blocking=True)
        torch.cuda.current_stream(next(iter(averaged.values())).device).synchronize()
        return OrderedDict((k, t.view(t.shape)) for k, t in bufs.items())  # caller-side tensor objects


    def _to_host_flat(self, averaged):
        groups = OrderedDict()  # device storage -> (dtype, storage, keys, element offsets, shapes)
        for k, v in averaged.items():
            if not v.is_cuda or not v.is_contiguous():
                return None
            st = v.untyped_storage()
            g = groups.get(st.data_ptr())
            if g is None:
                g = groups[st.data_ptr()] = (v.dtype, st, [], [], [])
            elif g[0] != v.dtype:
                return None
            g[2].append(k)
            g[3].append(v.storage_offset())
            g[4].append(tuple(v.shape))
        if len(groups) > 8:  # not the engine's grouped outputs: per-tensor copies
            return None
        dev = next(iter(averaged.values())).device
        cache = self._flat_host.setdefault(self.parity, [])
        if _storage_held(cache):
            # the caller still holds (part of) the result these buffers carried two rounds ago: leave
            # them to it and take fresh ones (the reference returns a dict that stays valid)
            cache = self._flat_host[self.parity] = []
        views = {}
        for gi, (dt, st, keys, offs, shapes) in enumerate(groups.values()):
            lo = min(offs)
            n = max(o + _numel(s) for o, s in zip(offs, shapes)) - lo
            if gi >= len(cache) or cache[gi].dtype != dt or cache[gi].numel() < n:
                if gi >= len(cache):
                    cache.append(None)
                cache[gi] = torch.empty(max(n, 1), dtype=dt, pin_memory=True)
            host = cache[gi][:n]
            src = torch.empty(0, dtype=dt, device=dev).set_(st, lo, (n,))
            host.copy_(src, non_blocking=True)
            for k, hv in zip(keys, _host.carve(host, [o - lo for o in offs], list(shapes))):
                views[k] = hv
        torch.cuda.current_stream(dev).synchronize()
        return OrderedDict((k, views[k]) for k in averaged.keys())


def _use_count_probe_ok() -> bool:
    """torch._C._storage_Use_Count is private: check once that it exists and that its baseline is
    the 2 references _storage_held assumes (the buffer's own tensor + the probe's storage object),
    and that a derived view adds one."""
    try:
        t = torch.empty(4)
        base = torch._C._storage_Use_Count(t.untyped_storage()._cdata)
        v = t[1:]
        held = torch._C._storage_Use_Count(t.untyped_storage()._cdata)
        del v
        return base == 2 and held == 3
    except Exception:  # noqa: BLE001 -- the private API moved: take the conservative path
        return False


_USE_COUNT_OK = _use_count_probe_ok()


def _storage_held(bufs) -> bool:
    """Is the storage of any of these (the ingest's own pinned buffers) still referenced from outside --
    by a tensor handed out from it or by ANY view derived from one (reshape, slice, ``.T``)?  Counted
    on the storage itself, not on the handed-out tensor objects: the buffer's own tensor and this
    probe's storage object account for 2 references.  If this torch's storage reference count does
    not behave that way (checked once at import), every buffer counts as held: fresh pinned buffers
    each round, never an overwritten result."""
    if not _USE_COUNT_OK:
        return any(b is not None for b in bufs)
    return any(torch._C._storage_Use_Count(b.untyped_storage()._cdata) > 2 for b in bufs if b is not None)


def _numel(shape) -> int:
    n = 1
    for s in shape:
        n *= s
    return n


def move_to_device(state_dict, device):
    """The reference's per-tensor move (ml_engine_adapter.model_params_to_device), in place."""
    for k in list(state_dict.keys()):
        state_dict[k] = state_dict[k].to(device)
    return state_dict
