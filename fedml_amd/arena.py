"""ClientArena: device-resident, client-major storage for one round of client updates.

Why: the aggregation is a pure HBM stream, and how the K client updates sit in HBM matters.
K separately allocated buffers read at ~5.9 TB/s on MI355X, the same bytes as K rows of ONE
allocation at ~6.8 TB/s (tools/hbm_probe.py, profiles/r01_hbm_probe*.json: address translation
over many independent allocations costs ~13 %).  A state_dict round also costs one pointer per
(client, key) -- 19,456 for ViT-B/16 at K = 128 -- where an arena needs one per client.

Layout: the model's keys are grouped by storage dtype; for each dtype group the arena holds one
tensor ``[capacity, P_group]`` in which client i's row carries that group's keys at fixed offsets,
each key padded to a 64-element (256-byte for fp32) boundary so every key and every row starts
16-byte aligned (the kernel's vector path).  Aggregating the round is then ONE flat launch per
dtype group over K row pointers (fa_weighted_sum with n = P_group), and the result lives in an
output arena with the same offsets, exposed as per-key views in the model's key order.

Tiled layout (``tiled=True``): each dtype group is stored tile-interleaved, ``[tiles, capacity, E]``
with E elements = 4 KiB (``FA_TILE_BYTES``): tile t of client r sits at (t * capacity + r) * 4 KiB.
A workgroup of the aggregation kernel reads tile t of all K clients -- with the client-major
layout those are K 4-KiB pieces 500 MB apart (at the metric size), tiled they are ONE contiguous
K * 4 KiB run.  Measured on MI355X at the metric size (tools/layout_probe.py): the bare read
pattern streams at 6.54-6.76 TB/s tiled vs 6.12-6.28 TB/s client-major.  The logical per-group
offsets are unchanged (same ArenaLayout), only the physical placement differs, so client rows are
not addressable as tensor views: ingest goes through ``write`` (one strided device copy per
dtype group) and ``read`` gathers a client back.

Ingest: ``write(i, state_dict)`` copies a client's tensors into row i (device -> device, or host
-> device).  Host updates (what the reference's transports deliver, e.g. mpi_receive_thread.py:25)
go through a pinned staging ring: the client's tensors are packed into pinned memory, one async
H2D per dtype group is issued on a copy stream, and the aggregation stream waits on its event.
"""
from __future__ import annotations

import os
import weakref
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _host
from .engine import MUL_N_DIV_N, MUL_W, SUM, AggEngine, get_engine, out_dtype

_ALIGN_ELEMS = 64
_SUPPORTED = (torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64)


def _pad(n: int) -> int:
    return (n + _ALIGN_ELEMS - 1) // _ALIGN_ELEMS * _ALIGN_ELEMS


class ArenaLayout:
    """Key -> (dtype group, offset, shape) map of a model state_dict."""

    def __init__(self, spec: Sequence[Tuple[str, Sequence[int], torch.dtype]]):
        self.keys: List[str] = []
        self.where: Dict[str, Tuple[torch.dtype, int, Tuple[int, ...], int]] = {}
        self.group_numel: Dict[torch.dtype, int] = {}
        for name, shape, dt in spec:
            if dt not in _SUPPORTED:
                raise TypeError(f"arena: key {name!r} has unsupported dtype {dt}")
            n = 1
            for s in shape:
                n *= int(s)
            off = self.group_numel.get(dt, 0)
            self.where[name] = (dt, off, tuple(int(s) for s in shape), n)
            self.group_numel[dt] = off + _pad(max(n, 1))
            self.keys.append(name)
        # per dtype group: (key positions, element offsets, shapes) for _host.carve
        self.group_keys: Dict[torch.dtype, Tuple[List[int], List[int], List[Tuple[int, ...]]]] = {}
        for pos, name in enumerate(self.keys):
            dt, off, shape, _ = self.where[name]
            g = self.group_keys.setdefault(dt, ([], [], []))
            g[0].append(pos)
            g[1].append(off)
            g[2].append(shape)

    def carve(self, outs: Dict[torch.dtype, torch.Tensor]) -> "OrderedDict[str, torch.Tensor]":
        """Per-key views of the flat per-dtype-group outputs, in key order (built in C++)."""
        views: List[Optional[torch.Tensor]] = [None] * len(self.keys)
        for dt, (pos, offs, shapes) in self.group_keys.items():
            for p_, v in zip(pos, _host.carve(outs[dt], offs, shapes)):
                views[p_] = v
        return OrderedDict(zip(self.keys, views))

    @classmethod
    def from_state_dict(cls, sd) -> "ArenaLayout":
        return cls([(k, tuple(v.shape), v.dtype) for k, v in sd.items()])

    def views(self, bufs: Dict[torch.dtype, torch.Tensor], row: Optional[int]) -> "OrderedDict[str, torch.Tensor]":
        out = OrderedDict()
        for k in self.keys:
            dt, off, shape, n = self.where[k]
            b = bufs[dt] if row is None else bufs[dt][row]
            out[k] = b[off:off + n].view(shape)
        return out


TILE_BYTES = 4096  # FA_TILE_BYTES (include/fedagg.h)

# state_dicts adopted into arena rows (ClientArena.adopt): id(dict) -> (arena, row).  A later
# aggregate() over such dicts is recognised (resident_rows) and runs as ONE launch per dtype group
# over the arena rows instead of walking a (key, client) pointer table.
_ADOPTED: Dict[int, Tuple["weakref.ref", int]] = {}


# c10::ScalarType codes (match_rows compares them with the values' scalar_type())
_SCALAR_TYPE = {torch.uint8: 0, torch.int8: 1, torch.int16: 2, torch.int32: 3, torch.int64: 4, torch.float16: 5,
                torch.float32: 6, torch.float64: 7, torch.bool: 11, torch.bfloat16: 15}


def tile_elems(dt: torch.dtype) -> int:
    return TILE_BYTES // torch.empty((), dtype=dt).element_size()


class ClientArena:
    def __init__(self, layout: ArenaLayout, capacity: int, device=None, engine: Optional[AggEngine] = None,
                 zero: bool = True, tiled: bool = False):
        self.layout = layout
        self.capacity = int(capacity)
        self.tiled = bool(tiled)
        self.engine = engine or get_engine(None if device is None else torch.device(device).index)
        self.device = self.engine.device
        self.alloc_kind: Dict[torch.dtype, str] = {}
        self.bufs: Dict[torch.dtype, torch.Tensor] = {}
        self.placement: Dict[torch.dtype, dict] = {}
        for dt, n in layout.group_numel.items():
            shape = (-(-n // tile_elems(dt)), self.capacity, tile_elems(dt)) if self.tiled else (self.capacity, n)
            self.bufs[dt] = self._place(shape, dt, zero, self._alloc(shape, dt, zero))
        self._scratch: Dict[torch.dtype, torch.Tensor] = {}
        self._stage_dev: Dict[torch.dtype, torch.Tensor] = {}  # copy-stream row staging (tiled host ingest)
        self._copy_stream = None
        self._staging: List[Tuple[Dict[torch.dtype, torch.Tensor], Optional[torch.cuda.Event]]] = []
        self._next_stage = 0
        self._pending: List[torch.cuda.Event] = []
        self._rows_adopted: Dict[int, int] = {}  # row -> id of the state_dict adopted into it
        self._handed: Dict[int, list] = {}        # row -> weakrefs of the row views adopt() handed out

    # Groups of at least CONTIG_MIN_BYTES live in physically contiguous device memory
    # (AggEngine.alloc_contiguous): the weighted-sum kernel's rate over a 64.5 GB arena depended on the
    # allocation -- 9.28-10.0 ms per K = 128 x 125 M step on one box with identical translation, L2
    # and request counters (profiles/r06n-r06q) -- and contiguous blocks ran at the fast end more
    # often (DESIGN A.3 item 11).  FEDML_AMD_ARENA_ALLOC=torch: the caching allocator for every group.
    CONTIG_MIN_BYTES = 1 << 30

    def _alloc(self, shape, dt: torch.dtype, zero: bool) -> torch.Tensor:
        n = 1
        for d in shape:
            n *= int(d)
        nbytes = n * torch.empty((), dtype=dt).element_size()
        if nbytes >= self.CONTIG_MIN_BYTES and os.environ.get("FEDML_AMD_ARENA_ALLOC", "contiguous") != "torch":
            raw = self.engine.alloc_contiguous(nbytes)
            if raw is not None:
                t = raw.view(dt).view(shape)
                if zero:  # zeroed padding keeps padded outputs finite
                    t.zero_()
                self.alloc_kind[dt] = "contiguous"
                return t
        self.alloc_kind[dt] = "torch"
        return (torch.zeros if zero else torch.empty)(shape, dtype=dt, device=self.device)

    # Placement check (r06): of contiguous blocks too, some ran the weighted-sum kernel 5-8 % slower
    # than others with the same read rate (profiles/r06p, r06z), and the kernel / read-probe time ratio
    # of three quick launches right after allocation tells them apart (1.02-1.055 vs 1.115-1.127 for
    # the 10.0 ms blocks of the metric size, profiles/r06aa).  A tiled float group of at least
    # PLACEMENT_MIN_BYTES whose ratio exceeds PLACEMENT_RATIO is allocated again (the old block kept
    # until the new one is measured), at most PLACEMENT_TRIES blocks in all, and the best one stays.
    # FEDML_AMD_ARENA_PLACEMENT=0 turns the check off.
    PLACEMENT_MIN_BYTES = 16 << 30
    PLACEMENT_RATIO = 1.07
    PLACEMENT_TRIES = 3

    def _placement_ratio(self, buf: torch.Tensor, dt: torch.dtype) -> float:
        """median(weighted-sum kernel) / median(read probe) over the group, 3 interleaved launches
        each (HIP events on the current stream)."""
        n, cap = self.layout.group_numel[dt], self.capacity
        out = torch.empty(n, dtype=dt, device=self.device)
        rows, w = list(range(cap)), [1.0 / cap] * cap
        st = torch.cuda.current_stream(self.device)
        km, pm = [], []
        for _ in range(3):
            for fn, acc in ((lambda: self.engine.read_probe(buf, cap), pm),
                            (lambda: self.engine.weighted_sum_tiled(buf, rows, MUL_W, w, n=n, out=out), km)):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                fn()
                b.record(st)
                b.synchronize()
                acc.append(a.elapsed_time(b))
        km.sort()
        pm.sort()
        return km[1] / pm[1]

    def _place(self, shape, dt: torch.dtype, zero: bool, buf: torch.Tensor) -> torch.Tensor:
        nbytes = buf.numel() * buf.element_size()
        if (not self.tiled or not dt.is_floating_point or self.alloc_kind.get(dt) != "contiguous"
                or nbytes < self.PLACEMENT_MIN_BYTES or self.capacity < 64
                or os.environ.get("FEDML_AMD_ARENA_PLACEMENT", "1") == "0"):
            return buf  # (the ratio's threshold holds for >= 64 client rows per workgroup)
        ratios = [self._placement_ratio(buf, dt)]
        best = buf
        del buf  # (at most two blocks alive at once: the best so far and the one being measured)
        while min(ratios) > self.PLACEMENT_RATIO and len(ratios) < self.PLACEMENT_TRIES:
            raw = self.engine.alloc_contiguous(nbytes)
            if raw is None:
                break
            nb = raw.view(dt).view(shape)
            del raw
            if zero:
                nb.zero_()
            ratios.append(self._placement_ratio(nb, dt))
            if ratios[-1] < min(ratios[:-1]):
                best = nb  # the previous best is freed when its last reference goes
            del nb
        self.placement[dt] = {"ratios": [round(r, 4) for r in ratios], "kept": ratios.index(min(ratios)),
                              "threshold": self.PLACEMENT_RATIO}
        return best

    @classmethod
    def for_model(cls, template_state_dict, capacity: int, device=None, **kw) -> "ClientArena":
        return cls(ArenaLayout.from_state_dict(template_state_dict), capacity, device, **kw)

    def slot(self, i: int) -> "OrderedDict[str, torch.Tensor]":
        """Client i's tensors (views into the arena), in the model's key order."""
        if self.tiled:
            raise TypeError("a tiled arena's rows are not tensor views: use write(i, sd) / read(i)")
        return self.layout.views(self.bufs, i)

    def rows(self, dt: torch.dtype, clients: Sequence[int]) -> List[torch.Tensor]:
        if self.tiled:
            raise TypeError("a tiled arena's rows are not tensor views: use write(i, sd) / read(i)")
        return [self.bufs[dt][i] for i in clients]

    def tile_view(self, dt: torch.dtype, i: int) -> torch.Tensor:
        """Tiled arena: client i's dtype group as a strided [tiles, E] view (row-major flat order)."""
        if not self.tiled:
            raise TypeError("tile_view: not a tiled arena")
        return self.bufs[dt][:, i, :]

    def _row_scratch(self, dt: torch.dtype) -> torch.Tensor:
        """A contiguous logical row of group dt, padded to whole tiles (tiled ingest/read)."""
        t = self._scratch.get(dt)
        if t is None:
            nt, _, E = self.bufs[dt].shape
            t = self._scratch[dt] = torch.zeros(nt * E, dtype=dt, device=self.device)
        return t

    def read(self, i: int) -> "OrderedDict[str, torch.Tensor]":
        """Client i's tensors as new device tensors (a copy; works for both layouts)."""
        if not 0 <= i < self.capacity:
            raise IndexError(f"arena row {i} out of range [0, {self.capacity})")
        self._wait_ingest()
        if not self.tiled:
            return OrderedDict((k, v.clone()) for k, v in self.slot(i).items())
        rows = {dt: self.tile_view(dt, i).reshape(-1) for dt in self.bufs}  # reshape of a strided view copies
        return OrderedDict((k, v.clone()) for k, v in self.layout.views(rows, None).items())

    # ------------------------------------------------------------------ ingest
    def write(self, i: int, state_dict) -> None:
        """Copy one client's update into row i (device tensors: D2D on the current stream; host
        tensors: packed into pinned staging and sent with one H2D per dtype group)."""
        if not 0 <= i < self.capacity:
            raise IndexError(f"arena row {i} out of range [0, {self.capacity})")
        self._detach(i)
        for k in self.layout.keys:
            dt, _, shape, _ = self.layout.where[k]
            t = state_dict[k]  # KeyError on a missing key, like the reference's per-key access
            if t.dtype != dt or tuple(t.shape) != shape:
                raise TypeError(f"arena: key {k!r} is {t.dtype}{tuple(t.shape)}, layout says {dt}{shape}")
        first = state_dict[self.layout.keys[0]]
        if first.is_cuda:
            if self.tiled and len(self.layout.keys) == 1 and first.is_contiguous():
                # one key at offset 0: scatter it straight into the tiles (2 P s bytes, no row scratch)
                dt = first.dtype
                nt, _, E = self.bufs[dt].shape
                x = first.reshape(-1)
                full = x.numel() // E
                tv = self.tile_view(dt, i)
                if full:
                    tv[:full].copy_(x[:full * E].view(full, E))
                if x.numel() > full * E:
                    tv[full, :x.numel() - full * E].copy_(x[full * E:])
                return
            if self.tiled:  # pack the logical row, then one strided tile scatter per dtype group
                rows = {dt: self._row_scratch(dt) for dt in self.bufs}
                for k, v in self.layout.views(rows, None).items():
                    v.copy_(state_dict[k])
                for dt, r in rows.items():
                    self.tile_view(dt, i).copy_(r.view(self.bufs[dt].shape[0], -1))
                return
            for k, v in self.slot(i).items():
                v.copy_(state_dict[k])
            return
        self._write_host(i, state_dict)

    def _detach(self, i: int) -> None:
        """Row i is about to be overwritten: every row view handed out by an earlier adopt(i) that is
        still alive (a caller kept the update dict, or one of its tensors) is moved to a private copy
        first (``t.set_(t.clone())``, on the compute stream, which the overwrite is ordered after), so
        it keeps its values -- in the reference each update owns its tensors.

        Scope: the protection covers the tensor OBJECTS adopt() handed out (the dict's entries, and
        the dict itself).  A view derived from one of them (``t.reshape(-1)``, ``t[0]``, ``t.T``) is a
        view of the arena row, not of the private copy; it follows the row once that is
        overwritten.  Callers that keep such a view across rounds clone it (the arena's storage is
        shared by every row, so it cannot tell which row a derived view points into).  Results of
        ``ArrivalIngest.to_host`` have no such limit (their guard counts references on the storage)."""
        refs = self._handed.pop(i, None)
        if not refs:
            return
        for r in refs:
            t = r()
            if t is not None:
                t.set_(t.clone())

    def adopt(self, i: int, state_dict) -> None:
        """On-arrival ingest (the reference moves an arriving update to the server device in place,
        cross_silo/server/fedml_aggregator.py:57-66 -> ml_engine_adapter.py:234-254): copy the update
        into row i and rebind the dict's entries to the row's device views, in place.  The compute
        stream is ordered after the copy (a stream wait, no host block), so the rebound tensors
        are safe to use on it at once.  Later aggregations over adopted dicts are recognised by
        ``resident_rows`` and run over the arena rows.

        Ownership: the row is reused by a later adopt/write of row i (the round drivers alternate
        rows by round); if the dict adopted now, or any of its tensors, is still referenced then,
        those tensors are first moved to private copies (``_detach``), so a caller that keeps a
        round's update never sees another round's values."""
        if self.tiled:
            raise TypeError("adopt: a tiled arena's rows are not tensor views (use a client-major arena)")
        if len(state_dict) != len(self.layout.keys) or any(k not in self.layout.where for k in state_dict):
            raise TypeError("adopt: the update's keys differ from the arena layout")
        self.write(i, state_dict)
        self._wait_ingest()
        views = self.slot(i)
        for k, v in views.items():
            state_dict[k] = v
        self._handed[i] = [weakref.ref(v) for v in views.values()]
        old = self._rows_adopted.get(i)  # the dict this row held before: no longer resident here
        if old is not None and _ADOPTED.get(old, (None, -1))[1] == i:
            _ADOPTED.pop(old, None)
        self._rows_adopted[i] = id(state_dict)
        _ADOPTED[id(state_dict)] = (weakref.ref(self), i)

    def _ptr_table(self):
        """Per key (layout order): device address of row 0's tensor, the row stride in bytes, and
        the view's (scalar type, ndim, sizes) record with its offsets (match_rows)."""
        t = getattr(self, "_ptr_tab", None)
        if t is None:
            base, stride, meta, moff = [], [], [], []
            for k in self.layout.keys:
                dt, off, shape, _ = self.layout.where[k]
                b = self.bufs[dt]
                base.append(b.data_ptr() + off * b.element_size())
                stride.append(b.stride(0) * b.element_size())
                moff.append(len(meta))
                meta += [_SCALAR_TYPE[dt], len(shape)] + [int(s) for s in shape]
            t = self._ptr_tab = (torch.tensor(base, dtype=torch.int64), torch.tensor(stride, dtype=torch.int64),
                                 torch.tensor(meta, dtype=torch.int64), torch.tensor(moff, dtype=torch.int64))
        return t

    def _stage_slot(self):
        if len(self._staging) < 2:
            bufs = {dt: torch.zeros(n, dtype=dt, pin_memory=True) for dt, n in self.layout.group_numel.items()}
            self._staging.append((bufs, None))
        idx = self._next_stage % len(self._staging)
        self._next_stage += 1
        bufs, ev = self._staging[idx]
        if ev is not None:
            ev.synchronize()  # the H2D that last used this pinned slot has finished
        return idx, bufs

    def _write_host(self, i: int, state_dict) -> None:
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(self.device)
        # the H2D overwrites row i: it must not start before every kernel already queued on the
        # compute stream (e.g. the previous round's aggregate() or read() of these rows) has run
        self._copy_stream.wait_stream(torch.cuda.current_stream(self.device))
        if not self.tiled and all(state_dict[k].is_pinned() for k in self.layout.keys):
            # already page-locked (e.g. a transport that receives into pinned buffers): DMA directly
            slot = self.slot(i)
            with torch.cuda.stream(self._copy_stream):
                for k, v in slot.items():
                    v.copy_(state_dict[k], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._copy_stream)
            self._pending.append(ev)
            return
        idx, pinned = self._stage_slot()
        if not self.tiled:
            self._pack_and_copy(i, state_dict, pinned)
            with torch.cuda.stream(self._copy_stream):
                ev = torch.cuda.Event()
                ev.record(self._copy_stream)
            self._staging[idx] = (pinned, ev)
            self._pending.append(ev)
            return
        views = self.layout.views(pinned, None)
        for k, v in views.items():
            v.copy_(state_dict[k])
        with torch.cuda.stream(self._copy_stream):
            for dt, buf in pinned.items():
                if self.tiled:  # H2D of the logical row, then the strided tile scatter, same stream
                    nt, _, E = self.bufs[dt].shape
                    r = self._stage_dev.get(dt)
                    if r is None:
                        r = self._stage_dev[dt] = torch.zeros(nt * E, dtype=dt, device=self.device)
                    r[:buf.numel()].copy_(buf, non_blocking=True)
                    self.tile_view(dt, i).copy_(r.view(nt, E))
                else:
                    self.bufs[dt][i].copy_(buf, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._copy_stream)
        self._staging[idx] = (pinned, ev)
        self._pending.append(ev)

    PACK_CHUNK_BYTES = 8 << 20  # H2D issued per ~8 MB packed

    def _pack_and_copy(self, i: int, state_dict, pinned) -> None:
        """Pack the update into the pinned row and issue the H2D of every ~8 MB packed on the copy
        stream at once, so the DMA of one piece runs while the next is packed (r02: the
        pack-then-copy form left 0.6 ms of H2D after a 1.1 ms pack of a 47 MB update).  The pack is
        torch's per-key copy_ (its OpenMP pool); the C++ thread-pool memcpy used for whole-round host
        packing (_host.pack_range) measured slower here (K = 32 ResNet-18-GN last arrival: pack
        1.30 ms with copy_ vs 1.8-2.4 ms with 4-16 threads, profiles/r02ah)."""
        issued = {dt: 0 for dt in pinned}  # elements of each dtype group already handed to the DMA
        packed = dict(issued)
        pending = 0

        def issue(final: bool):
            with torch.cuda.stream(self._copy_stream):
                for dt, buf in pinned.items():
                    hi = buf.numel() if final else packed[dt]
                    if hi > issued[dt]:
                        self.bufs[dt][i][issued[dt]:hi].copy_(buf[issued[dt]:hi], non_blocking=True)
                        issued[dt] = hi

        for k in self.layout.keys:
            dt, off, shape, n = self.layout.where[k]
            pinned[dt][off:off + n].view(shape).copy_(state_dict[k])
            packed[dt] = off + n
            pending += n * pinned[dt].element_size()
            if pending >= self.PACK_CHUNK_BYTES:
                issue(False)
                pending = 0
        issue(True)

    def _wait_ingest(self):
        cur = torch.cuda.current_stream(self.device)
        for ev in self._pending:
            cur.wait_event(ev)
        self._pending.clear()

    # ------------------------------------------------------------------ aggregation
    def aggregate(self, mode: int, coef: Optional[Sequence[float]] = None, divisor: float = 1.0,
                  clients: Optional[Sequence[int]] = None,
                  out: Optional[Dict[torch.dtype, torch.Tensor]] = None) -> "OrderedDict[str, torch.Tensor]":
        """Ordered reduction over the given client rows (default: all), one launch per dtype group
        (one launch in all for a float group + the int64 counter group, fa_weighted_sum_pair).
        ``out`` (optional): preallocated flat output per INPUT dtype group (reused across rounds).
        Returns per-key views of the result in the model's key order."""
        clients = list(range(self.capacity)) if clients is None else list(clients)
        if not clients:
            raise IndexError("list index out of range")
        self._wait_ingest()
        outs: Dict[torch.dtype, torch.Tensor] = {}
        pair = self._pair_groups()
        if pair is not None:  # a float group + the int64 counters: one launch (fa_weighted_sum_pair)
            fdt = pair
            gn = self.layout.group_numel
            outs[fdt], outs[torch.int64] = self.engine.weighted_sum_pair(
                self.bufs[fdt], self.bufs[torch.int64], clients, mode, coef, divisor, n=gn[fdt],
                n_i64=gn[torch.int64], out=out.get(fdt) if out is not None else None,
                out_i64=out.get(torch.int64) if out is not None else None)
            return self.layout.carve(outs)
        for dt, buf in self.bufs.items():
            o = out[dt] if out is not None else None
            if self.tiled:
                outs[dt] = self.engine.weighted_sum_tiled(buf, clients, mode, coef, divisor,
                                                          n=self.layout.group_numel[dt], out=o)
            else:
                outs[dt] = self.engine.weighted_sum_rows(buf, clients, mode, coef, divisor, out=o)
        return self.layout.carve(outs)

    def median(self, clients: Optional[Sequence[int]] = None,
               out: Optional[Dict[torch.dtype, torch.Tensor]] = None) -> "OrderedDict[str, torch.Tensor]":
        """Coordinate-wise median over the given client rows (default: all), one launch per dtype
        group (coordinate_wise_median_defense.py:18-44's torch.median(dim=-1) per coordinate; a
        selection, bit for bit): tiled arenas through fa_coord_median_tiled (the layout whose K tiles
        of a workgroup are one contiguous run), client-major arenas over the row views.  Float groups
        only (the reference's median runs over weight tensors).  Returns per-key views."""
        clients = list(range(self.capacity)) if clients is None else list(clients)
        if not clients:
            raise RuntimeError("torch.cat(): expected a non-empty list of Tensors")
        if any(dt not in (torch.float32, torch.bfloat16, torch.float16, torch.float64) for dt in self.bufs):
            raise TypeError("median: the arena holds a non-float dtype group")
        self._wait_ingest()
        outs: Dict[torch.dtype, torch.Tensor] = {}
        for dt, buf in self.bufs.items():
            o = out[dt] if out is not None else None
            n = self.layout.group_numel[dt]
            if self.tiled:
                outs[dt] = self.engine.coord_median_tiled(buf, clients, n=n, out=o)
            else:
                o = o if o is not None else torch.empty(n, dtype=dt, device=buf.device)
                self.engine.coord_median([[buf[i][:n] for i in clients]], outs=[o])
                outs[dt] = o
        return self.layout.carve(outs)

    def _pair_groups(self) -> Optional[torch.dtype]:
        """The float dtype when the arena holds exactly one float group and one int64 group."""
        dts = list(self.bufs)
        if len(dts) != 2 or torch.int64 not in dts:
            return None
        fdt = dts[0] if dts[1] == torch.int64 else dts[1]
        return fdt if fdt in (torch.float32, torch.bfloat16, torch.float16, torch.float64) else None

    def aggregate_grouped(self, groups: Sequence[Sequence[int]], mode: int, coef: Optional[Sequence[float]],
                          divisor: float, group_mode: int, group_coef: Optional[Sequence[float]] = None,
                          group_divisor: Optional[Sequence[float]] = None) -> "OrderedDict[str, torch.Tensor]":
        """Two-level reduction over client groups in ONE pass per dtype group (fa_weighted_sum_grouped).
        ``coef`` is indexed like the concatenation of ``groups``.  Float dtype groups only."""
        self._wait_ingest()
        order = [i for g in groups for i in g]
        gptr = [0]
        for g in groups:
            gptr.append(gptr[-1] + len(g))
        outs: Dict[torch.dtype, torch.Tensor] = {}
        for dt, buf in self.bufs.items():
            if self.tiled:
                outs[dt] = self.engine.weighted_sum_grouped_tiled(buf, order, mode, coef, divisor, gptr, group_mode,
                                                                  group_coef, group_divisor,
                                                                  n=self.layout.group_numel[dt])
            else:
                outs[dt] = self.engine.weighted_sum_grouped([buf[i] for i in order], mode, coef, divisor, gptr,
                                                            group_mode, group_coef, group_divisor)
        return self.layout.carve(outs)

    def hierarchical(self, groups: Sequence[Sequence[int]], counts: Sequence[int], formula: str = "sp"):
        """Hierarchical FedAvg of a round in one pass: group FedAvg (weights n_i / N_g), then
        formula "sp": global = sum_g G_g * (N_g / N)       (sp/hierarchical_fl/trainer.py:108-110)
        formula "cloud": global = sum_g (G_g * N_g) / N   (HierFedAvgCloudAggregator.py:140-157)."""
        w, gn = [], []
        for g in groups:
            Ng = sum(counts[i] for i in g)
            gn.append(Ng)
            w += [counts[i] / Ng for i in g]
        N = sum(gn)
        if formula == "sp":
            return self.aggregate_grouped(groups, MUL_W, w, 1.0, MUL_W, [n / N for n in gn])
        return self.aggregate_grouped(groups, MUL_W, w, 1.0, MUL_N_DIV_N, gn, [float(N)] * len(gn))

    def fedavg(self, counts: Sequence[int], clients: Optional[Sequence[int]] = None):
        """FedMLAggOperator.agg FedAvg branch (agg_operator.py:35-44) over the arena rows."""
        N = sum(counts)
        return self.aggregate(MUL_W, [c / N for c in counts], clients=clients)




def resident_rows(dicts, keys=None):
    """(arena, rows) when every dict of ``dicts`` was adopted by ONE client-major arena and still
    holds exactly that arena's row views, keys in the layout's order (checked in C++ by
    fedml_amd._host.match_rows: the key order, each value's address, contiguity, dtype and shape);
    else None."""
    first = _ADOPTED.get(id(dicts[0]))
    if first is None:
        return None
    arena = first[0]()
    if arena is None:
        return None
    rows = []
    for d in dicts:
        e = _ADOPTED.get(id(d))
        if e is None or e[0]() is not arena:
            return None
        rows.append(e[1])
    base, stride, meta, moff = arena._ptr_table()
    if not _host.match_rows(list(dicts), arena.layout.keys, base, stride, rows, meta, moff):
        return None
    return arena, rows
