"""AggEngine: the device-side aggregation engine over torch tensors (one per HIP device).

Thin host layer over libfedagg.so: validates tensors, builds the pointer tables the C ABI takes,
and launches on the current torch stream.  All arithmetic happens in the HIP kernels
(fedml_amd/csrc/fedagg.hip); this module never computes results on the CPU.
"""
from __future__ import annotations

import os
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _native as N

MUL_W, MUL_N_DIV_N, SUM = N.MUL_W, N.MUL_N_DIV_N, N.SUM

DTYPE_CODE = {
    torch.float32: N.F32,
    torch.bfloat16: N.BF16,
    torch.float16: N.F16,
    torch.float64: N.F64,
    torch.int64: N.I64,
}


def out_dtype(dtype: torch.dtype, mode: int) -> torch.dtype:
    """Result dtype of the reference's op sequence for an input dtype (PyTorch promotion)."""
    if dtype == torch.int64 and mode != SUM:
        return torch.float32
    return dtype


def _require_device(t: torch.Tensor, dev: torch.device, what: str):
    if t.device != dev:
        raise ValueError(f"{what}: tensor on {t.device}, engine on {dev}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: tensor must be contiguous")


class _LockedLib:
    """The native library with every call made under the engine's lock.  One fa_ctx per device is
    shared by every thread of the process (the engine is a per-device singleton), while the C ABI
    allows one thread per context at a time (include/fedagg.h: the staging-slot ring); ctypes
    releases the GIL during the call, so the lock is what serialises two receive threads."""

    def __init__(self, lib, lock):
        self._l = lib
        self._lock = lock

    def __getattr__(self, name):
        fn = getattr(self._l, name)
        lock = self._lock

        def call(*a):
            with lock:
                return fn(*a)
        call.__name__ = name
        setattr(self, name, call)
        return call


class AggEngine:
    """One native context bound to one HIP device.  Thread-safe: native launches and the host
    staging of ``state_dict_agg`` are serialised by ``self.lock`` (a re-entrant lock)."""

    _engines: Dict[int, "AggEngine"] = {}
    _elock = threading.Lock()

    def __init__(self, device: Optional[int] = None):
        if not torch.cuda.is_available():
            raise N.FedAggNativeError("no HIP device visible: the aggregation engine runs on MI355X only")
        self.device_index = torch.cuda.current_device() if device is None else int(device)
        self.device = torch.device("cuda", self.device_index)
        L = N.lib()
        h = N.ctypes.c_void_p()
        N.check(L.fa_ctx_create(self.device_index, N.ctypes.byref(h)), "fa_ctx_create")
        self._ctx = h
        self.lock = threading.RLock()
        self._lib = _LockedLib(L, self.lock)

    @classmethod
    def get(cls, device: Optional[int] = None) -> "AggEngine":
        idx = torch.cuda.current_device() if device is None else int(device)
        with cls._elock:
            eng = cls._engines.get(idx)
            if eng is None:
                eng = cls._engines[idx] = AggEngine(idx)
            return eng

    def close(self):
        for h in getattr(self, "_owned_streams", []):
            self._lib.fa_stream_destroy(N.ctypes.c_void_p(h))
        self._owned_streams = []
        if getattr(self, "_ctx", None) is not None and self._ctx.value:
            self._lib.fa_ctx_destroy(self._ctx)
            self._ctx = N.ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_variant(self, variant: int):
        N.check(self._lib.fa_ctx_set_variant(self._ctx, int(variant)), "fa_ctx_set_variant")

    def set_mix_band(self, enable: bool):
        N.check(self._lib.fa_ctx_set_mix_band(self._ctx, int(bool(enable))), "fa_ctx_set_mix_band")

    def cu_masked_stream(self, cu_count: int) -> torch.cuda.ExternalStream:
        """A torch stream whose kernels run on ``cu_count`` CUs of this device
        (fa_stream_create_cu_masked); kept alive for the engine's lifetime."""
        h = N.ctypes.c_void_p()
        N.check(self._lib.fa_stream_create_cu_masked(self.device_index, int(cu_count), N.ctypes.byref(h)),
                "fa_stream_create_cu_masked")
        self._owned_streams = getattr(self, "_owned_streams", []) + [h.value]
        return torch.cuda.ExternalStream(h.value, device=self.device)

    def _stream(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return N.ctypes.c_void_p(s.cuda_stream)

    def read_probe(self, buf: torch.Tensor, rows_per_workgroup: int, stream=None) -> None:
        """Measurement only (fa_read_probe): stream ``buf``'s bytes in the weighted-sum kernel's
        tiled read pattern -- ``rows_per_workgroup`` consecutive 4-KiB rows per workgroup, no
        arithmetic, no output stream.  Asynchronous; time it with events on ``stream``."""
        if buf.device != self.device or not buf.is_contiguous():
            raise ValueError("read_probe: a contiguous tensor on this engine's device is required")
        word = self.__dict__.get("_probe_word")
        if word is None:
            word = self._probe_word = torch.zeros(1, dtype=torch.int32, device=self.device)
        N.check(self._lib.fa_read_probe(self._ctx, N.ctypes.c_void_p(buf.data_ptr()),
                                        buf.numel() * buf.element_size(), int(rows_per_workgroup),
                                        N.ctypes.c_void_p(word.data_ptr()), self._stream(stream)), "fa_read_probe")

    def alloc_contiguous(self, nbytes: int) -> Optional[torch.Tensor]:
        """``nbytes`` of physically contiguous device memory (fa_device_alloc_contiguous) as a uint8
        tensor (view it as the arena's dtype), freed when its storage is; None when the device has
        no contiguous range that large.  Arena storage: see ClientArena."""
        p = N.ctypes.c_void_p()
        if self._lib.fa_device_alloc_contiguous(self._ctx, int(nbytes), N.ctypes.byref(p)) != N.FA_OK or not p.value:
            return None
        return torch.as_tensor(_DeviceBlock(self, p.value, int(nbytes)), device=self.device)

    def _scratch(self, name: str, need: int, stream=None) -> torch.Tensor:
        """Device scratch of >= need bytes, cached per (name, stream): calls queued on different
        streams never share one, and a buffer replaced while a kernel on ``stream`` may still read it
        is only reused by the allocator after that stream's queued work (record_stream)."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        cache = self.__dict__.setdefault("_scratch_cache", {})
        key = (name, s.cuda_stream)
        t = cache.get(key)
        if t is None or t.numel() < need:
            t = torch.empty(max(int(need), 1), dtype=torch.uint8, device=self.device)
            t.record_stream(s)
            cache[key] = t
        return t

    # ------------------------------------------------------------------ weighted sums
    def weighted_sum(self, xs: Sequence[torch.Tensor], mode: int, coef: Optional[Sequence[float]] = None,
                     divisor: float = 1.0, out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """Ordered reduction over clients of same-shape device tensors (include/fedagg.h)."""
        return self.weighted_sum_multi([list(xs)], mode, coef, divisor,
                                       outs=None if out is None else [out], stream=stream)[0]

    def weighted_sum_multi(self, segments: Sequence[Sequence[torch.Tensor]], mode: int,
                           coef: Optional[Sequence[float]] = None, divisor: float = 1.0,
                           outs: Optional[Sequence[torch.Tensor]] = None, stream=None) -> List[torch.Tensor]:
        """segments[s][i] = client i's tensor for key s (one dtype for all); one launch."""
        if len(segments) == 0:
            return []
        k = len(segments[0])
        if k == 0:
            raise ValueError("weighted_sum: no client tensors")
        dt = segments[0][0].dtype
        if dt not in DTYPE_CODE:
            raise TypeError(f"weighted_sum: unsupported dtype {dt}")
        if mode != SUM and (coef is None or len(coef) != k):
            raise ValueError("weighted_sum: need one coefficient per client")
        odt = out_dtype(dt, mode)
        numels, in_ptrs, out_ptrs, results = [], [], [], []
        for s, seg in enumerate(segments):
            if len(seg) != k:
                raise ValueError(f"segment {s}: {len(seg)} clients, expected {k}")
            shape = seg[0].shape
            for i, t in enumerate(seg):
                if t.dtype != dt:
                    raise TypeError(f"segment {s} client {i}: dtype {t.dtype} != {dt}")
                if t.shape != shape:
                    raise RuntimeError(f"segment {s} client {i}: shape {tuple(t.shape)} != {tuple(shape)}")
                _require_device(t, self.device, f"segment {s} client {i}")
                in_ptrs.append(t.data_ptr())
            if outs is not None:
                o = outs[s]
                if o.dtype != odt or o.numel() != seg[0].numel():
                    raise ValueError(f"segment {s}: output must be {odt} with {seg[0].numel()} elements")
                _require_device(o, self.device, f"segment {s} output")
            else:
                o = torch.empty(shape, dtype=odt, device=self.device)
            results.append(o)
            out_ptrs.append(o.data_ptr())
            numels.append(seg[0].numel())
        c = N.f64_array(coef if coef is not None else [0.0] * k)
        rc = self._lib.fa_weighted_sum_multi(
            self._ctx, DTYPE_CODE[dt], int(mode), len(segments), N.i64_array(numels), k,
            N.ptr_array(in_ptrs), c, float(divisor), N.ptr_array(out_ptrs), self._stream(stream))
        N.check(rc, "fa_weighted_sum_multi")
        return results

    def weighted_sum_rows(self, buf: torch.Tensor, rows: Sequence[int], mode: int,
                          coef: Optional[Sequence[float]] = None, divisor: float = 1.0,
                          out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """Ordered reduction over rows of ONE 2-D device tensor (a ClientArena dtype group):
        pointers are computed from the base address, so the host cost is O(1) tensor checks."""
        if buf.dim() != 2 or not buf.is_contiguous():
            raise ValueError("weighted_sum_rows: buf must be a contiguous 2-D tensor")
        _require_device(buf, self.device, "arena")
        dt = buf.dtype
        if dt not in DTYPE_CODE:
            raise TypeError(f"weighted_sum_rows: unsupported dtype {dt}")
        k = len(rows)
        if k == 0:
            raise ValueError("weighted_sum_rows: no rows")
        nrow, ncol = buf.shape
        if min(rows) < 0 or max(rows) >= nrow:
            raise IndexError("weighted_sum_rows: row out of range")
        if mode != SUM and (coef is None or len(coef) != k):
            raise ValueError("weighted_sum_rows: need one coefficient per row")
        odt = out_dtype(dt, mode)
        if out is None:
            out = torch.empty(ncol, dtype=odt, device=self.device)
        elif out.dtype != odt or out.numel() != ncol:
            raise ValueError(f"weighted_sum_rows: output must be {odt} with {ncol} elements")
        _require_device(out, self.device, "output")
        base, stride = buf.data_ptr(), ncol * buf.element_size()
        rc = self._lib.fa_weighted_sum(
            self._ctx, DTYPE_CODE[dt], int(mode), ncol, k, N.ptr_array([base + r * stride for r in rows]),
            N.f64_array(coef) if coef is not None else None, float(divisor), out.data_ptr(), self._stream(stream))
        N.check(rc, "fa_weighted_sum")
        return out

    def _tiled_args(self, buf: torch.Tensor, rows: Sequence[int], t0: int, n: Optional[int], what: str):
        """Pointer table of a tile-interleaved arena group ``buf`` = [tiles, capacity, E] (E elements =
        N.TILE_BYTES): rows ``rows`` starting at tile ``t0``, ``n`` logical elements."""
        if buf.dim() != 3 or not buf.is_contiguous() or buf.shape[2] * buf.element_size() != N.TILE_BYTES:
            raise ValueError(f"{what}: buf must be a contiguous [tiles, capacity, {N.TILE_BYTES}-byte tile] tensor")
        _require_device(buf, self.device, "arena")
        if buf.dtype not in DTYPE_CODE:
            raise TypeError(f"{what}: unsupported dtype {buf.dtype}")
        ntile, cap, E = buf.shape
        if len(rows) == 0:
            raise ValueError(f"{what}: no rows")
        if min(rows) < 0 or max(rows) >= cap:
            raise IndexError(f"{what}: row out of range")
        if not 0 <= t0 <= ntile:
            raise IndexError(f"{what}: first tile {t0} out of range")
        avail = (ntile - t0) * E
        n = avail if n is None else int(n)
        if not 0 <= n <= avail:
            raise ValueError(f"{what}: {n} elements from tile {t0} exceed the arena ({avail})")
        stride = cap * N.TILE_BYTES
        base = buf.data_ptr() + t0 * stride
        return n, N.ptr_array([base + r * N.TILE_BYTES for r in rows]), stride

    def weighted_sum_tiled(self, buf: torch.Tensor, rows: Sequence[int], mode: int,
                           coef: Optional[Sequence[float]] = None, divisor: float = 1.0, n: Optional[int] = None,
                           t0: int = 0, out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """Ordered reduction over rows of a TILE-INTERLEAVED arena group (fa_weighted_sum_tiled):
        ``buf[t, r, :]`` is tile t of client row r, so one workgroup's K tiles are one contiguous run.
        Reduces ``n`` elements (default: all) starting at tile ``t0``; the output is flat."""
        n, ptrs, stride = self._tiled_args(buf, rows, t0, n, "weighted_sum_tiled")
        k = len(rows)
        if mode != SUM and (coef is None or len(coef) != k):
            raise ValueError("weighted_sum_tiled: need one coefficient per row")
        odt = out_dtype(buf.dtype, mode)
        if out is None:
            out = torch.empty(n, dtype=odt, device=self.device)
        elif out.dtype != odt or out.numel() != n:
            raise ValueError(f"weighted_sum_tiled: output must be {odt} with {n} elements")
        _require_device(out, self.device, "output")
        rc = self._lib.fa_weighted_sum_tiled(
            self._ctx, DTYPE_CODE[buf.dtype], int(mode), n, k, ptrs, stride,
            N.f64_array(coef) if coef is not None else None, float(divisor), out.data_ptr(), self._stream(stream))
        N.check(rc, "fa_weighted_sum_tiled")
        return out

    def weighted_sum_pair(self, buf: torch.Tensor, buf_i64: torch.Tensor, rows: Sequence[int], mode: int,
                          coef: Optional[Sequence[float]] = None, divisor: float = 1.0, n: Optional[int] = None,
                          n_i64: Optional[int] = None, out: Optional[torch.Tensor] = None,
                          out_i64: Optional[torch.Tensor] = None, stream=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """A float arena group and the int64 arena group of the same clients in ONE launch
        (fa_weighted_sum_pair).  Both groups are row-major [capacity, numel] or both tiled
        [tiles, capacity, E]; returns the two flat outputs (same bits as two separate launches)."""
        if buf_i64.dtype != torch.int64 or buf.dtype not in (torch.float32, torch.bfloat16, torch.float16,
                                                             torch.float64):
            raise TypeError("weighted_sum_pair: a float group and an int64 group")
        if buf.dim() != buf_i64.dim() or buf.dim() not in (2, 3):
            raise ValueError("weighted_sum_pair: both groups row-major (2-D) or both tiled (3-D)")
        k = len(rows)
        if mode != SUM and (coef is None or len(coef) != k):
            raise ValueError("weighted_sum_pair: need one coefficient per row")
        tabs = []
        for b, nn in ((buf, n), (buf_i64, n_i64)):
            if b.dim() == 3:
                nn, ptrs, stride = self._tiled_args(b, rows, 0, nn, "weighted_sum_pair")
            else:
                if not b.is_contiguous():
                    raise ValueError("weighted_sum_pair: buf must be contiguous")
                _require_device(b, self.device, "arena")
                if k == 0:
                    raise ValueError("weighted_sum_pair: no rows")
                if min(rows) < 0 or max(rows) >= b.shape[0]:
                    raise IndexError("weighted_sum_pair: row out of range")
                ncol = b.shape[1]
                nn = ncol if nn is None else int(nn)
                if not 0 <= nn <= ncol:
                    raise ValueError("weighted_sum_pair: n exceeds the row")
                rs = ncol * b.element_size()
                ptrs, stride = N.ptr_array([b.data_ptr() + r * rs for r in rows]), 0
            tabs.append((nn, ptrs, stride))
        outs = []
        for b, o, (nn, _, _) in ((buf, out, tabs[0]), (buf_i64, out_i64, tabs[1])):
            odt = out_dtype(b.dtype, mode)
            if o is None:
                o = torch.empty(nn, dtype=odt, device=self.device)
            elif o.dtype != odt or o.numel() != nn:
                raise ValueError(f"weighted_sum_pair: output must be {odt} with {nn} elements")
            _require_device(o, self.device, "output")
            outs.append(o)
        rc = self._lib.fa_weighted_sum_pair(
            self._ctx, DTYPE_CODE[buf.dtype], int(mode), tabs[0][0], tabs[1][0], k, tabs[0][1], tabs[1][1],
            tabs[0][2], tabs[1][2], N.f64_array(coef) if coef is not None else None, float(divisor),
            outs[0].data_ptr(), outs[1].data_ptr(), self._stream(stream))
        N.check(rc, "fa_weighted_sum_pair")
        return outs[0], outs[1]

    def weighted_sum_tiled_multi(self, buf: torch.Tensor, rows: Sequence[int], mode: int,
                                 coef: Optional[Sequence[float]], divisor: float,
                                 ranges: Sequence[Tuple[int, int]], outs: Sequence[torch.Tensor],
                                 stream=None) -> None:
        """Several element ranges [lo, hi) (tile-aligned starts) of a tiled arena group reduced in ONE
        launch (fa_weighted_sum_tiled_multi) into ``outs`` (flat, hi - lo elements each)."""
        ntile, cap, E = buf.shape
        k = len(rows)
        if mode != SUM and (coef is None or len(coef) != k):
            raise ValueError("weighted_sum_tiled_multi: need one coefficient per row")
        odt = out_dtype(buf.dtype, mode)
        if len(ranges) != len(outs) or not ranges:
            raise ValueError("weighted_sum_tiled_multi: one output per range")
        ptrs, numels = [], []
        for (lo, hi), o in zip(ranges, outs):
            if lo % E:
                raise ValueError("weighted_sum_tiled_multi: ranges must start on a tile")
            n, p, stride = self._tiled_args(buf, rows, lo // E, hi - lo, "weighted_sum_tiled_multi")
            if o.dtype != odt or o.numel() != n:
                raise ValueError(f"weighted_sum_tiled_multi: output must be {odt} with {n} elements")
            _require_device(o, self.device, "output")
            ptrs.extend(p)
            numels.append(n)
        rc = self._lib.fa_weighted_sum_tiled_multi(
            self._ctx, DTYPE_CODE[buf.dtype], int(mode), len(ranges), N.i64_array(numels), k,
            N.ptr_array(ptrs), cap * N.TILE_BYTES, N.f64_array(coef) if coef is not None else None, float(divisor),
            N.ptr_array([o.data_ptr() for o in outs]), self._stream(stream))
        N.check(rc, "fa_weighted_sum_tiled_multi")

    def weighted_sum_grouped_tiled(self, buf: torch.Tensor, rows: Sequence[int], mode: int,
                                   coef: Optional[Sequence[float]], divisor: float, group_ptr: Sequence[int],
                                   group_mode: int, group_coef: Optional[Sequence[float]] = None,
                                   group_divisor: Optional[Sequence[float]] = None, n: Optional[int] = None,
                                   t0: int = 0, out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """fa_weighted_sum_grouped over rows of a tile-interleaved arena group (see weighted_sum_tiled)."""
        if buf.dtype not in (torch.float32, torch.bfloat16, torch.float16, torch.float64):
            raise TypeError(f"weighted_sum_grouped_tiled: unsupported dtype {buf.dtype}")
        n, ptrs, stride = self._tiled_args(buf, rows, t0, n, "weighted_sum_grouped_tiled")
        if out is None:
            out = torch.empty(n, dtype=buf.dtype, device=self.device)
        elif out.dtype != buf.dtype or out.numel() != n:
            raise ValueError(f"weighted_sum_grouped_tiled: output must be {buf.dtype} with {n} elements")
        _require_device(out, self.device, "output")
        rc = self._lib.fa_weighted_sum_grouped_tiled(
            self._ctx, DTYPE_CODE[buf.dtype], int(mode), n, len(rows), ptrs, stride,
            N.f64_array(coef) if coef is not None else None, float(divisor), len(group_ptr) - 1,
            N.i32_array(group_ptr), int(group_mode), N.f64_array(group_coef) if group_coef is not None else None,
            N.f64_array(group_divisor) if group_divisor is not None else None, out.data_ptr(), self._stream(stream))
        N.check(rc, "fa_weighted_sum_grouped_tiled")
        return out

    def weighted_sum_grouped(self, xs: Sequence[torch.Tensor], mode: int, coef: Optional[Sequence[float]],
                             divisor: float, group_ptr: Sequence[int], group_mode: int,
                             group_coef: Optional[Sequence[float]] = None,
                             group_divisor: Optional[Sequence[float]] = None,
                             out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """Two-level ordered reduction in one pass (fa_weighted_sum_grouped): groups of clients
        [group_ptr[g], group_ptr[g+1]), group epilogue `group_mode`, ordered sum over groups."""
        k = len(xs)
        if k == 0:
            raise ValueError("weighted_sum_grouped: no client tensors")
        dt, shape = xs[0].dtype, xs[0].shape
        if dt not in (torch.float32, torch.bfloat16, torch.float16, torch.float64):
            raise TypeError(f"weighted_sum_grouped: unsupported dtype {dt}")
        for i, t in enumerate(xs):
            if t.dtype != dt or t.shape != shape:
                raise ValueError(f"client {i}: dtype/shape mismatch")
            _require_device(t, self.device, f"client {i}")
        G = len(group_ptr) - 1
        if out is None:
            out = torch.empty(shape, dtype=dt, device=self.device)
        _require_device(out, self.device, "output")
        rc = self._lib.fa_weighted_sum_grouped(
            self._ctx, DTYPE_CODE[dt], int(mode), xs[0].numel(), k, N.ptr_array([t.data_ptr() for t in xs]),
            N.f64_array(coef) if coef is not None else None, float(divisor), G, N.i32_array(group_ptr),
            int(group_mode), N.f64_array(group_coef) if group_coef is not None else None,
            N.f64_array(group_divisor) if group_divisor is not None else None, out.data_ptr(),
            self._stream(stream))
        N.check(rc, "fa_weighted_sum_grouped")
        return out

    def fedavg_sgd(self, segments: Sequence[Sequence[torch.Tensor]], coef: Sequence[float],
                   params: Sequence[torch.Tensor], momentum_bufs: Optional[Sequence[torch.Tensor]],
                   lr: float, momentum: float = 0.0, dampening: float = 0.0, weight_decay: float = 0.0,
                   nesterov: bool = False, first_step: bool = True, stream=None) -> None:
        """FedAvg + torch.optim.SGD server step in one pass (fa_fedavg_sgd); params and momentum
        buffers (fp32, contiguous, on this device) are updated in place."""
        k = len(segments[0]) if segments else 0
        if k == 0:
            raise ValueError("fedavg_sgd: no client tensors")
        if len(coef) != k or len(params) != len(segments):
            raise ValueError("fedavg_sgd: one coefficient per client and one parameter per segment")
        in_ptrs, numels = [], []
        for s, (seg, p) in enumerate(zip(segments, params)):
            if p.dtype != torch.float32:
                raise TypeError(f"fedavg_sgd: parameter {s} is {p.dtype} (float32 only)")
            _require_device(p, self.device, f"parameter {s}")
            if len(seg) != k:
                raise ValueError(f"segment {s}: {len(seg)} clients, expected {k}")
            for i, t in enumerate(seg):
                if t.dtype != torch.float32 or t.shape != p.shape:
                    raise ValueError(f"segment {s} client {i}: must be float32 of shape {tuple(p.shape)}")
                _require_device(t, self.device, f"segment {s} client {i}")
                in_ptrs.append(t.data_ptr())
            numels.append(p.numel())
        if momentum != 0.0:
            if momentum_bufs is None or len(momentum_bufs) != len(params):
                raise ValueError("fedavg_sgd: momentum needs one buffer per parameter")
            for b, p in zip(momentum_bufs, params):
                if b.dtype != torch.float32 or b.shape != p.shape:
                    raise ValueError("fedavg_sgd: momentum buffer dtype/shape mismatch")
                _require_device(b, self.device, "momentum buffer")
            mptr = N.ptr_array([b.data_ptr() for b in momentum_bufs])
        else:
            mptr = None
        rc = self._lib.fa_fedavg_sgd(
            self._ctx, len(params), N.i64_array(numels), k, N.ptr_array(in_ptrs), N.f64_array(coef),
            N.ptr_array([p.data_ptr() for p in params]), mptr, float(lr), float(momentum), float(dampening),
            float(weight_decay), int(bool(nesterov)), int(bool(first_step)), self._stream(stream))
        N.check(rc, "fa_fedavg_sgd")

    def fedavg_rmsprop(self, segments: Sequence[Sequence[torch.Tensor]], coef: Sequence[float],
                       params: Sequence[torch.Tensor], square_avgs: Sequence[torch.Tensor],
                       momentum_bufs: Optional[Sequence[torch.Tensor]], lr: float, alpha: float = 0.99,
                       eps: float = 1e-8, weight_decay: float = 0.0, momentum: float = 0.0,
                       first_step: bool = True, stream=None) -> None:
        """FedAvg + torch.optim.RMSprop server step in one pass (fa_fedavg_rmsprop); params, square
        averages and momentum buffers (fp32, contiguous, on this device) are updated in place."""
        k = len(segments[0]) if segments else 0
        if k == 0:
            raise ValueError("fedavg_rmsprop: no client tensors")
        if len(coef) != k or len(params) != len(segments) or len(square_avgs) != len(params):
            raise ValueError("fedavg_rmsprop: one coefficient per client, one parameter and state per segment")
        in_ptrs, numels = [], []
        for s, (seg, p, q) in enumerate(zip(segments, params, square_avgs)):
            for t, what in ((p, "parameter"), (q, "square_avg")):
                if t.dtype != torch.float32 or t.shape != p.shape:
                    raise TypeError(f"fedavg_rmsprop: {what} {s} must be float32 of shape {tuple(p.shape)}")
                _require_device(t, self.device, f"{what} {s}")
            if len(seg) != k:
                raise ValueError(f"segment {s}: {len(seg)} clients, expected {k}")
            for i, t in enumerate(seg):
                if t.dtype != torch.float32 or t.shape != p.shape:
                    raise ValueError(f"segment {s} client {i}: must be float32 of shape {tuple(p.shape)}")
                _require_device(t, self.device, f"segment {s} client {i}")
                in_ptrs.append(t.data_ptr())
            numels.append(p.numel())
        mptr = None
        if momentum != 0.0:
            if momentum_bufs is None or len(momentum_bufs) != len(params):
                raise ValueError("fedavg_rmsprop: momentum needs one buffer per parameter")
            for b, p in zip(momentum_bufs, params):
                if b.dtype != torch.float32 or b.shape != p.shape:
                    raise ValueError("fedavg_rmsprop: momentum buffer dtype/shape mismatch")
                _require_device(b, self.device, "momentum buffer")
            mptr = N.ptr_array([b.data_ptr() for b in momentum_bufs])
        rc = self._lib.fa_fedavg_rmsprop(
            self._ctx, len(params), N.i64_array(numels), k, N.ptr_array(in_ptrs), N.f64_array(coef),
            N.ptr_array([p.data_ptr() for p in params]), N.ptr_array([q.data_ptr() for q in square_avgs]), mptr,
            float(lr), float(alpha), float(eps), float(weight_decay), float(momentum), int(bool(first_step)),
            self._stream(stream))
        N.check(rc, "fa_fedavg_rmsprop")

    def fedavg_sgd_tiled(self, buf: torch.Tensor, rows: Sequence[int], coef: Sequence[float], param: torch.Tensor,
                         momentum_buf: Optional[torch.Tensor], lr: float, momentum: float = 0.0,
                         dampening: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False,
                         first_step: bool = True, stream=None) -> None:
        """fedavg_sgd of ONE flat fp32 parameter over rows of a tile-interleaved arena group
        (fa_fedavg_sgd_tiled); ``param`` / ``momentum_buf`` updated in place."""
        if buf.dtype != torch.float32 or param.dtype != torch.float32:
            raise TypeError("fedavg_sgd_tiled: float32 only")
        n, ptrs, stride = self._tiled_args(buf, rows, 0, param.numel(), "fedavg_sgd_tiled")
        if len(coef) != len(rows):
            raise ValueError("fedavg_sgd_tiled: one coefficient per row")
        _require_device(param, self.device, "parameter")
        if momentum != 0.0:
            if momentum_buf is None or momentum_buf.dtype != torch.float32 or momentum_buf.numel() != n:
                raise ValueError("fedavg_sgd_tiled: momentum needs a float32 buffer like the parameter")
            _require_device(momentum_buf, self.device, "momentum buffer")
        rc = self._lib.fa_fedavg_sgd_tiled(
            self._ctx, n, len(rows), ptrs, stride, N.f64_array(coef), param.data_ptr(),
            momentum_buf.data_ptr() if momentum != 0.0 else None, float(lr), float(momentum), float(dampening),
            float(weight_decay), int(bool(nesterov)), int(bool(first_step)), self._stream(stream))
        N.check(rc, "fa_fedavg_sgd_tiled")

    def weighted_sum_table(self, dtype_code: int, mode: int, seg_numel: torch.Tensor, k: int,
                           in_ptrs: torch.Tensor, out_ptrs: torch.Tensor, coef: Optional[Sequence[float]] = None,
                           divisor: float = 1.0, stream=None) -> None:
        """Raw multi-segment launch from prebuilt host tables (int64 CPU tensors):
        seg_numel[T], in_ptrs[T*k] (key-major device pointers), out_ptrs[T].  Used by the
        state_dict path, whose tables are built and validated by fedml_amd._host."""
        T = seg_numel.numel()
        assert in_ptrs.dtype == torch.int64 and in_ptrs.numel() == T * k and in_ptrs.is_contiguous()
        assert out_ptrs.dtype == torch.int64 and out_ptrs.numel() == T and out_ptrs.is_contiguous()
        assert seg_numel.dtype == torch.int64 and seg_numel.is_contiguous()
        if mode != SUM and (coef is None or len(coef) != k):
            raise ValueError("weighted_sum: need one coefficient per client")
        c = N.f64_array(coef if coef is not None else [0.0] * k)
        rc = self._lib.fa_weighted_sum_multi(
            self._ctx, int(dtype_code), int(mode), T,
            N.ctypes.cast(seg_numel.data_ptr(), N._P_i64), k,
            N.ctypes.cast(in_ptrs.data_ptr(), N._P_vp), c, float(divisor),
            N.ctypes.cast(out_ptrs.data_ptr(), N._P_vp), self._stream(stream))
        N.check(rc, "fa_weighted_sum_multi")

    def host_round_abi(self):
        """(fa_weighted_sum_host, fa_last_error, fa_ctx*) as integer addresses, for the one-call small
        host round (_host.small_host_round), which calls the C ABI directly."""
        a = getattr(self, "_host_round_abi", None)
        if a is None:
            L = N.lib()
            a = self._host_round_abi = (N.ctypes.cast(L.fa_weighted_sum_host, N.ctypes.c_void_p).value,
                                        N.ctypes.cast(L.fa_last_error, N.ctypes.c_void_p).value, self._ctx.value)
        return a

    def weighted_sum_host_table(self, dtype_code: int, mode: int, seg_numel: torch.Tensor, k: int,
                                in_ptrs: torch.Tensor, out_ptrs: torch.Tensor, coef: Optional[Sequence[float]] = None,
                                divisor: float = 1.0, stream=None) -> None:
        """fa_weighted_sum_host from prebuilt tables of HOST pointers (int64 CPU tensors, as
        weighted_sum_table): synchronous, the kernel reads and writes mapped pinned memory."""
        T = seg_numel.numel()
        assert in_ptrs.dtype == torch.int64 and in_ptrs.numel() == T * k and in_ptrs.is_contiguous()
        assert out_ptrs.dtype == torch.int64 and out_ptrs.numel() == T and out_ptrs.is_contiguous()
        assert seg_numel.dtype == torch.int64 and seg_numel.is_contiguous()
        if mode != SUM and (coef is None or len(coef) != k):
            raise ValueError("weighted_sum: need one coefficient per client")
        c = N.f64_array(coef if coef is not None else [0.0] * k)
        rc = self._lib.fa_weighted_sum_host(
            self._ctx, int(dtype_code), int(mode), T, N.ctypes.cast(seg_numel.data_ptr(), N._P_i64), k,
            N.ctypes.cast(in_ptrs.data_ptr(), N._P_vp), c, float(divisor),
            N.ctypes.cast(out_ptrs.data_ptr(), N._P_vp), self._stream(stream))
        N.check(rc, "fa_weighted_sum_host")

    def weighted_sum_table_pair(self, dtype_code: int, mode: int, numel0: torch.Tensor, in0: torch.Tensor,
                                out0: torch.Tensor, numel1: torch.Tensor, in1: torch.Tensor, out1: torch.Tensor,
                                k: int, coef: Optional[Sequence[float]] = None, divisor: float = 1.0,
                                stream=None) -> None:
        """A float group and the int64 group of a state_dict (prebuilt host tables as in
        weighted_sum_table) in ONE launch (fa_weighted_sum_pair_multi)."""
        for nm, it, ot in ((numel0, in0, out0), (numel1, in1, out1)):
            T = nm.numel()
            assert nm.dtype == torch.int64 and nm.is_contiguous()
            assert it.dtype == torch.int64 and it.numel() == T * k and it.is_contiguous()
            assert ot.dtype == torch.int64 and ot.numel() == T and ot.is_contiguous()
        if mode != SUM and (coef is None or len(coef) != k):
            raise ValueError("weighted_sum: need one coefficient per client")
        c = N.f64_array(coef if coef is not None else [0.0] * k)
        cast = N.ctypes.cast
        rc = self._lib.fa_weighted_sum_pair_multi(
            self._ctx, int(dtype_code), int(mode), numel0.numel(), cast(numel0.data_ptr(), N._P_i64),
            numel1.numel(), cast(numel1.data_ptr(), N._P_i64), k, cast(in0.data_ptr(), N._P_vp),
            cast(in1.data_ptr(), N._P_vp), c, float(divisor), cast(out0.data_ptr(), N._P_vp),
            cast(out1.data_ptr(), N._P_vp), self._stream(stream))
        N.check(rc, "fa_weighted_sum_pair_multi")

    def promote_add(self, acc: torch.Tensor, t: torch.Tensor, out: Optional[torch.Tensor] = None,
                    stream=None) -> torch.Tensor:
        """``acc += t`` across dtypes, PyTorch's in-place semantics (fa_promote_add): computed in
        promote_types(acc, t), rounded to acc's dtype.  acc a float tensor; returns ``out`` (default:
        a new tensor like acc; ``out=acc`` updates in place)."""
        if acc.dtype not in (torch.float32, torch.bfloat16, torch.float16, torch.float64):
            raise TypeError(f"promote_add: accumulator dtype {acc.dtype} must be a float type")
        if t.dtype not in DTYPE_CODE:
            raise TypeError(f"promote_add: term dtype {t.dtype} not supported")
        if t.numel() != acc.numel():
            raise RuntimeError(f"promote_add: {t.numel()} elements vs {acc.numel()}")
        _require_device(acc, self.device, "accumulator")
        _require_device(t, self.device, "term")
        if out is None:
            out = torch.empty_like(acc)
        elif out.dtype != acc.dtype or out.numel() != acc.numel():
            raise ValueError("promote_add: out must be like acc")
        _require_device(out, self.device, "output")
        rc = self._lib.fa_promote_add(self._ctx, DTYPE_CODE[acc.dtype], DTYPE_CODE[t.dtype], acc.numel(),
                                      acc.data_ptr(), t.data_ptr(), out.data_ptr(), self._stream(stream))
        N.check(rc, "fa_promote_add")
        return out

    # ------------------------------------------------------------------ mixing / gossip
    def mix(self, xs: Sequence[torch.Tensor], row_ptr: Sequence[int], cols: Sequence[int],
            vals: Sequence[float], post_scale: Optional[Sequence[float]] = None,
            outs: Optional[Sequence[torch.Tensor]] = None, outs2: Optional[Sequence[torch.Tensor]] = None,
            stream=None) -> Tuple[List[torch.Tensor], Optional[List[torch.Tensor]]]:
        """CSR-ordered mixing rows over same-shape device tensors (fa_mix)."""
        if len(xs) == 0:
            raise ValueError("mix: no inputs")
        dt, shape = xs[0].dtype, xs[0].shape
        for i, t in enumerate(xs):
            if t.dtype != dt or t.shape != shape:
                raise ValueError(f"mix: input {i} dtype/shape mismatch")
            _require_device(t, self.device, f"mix input {i}")
        rows = len(row_ptr) - 1
        if outs is None:
            outs = [torch.empty(shape, dtype=dt, device=self.device) for _ in range(rows)]
        if post_scale is not None and outs2 is None:
            outs2 = [torch.empty(shape, dtype=dt, device=self.device) for _ in range(rows)]
        in_set = {t.data_ptr() for t in xs}
        for o in list(outs) + list(outs2 or []):
            _require_device(o, self.device, "mix output")
            if o.data_ptr() in in_set:
                raise ValueError("mix: outputs must not alias inputs")
        rc = self._lib.fa_mix(
            self._ctx, DTYPE_CODE.get(dt, -1), xs[0].numel(), rows, N.i32_array(row_ptr), N.i32_array(cols),
            N.f64_array(vals), len(xs), N.ptr_array([t.data_ptr() for t in xs]),
            N.ptr_array([o.data_ptr() for o in outs]),
            N.f64_array(post_scale) if post_scale is not None else None,
            N.ptr_array([o.data_ptr() for o in outs2]) if outs2 is not None else None,
            self._stream(stream))
        N.check(rc, "fa_mix")
        return list(outs), (list(outs2) if outs2 is not None else None)

    def pushsum(self, xs: Sequence[torch.Tensor], row_ptr: Sequence[int], cols: Sequence[int], vals: Sequence[float],
                omega_in: torch.Tensor, outs: Optional[Sequence[torch.Tensor]] = None,
                outs2: Optional[Sequence[torch.Tensor]] = None, omega_out: Optional[torch.Tensor] = None,
                stream=None) -> Tuple[List[torch.Tensor], List[torch.Tensor], torch.Tensor]:
        """One PushSum step with the weights on the device (fa_pushsum): mixed models, their z = x /
        omega', and omega' (float32, one per row), all computed on the GPU."""
        if len(xs) == 0:
            raise ValueError("pushsum: no inputs")
        dt, shape = xs[0].dtype, xs[0].shape
        for i, t in enumerate(xs):
            if t.dtype != dt or t.shape != shape:
                raise ValueError(f"pushsum: input {i} dtype/shape mismatch")
            _require_device(t, self.device, f"pushsum input {i}")
        rows = len(row_ptr) - 1
        if omega_in.dtype != torch.float32 or omega_in.numel() != len(xs):
            raise ValueError("pushsum: omega_in must be float32 with one weight per input")
        _require_device(omega_in, self.device, "omega_in")
        outs = list(outs) if outs is not None else [torch.empty(shape, dtype=dt, device=self.device) for _ in range(rows)]
        outs2 = list(outs2) if outs2 is not None else [torch.empty(shape, dtype=dt, device=self.device) for _ in range(rows)]
        if omega_out is None:
            omega_out = torch.empty(rows, dtype=torch.float32, device=self.device)
        elif omega_out.dtype != torch.float32 or omega_out.numel() != rows:
            raise ValueError("pushsum: omega_out must be float32 with one weight per row")
        _require_device(omega_out, self.device, "omega_out")
        in_set = {t.data_ptr() for t in xs}
        for o in outs + outs2:
            _require_device(o, self.device, "pushsum output")
            if o.data_ptr() in in_set:
                raise ValueError("pushsum: outputs must not alias inputs")
        rc = self._lib.fa_pushsum(
            self._ctx, DTYPE_CODE.get(dt, -1), xs[0].numel(), rows, N.i32_array(row_ptr), N.i32_array(cols),
            N.f64_array(vals), len(xs), N.ptr_array([t.data_ptr() for t in xs]), omega_in.data_ptr(),
            N.ptr_array([o.data_ptr() for o in outs]), N.ptr_array([o.data_ptr() for o in outs2]),
            omega_out.data_ptr(), self._stream(stream))
        N.check(rc, "fa_pushsum")
        return outs, outs2, omega_out

    def mix_tiled(self, buf_in: torch.Tensor, in_rows: Sequence[int], row_ptr: Sequence[int], cols: Sequence[int],
                  vals: Sequence[float], buf_out: torch.Tensor, out_rows: Sequence[int],
                  post_scale: Optional[Sequence[float]] = None, buf_out2: Optional[torch.Tensor] = None,
                  n: Optional[int] = None, stream=None) -> None:
        """fa_mix between tile-interleaved arena groups: input j = row in_rows[j] of ``buf_in``
        ([tiles, cap, E]); output row r -> row out_rows[r] of ``buf_out`` (and ``buf_out2`` with
        post_scale).  ``n`` logical elements (default: all)."""
        n, iptr, istride = self._tiled_args(buf_in, in_rows, 0, n, "mix_tiled")
        rows = len(row_ptr) - 1
        if len(out_rows) != rows:
            raise ValueError("mix_tiled: one output row per CSR row")
        for b in [buf_out] + ([buf_out2] if buf_out2 is not None else []):
            if b.dtype != buf_in.dtype or b.shape[0] != buf_in.shape[0] or b.shape[2] != buf_in.shape[2]:
                raise ValueError("mix_tiled: output arena must match the input arena's dtype and tiles")
            if b.data_ptr() == buf_in.data_ptr():
                raise ValueError("mix_tiled: outputs must not alias inputs")
        _, optr, ostride = self._tiled_args(buf_out, out_rows, 0, n, "mix_tiled output")
        optr2 = None
        if post_scale is not None:
            if buf_out2 is None:
                raise ValueError("mix_tiled: post_scale needs buf_out2")
            _, optr2, ostride2 = self._tiled_args(buf_out2, out_rows, 0, n, "mix_tiled output2")
            if ostride2 != ostride:
                raise ValueError("mix_tiled: buf_out2 must have buf_out's capacity")
        rc = self._lib.fa_mix_tiled(
            self._ctx, DTYPE_CODE.get(buf_in.dtype, -1), n, rows, N.i32_array(row_ptr), N.i32_array(cols),
            N.f64_array(vals), len(in_rows), iptr, istride, optr, ostride,
            N.f64_array(post_scale) if post_scale is not None else None, optr2, self._stream(stream))
        N.check(rc, "fa_mix_tiled")

    # ------------------------------------------------------------------ finite field (SecAgg)
    def finite_sum(self, segments: Sequence[Sequence[torch.Tensor]], prime: int, flags: int,
                   masks: Optional[Sequence[Optional[torch.Tensor]]] = None, finite: bool = True,
                   q_bits: Optional[int] = None, scale: float = 1.0,
                   stream=None) -> Tuple[Optional[List[torch.Tensor]], Optional[List[torch.Tensor]]]:
        """Finite-field client sum (fa_finite_sum) over int64 segments[s][i]; returns
        (finite int64 outputs or None, dequantized outputs or None): float32 (* scale), or my_q_inv's
        float64 with the REAL_F64 flag."""
        k = len(segments[0]) if segments else 0
        if k == 0:
            raise ValueError("finite_sum: no client tensors")
        if not finite and q_bits is None:
            raise ValueError("finite_sum: nothing to output")
        in_ptrs, numels, mptrs, fin, real = [], [], [], [], []
        for s, seg in enumerate(segments):
            if len(seg) != k:
                raise ValueError(f"segment {s}: {len(seg)} clients, expected {k}")
            shape = seg[0].shape
            for i, t in enumerate(seg):
                if t.dtype != torch.int64:
                    raise TypeError(f"finite_sum: segment {s} client {i} is {t.dtype} (int64 only)")
                if t.shape != shape:
                    raise RuntimeError(f"segment {s} client {i}: shape {tuple(t.shape)} != {tuple(shape)}")
                _require_device(t, self.device, f"segment {s} client {i}")
                in_ptrs.append(t.data_ptr())
            m = masks[s] if masks is not None else None
            if m is not None:
                if m.dtype != torch.int64 or m.numel() != seg[0].numel():
                    raise ValueError(f"finite_sum: mask {s} must be int64 with {seg[0].numel()} elements")
                _require_device(m, self.device, f"mask {s}")
            mptrs.append(m.data_ptr() if m is not None else None)
            numels.append(seg[0].numel())
            if finite:
                fin.append(torch.empty(shape, dtype=torch.int64, device=self.device))
            if q_bits is not None:
                rdt = torch.float64 if flags & N.REAL_F64 else torch.float32
                real.append(torch.empty(shape, dtype=rdt, device=self.device))
        rc = self._lib.fa_finite_sum(
            self._ctx, len(segments), N.i64_array(numels), k, N.ptr_array(in_ptrs),
            N.ptr_array(mptrs) if masks is not None else None, int(prime), int(flags),
            N.ptr_array([t.data_ptr() for t in fin]) if finite else None, int(q_bits or 0), float(scale),
            N.ptr_array([t.data_ptr() for t in real]) if q_bits is not None else None, self._stream(stream))
        N.check(rc, "fa_finite_sum")
        return (fin if finite else None), (real if q_bits is not None else None)

    def finite_sum_tiled(self, buf: torch.Tensor, rows: Sequence[int], prime: int, flags: int,
                         mask: Optional[torch.Tensor] = None, finite: bool = True, q_bits: Optional[int] = None,
                         scale: float = 1.0, n: Optional[int] = None, stream=None):
        """finite_sum over rows of a tile-interleaved int64 arena group (fa_finite_sum_tiled);
        returns (finite int64 output or None, dequantized output or None), flat."""
        if buf.dtype != torch.int64:
            raise TypeError("finite_sum_tiled: int64 arena only")
        if not finite and q_bits is None:
            raise ValueError("finite_sum_tiled: nothing to output")
        n, ptrs, stride = self._tiled_args(buf, rows, 0, n, "finite_sum_tiled")
        if mask is not None:
            if mask.dtype != torch.int64 or mask.numel() != n:
                raise ValueError(f"finite_sum_tiled: mask must be int64 with {n} elements")
            _require_device(mask, self.device, "mask")
        fin = torch.empty(n, dtype=torch.int64, device=self.device) if finite else None
        real = None
        if q_bits is not None:
            real = torch.empty(n, dtype=torch.float64 if flags & N.REAL_F64 else torch.float32, device=self.device)
        rc = self._lib.fa_finite_sum_tiled(
            self._ctx, n, len(rows), ptrs, stride, mask.data_ptr() if mask is not None else None, int(prime),
            int(flags), fin.data_ptr() if fin is not None else None, int(q_bits or 0), float(scale),
            real.data_ptr() if real is not None else None, self._stream(stream))
        N.check(rc, "fa_finite_sum_tiled")
        return fin, real

    def finite_quantize(self, xs: Sequence[torch.Tensor], prime: int, q_bits: int,
                        masks: Optional[Sequence[torch.Tensor]] = None, stream=None) -> List[torch.Tensor]:
        """my_q (+ model_masking with masks) of same-dtype device tensors (fa_finite_quantize)."""
        if len(xs) == 0:
            return []
        dt = xs[0].dtype
        if dt not in (torch.float32, torch.float64, torch.int64):
            raise TypeError(f"finite_quantize: unsupported dtype {dt} (float32, float64, int64)")
        outs = []
        for s, t in enumerate(xs):
            if t.dtype != dt:
                raise TypeError(f"finite_quantize: tensor {s} is {t.dtype}, expected {dt}")
            _require_device(t, self.device, f"tensor {s}")
            outs.append(torch.empty(t.shape, dtype=torch.int64, device=self.device))
            if masks is not None:
                m = masks[s]
                if m.dtype != torch.int64 or m.numel() != t.numel():
                    raise ValueError(f"finite_quantize: mask {s} must be int64 with {t.numel()} elements")
                _require_device(m, self.device, f"mask {s}")
        rc = self._lib.fa_finite_quantize(
            self._ctx, DTYPE_CODE[dt], len(xs), N.i64_array([t.numel() for t in xs]),
            N.ptr_array([t.data_ptr() for t in xs]),
            N.ptr_array([m.data_ptr() for m in masks]) if masks is not None else None, int(prime), int(q_bits),
            N.ptr_array([o.data_ptr() for o in outs]), self._stream(stream))
        N.check(rc, "fa_finite_quantize")
        return outs

    def lcc_decode(self, coef: Sequence[Sequence[int]], f: torch.Tensor, prime: int, n_out: int,
                   stream=None) -> torch.Tensor:
        """First n_out entries of np.mod(coef.dot(f), p) (int64 wrap), f an int64 (k x m) device tensor."""
        if f.dtype != torch.int64 or f.dim() != 2:
            raise ValueError("lcc_decode: f must be a 2-D int64 tensor")
        _require_device(f, self.device, "lcc f")
        rows = len(coef)
        k, m = f.shape
        flat = [int(v) for row in coef for v in row]
        if rows == 0 or len(flat) != rows * k:
            raise ValueError(f"lcc_decode: coef must be rows x {k}")
        out = torch.empty(int(n_out), dtype=torch.int64, device=self.device)
        rc = self._lib.fa_lcc_decode(self._ctx, rows, k, m, N.i64_array(flat), f.data_ptr(), int(prime), int(n_out),
                                     out.data_ptr(), self._stream(stream))
        N.check(rc, "fa_lcc_decode")
        return out

    # ------------------------------------------------------------------ robust aggregation
    def mt_randint_sum(self, seeds: Sequence[int], signs: Sequence[int], prime: int, n: int,
                       out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """sum_s sign_s * np.random.RandomState(seed_s).randint(0, prime, size=n), mod prime, as an
        int64 device tensor (fa_mt_randint_sum: numpy's legacy MT19937 streams expanded on the
        device, bit-exact) -- SecAgg's mask re-expansion (sa_fedml_aggregator.py:92-136)."""
        if len(seeds) != len(signs):
            raise ValueError("mt_randint_sum: one sign per seed")
        for v in seeds:
            if not 0 <= int(v) <= 0xFFFFFFFF:
                raise ValueError("Seed must be between 0 and 2**32 - 1")
        n = int(n)
        if out is None:
            out = torch.empty(max(n, 0), dtype=torch.int64, device=self.device)
        _require_device(out, self.device, "out")
        if out.dtype != torch.int64 or out.numel() < n:
            raise ValueError(f"mt_randint_sum: out must be int64 with >= {n} elements")
        S = len(seeds)
        sd = (N.ctypes.c_uint32 * max(S, 1))(*[int(v) for v in seeds])
        sg = (N.ctypes.c_int8 * max(S, 1))(*[int(v) for v in signs])
        with self.lock:
            need = self._lib.fa_mt_randint_sum_scratch_bytes(n)
            scratch = self._scratch("mt", need, stream) if need else None
            rc = self._lib.fa_mt_randint_sum(self._ctx, S, sd, sg, int(prime), n, out.data_ptr(),
                                             scratch.data_ptr() if need else None, need, self._stream(stream))
        N.check(rc, "fa_mt_randint_sum")
        return out

    def coord_median(self, segments: Sequence[Sequence[torch.Tensor]],
                     outs: Optional[Sequence[torch.Tensor]] = None, stream=None) -> List[torch.Tensor]:
        """Coordinate-wise median over clients (fa_coord_median): segments[s][i] = client i's
        tensor of segment s (one dtype: float32, bfloat16, float16, float64); one launch."""
        k = len(segments[0]) if segments else 0
        if k == 0:
            raise ValueError("coord_median: no client tensors")
        dt = segments[0][0].dtype
        if dt not in (torch.float32, torch.bfloat16, torch.float16, torch.float64):
            raise TypeError(f"coord_median: unsupported dtype {dt}")
        in_ptrs, numels, results = [], [], []
        for s, seg in enumerate(segments):
            if len(seg) != k:
                raise ValueError(f"segment {s}: {len(seg)} clients, expected {k}")
            for i, t in enumerate(seg):
                if t.dtype != dt or t.shape != seg[0].shape:
                    raise ValueError(f"segment {s} client {i}: dtype/shape mismatch")
                _require_device(t, self.device, f"segment {s} client {i}")
                in_ptrs.append(t.data_ptr())
            if outs is not None:
                o = outs[s]
                if o.dtype != dt or o.numel() != seg[0].numel():
                    raise ValueError(f"segment {s}: output must be {dt} with {seg[0].numel()} elements")
                _require_device(o, self.device, f"segment {s} output")
            else:
                o = torch.empty(seg[0].shape, dtype=dt, device=self.device)
            results.append(o)
            numels.append(seg[0].numel())
        rc = self._lib.fa_coord_median(self._ctx, DTYPE_CODE[dt], len(segments), N.i64_array(numels), k,
                                       N.ptr_array(in_ptrs), N.ptr_array([o.data_ptr() for o in results]),
                                       self._stream(stream))
        N.check(rc, "fa_coord_median")
        return results

    def coord_median_tiled(self, buf: torch.Tensor, rows: Sequence[int], n: Optional[int] = None,
                           out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """Coordinate-wise median over rows of a TILE-INTERLEAVED arena group ``buf`` [tiles, capacity,
        E] (fa_coord_median_tiled): the same selection, bit for bit, as ``coord_median`` over the
        logical rows, read in the layout whose K tiles of a workgroup are one contiguous run."""
        if buf.dtype not in (torch.float32, torch.bfloat16, torch.float16, torch.float64):
            raise TypeError(f"coord_median_tiled: unsupported dtype {buf.dtype}")
        n, ptrs, stride = self._tiled_args(buf, rows, 0, n, "coord_median_tiled")
        if out is None:
            out = torch.empty(n, dtype=buf.dtype, device=self.device)
        elif out.dtype != buf.dtype or out.numel() != n or not out.is_contiguous():
            raise ValueError(f"coord_median_tiled: output must be a contiguous {buf.dtype} tensor of {n} elements")
        _require_device(out, self.device, "output")
        if n == 0:
            return out
        rc = self._lib.fa_coord_median_tiled(self._ctx, DTYPE_CODE[buf.dtype], 1, N.i64_array([n]), len(rows), ptrs,
                                             stride, N.ptr_array([out.data_ptr()]), self._stream(stream))
        N.check(rc, "fa_coord_median_tiled")
        return out

    MAX_PAIR_K = 128  # kMaxPairK (fedml_amd/csrc/robust.hip): clients per fa_pairwise_sqdist launch

    def pairwise_sqdist(self, segments: Sequence[Sequence[torch.Tensor]], stream=None,
                        diff_dtype: torch.dtype = torch.float32) -> torch.Tensor:
        """K x K float64 matrix of squared Euclidean distances between the clients' float32 vectors
        (segments[s][i] = client i's piece s), fa_pairwise_sqdist.  K > 128 (one launch holds at
        most 128 clients): clients in blocks of 64, one launch per pair of blocks (each launch the
        union of two blocks, its cross distances kept) -- every distance is still one device pass
        over the two clients' vectors, the same per-pair arithmetic as the single launch.
        ``diff_dtype`` bfloat16 / float16: every difference rounded to that dtype before it is
        squared (fa_pairwise_sqdist_rt; the reference's arithmetic for a bf16 / f16 model);
        float64: the inputs are float64 vectors, measured in float64 throughout (a float64 model)."""
        if diff_dtype not in _DIFF_DT:
            raise ValueError("pairwise_sqdist: diff_dtype must be float32, bfloat16, float16 or float64, "
                             f"not {diff_dtype}")
        in_dt = torch.float64 if diff_dtype == torch.float64 else torch.float32
        k = len(segments[0]) if segments else 0
        if k < 2:
            raise ValueError("pairwise_sqdist: need at least two clients")
        for s, seg in enumerate(segments):
            if len(seg) != k:
                raise ValueError(f"segment {s}: {len(seg)} clients, expected {k}")
            for i, t in enumerate(seg):
                if t.dtype != in_dt or t.numel() != seg[0].numel():
                    raise ValueError(f"segment {s} client {i}: {in_dt} of {seg[0].numel()} elements expected")
                _require_device(t, self.device, f"segment {s} client {i}")
        if k <= self.MAX_PAIR_K:
            return self._pairwise_launch(segments, stream, diff_dtype)
        B = self.MAX_PAIR_K // 2
        blocks = [list(range(lo, min(k, lo + B))) for lo in range(0, k, B)]
        d = torch.zeros((k, k), dtype=torch.float64, device=self.device)
        for a in range(len(blocks)):
            for b in range(a + 1, len(blocks)):
                ids = blocks[a] + blocks[b]
                sub = self._pairwise_launch([[seg[i] for i in ids] for seg in segments], stream, diff_dtype)
                idx = torch.tensor(ids, device=self.device)
                d.index_put_((idx.view(-1, 1), idx.view(1, -1)), sub)  # diagonal blocks rewritten, same values
        return d

    # Gram form (fa_pairwise_sqdist_gram) for float32 models: its result stands when the largest
    # cancellation factor kappa = (A_i + A_j) / D_ij is at most min(KAPPA_MAX, the error model's
    # bound at this size) -- fa_pairwise_sqdist_gram_limit: 6 sigma of the modelled float32 run error
    # <= 1e-6 relative (tests/test_gpu_robust.py's kappa band); otherwise -- and for non-finite
    # inputs or D_ij <= 0 -- the direct kernels queued behind it recompute the matrix, decided on the
    # device (no host round trip)
    KAPPA_MAX = 16.0
    # A shape whose last guarded call fell back (e.g. the reference's ByzantineAttack "zero" mode:
    # identical attacker vectors, D = 0 every round) goes straight to the direct kernels, re-trying
    # the Gram form every GRAM_RETRY-th call (FEDML_AMD_KRUM_STICKY=0: always the guarded Gram form)
    GRAM_RETRY = 8

    @property
    def last_kappa_max(self) -> Optional[float]:
        """kappa_max of the last Gram-form call (reads the device value: synchronises)."""
        km = getattr(self, "_last_km", None)
        return None if km is None else float(km.item())

    @property
    def last_kappa_limit(self) -> Optional[float]:
        """The kappa limit the last guarded Gram-form call applied (fa_pairwise_sqdist_gram_limit)."""
        return getattr(self, "_last_limit", None)

    @property
    def last_pair_form(self) -> str:
        """"gram" or "direct": which form's result the last float32 pairwise call returned."""
        if getattr(self, "_last_form", None) != "auto":
            return self._last_form
        return "gram" if self.last_kappa_max <= self._last_limit else "direct"

    def _gram_memo_form(self, key) -> Tuple[bool, bool]:
        """(go straight to the direct kernels, copy this call's kappa_max) for a guarded call of this
        shape.  kappa_max is copied to pinned memory on the first call and every GRAM_RETRY-th call
        after it only, and read once that copy's event has completed (never waited on): in the
        common case -- no fallback -- the memo costs one 8-byte copy per GRAM_RETRY calls."""
        m = self.__dict__.setdefault("_gram_memo", {}).get(key)
        if m is None:
            return False, True
        if m["pending"] and m["ev"].query():
            m["fell"], m["pending"] = not (float(m["km"][0]) <= m["limit"]), False
        m["calls"] += 1
        check = m["calls"] % self.GRAM_RETRY == 0
        return m["fell"] and not check, check

    def _pairwise_launch(self, segments, stream=None, diff_dtype=torch.float32, form=None) -> torch.Tensor:
        k = len(segments[0])
        in_ptrs = [t.data_ptr() for seg in segments for t in seg]
        nl = N.i64_array([seg[0].numel() for seg in segments])
        form = form or os.environ.get("FEDML_AMD_KRUM_FORM", "auto")
        key = (k, tuple(seg[0].numel() for seg in segments))
        copy = False
        if diff_dtype == torch.float32 and form == "auto" and os.environ.get("FEDML_AMD_KRUM_STICKY", "1") != "0":
            skip, copy = self._gram_memo_form(key)
            if skip:
                form = "direct"
        if diff_dtype == torch.float32 and form in ("auto", "gram"):
            ptrs = N.ptr_array(in_ptrs)
            limit = self._lib.fa_pairwise_sqdist_gram_limit(len(segments), nl, k, ptrs, self.KAPPA_MAX) \
                if form == "auto" else 0.0
            with self.lock:
                need = self._lib.fa_pairwise_sqdist_gram_scratch_bytes(len(segments), nl, k)
                scratch = self._scratch("pdg", need, stream)
                d = torch.empty((k, k), dtype=torch.float64, device=self.device)
                km = torch.empty(1, dtype=torch.float64, device=self.device)
                rc = self._lib.fa_pairwise_sqdist_gram(self._ctx, len(segments), nl, k, ptrs,
                                                       d.data_ptr(), km.data_ptr(),
                                                       self.KAPPA_MAX if form == "auto" else 0.0,
                                                       scratch.data_ptr(), scratch.numel(), self._stream(stream))
            N.check(rc, "fa_pairwise_sqdist_gram")
            self._last_km, self._last_form, self._last_limit = km, form if form == "gram" else "auto", limit
            if copy:  # kappa_max to pinned host memory, read by a later call of this shape
                memo = self._gram_memo
                m = memo.get(key) or {"km": torch.zeros(1, dtype=torch.float64, pin_memory=True), "calls": 0,
                                      "fell": False, "ev": torch.cuda.Event(), "done": torch.cuda.Event()}
                s = stream if stream is not None else torch.cuda.current_stream(self.device)
                # the 8-byte copy runs on a side stream behind this call, off the caller's stream (a
                # blit kernel there put ~4 us between this call and the next one, r06c)
                side = self.__dict__.get("_memo_stream")
                if side is None:
                    side = self._memo_stream = torch.cuda.Stream(self.device)
                m["done"].record(s)
                side.wait_event(m["done"])
                with torch.cuda.stream(side):
                    m["km"].copy_(km, non_blocking=True)
                km.record_stream(side)
                m["ev"].record(side)
                m["limit"], m["pending"] = limit, True
                memo[key] = m
            return d
        self._last_km, self._last_form = None, "direct"
        with self.lock:
            need = self._lib.fa_pairwise_sqdist_scratch_bytes(len(segments), nl, k)
            scratch = self._scratch("pd", need, stream)
            d = torch.empty((k, k), dtype=torch.float64, device=self.device)
            rc = self._lib.fa_pairwise_sqdist_rt(self._ctx, _DIFF_DT[diff_dtype], len(segments), nl, k,
                                                 N.ptr_array(in_ptrs), d.data_ptr(), scratch.data_ptr(),
                                                 scratch.numel(), self._stream(stream))
        N.check(rc, "fa_pairwise_sqdist")
        return d


class _DeviceBlock:
    """Owner of one fa_device_alloc_contiguous block, exposed through __cuda_array_interface__ (the
    tensor torch builds from it holds this object until its storage dies, then fa_device_free)."""
    _exiting = False  # interpreter teardown: the process's exit returns the memory

    def __init__(self, eng: "AggEngine", ptr: int, nbytes: int):
        self.eng, self.ptr = eng, ptr
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}

    def __del__(self):
        if self.ptr and not _DeviceBlock._exiting:
            try:
                self.eng._lib.fa_device_free(self.eng._ctx, N.ctypes.c_void_p(self.ptr))
            except Exception:
                pass
        self.ptr = 0


def _mark_exiting():
    _DeviceBlock._exiting = True


import atexit  # noqa: E402

atexit.register(_mark_exiting)

_DIFF_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3}  # FA_DTYPE_*


def get_engine(device: Optional[int] = None) -> AggEngine:
    return AggEngine.get(device)
