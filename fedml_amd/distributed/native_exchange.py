"""The group -> global step through the C ABI (include/fedagg_comm.h): one native call per step.

``NativeComm`` holds this rank's RCCL communicators, created by libfedagg.so itself
(fa_comm_init) from a unique id that rank 0 broadcasts over the caller's process group -- the
binding creates the communicator, as SURVEY.md §8(b) asks, and a non-Python host would do the same
over MPI.  ``NativeExchange.run`` issues every chunk's local partial, the RCCL traffic and the
owners' rank-ordered sums in ONE fa_group_reduce call (no Python per chunk).

Reference: simulation/nccl/base_framework/common.py:106-122 (process group setup), :196-228
(reduce to rank 0 and the broadcast), params.py:98-128 (per-tensor reduce).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import _native as N
from ..engine import DTYPE_CODE, get_engine, out_dtype

EXCHANGE_CODE = {"ordered": N.XCHG_ORDERED, "ordered_all": N.XCHG_ORDERED_ALL, "reduce": N.XCHG_REDUCE,
                 "all_reduce": N.XCHG_ALL_REDUCE, "reduce_scatter": N.XCHG_REDUCE_SCATTER}


def group_plan(n: int, chunks: int, align: int, world: int, root: int, loopback: bool = False):
    """fa_group_plan_ex: [(lo, hi, [piece (start, size) per rank])] per chunk -- the C library's plan
    (a pure function, also callable without a GPU).  ``loopback``: the root owns a piece too."""
    L = N.lib()
    cap = max(1, chunks)
    lo, hi = (ctypes.c_int64 * cap)(), (ctypes.c_int64 * cap)()
    ps, pz = (ctypes.c_int64 * (cap * world))(), (ctypes.c_int64 * (cap * world))()
    c = L.fa_group_plan_ex(int(n), int(chunks), int(align), int(world), int(root),
                           N.XFLAG_LOOPBACK if loopback else 0, cap, lo, hi, ps, pz)
    if c < 0:
        N.check(c, "fa_group_plan")
    return [(lo[i], hi[i], [(ps[i * world + r], pz[i * world + r]) for r in range(world)]) for i in range(c)]


class NativeComm:
    """This rank's fa_comm (two RCCL communicators over the process group's ranks, on ``device``)."""

    def __init__(self, group=None, device: Optional[int] = None):
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        L = N.lib()
        uid = (ctypes.c_uint8 * N.COMM_ID_BYTES)()
        if self.rank == 0:
            N.check(L.fa_comm_unique_id(uid, N.COMM_ID_BYTES), "fa_comm_unique_id")
        t = torch.tensor(list(uid), dtype=torch.uint8, device=self._bcast_device(group))
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast(t, src=src, group=group)
        uid = (ctypes.c_uint8 * N.COMM_ID_BYTES)(*t.cpu().tolist())
        h = ctypes.c_void_p()
        N.check(L.fa_comm_init(self.device, self.world, self.rank, uid, ctypes.byref(h)), "fa_comm_init")
        self._h = h
        self._lib = L

    def _bcast_device(self, group):
        backend = dist.get_backend(group)
        return torch.device("cuda", self.device) if backend == "nccl" else torch.device("cpu")

    @property
    def handle(self):
        return self._h

    def set_timing(self, enable: bool):
        N.check(self._lib.fa_comm_set_timing(self._h, int(bool(enable))), "fa_comm_set_timing")

    def local_time(self, reset: bool = True) -> Tuple[float, int]:
        """(summed ms, launches) of the local-step kernels since the last reset (timing on)."""
        ms, cnt = ctypes.c_double(), ctypes.c_int64()
        N.check(self._lib.fa_comm_local_time(self._h, int(reset), ctypes.byref(ms), ctypes.byref(cnt)),
                "fa_comm_local_time")
        return ms.value, cnt.value

    def op_counts(self) -> Tuple[int, int, int, int]:
        """(sends, receives) issued on communicator 1, then on communicator 2, since creation."""
        c = (ctypes.c_int64 * 4)()
        N.check(self._lib.fa_comm_op_counts(self._h, c), "fa_comm_op_counts")
        return tuple(c)

    def last_op(self) -> str:
        buf = ctypes.create_string_buffer(256)
        if self._lib.fa_comm_last_op(self._h, buf, 256) != N.FA_OK:
            return ""
        return buf.value.decode()

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.fa_comm_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NativeExchange:
    """fa_group_reduce over a NativeComm: the local-step descriptors and the scratch buffer."""

    def __init__(self, comm: NativeComm, collective: str, root: int = 0, chunks: int = 8, loopback: bool = False):
        if collective not in EXCHANGE_CODE:
            raise ValueError(f"unknown collective {collective!r}")
        if loopback and collective not in ("ordered", "ordered_all"):
            raise ValueError("loopback applies to the ordered exchanges only")
        self.comm = comm
        self.collective = collective
        self.loopback = bool(loopback)
        # FA_XCHG_LOOPBACK: every rank (root included) owns a piece and sends its own piece to itself
        # through RCCL -- at world 1 the whole ordered exchange runs on one GPU
        self.code = EXCHANGE_CODE[collective] | (N.XCHG_LOOPBACK if loopback else 0)
        self.root = root
        self.chunks = chunks
        self._scratch = None
        self._keep = None

    # -------------------------------------------------------------- local-step descriptors
    @staticmethod
    def flat(xs: Sequence[torch.Tensor], mode: int, coef: Optional[Sequence[float]], divisor: float = 1.0):
        dt = xs[0].dtype
        if dt not in DTYPE_CODE:
            raise TypeError(f"unsupported dtype {dt}")
        ptrs = N.ptr_array([x.data_ptr() for x in xs])
        cf = N.f64_array(coef if coef is not None else [1.0] * len(xs))
        st = N.LocalStep(kind=N.LOCAL_FLAT, dtype=DTYPE_CODE[dt], mode=int(mode), k=len(xs), d_in=ptrs,
                         tile_stride=0, coef=cf, divisor=float(divisor))
        return st, (ptrs, cf), dt

    @staticmethod
    def grouped(xs, mode, coef, divisor, gptr, gmode, gcoef, gdiv):
        st, keep, dt = NativeExchange.flat(xs, mode, coef, divisor)
        gp, gc, gd = N.i32_array(gptr), N.f64_array(gcoef), N.f64_array(gdiv)
        st.kind, st.num_groups, st.group_mode = N.LOCAL_GROUPED, len(gptr) - 1, int(gmode)
        st.group_ptr, st.group_coef, st.group_divisor = gp, gc, gd
        return st, keep + (gp, gc, gd), dt

    @staticmethod
    def tiled(buf: torch.Tensor, rows: Sequence[int], mode: int, coef: Sequence[float], divisor: float = 1.0):
        if buf.dim() != 3 or not buf.is_contiguous() or buf.shape[2] * buf.element_size() != N.TILE_BYTES:
            raise ValueError("tiled local step: buf must be a contiguous [tiles, capacity, tile] tensor")
        cap = buf.shape[1]
        if not rows or min(rows) < 0 or max(rows) >= cap:
            raise IndexError("tiled local step: row out of range")
        ptrs = N.ptr_array([buf.data_ptr() + r * N.TILE_BYTES for r in rows])
        cf = N.f64_array(coef)
        st = N.LocalStep(kind=N.LOCAL_TILED, dtype=DTYPE_CODE[buf.dtype], mode=int(mode), k=len(rows), d_in=ptrs,
                         tile_stride=cap * N.TILE_BYTES, coef=cf, divisor=float(divisor))
        return st, (ptrs, cf), buf.dtype

    @staticmethod
    def partial(part: torch.Tensor):
        st = N.LocalStep(kind=N.LOCAL_PARTIAL, dtype=DTYPE_CODE[part.dtype], mode=N.SUM, k=0,
                         d_partial=part.data_ptr())
        return st, (), part.dtype

    # -------------------------------------------------------------- the step
    def shard_elems(self, n: int, align: int) -> int:
        w = self.comm.world
        return -(-n // (w * align)) * align

    def run(self, desc, n: int, align: int, out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        st, keep, in_dt = desc
        dev = torch.device("cuda", self.comm.device)
        odt = out_dtype(in_dt, st.mode) if st.kind != N.LOCAL_PARTIAL else in_dt
        numel = self.shard_elems(n, align) if self.code == N.XCHG_REDUCE_SCATTER else n
        if out is None:
            out = torch.empty(max(numel, 0), dtype=odt, device=dev)
        if out.dtype != odt or out.numel() < numel or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous {odt} tensor of >= {numel} elements")
        L = N.lib()
        need = ctypes.c_int64()
        N.check(L.fa_group_reduce_scratch_bytes(self.comm.handle, self.code, ctypes.byref(st), int(n), self.chunks,
                                                int(align), self.root, ctypes.byref(need)),
                "fa_group_reduce_scratch_bytes")
        if need.value and (self._scratch is None or self._scratch.numel() < need.value):
            self._scratch = torch.empty(need.value, dtype=torch.uint8, device=dev)
        scr = self._scratch.data_ptr() if need.value else None
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        eng = get_engine(self.comm.device)
        with eng.lock:  # one thread per fa_ctx at a time (include/fedagg.h)
            rc = L.fa_group_reduce(eng._ctx, self.comm.handle, self.code, ctypes.byref(st), int(n), self.chunks,
                                   int(align), self.root, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(scr),
                                   need.value, ctypes.c_void_p(s.cuda_stream))
        N.check(rc, f"fa_group_reduce({self.collective})")
        # the scratch and the caller's inputs are in use until the stream passes this call
        if self._scratch is not None:
            self._scratch.record_stream(s)
        self._keep = keep
        if self.code == N.XCHG_REDUCE_SCATTER:
            valid = max(0, min(numel, n - self.comm.rank * numel))
            return out[:valid]
        return out

    def owned(self, n: int, align: int) -> List[tuple]:
        """The pieces this rank summed in the ordered exchanges AND holds in its d_out.  Under
        FA_XCHG_LOOPBACK with "ordered" a non-root owner sums into the library's scratch and sends the
        sum to the root only, so its d_out holds none of it: []."""
        if self.collective not in ("ordered", "ordered_all") or (self.comm.world == 1 and not self.loopback):
            return []
        me = self.comm.rank
        if self.loopback and self.collective == "ordered" and me != self.root:
            return []
        return [(pc[me][0], pc[me][0] + pc[me][1])
                for _, _, pc in group_plan(n, self.chunks, align, self.comm.world, self.root, self.loopback)
                if pc[me][1]]
