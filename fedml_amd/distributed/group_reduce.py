"""Multi-GPU group -> global aggregation: one client group per GPU, RCCL over xGMI for the exchange.

One process per GPU (torch.distributed, backend "nccl" = RCCL).  Rank r holds client group r.

* Group step (local, the HIP kernel): the ordered weighted partial of the rank's clients,
  ``S_r = sum_{i in r} x_i * w_i`` (flat FedAvg with GLOBAL weights w_i = n_i / N), or, for the
  hierarchical formula, the group FedAvg ``G_r`` (weights n_i / N_r) pre-scaled to the cloud
  formula's term ``(G_r * N_r) / N`` (HierFedAvgCloudAggregator.py:146-156) -- the exact per-element
  ops the reference applies before its cloud-side accumulation.
* Global step (the exchange), ``collective``:
    "ordered"         (default) the full global model on ``dst``, summed IN RANK ORDER -- bit-identical
                      to the reference's two-level reduces: fedavg_seq (worker partials, then an
                      ordered sum; FedAVGAggregator.py:201-236), the hierarchical cloud step (ordered
                      sum of the pre-scaled group terms) and the oracle's rank-ordered sum.  The
                      summation is spread over the G-1 ranks other than ``dst`` ("owners"): chunk
                      [a, b) is split into G-1 consecutive pieces, one per owner in rank order; an
                      all-to-all sends every rank's partial of piece o to owner o (``dst`` owns
                      nothing, so its links carry only its own partial out and the results in);
                      owner o sums the G partials of its piece in rank order with the engine's SUM
                      kernel; a second all-to-all, on a second communicator so that it runs beside
                      the next chunk's first one, lands the summed pieces in ``out[a:b]`` on ``dst``
                      -- they are consecutive, so no copy.  Per chunk every directed xGMI link
                      carries at most (b - a)/(G - 1) elements, vs (b - a)/G * 2 into ``dst`` for a
                      reduce-scatter + gather and (b - a) per ring link for a ring reduce;
    "ordered_all"     the same, summed pieces delivered to EVERY rank (the reference's reduce followed
                      by its broadcast of the global model, simulation/nccl/base_framework/
                      common.py:196-228);
    "reduce"          SUM-reduce to ``dst`` with RCCL's reduce -- the reference's NCCL simulator call
                      (simulation/nccl/base_framework/params.py:98-105, common.py:196-210); the
                      cross-rank summation order is RCCL's, so the result matches the sequential
                      reference normwise (~1e-7), not bit-for-bit;
    "all_reduce"      the same, result on every rank;
    "reduce_scatter"  the same, result SHARDED: rank r owns elements [r*S, min((r+1)*S, P)) with
                      S = P/G rounded up to whole tiles, and no rank holds the whole model (a
                      sharded broadcast would follow); the least xGMI traffic of all.
* Pipelining: P is cut into ``chunks``; chunk c's exchange is issued (async, stream-ordered behind
  chunk c's kernel) while chunk c+1's partial is computed, so the xGMI transfer hides behind HBM
  streaming.  ("ordered": the owners' sum of chunk c is queued after chunk c+1's partial.)

The local reduction is injectable (``local_sum``) so the exchange logic can be tested with the
gloo backend on CPU; in the product it is the HIP engine and there is no CPU path.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..engine import MUL_N_DIV_N, MUL_W, SUM

LocalSum = Callable[..., torch.Tensor]  # (xs, mode, coef, divisor, out) -> out

COLLECTIVES = ("ordered", "ordered_all", "reduce", "all_reduce", "reduce_scatter")
NATIVE_ALIGN = 256  # chunk / piece granularity (elements) of the native path on flat inputs
_SECOND_GROUP: dict = {}  # process group -> a second communicator over the same ranks ("ordered")
_LAST = [None]            # the last exchange operation this process issued (hang diagnostics)


def last_issued():
    """Name of the last exchange operation issued by this process ("chunk c/C <op>"), or None --
    what a watchdog prints when a collective never completes.  For the native exchange this is
    the last RCCL operation libfedagg issued (fa_comm_last_op)."""
    ops = [_LAST[0]] if _LAST[0] else []
    for key, c in list(_SECOND_GROUP.items()):
        if isinstance(key, tuple) and key[0] == "native":
            op = c.last_op()
            if op:
                ops.append(f"libfedagg: {op}")
    return "; ".join(ops) or None


def _engine_local_sum(xs, mode, coef, divisor, out):
    from ..engine import get_engine
    return get_engine(out.device.index).weighted_sum(xs, mode, coef, divisor, out=out)


def _engine_local_grouped(xs, mode, coef, divisor, gptr, gmode, gcoef, gdiv, out):
    from ..engine import get_engine
    return get_engine(out.device.index).weighted_sum_grouped(xs, mode, coef, divisor, gptr, gmode, gcoef,
                                                             gdiv, out=out)


def split_bounds(n: int, parts: int, align: int = 1) -> List[tuple]:
    """Exactly ``parts`` consecutive ranges covering [0, n) (some may be empty); inner bounds are
    multiples of ``align``."""
    units = -(-n // align)
    return [(min(n, units * j // parts * align), min(n, units * (j + 1) // parts * align)) for j in range(parts)]


def chunk_bounds(n: int, chunks: int, align: int = 1) -> List[tuple]:
    """``chunks`` consecutive ranges covering [0, n); inner bounds are multiples of ``align``."""
    units = -(-n // align)
    chunks = max(1, min(chunks, units)) if units > 0 else 1
    return [(min(n, units * c // chunks * align), min(n, units * (c + 1) // chunks * align)) for c in range(chunks)]


class GroupReducer:
    """Group -> global reduction of flat parameter vectors over a process group."""

    def __init__(self, group=None, collective: str = "ordered", dst: int = 0, chunks: int = 8,
                 local_sum: Optional[LocalSum] = None, local_grouped: Optional[Callable] = None,
                 stream: Optional[torch.cuda.Stream] = None, combine_sum: Optional[LocalSum] = None,
                 native: Optional[bool] = None, timing: bool = False, loopback: bool = False):
        if collective not in COLLECTIVES:
            raise ValueError(f"unknown collective {collective!r}")
        self.group = group
        self.collective = collective
        self.dst = dst
        self.chunks = chunks
        self.local_sum = local_sum or _engine_local_sum
        # the owners' rank-ordered sum of the G partials ("ordered"): SUM mode of the same engine
        self.combine_sum = combine_sum or self.local_sum
        # fused two-level local step (group partial + epilogue in one kernel pass); with an injected
        # local_sum and no local_grouped the levels run as separate passes (same arithmetic)
        self.local_grouped = local_grouped if local_grouped is not None else (
            _engine_local_grouped if local_sum is None else None)
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if not 0 <= dst < self.world:
            raise ValueError(f"dst {dst} outside the group of {self.world}")
        # optional stream for the local partials and the collectives' dependencies, e.g. a CU-masked
        # stream (AggEngine.cu_masked_stream) that leaves CUs free for RCCL's kernels
        self.stream = stream
        self._group2 = None
        # native (the product path on GPUs): the whole step is ONE fa_group_reduce call of the C ABI
        # (include/fedagg_comm.h) over libfedagg's own RCCL communicators; the torch.distributed form
        # below is the same algorithm for CPU (gloo) tests and the one-GPU rehearsal, or with an
        # injected local reduction
        # loopback (native only): the ordered exchanges with a piece for every rank, the own piece sent
        # to itself through RCCL (FA_XCHG_LOOPBACK) -- runs the whole exchange even at world 1
        if native is None:
            native = (local_sum is None and combine_sum is None and local_grouped is None
                      and (self.world > 1 or loopback) and dist.get_backend(group) == "nccl")
        if loopback and not native:
            raise ValueError("loopback: only the native exchange (RCCL) has it")
        self.native = None
        if native:
            from .native_exchange import NativeExchange
            self.native = NativeExchange(_native_comm(group), collective, dst, chunks, loopback=loopback)
            self.native.comm.set_timing(timing)
        elif collective in ("ordered", "ordered_all") and self.world > 1:
            self._group2 = _second_group(group)
        self._bufs: dict = {}
        self.owned = None  # "ordered": (lo, hi) pieces of the global model this rank summed, last call

    # -------------------------------------------------------------- public entry points
    def fedavg(self, xs: Sequence[torch.Tensor], weights: Sequence[float], out: Optional[torch.Tensor] = None):
        """Global FedAvg of all ranks' clients; ``weights`` = this rank's GLOBAL w_i = n_i / N."""
        flat = [x.reshape(-1) for x in xs]
        w = list(weights)
        if self.native is not None:
            from .native_exchange import NativeExchange
            return self._native_run(NativeExchange.flat(flat, MUL_W, w), flat[0].numel(), NATIVE_ALIGN, out)
        return self._run(flat, lambda part, a, b: self.local_sum([x[a:b] for x in flat], MUL_W, w, 1.0, part),
                         out, mode=MUL_W)

    def hierarchical(self, xs: Sequence[torch.Tensor], counts: Sequence[int], total: int,
                     out: Optional[torch.Tensor] = None):
        """This rank's clients form ONE group: group FedAvg (weights n_i / N_r,
        sp/fedavg_api.py:144-159), cloud term (G_r * N_r) / N (MPI cloud formula), global sum."""
        return self.hierarchical_groups(xs, [list(counts)], total, out)

    def hierarchical_groups(self, xs: Sequence[torch.Tensor], group_counts: Sequence[Sequence[int]], total: int,
                            out: Optional[torch.Tensor] = None):
        """This rank holds several consecutive groups (xs concatenated in group order): per group the
        group FedAvg and cloud term, the ordered sum over this rank's groups, then the global sum."""
        flat = [x.reshape(-1) for x in xs]
        w, gn, gptr = [], [], [0]
        for cnts in group_counts:
            ng = sum(cnts)
            gn.append(ng)
            w += [c / ng for c in cnts]
            gptr.append(gptr[-1] + len(cnts))
        if len(flat) != gptr[-1]:
            raise ValueError("hierarchical_groups: client count does not match the groups")
        T = float(total)
        if self.native is not None:
            from .native_exchange import NativeExchange
            return self._native_run(NativeExchange.grouped(flat, MUL_W, w, 1.0, gptr, MUL_N_DIV_N, gn, [T] * len(gn)),
                                    flat[0].numel(), NATIVE_ALIGN, out)

        def local(part, a, b):
            sl = [x[a:b] for x in flat]
            if self.local_grouped is not None:
                self.local_grouped(sl, MUL_W, w, 1.0, gptr, MUL_N_DIV_N, gn, [T] * len(gn), part)
                return
            terms = []
            for g in range(len(gn)):  # two-pass form (injected local_sum): same arithmetic
                G = torch.empty_like(part)
                self.local_sum(sl[gptr[g]:gptr[g + 1]], MUL_W, w[gptr[g]:gptr[g + 1]], 1.0, G)
                t = torch.empty_like(part)
                self.local_sum([G], MUL_N_DIV_N, [gn[g]], T, t)
                terms.append(t)
            if len(terms) == 1:
                part.copy_(terms[0])
            else:
                self.local_sum(terms, SUM, None, 1.0, part)
        return self._run(flat, local, out, mode=MUL_W)

    def fedavg_tiled(self, engine, buf: torch.Tensor, rows: Sequence[int], weights: Sequence[float], n: int,
                     out: Optional[torch.Tensor] = None):
        """``fedavg`` over rows of a tile-interleaved ClientArena group ``buf`` ([tiles, capacity, E],
        fedml_amd/arena.py): chunks are whole tiles, each chunk one fa_weighted_sum_tiled launch."""
        E = buf.shape[2]
        w = list(weights)
        rows = list(rows)
        if self.native is not None:
            from .native_exchange import NativeExchange
            return self._native_run(NativeExchange.tiled(buf, rows, MUL_W, w), n, E, out)

        def local(part, a, b):
            if a % E:
                raise ValueError("fedavg_tiled: chunk does not start on a tile boundary")
            engine.weighted_sum_tiled(buf, rows, MUL_W, w, n=b - a, t0=a // E, out=part)

        local_multi = None
        if hasattr(engine, "weighted_sum_tiled_multi"):  # reduce_scatter: a chunk's G slices, one launch
            def local_multi(pieces):
                engine.weighted_sum_tiled_multi(buf, rows, MUL_W, w, 1.0, [(lo, hi) for _, lo, hi in pieces],
                                                [p for p, _, _ in pieces])
        return self._run_n(n, buf.dtype, buf.device, local, out, MUL_W, align=E, local_multi=local_multi)

    def sum(self, xs: Sequence[torch.Tensor], out: Optional[torch.Tensor] = None):
        """Plain global sum (FedAvg_seq / FedDyn branches)."""
        flat = [x.reshape(-1) for x in xs]
        if self.native is not None:
            from .native_exchange import NativeExchange
            return self._native_run(NativeExchange.flat(flat, SUM, None), flat[0].numel(), NATIVE_ALIGN, out)
        return self._run(flat, lambda part, a, b: self.local_sum([x[a:b] for x in flat], SUM, None, 1.0, part),
                         out, mode=SUM)

    def local_time(self, reset: bool = True):
        """Native path with ``timing=True``: (summed ms, launches) of the local-step kernels."""
        if self.native is None:
            raise RuntimeError("local_time: only the native exchange records local-step timing")
        return self.native.comm.local_time(reset)

    # -------------------------------------------------------------- implementation
    def _native_run(self, desc, n, align, out):
        dev = torch.device("cuda", self.native.comm.device)
        _LAST[0] = f"native fa_group_reduce ({self.collective}, {n} elements)"
        if self.stream is None:
            res = self.native.run(desc, n, align, out)
        else:
            caller = torch.cuda.current_stream(dev)
            self.stream.wait_stream(caller)
            if out is not None:
                out.record_stream(self.stream)
            res = self.native.run(desc, n, align, out, stream=self.stream)
            caller.wait_stream(self.stream)
            if res is not out:
                res.record_stream(caller)
        self.owned = self.native.owned(n, align) or None
        return res

    def _run(self, flat, local, out, mode):
        return self._run_n(flat[0].numel(), flat[0].dtype, flat[0].device, local, out, mode)

    def _run_n(self, n, dtype, dev, local, out, mode, align: int = 1, local_multi=None):
        if out is None:
            out = torch.empty(n, dtype=torch.float32 if dtype == torch.int64 and mode != SUM else dtype, device=dev)
        if self.stream is None:
            return self._run_body(n, dev, local, out, align, local_multi)
        caller = torch.cuda.current_stream(dev)
        self.stream.wait_stream(caller)      # inputs / out were produced on the caller's stream
        out.record_stream(self.stream)
        with torch.cuda.stream(self.stream):
            res = self._run_body(n, dev, local, out, align, local_multi)
        caller.wait_stream(self.stream)      # the result is consumed on the caller's stream
        if res is not out:
            res.record_stream(caller)        # allocated on self.stream, used on the caller's
        return res

    def _scratch(self, name, numel, dtype, dev):
        """Internal staging, kept across calls (never the caller's ``out``)."""
        t = self._bufs.get(name)
        if t is None or t.numel() < numel or t.dtype != dtype or t.device != dev:
            t = self._bufs[name] = torch.empty(max(numel, 1), dtype=dtype, device=dev)
        return t

    def _run_body(self, n, dev, local, out, align, local_multi=None):
        if self.world == 1:
            for a, b in chunk_bounds(n, self.chunks, align):
                local(out[a:b], a, b)
            return out
        if self.collective in ("ordered", "ordered_all"):
            return self._run_ordered(n, dev, local, out, align)
        if self.collective == "reduce_scatter":
            return self._run_reduce_scatter(n, dev, local, out, align, local_multi)
        works = []
        for a, b in chunk_bounds(n, self.chunks, align):
            part = out[a:b]
            local(part, a, b)
            _LAST[0] = f"{self.collective} of [{a}, {b}) of {n}"
            if self.collective == "reduce":
                works.append(dist.reduce(part, dst=self.dst, op=dist.ReduceOp.SUM, group=self.group,
                                         async_op=True))
            else:  # all_reduce
                works.append(dist.all_reduce(part, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        for w in works:
            w.wait()
        return out

    def _run_reduce_scatter(self, n, dev, local, out, align, local_multi):
        # shards of S elements (whole tiles), the last one zero-padded past n: rank r owns the
        # global model's elements [r*S, min((r+1)*S, n)); staging is internal
        S = -(-n // (self.world * align)) * align
        stage = self._scratch("rs_stage", S * self.world, out.dtype, dev)
        shard = torch.empty(S, dtype=out.dtype, device=dev)
        works = []
        # chunk-major staging: chunk [a, b) of every rank's shard is laid out contiguously
        # (rank-major inside the chunk), which is what reduce_scatter_tensor consumes
        for a, b in chunk_bounds(S, self.chunks, align):
            L = b - a
            base = self.world * a
            pieces = []
            for r in range(self.world):
                lo, hi = r * S + a, min(r * S + b, n)
                dstv = stage[base + r * L: base + (r + 1) * L]
                if hi > lo:
                    pieces.append((dstv[:hi - lo], lo, hi))
                if hi - lo < L:
                    dstv[max(hi - lo, 0):].zero_()
            if local_multi is not None:  # every rank's slice of the chunk in ONE launch
                local_multi(pieces)
            else:
                for dstv, lo, hi in pieces:
                    local(dstv, lo, hi)
            _LAST[0] = f"reduce_scatter of shard range [{a}, {b}) of {S}"
            works.append(dist.reduce_scatter_tensor(shard[a:b], stage[base: base + self.world * L],
                                                    op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        for w in works:
            w.wait()
        return shard[:max(0, min(S, n - self.rank * S))]

    def _run_ordered(self, n, dev, local, out, align):
        """Rank-ordered global sum, summed by the owners (every rank but ``dst``), delivered to
        ``dst`` (or to every rank, "ordered_all").  See the module docstring."""
        world, me, dst = self.world, self.rank, self.dst
        to_all = self.collective == "ordered_all"
        owners = [r for r in range(world) if r != dst]
        plan = []  # per chunk: (a, b, piece size per rank, piece start per rank)
        for a, b in chunk_bounds(n, self.chunks, align):
            sizes, starts = [0] * world, [a] * world
            for o, (lo, hi) in zip(owners, split_bounds(b - a, len(owners), align)):
                sizes[o], starts[o] = hi - lo, a + lo
            plan.append((a, b, sizes, starts))
        dt = out.dtype
        send = self._scratch("send", n, dt, dev)
        mine = sum(p[2][me] for p in plan)
        recv = self._scratch("recv", world * mine, dt, dev)
        own = self._scratch("own", mine, dt, dev)
        offs, o = [], 0
        for p in plan:
            offs.append(o)
            o += p[2][me]
        first, second = [], []

        def finish(c):
            a, b, sizes, starts = plan[c]
            L, o0 = sizes[me], offs[c]
            first[c].wait()  # this chunk's G partials of my piece have landed (stream-ordered on device)
            if L:
                r0 = world * o0
                self.combine_sum([recv[r0 + r * L: r0 + (r + 1) * L] for r in range(world)], SUM, None, 1.0,
                                 own[o0:o0 + L])
            _LAST[0] = f"ordered chunk {c + 1}/{len(plan)}: delivery (second communicator)"
            if not to_all:  # deliver the summed pieces owner -> dst, consecutive in out[a:b]
                osz = list(sizes) if me == dst else [0] * world
                isz = [L if r == dst else 0 for r in range(world)]
                second.append(dist.all_to_all_single(out[a:b] if me == dst else out[a:a], own[o0:o0 + L], osz,
                                                     isz, group=self._group2, async_op=True))
                return
            # "ordered_all": every owner's piece to every rank (one buffer, G-1 sends: P2P)
            ops = []
            for r in range(world):
                if r == me:
                    if L:
                        out[starts[me]:starts[me] + L].copy_(own[o0:o0 + L])
                    continue
                if sizes[r]:
                    ops.append(dist.P2POp(dist.irecv, out[starts[r]:starts[r] + sizes[r]], r, self._group2))
                if L:
                    ops.append(dist.P2POp(dist.isend, own[o0:o0 + L], r, self._group2))
            if ops:
                second.extend(dist.batch_isend_irecv(ops))

        for c, (a, b, sizes, starts) in enumerate(plan):
            local(send[a:b], a, b)
            L, o0 = sizes[me], offs[c]
            _LAST[0] = f"ordered chunk {c + 1}/{len(plan)}: all_to_all to the owners"
            first.append(dist.all_to_all_single(recv[world * o0: world * (o0 + L)], send[a:b], [L] * world,
                                                list(sizes), group=self.group, async_op=True))
            if c >= 1:  # software pipeline: chunk c-1's owner sum queues behind chunk c's partial
                finish(c - 1)
        finish(len(plan) - 1)
        for w in second:
            w.wait()
        self.owned = [(p[3][me], p[3][me] + p[2][me]) for p in plan if p[2][me]]
        return out


def release_groups():
    """Destroy this process's extra torch.distributed groups (the "ordered" second groups) -- call
    before dist.destroy_process_group(), so none is left for interpreter teardown to destroy (gloo
    aborts with "terminate called without an active exception" when one is finalised at exit)."""
    import gc
    for key in list(_SECOND_GROUP):
        if isinstance(key, tuple) and key[0] == "native":
            continue  # libfedagg's RCCL communicators: owned by their reducers (fa_comm_destroy)
        g = _SECOND_GROUP.pop(key)
        try:
            dist.destroy_process_group(g)
        except Exception:  # noqa: BLE001 -- already gone with the default group
            pass
    gc.collect()


def _native_comm(group):
    """This process's NativeComm over ``group`` (created collectively, once per group)."""
    from .native_exchange import NativeComm
    key = ("native", group if group is not None else dist.group.WORLD)
    c = _SECOND_GROUP.get(key)
    if c is None:
        c = _SECOND_GROUP[key] = NativeComm(group)
    return c


def _second_group(group):
    """A second communicator over ``group``'s ranks (created collectively, once per group)."""
    key = group if group is not None else dist.group.WORLD  # a re-created default group is a new key
    g2 = _SECOND_GROUP.get(key)
    if g2 is None:
        ranks = dist.get_process_group_ranks(group) if group is not None else list(range(dist.get_world_size()))
        # only the group's members enter (a reducer built over a subgroup must not need the others)
        g2 = _SECOND_GROUP[key] = dist.new_group(ranks, use_local_synchronization=True)
    return g2
