"""Multi-GPU group -> global aggregation: one client group per GPU, RCCL over xGMI for the exchange.

One process per GPU (torch.distributed, backend "nccl" = RCCL).  Rank r holds client group r.

* Group step (local, the HIP kernel): the ordered weighted partial of the rank's clients,
  ``S_r = sum_{i in r} x_i * w_i`` (flat FedAvg with GLOBAL weights w_i = n_i / N), or, for the
  hierarchical formula, the group FedAvg ``G_r`` (weights n_i / N_r) pre-scaled to the cloud
  formula's term ``(G_r * N_r) / N`` (HierFedAvgCloudAggregator.py:146-156) -- the exact per-element
  ops the reference applies before its cloud-side accumulation.
* Global step (the exchange), ``collective``:
    "reduce"          SUM-reduce to ``dst`` -- the reference's NCCL simulator pattern
                      (simulation/nccl/base_framework/params.py:98-105, common.py:196-210); the
                      cross-rank summation order is RCCL's, so the result matches the sequential
                      reference normwise (~1e-7), not bit-for-bit;
    "all_reduce"      the same, result on every rank;
    "reduce_scatter"  the same, result sharded: rank r owns elements [r*S, min((r+1)*S, P)) with
                      S = P/G rounded up to whole tiles -- the least xGMI traffic (each link
                      carries 1/G of a partial per direction), and the global model is already
                      partitioned for a sharded broadcast;
    "ordered"         gather the G partials to ``dst`` and sum them there IN RANK ORDER with the
                      engine's SUM mode: bit-identical to the reference's two-level reduces --
                      fedavg_seq (worker partials, then an ordered sum; FedAVGAggregator.py:201-236)
                      and the hierarchical cloud step (ordered sum of the pre-scaled group terms).
* Pipelining: P is cut into ``chunks``; chunk c's collective is issued (async, stream-ordered
  behind chunk c's kernel) while chunk c+1's partial is computed, so the xGMI transfer hides
  behind HBM streaming.

The local reduction is injectable (``local_sum``) so the exchange logic can be tested with the
gloo backend on CPU; in the product it is the HIP engine and there is no CPU path.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..engine import MUL_N_DIV_N, MUL_W, SUM

LocalSum = Callable[..., torch.Tensor]  # (xs, mode, coef, divisor, out) -> out


def _engine_local_sum(xs, mode, coef, divisor, out):
    from ..engine import get_engine
    return get_engine(out.device.index).weighted_sum(xs, mode, coef, divisor, out=out)


def _engine_local_grouped(xs, mode, coef, divisor, gptr, gmode, gcoef, gdiv, out):
    from ..engine import get_engine
    return get_engine(out.device.index).weighted_sum_grouped(xs, mode, coef, divisor, gptr, gmode, gcoef,
                                                             gdiv, out=out)


def chunk_bounds(n: int, chunks: int, align: int = 1) -> List[tuple]:
    """``chunks`` consecutive ranges covering [0, n); inner bounds are multiples of ``align``."""
    units = -(-n // align)
    chunks = max(1, min(chunks, units)) if units > 0 else 1
    return [(min(n, units * c // chunks * align), min(n, units * (c + 1) // chunks * align)) for c in range(chunks)]


class GroupReducer:
    """Group -> global reduction of flat parameter vectors over a process group."""

    def __init__(self, group=None, collective: str = "reduce", dst: int = 0, chunks: int = 8,
                 local_sum: Optional[LocalSum] = None, local_grouped: Optional[Callable] = None,
                 stream: Optional[torch.cuda.Stream] = None):
        if collective not in ("reduce", "all_reduce", "reduce_scatter", "ordered"):
            raise ValueError(f"unknown collective {collective!r}")
        self.group = group
        self.collective = collective
        self.dst = dst
        self.chunks = chunks
        self.local_sum = local_sum or _engine_local_sum
        # fused two-level local step (group partial + epilogue in one kernel pass); with an injected
        # local_sum and no local_grouped the levels run as separate passes (same arithmetic)
        self.local_grouped = local_grouped if local_grouped is not None else (
            _engine_local_grouped if local_sum is None else None)
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        # optional stream for the local partials and the collectives' dependencies, e.g. a CU-masked
        # stream (AggEngine.cu_masked_stream) that leaves CUs free for RCCL's kernels
        self.stream = stream

    # -------------------------------------------------------------- public entry points
    def fedavg(self, xs: Sequence[torch.Tensor], weights: Sequence[float], out: Optional[torch.Tensor] = None):
        """Global FedAvg of all ranks' clients; ``weights`` = this rank's GLOBAL w_i = n_i / N."""
        flat = [x.reshape(-1) for x in xs]
        w = list(weights)
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
        return self._run(flat, lambda part, a, b: self.local_sum([x[a:b] for x in flat], SUM, None, 1.0, part),
                         out, mode=SUM)

    # -------------------------------------------------------------- implementation
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

    def _run_body(self, n, dev, local, out, align, local_multi=None):
        works = []
        gathered = []
        if self.collective == "reduce_scatter":
            # shards of S elements (whole tiles), the last one zero-padded past n: rank r owns the
            # global model's elements [r*S, min((r+1)*S, n))
            S = -(-n // (self.world * align)) * align
            stage = out if out.numel() >= S * self.world else torch.empty(S * self.world, dtype=out.dtype, device=dev)
            shard = torch.empty(S, dtype=out.dtype, device=dev)
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
                if self.world > 1:
                    works.append(dist.reduce_scatter_tensor(shard[a:b], stage[base: base + self.world * L],
                                                            op=dist.ReduceOp.SUM, group=self.group,
                                                            async_op=True))
                else:
                    shard[a:b].copy_(stage[base: base + L])
            for w in works:
                w.wait()
            return shard[:max(0, min(S, n - self.rank * S))]
        for a, b in chunk_bounds(n, self.chunks, align):
            part = out[a:b]
            local(part, a, b)
            if self.world == 1:
                continue
            if self.collective == "reduce":
                works.append(dist.reduce(part, dst=self.dst, op=dist.ReduceOp.SUM, group=self.group,
                                         async_op=True))
            elif self.collective == "all_reduce":
                works.append(dist.all_reduce(part, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            else:  # ordered
                bufs = [torch.empty_like(part) for _ in range(self.world)] if self.rank == self.dst else None
                works.append(dist.gather(part, bufs, dst=self.dst, group=self.group, async_op=True))
                gathered.append((a, b, bufs))
        for w in works:
            w.wait()
        if self.collective == "ordered" and self.rank == self.dst and self.world > 1:
            for a, b, bufs in gathered:
                self.local_sum(bufs, SUM, None, 1.0, out[a:b])
        return out
