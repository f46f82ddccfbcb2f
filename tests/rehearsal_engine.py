"""Test infrastructure: the local reductions of the CPU N-rank bench rehearsal.

``FEDML_AMD_BENCH_REHEARSAL=cpu FEDML_AMD_BENCH_ENGINE=rehearsal_engine:make python bench.py --gpus 8 ...``
runs bench.py's own N > 1 code paths (launcher -> torch.distributed.run -> 8 gloo ranks ->
GroupReducer / DistributedGossip -> per-rank parity) on a CPU container.  What the GPU ranks do with
the HIP kernels, this stand-in does with the C oracle (oracle/orc.py), on host tensors, with the
same argument conventions as fedml_amd.engine.AggEngine.  It exercises the exchange orchestration,
not the kernels (those are the -m gpu parity tests), and lives under tests/ because the oracle may
only be called from test infrastructure.
"""
from __future__ import annotations

import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import orc  # noqa: E402

SUM = 2


class OracleEngine:
    device = torch.device("cpu")

    def set_variant(self, v):
        raise SystemExit("CPU rehearsal: kernel variants are a GPU notion")

    def weighted_sum(self, xs, mode, coef=None, divisor=1.0, out=None, stream=None):
        r = orc.weighted_sum([x.reshape(-1) for x in xs], mode, coef, divisor)
        if out is None:
            return r
        out.copy_(r.reshape(out.shape))
        return out

    def _tiled_rows(self, buf, rows, lo, hi):
        E = buf.shape[2]
        if lo % E:
            raise ValueError("tiled range does not start on a tile boundary")
        return [buf[lo // E:, r, :].reshape(-1)[:hi - lo] for r in rows]

    def weighted_sum_tiled(self, buf, rows, mode, coef=None, divisor=1.0, n=None, t0=0, out=None, stream=None):
        E = buf.shape[2]
        n = buf.shape[0] * E - t0 * E if n is None else n
        return self.weighted_sum(self._tiled_rows(buf, rows, t0 * E, t0 * E + n), mode, coef, divisor, out)

    def weighted_sum_tiled_multi(self, buf, rows, mode, coef, divisor, ranges, outs, stream=None):
        for (lo, hi), o in zip(ranges, outs):
            self.weighted_sum(self._tiled_rows(buf, rows, lo, hi), mode, coef, divisor, o)

    def weighted_sum_grouped(self, xs, mode, coef, divisor, group_ptr, group_mode, group_coef=None,
                             group_divisor=None, out=None, stream=None):
        """Per group the ordered partial, its epilogue, then the ordered sum over groups -- the
        arithmetic of fa_weighted_sum_grouped (include/fedagg.h) as separate oracle passes."""
        terms = []
        for g in range(len(group_ptr) - 1):
            a, b = group_ptr[g], group_ptr[g + 1]
            G = orc.weighted_sum([x.reshape(-1) for x in xs[a:b]], mode, None if coef is None else coef[a:b], divisor)
            terms.append(orc.weighted_sum([G], group_mode, None if group_coef is None else [group_coef[g]],
                                          1.0 if group_divisor is None else group_divisor[g]))
        r = orc.weighted_sum(terms, SUM) if len(terms) > 1 else terms[0]
        if out is None:
            return r
        out.copy_(r.reshape(out.shape))
        return out

    def mix(self, xs, row_ptr, cols, vals, post_scale=None, outs=None, outs2=None, stream=None):
        o, o2 = orc.mix([x.reshape(-1) for x in xs], row_ptr, cols, vals, post_scale)
        if outs is None:
            return o, o2
        for a, b in zip(outs, o):
            a.copy_(b.reshape(a.shape))
        if outs2 is not None:
            for a, b in zip(outs2, o2):
                a.copy_(b.reshape(a.shape))
        return list(outs), (list(outs2) if outs2 is not None else None)


def make():
    return OracleEngine()
