"""Coordinate-wise median on the HIP engine (drop-in for the reference's
python/fedml/core/security/defense/coordinate_wise_median_defense.py).

The reference vectorizes every client's weights (BatchNorm statistics skipped, utils.py:8-21),
stacks them and takes ``torch.median(dim=-1)``, then walks ALL keys of client 0's dict, slicing
the median vector by each key's size (:33-43) -- so a model with BatchNorm statistics misaligns
and ends in a ``view`` RuntimeError; client 0's dict is modified in place and returned.  This
mirror keeps all of that; the median itself is ONE ``fa_coord_median`` launch over the weight
keys (a selection, bit-identical to ATen's: NaN first, lower median, ties by client index;
tests/golden/g16_*).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Any, Callable, List, Tuple

import torch

from ....arena import resident_rows
from ....engine import get_engine
from ..common.utils import is_weight_param

_NATIVE = (torch.float32, torch.bfloat16, torch.float16, torch.float64)


class CoordinateWiseMedianDefense(object):
    def __init__(self, config):
        pass

    def defend_on_aggregation(self, raw_client_grad_list: List[Tuple[float, OrderedDict]],
                              base_aggregation_func: Callable = None, extra_auxiliary_info: Any = None):
        grads = [g for _, g in raw_client_grad_list]
        if len(grads) == 0:
            raise RuntimeError("torch.cat(): expected a non-empty list of Tensors")
        keys = [k for k in grads[0].keys() if is_weight_param(k)]
        if not keys:
            raise RuntimeError("torch.cat(): expected a non-empty list of Tensors")
        hit = resident_rows(grads) if len(keys) == len(grads[0]) else None
        if hit is not None and len(hit[0].bufs) == 1 and next(iter(hit[0].bufs)) in _NATIVE:
            # updates adopted into ONE arena's rows, one float dtype group, weights only: the median
            # is one launch over the rows (tiled arenas read tile-interleaved); same bits, and the
            # write-back below gives client 0's dict the same per-key values
            arena, rows = hit
            med = arena.median(rows)
            averaged_params = raw_client_grad_list[0][1]
            for k in list(averaged_params.keys()):
                averaged_params[k] = med[k]
            return averaged_params
        dev = next((g[k].device for g in grads for k in keys if g[k].is_cuda), None)
        eng = get_engine(dev.index if dev is not None else None)
        cat_dtype = grads[0][keys[0]].dtype
        for k in keys[1:]:
            cat_dtype = torch.promote_types(cat_dtype, grads[0][k].dtype)
        if cat_dtype not in _NATIVE:
            raise TypeError(f"coordinate-wise median of {cat_dtype} weights is not supported")
        segs, numels = [], []
        for k in keys:
            col = []
            for g in grads:
                t = g[k]
                if t.device != eng.device:
                    t = t.to(eng.device)
                if t.dtype != cat_dtype:
                    t = t.to(cat_dtype)  # torch.cat's type promotion
                col.append(t.contiguous().reshape(-1))
            if any(c.numel() != col[0].numel() for c in col):
                raise RuntimeError(f"Sizes of tensors must match (key {k!r})")
            segs.append(col)
            numels.append(col[0].numel())
        vec = torch.empty(sum(numels), dtype=cat_dtype, device=eng.device)
        outs, pos = [], 0
        for n in numels:
            outs.append(vec[pos:pos + n])
            pos += n
        eng.coord_median(segs, outs=outs)
        if dev is None:
            vec = vec.cpu()
        # the reference's write-back walk over every key of client 0's dict (:36-43)
        index = 0
        averaged_params = raw_client_grad_list[0][1]
        for k, params in averaged_params.items():
            median_params = vec[index: index + params.numel()].view(params.size())
            index += params.numel()
            averaged_params[k] = median_params
        return averaged_params
