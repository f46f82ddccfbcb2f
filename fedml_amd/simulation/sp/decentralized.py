"""Decentralized gossip steps (reference: python/fedml/simulation/sp/decentralized/client_dsgd.py:
92-122 and client_pushsum.py:111-156), one launch of the mixing kernel per tensor for ALL nodes.

The reference's single-process simulator shares one model object between all clients and updates
them in place one after another (decentralized_fl_api.py:54-106), which makes its trajectory
degenerate; the step here is the per-node function the reference defines -- node i mixes the
neighbour models it received this round (synchronous / Jacobi semantics):

  DSGD:     x_i <- x_i * W_ii, then x_i += x_j * W_ji for every in-neighbour j in ascending order
  PushSum:  the same x update, omega_i <- omega_i * W_ii + sum_j omega_j * W_ji,  z_i = x_i * (1/omega_i)
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional, Sequence

import numpy as np
import torch

from ...core.distributed.topology.topology_manager import gossip_rows
from ...ml.aggregator.state_dict_agg import mix


def dsgd_step(models: Sequence[dict], W: np.ndarray):
    """models[i] = node i's parameter dict; returns the list of updated dicts."""
    rows, _ = mix(models, *gossip_rows(W))
    return rows


def pushsum_step(models: Sequence[dict], W: np.ndarray, omegas):
    """Returns (x_new, z_new, omega_new); z = x * (1 / omega) on the GPU in the same pass.

    ``omegas`` a float32 DEVICE tensor: the weights stay on the device (fa_pushsum -- omega' is
    mixed by the same rows in float32 and 1/omega' computed on the GPU) and omega_new is returned
    as a device tensor; a sequence of numbers: the host bookkeeping, omega_new a list."""
    if isinstance(omegas, torch.Tensor) and omegas.is_cuda:
        return _pushsum_step_device(models, W, omegas)
    n = W.shape[0]
    new_omega: List[float] = []
    for i in range(n):
        om = omegas[i] * W[i, i]
        for j in range(n):
            if j != i and W[j, i] != 0:
                om += omegas[j] * W[j, i]
        new_omega.append(om)
    rows, z = mix(models, *gossip_rows(W), post_scale=[1.0 / o for o in new_omega])
    return rows, z, new_omega


def _pushsum_step_device(models: Sequence[dict], W: np.ndarray, omegas: torch.Tensor):
    from ...engine import get_engine
    eng = get_engine(omegas.device.index)
    row_ptr, cols, vals = gossip_rows(W)
    keys = list(models[0].keys())
    n = len(row_ptr) - 1
    rows = [OrderedDict() for _ in range(n)]
    z = [OrderedDict() for _ in range(n)]
    omega_out = torch.empty(n, dtype=torch.float32, device=omegas.device)
    for k in keys:
        col = [m[k] for m in models]
        shape = col[0].shape
        if col[0].dtype not in (torch.float32, torch.bfloat16, torch.float16):
            col = [t.to(torch.float32) for t in col]  # integer buffers: int -> float32 (x * float32 weight)
        col = [t.to(eng.device).contiguous().reshape(-1) for t in col]
        o, o2, _ = eng.pushsum(col, row_ptr, cols, vals, omegas, omega_out=omega_out)
        for r in range(n):
            rows[r][k] = o[r].reshape(shape)
            z[r][k] = o2[r].reshape(shape)
    return rows, z, omega_out
