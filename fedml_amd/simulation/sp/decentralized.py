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

from typing import List, Optional, Sequence

import numpy as np

from ...core.distributed.topology.topology_manager import gossip_rows
from ...ml.aggregator.state_dict_agg import mix


def dsgd_step(models: Sequence[dict], W: np.ndarray):
    """models[i] = node i's parameter dict; returns the list of updated dicts."""
    rows, _ = mix(models, *gossip_rows(W))
    return rows


def pushsum_step(models: Sequence[dict], W: np.ndarray, omegas: Sequence[float]):
    """Returns (x_new, z_new, omega_new) lists; z = x * (1 / omega) on the GPU in the same pass."""
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
