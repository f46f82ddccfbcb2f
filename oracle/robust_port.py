"""PyTorch-CPU restatement of the reference's robust aggregators -- TEST INFRASTRUCTURE ONLY.

Op-for-op the tensor work of core/security/defense/coordinate_wise_median_defense.py:26-31
(vectorize, unsqueeze, cat, torch.median) and krum_defense.py:52-66 (one `(v_i - v_j).norm()`
per ordered pair).  bench.py times them as the CPU baselines of its median / krum configs.
"""
from __future__ import annotations

import torch


def median_port(vectors):
    stacked = torch.cat([v.unsqueeze(-1) for v in vectors], dim=-1)
    return torch.median(stacked, dim=-1).values


def krum_distances_port(vectors):
    k = len(vectors)
    d = [[0.0] * k for _ in range(k)]
    for i in range(k):
        for j in range(k):
            if i != j:
                d[i][j] = (vectors[i] - vectors[j]).norm().item() ** 2
    return d
