"""numpy restatement of the reference's LightSecAgg server reconstruction -- TEST INFRASTRUCTURE ONLY.

Op-for-op the per-key arithmetic of python/fedml/cross_silo/lightsecagg/lsa_fedml_aggregator.py:
140-166 (sum of the masked finite models with numpy int64 `+=`, `-= mask`, `np.mod(., p)`) and
core/mpc/lightsecagg.py:157-185 (my_q_inv, torch.Tensor conversion) followed by `* (1/len)`.
Used as the CPU baseline of bench.py's secagg config and pinned by tests/test_oracle_finite.py
against the g14 fixtures.
"""
from __future__ import annotations

import numpy as np
import torch


def my_q_inv(X_q, q_bit, p):
    flag = X_q - (p - 1) / 2
    is_negative = (abs(np.sign(flag)) + np.sign(flag)) / 2
    X_q = X_q - p * is_negative
    return X_q.astype(float) / (2 ** q_bit)


def lsa_reconstruct(models, mask_flat, dims, p, q_bits):
    """models: list of dicts key -> int64 ndarray (first-round active clients, in order);
    mask_flat: int64 ndarray (>= sum(dims)).  Returns dict key -> float32 CPU tensor."""
    out = {}
    pos = 0
    keys = list(models[0].keys())
    for j, k in enumerate(keys):
        acc = np.array(models[0][k], copy=True)
        for m in models[1:]:
            acc += m[k]
        d = dims[j]
        acc -= np.reshape(mask_flat[pos:pos + d], np.shape(acc))
        acc = np.mod(acc, p)
        real = my_q_inv(np.array(acc), q_bits, p)
        t = torch.Tensor([real]) if isinstance(real, np.floating) else torch.Tensor(real)
        out[k] = t * (1 / len(models))
        pos += d
    return out
