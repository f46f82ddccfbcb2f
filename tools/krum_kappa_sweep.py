#!/usr/bin/env python
"""r06: the Gram form's error against kappa, P and K -- calibration of the
guard.  For each (P, K, construction, target kappa) the Gram form is FORCED (no guard) and compared
pair by pair with a float64 reference computed on the device (the centred float64 Gram form:
relative error ~1e-16 kappa, negligible at the 1e-6 scale; the CPU oracle is what the -m gpu tests
use).  Constructions:
  offset -- clients 0, 1, 2 shifted by delta (3 of the 5 that define the kernel's centre, the
            median of clients 0..4), the rest honest around a common model: every honest pair has
            kappa ~ (delta^2 + s^2) / s^2 (VERDICT: honest clients at a controlled offset from the centre)
  pair   -- all honest, and the last client a near copy of the one before it (x + eps z): one pair
            at the target kappa (near-duplicate attackers)
Prints one JSON line per case: realised kappa_max (exact, float64), the kernel's kappa_max, the max
relative error over pairs and the max of (relative error / kappa_ij), plus the modelled bound
(fedml_amd/csrc/robust.hip gram_kappa_bound) at that P and run length.
"""
from __future__ import annotations

import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make(P, K, kind, kappa, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    m = torch.randn(P, generator=g, device="cuda") * 0.05
    s = 1e-2
    z = torch.randn((K, P), generator=g, device="cuda")
    x = m + s * z
    if kind == "offset":
        d = s * max(kappa - 1.3, 0.0) ** 0.5
        x[:3] += d
    else:
        eps = s * (2 * 1.29 / kappa) ** 0.5
        x[K - 1] = x[K - 2] + eps * torch.randn(P, generator=g, device="cuda")
    Ppad = -(-P // 64) * 64  # rows 256-byte aligned, as arena rows (the 16-byte load paths)
    buf = torch.zeros((K, Ppad), device="cuda")
    buf[:, :P] = x
    return buf[:, :P]


def ref64(x):
    """float64 pairwise squared distances and the exact kappa_ij of the kernel's centre."""
    K = x.shape[0]
    xd = x.double()  # (a strided [K, P] view: torch ops below copy as needed)
    xc = xd - xd.mean(0, keepdim=True)
    G = xc @ xc.T
    a = G.diag()
    D = (a[:, None] + a[None, :] - 2 * G).clamp_min(0)
    D.fill_diagonal_(0)
    c = x[:5].median(0).values if K >= 5 else (x[:3].median(0).values if K >= 3 else x[0])
    y = xd - c.double()
    A = (y * y).sum(1)
    kap = (A[:, None] + A[None, :]) / D
    kap.fill_diagonal_(0)
    return D, kap


def main():
    from fedml_amd.engine import get_engine
    eng = get_engine(0)
    Ps = [int(v) for v in os.environ.get("PS", "7850,9001,1000000,11699132").split(",")]
    Ks = [int(v) for v in os.environ.get("KS", "5,32,64,128").split(",")]
    kappas = [float(v) for v in os.environ.get("KAPPAS", "2,4,8,12,15.9").split(",")]
    kinds = os.environ.get("KINDS", "offset,pair").split(",")
    seeds = int(os.environ.get("SEEDS", "1"))
    for P in Ps:
        for K in Ks:
            for kind in kinds:
                for kap in kappas:
                    for sd in range(seeds):
                        x = make(P, K, kind, kap, 1000 * K + 7 * sd + int(kap * 10))
                        D, kij = ref64(x)
                        rows = list(x)
                        Dg = eng._pairwise_launch([rows], form="gram")
                        kg = eng.last_kappa_max
                        iu = torch.triu_indices(K, K, 1, device="cuda")
                        d0, d1, kk = D[iu[0], iu[1]], Dg[iu[0], iu[1]], kij[iu[0], iu[1]]
                        rel = ((d1 - d0).abs() / d0)
                        print(json.dumps({"P": P, "K": K, "kind": kind, "target": kap, "seed": sd,
                                          "kappa_max": round(float(kk.max()), 3), "kernel_kappa_max": round(kg, 3),
                                          "max_rel": float(rel.max()), "max_rel_over_kappa": float((rel / kk).max()),
                                          "pairs": int(kk.numel())}), flush=True)
                        del x, D, kij, Dg


if __name__ == "__main__":
    main()
