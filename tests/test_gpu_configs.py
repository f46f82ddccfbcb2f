"""Every BASELINE.json configuration at its own shape, through the paths a caller uses, against the
C oracle (which tests/test_oracle.py pins to the reference's own outputs):

* cfg1 LR-MNIST (784 -> 10 + bias), K = 2: FedMLAggOperator.agg, every element;
* cfg2 ResNet-18-GN state_dict (122 tensors, 20 int64), K = 32: FedMLAggOperator.agg on device
  state_dicts, FedAvgAPI._aggregate, and a tiled ClientArena; strided sample of every key;
* cfg3 ViT-B/16 bf16 layout (152 tensors, 86.6 M elements), K = 128: the same three paths;
* cfg4 hierarchical 8 groups x 64 clients x 11,699,132 fp32: fa_weighted_sum_grouped over separate
  client tensors and over a tiled arena (group FedAvg -> cloud term -> ordered sum over groups);
* cfg5 gossip, 256 ring nodes x 11,699,132 fp32: the 8 per-rank local problems of an 8-GPU run
  (32 nodes + 2 halo models each, interior rows then boundary rows, GossipPlan ordering) on one GPU,
  every node's row bit-exact to the single-device DSGD rows.

Sampled comparisons take whole 4-KiB tiles by slicing (torch's index_select faults on tensors of
more than 2^31 elements on this ROCm build, tools/diag_large.py)."""
from __future__ import annotations

import json
import os
import types
from collections import OrderedDict

import numpy as np
import pytest
import torch

from refcases import MUL_N_DIV_N, MUL_W

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RESNET18_P = 11_699_132
E = 1024


@pytest.fixture(scope="module")
def eng():
    from fedml_amd.engine import get_engine
    return get_engine(0)


def _layout(name):
    with open(os.path.join(ROOT, "tests", "golden", "layouts.json")) as f:
        return [(k, tuple(s), getattr(torch, dt)) for k, s, dt in json.load(f)[name]]


def _counts(K, seed=7):
    return [int(v) for v in np.random.RandomState(seed).randint(50, 601, size=K)]


def _dicts(K, layout, seed0=1000):
    out = []
    for i in range(K):
        g = torch.Generator(device="cuda").manual_seed(seed0 + i)
        d = OrderedDict()
        for name, shape, dt in layout:
            d[name] = (torch.randint(0, 100, shape, generator=g, device="cuda", dtype=dt) if dt == torch.int64
                       else torch.randn(shape, generator=g, device="cuda").to(dt))
        out.append(d)
    return out


def _bad(got, exp):
    ib = {4: torch.int32, 2: torch.int16, 8: torch.int64}[got.element_size()]
    assert got.dtype == exp.dtype, (got.dtype, exp.dtype)
    return int((got.reshape(-1).view(ib) != exp.reshape(-1).view(ib)).sum())


def _check_dict(result, dicts, layout, w, per_key=512):
    """Oracle FedAvg on a strided sample of every key; returns the number of differing elements."""
    from oracle import orc
    bad = 0
    for name, shape, _ in layout:
        n = int(np.prod(shape))
        idx = torch.arange(0, n, max(1, n // per_key), device="cuda")
        exp = orc.weighted_sum([d[name].reshape(-1).index_select(0, idx).cpu() for d in dicts], MUL_W, w)
        bad += _bad(result[name].reshape(-1).index_select(0, idx).cpu(), exp)
    return bad


def _tiles(P, count, seed):
    nt = -(-P // E)
    return sorted(torch.randperm(nt, generator=torch.Generator().manual_seed(seed))[:min(count, nt)].tolist())


def _pick(x, tiles, P):
    return torch.cat([x[t * E:min((t + 1) * E, P)] for t in tiles]).cpu()


def _arena_pick(buf, tiles, P):
    blk = torch.stack([buf[t] for t in tiles]).cpu()
    return torch.cat([blk[j, :, :min(E, P - t * E)] for j, t in enumerate(tiles)], dim=1)


# ------------------------------------------------------------------------------------------ cfg1
def test_cfg1_lr_mnist_K2():
    from oracle import orc
    from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator
    layout = [("linear.weight", (10, 784), torch.float32), ("linear.bias", (10,), torch.float32)]
    dicts = _dicts(2, layout)
    counts = _counts(2)
    w = [c / sum(counts) for c in counts]
    for where, thr in (("cuda", None), ("cpu", None), ("cpu", "0")):
        # CPU dicts: summed on the host below the break-even (host_sum.h, the default for cfg1's
        # 63 KB), or through the device's zero-copy kernel (FEDML_AMD_HOST_CPU_BYTES=0)
        old = os.environ.pop("FEDML_AMD_HOST_CPU_BYTES", None)
        if thr is not None:
            os.environ["FEDML_AMD_HOST_CPU_BYTES"] = thr
        try:
            raw = [(n, OrderedDict((k, v.to(where)) for k, v in d.items())) for n, d in zip(counts, dicts)]
            got = FedMLAggOperator.agg(types.SimpleNamespace(federated_optimizer="FedAvg"), raw)
        finally:
            os.environ.pop("FEDML_AMD_HOST_CPU_BYTES", None)
            if old is not None:
                os.environ["FEDML_AMD_HOST_CPU_BYTES"] = old
        for name, _, _ in layout:
            exp = orc.weighted_sum([d[name].cpu() for d in dicts], MUL_W, w)
            assert got[name].device.type == where and _bad(got[name].cpu(), exp) == 0, (where, thr, name)


# ------------------------------------------------------------------------------------ cfg2 / cfg3
@pytest.mark.parametrize("cfg,K", [("resnet18_gn", 32), ("vit_b16_bf16", 128)])
def test_cfg2_cfg3_state_dict_paths(eng, cfg, K):
    from fedml_amd.arena import ArenaLayout, ClientArena
    from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator
    from fedml_amd.simulation.sp.fedavg_api import FedAvgAPI
    layout = _layout(cfg)
    assert len(layout) == (122 if cfg == "resnet18_gn" else 152)
    dicts = _dicts(K, layout)
    counts = _counts(K)
    w = [c / sum(counts) for c in counts]
    # the drop-in operator on device state_dicts (one allocation per tensor, as callers hold them)
    got = FedMLAggOperator.agg(types.SimpleNamespace(federated_optimizer="FedAvg"), list(zip(counts, dicts)))
    assert list(got.keys()) == [k for k, _, _ in layout]
    assert _check_dict(got, dicts, layout, w) == 0
    del got
    # the SP simulator's inline loop (fedavg_api.py:144-159)
    got = FedAvgAPI(None, None, None)._aggregate(list(zip(counts, dicts)))
    assert _check_dict(got, dicts, layout, w) == 0
    del got
    # a tile-interleaved ClientArena (the bench layout)
    arena = ClientArena(ArenaLayout(layout), capacity=K, tiled=True)
    for i, d in enumerate(dicts):
        arena.write(i, d)
    got = arena.fedavg(counts)
    assert _check_dict(got, dicts, layout, w) == 0
    del arena, got, dicts
    torch.cuda.empty_cache()


# ------------------------------------------------------------------------------------------ cfg4
@pytest.mark.parametrize("form", ["tensors", "tiled"])
def test_cfg4_hierarchical_8x64_resnet_size(eng, form):
    from oracle import orc
    G, M, P = 8, 64, RESNET18_P
    counts = _counts(G * M)
    N = sum(counts)
    gcounts = [counts[g * M:(g + 1) * M] for g in range(G)]
    gn = [sum(c) for c in gcounts]
    w = [c / gn[g] for g in range(G) for c in gcounts[g]]
    gptr = [g * M for g in range(G + 1)]
    tiles = _tiles(P, 8, 4)
    if form == "tensors":
        xs = []
        for i in range(G * M):
            xs.append(torch.randn(P, generator=torch.Generator(device="cuda").manual_seed(1000 + i), device="cuda"))
        out = eng.weighted_sum_grouped(xs, MUL_W, w, 1.0, gptr, MUL_N_DIV_N, gn, [float(N)] * G)
        sample = [_pick(x, tiles, P) for x in xs]
    else:
        from fedml_amd.arena import ArenaLayout, ClientArena
        arena = ClientArena(ArenaLayout([("w", (P,), torch.float32)]), capacity=G * M, tiled=True, zero=False)
        for i in range(G * M):
            arena.write(i, {"w": torch.randn(P, generator=torch.Generator(device="cuda").manual_seed(1000 + i),
                                             device="cuda")})
        groups = [list(range(g * M, (g + 1) * M)) for g in range(G)]
        out = arena.hierarchical(groups, counts, formula="cloud")["w"]
        buf = arena.bufs[torch.float32]
        sample = list(_arena_pick(buf, tiles, P))
    terms = []
    for g in range(G):
        Gg = orc.weighted_sum(sample[gptr[g]:gptr[g + 1]], MUL_W, w[gptr[g]:gptr[g + 1]])
        terms.append(orc.weighted_sum([Gg], MUL_N_DIV_N, [gn[g]], float(N)))
    exp = orc.weighted_sum(terms, 2)
    assert _bad(_pick(out, tiles, P), exp) == 0
    torch.cuda.empty_cache()


# ------------------------------------------------------------------------------------------ cfg5
def test_cfg5_gossip_256_ring_as_8_rank_local_problems(eng):
    """The exact local problems an 8-GPU DistributedGossip step runs (fedml_amd/distributed/
    gossip.py): per rank 32 own nodes + 2 halo models in ring order, interior rows then boundary
    rows, on one device; every node's mixed model on sampled tiles == the oracle's DSGD rows of the
    whole 256-node ring (client_dsgd.py:104-122 order)."""
    from oracle import orc
    from fedml_amd.core.distributed.topology.topology_manager import SymmetricTopologyManager, gossip_rows
    from fedml_amd.distributed.gossip import GossipPlan
    n, P, world = 256, RESNET18_P, 8
    m = SymmetricTopologyManager(n, 2)
    m.generate_topology()
    W = m.topology
    models = {i: torch.randn(P, generator=torch.Generator(device="cuda").manual_seed(1000 + i), device="cuda")
              for i in range(n)}
    mixed = {}

    def local_mix(xs, rp, cs, vs, ps, outs, outs2):
        eng.mix(xs, rp, cs, vs, ps, outs, outs2)
    for r in range(world):
        plan = GossipPlan(W, r, world)
        assert len(plan.mine) == 32 and len(plan.halo_in) == 2 and len(plan.boundary) == 2
        outs = [torch.empty(P, device="cuda") for _ in plan.mine]
        plan.mix_local(models, local_mix, plan.interior, outs)
        plan.mix_local(models, local_mix, plan.boundary, outs)
        for node, o in zip(plan.mine, outs):
            mixed[node] = o
    tiles = _tiles(P, 8, 5)
    exp, _ = orc.mix([_pick(models[i], tiles, P) for i in range(n)], *gossip_rows(W))
    bad = sum(_bad(_pick(mixed[i], tiles, P), exp[i]) for i in range(n))
    assert bad == 0
    del models, mixed
    torch.cuda.empty_cache()
