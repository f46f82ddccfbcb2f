"""N > 1 exchange logic on CPU: world_size-2 gloo runs of the group -> global reducer and the
distributed gossip step, with the C oracle injected as the local reduction (the product path uses
the HIP kernels; these tests check the orchestration: chunking, collectives, ordering, halos)."""
from __future__ import annotations

import os
import socket
import sys
import traceback

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_sum(xs, mode, coef, divisor, out):
    from oracle import orc
    out.copy_(orc.weighted_sum([x.contiguous() for x in xs], mode, coef, divisor).reshape(out.shape))
    return out


def _oracle_mix(xs, row_ptr, cols, vals, post_scale, outs, outs2):
    from oracle import orc
    o, o2 = orc.mix(xs, row_ptr, cols, vals, post_scale)
    for a, b in zip(outs, o):
        a.copy_(b)
    if outs2 is not None:
        for a, b in zip(outs2, o2):
            a.copy_(b)


def _clients(K, P, seed=0):
    g = torch.Generator().manual_seed(seed)
    xs = [torch.randn(P, generator=g) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    return xs, counts


def _bits(a, b):
    return torch.equal(a.view(torch.int32), b.view(torch.int32))


def _worker(rank, world, port, fn, errq):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world)
        dist.barrier()  # teardown only once every rank is done
        from fedml_amd.distributed.group_reduce import release_groups
        release_groups()  # no gloo group left for interpreter teardown (it can abort there)
    except Exception:  # noqa: BLE001
        errq.put(f"rank {rank}: {traceback.format_exc()}")
    finally:
        dist.destroy_process_group()


def _spawn(fn, world=2):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


# ------------------------------------------------------------------------------ group reduce
def _case_group_reduce(rank, world):
    from oracle import orc
    from fedml_amd.distributed.group_reduce import GroupReducer
    K, P = 6, 10_001
    xs, counts = _clients(K, P)
    N = sum(counts)
    per = K // world
    mine = list(range(rank * per, (rank + 1) * per))
    w = [counts[i] / N for i in mine]
    # expected: ordered partial per rank, then rank-ordered sum (two ranks: any order is exact)
    parts = [orc.weighted_sum([xs[i] for i in range(r * per, (r + 1) * per)], 0,
                              [counts[i] / N for i in range(r * per, (r + 1) * per)]) for r in range(world)]
    exp = orc.weighted_sum(parts, 2)
    for coll in ("reduce", "all_reduce", "ordered", "ordered_all"):
        for chunks in (1, 3, 8):
            red = GroupReducer(collective=coll, chunks=chunks, local_sum=_oracle_sum)
            got = red.fedavg([xs[i] for i in mine], w)
            if rank == 0 or coll in ("all_reduce", "ordered_all"):
                assert _bits(got, exp), (coll, chunks)
    # hierarchical: group FedAvg, cloud term (G*N_r)/N, ordered sum over groups
    red = GroupReducer(collective="ordered", chunks=4, local_sum=_oracle_sum)
    got = red.hierarchical([xs[i] for i in mine], [counts[i] for i in mine], N)
    terms = []
    for r in range(world):
        idx = list(range(r * per, (r + 1) * per))
        nr = sum(counts[i] for i in idx)
        G = orc.weighted_sum([xs[i] for i in idx], 0, [counts[i] / nr for i in idx])
        terms.append(orc.weighted_sum([G], 1, [nr], float(N)))
    if rank == 0:
        assert _bits(got, orc.weighted_sum(terms, 2))


def test_group_reduce_gloo_world2():
    _spawn(_case_group_reduce)


def _case_reduce_scatter(rank, world):
    from oracle import orc
    from fedml_amd.distributed.group_reduce import GroupReducer
    K, P = 4, 4000
    xs, counts = _clients(K, P, seed=5)
    N = sum(counts)
    mine = [rank * 2, rank * 2 + 1]
    parts = [orc.weighted_sum([xs[2 * r], xs[2 * r + 1]], 0, [counts[2 * r] / N, counts[2 * r + 1] / N])
             for r in range(world)]
    exp = orc.weighted_sum(parts, 2)
    red = GroupReducer(collective="reduce_scatter", chunks=3, local_sum=_oracle_sum)
    shard = red.fedavg([xs[i] for i in mine], [counts[i] / N for i in mine])
    S = P // world
    assert _bits(shard, exp[rank * S:(rank + 1) * S])


def test_reduce_scatter_gloo_world2():
    _spawn(_case_reduce_scatter)


def _case_reduce_scatter_ragged(rank, world):
    """P not divisible by the world size: padded shards, rank r owns [r*S, min((r+1)*S, P))."""
    from oracle import orc
    from fedml_amd.distributed.group_reduce import GroupReducer
    K, P = 4, 4001
    xs, counts = _clients(K, P, seed=6)
    N = sum(counts)
    mine = [rank * 2, rank * 2 + 1]
    exp = orc.weighted_sum([orc.weighted_sum([xs[2 * r], xs[2 * r + 1]], 0, [counts[2 * r] / N, counts[2 * r + 1] / N])
                            for r in range(world)], 2)
    for chunks in (1, 3):
        red = GroupReducer(collective="reduce_scatter", chunks=chunks, local_sum=_oracle_sum)
        shard = red.fedavg([xs[i] for i in mine], [counts[i] / N for i in mine])
        S = -(-P // world)
        assert _bits(shard, exp[rank * S:min((rank + 1) * S, P)]), chunks
    # tiled, shards of whole 1024-element tiles, P = 10 tiles + 77
    P2 = 1024 * 10 + 77
    xs2 = [x[:P2].contiguous() for x in _clients(K, P2, seed=7)[0]]
    exp2 = orc.weighted_sum([orc.weighted_sum([xs2[2 * r], xs2[2 * r + 1]], 0,
                                              [counts[2 * r] / N, counts[2 * r + 1] / N]) for r in range(world)], 2)
    red = GroupReducer(collective="reduce_scatter", chunks=2, local_sum=_oracle_sum)
    shard = red.fedavg_tiled(_OracleTiledEngine(), _tiled_buf([xs2[i] for i in mine]), [0, 1],
                             [counts[i] / N for i in mine], P2)
    S = -(-P2 // (world * 1024)) * 1024
    assert _bits(shard, exp2[rank * S:min((rank + 1) * S, P2)])


def test_reduce_scatter_ragged_gloo_world2():
    _spawn(_case_reduce_scatter_ragged)


# ------------------------------------------------------------------------------ gossip
def _case_gossip(rank, world):
    from oracle import orc
    from fedml_amd.core.distributed.topology.topology_manager import SymmetricTopologyManager, gossip_rows
    from fedml_amd.distributed.gossip import DistributedGossip
    n, P = 8, 3001
    m = SymmetricTopologyManager(n, 4)
    m.generate_topology()
    W = m.topology
    xs, _ = _clients(n, P, seed=9)
    exp_rows, exp2 = orc.mix(xs, *gossip_rows(W), post_scale=[1.0 / (1 + i) for i in range(n)])
    dg = DistributedGossip(W, local_mix=_oracle_mix)
    mine = dg.mine
    assert mine == list(range(rank * 4, rank * 4 + 4))
    outs, outs2 = dg.step([xs[i] for i in mine], post_scale=[1.0 / (1 + i) for i in mine])
    for k, i in enumerate(mine):
        assert _bits(outs[k], exp_rows[i]), i
        assert _bits(outs2[k], exp2[i]), i
    assert dg.halo_in and dg.boundary


def test_gossip_gloo_world2():
    _spawn(_case_gossip)


def test_chunk_bounds_alignment():
    from fedml_amd.distributed.group_reduce import chunk_bounds
    for n, c, a in [(10, 3, 1), (10_000, 3, 1024), (5, 8, 1024), (1024 * 8, 8, 1024), (1024 * 8 + 1, 16, 1024)]:
        b = chunk_bounds(n, c, a)
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
        assert all(lo % a == 0 for lo, _ in b)
        assert len(b) <= c
    assert chunk_bounds(10, 3) == [(0, 3), (3, 6), (6, 10)]


class _OracleTiledEngine:
    """Stands in for AggEngine.weighted_sum_tiled on CPU: gathers the logical elements of a
    [tiles, capacity, E] buffer and reduces them with the oracle."""

    def weighted_sum_tiled(self, buf, rows, mode, coef=None, divisor=1.0, n=None, t0=0, out=None):
        _, cap, E = buf.shape
        assert t0 >= 0 and n is not None
        xs = [buf[t0:, r, :].reshape(-1)[:n] for r in rows]
        return _oracle_sum(xs, mode, coef, divisor, out)


def _tiled_buf(xs, E=1024):
    n = xs[0].numel()
    nt = -(-n // E)
    buf = torch.zeros(nt, len(xs), E)
    for j, x in enumerate(xs):
        f = torch.zeros(nt * E)
        f[:n] = x
        buf[:, j, :] = f.view(nt, E)
    return buf


def _case_group_reduce_tiled(rank, world):
    from oracle import orc
    from fedml_amd.distributed.group_reduce import GroupReducer
    K, P = 6, 1024 * 13 + 77
    xs, counts = _clients(K, P, seed=11)
    N = sum(counts)
    per = K // world
    mine = list(range(rank * per, (rank + 1) * per))
    parts = [orc.weighted_sum([xs[i] for i in range(r * per, (r + 1) * per)], 0,
                              [counts[i] / N for i in range(r * per, (r + 1) * per)]) for r in range(world)]
    exp = orc.weighted_sum(parts, 2)
    buf = _tiled_buf([xs[i] for i in mine])
    for coll in ("reduce", "all_reduce", "ordered", "ordered_all"):
        for chunks in (1, 3, 8):
            red = GroupReducer(collective=coll, chunks=chunks, local_sum=_oracle_sum)
            got = red.fedavg_tiled(_OracleTiledEngine(), buf, list(range(per)), [counts[i] / N for i in mine], P)
            if rank == 0 or coll in ("all_reduce", "ordered_all"):
                assert _bits(got, exp), (coll, chunks)
    # reduce_scatter: shards of whole tiles
    P2 = 1024 * 8
    xs2 = [x[:P2].contiguous() for x in xs]
    exp2 = orc.weighted_sum([orc.weighted_sum([xs2[i] for i in range(r * per, (r + 1) * per)], 0,
                                              [counts[i] / N for i in range(r * per, (r + 1) * per)])
                             for r in range(world)], 2)
    red = GroupReducer(collective="reduce_scatter", chunks=3, local_sum=_oracle_sum)
    shard = red.fedavg_tiled(_OracleTiledEngine(), _tiled_buf([xs2[i] for i in mine]), list(range(per)),
                             [counts[i] / N for i in mine], P2)
    S = P2 // world
    assert _bits(shard, exp2[rank * S:(rank + 1) * S])


def test_group_reduce_tiled_gloo_world2():
    _spawn(_case_group_reduce_tiled)


# ------------------------------------------------------------------------------ ordered, G > 2
def _case_ordered_multi(rank, world):
    """The owner-summed "ordered" exchange at G = 3 / 4: every chunk split over the G-1 owners (some
    pieces empty at small n), rank-ordered sums, delivered to dst (0 or the last rank) or to all;
    bit-identical to the oracle's rank-ordered sum of per-rank partials, flat and tiled, and for the
    hierarchical cloud formula with one group per rank."""
    from oracle import orc
    from fedml_amd.distributed.group_reduce import GroupReducer
    per = 3
    K = per * world
    for P in (1, 5, 1024 * 7 + 13, 40_001):
        xs, counts = _clients(K, P, seed=P)
        N = sum(counts)
        ids = [list(range(r * per, (r + 1) * per)) for r in range(world)]
        parts = [orc.weighted_sum([xs[i] for i in ids[r]], 0, [counts[i] / N for i in ids[r]]) for r in range(world)]
        exp = orc.weighted_sum(parts, 2)
        mine = ids[rank]
        for coll, dst in (("ordered", 0), ("ordered", world - 1), ("ordered_all", 0)):
            for chunks in (1, 4):
                red = GroupReducer(collective=coll, dst=dst, chunks=chunks, local_sum=_oracle_sum)
                out = torch.full((P,), float("nan"))
                got = red.fedavg([xs[i] for i in mine], [counts[i] / N for i in mine], out=out)
                if rank == dst or coll == "ordered_all":
                    assert got is out and _bits(got, exp), (P, coll, dst, chunks)
                owned = sum(hi - lo for lo, hi in red.owned)
                assert owned == 0 if rank == dst else (owned > 0 or P < 1000), (rank, red.owned)
        if P > 1024:
            red = GroupReducer(collective="ordered", chunks=3, local_sum=_oracle_sum)
            got = red.fedavg_tiled(_OracleTiledEngine(), _tiled_buf([xs[i] for i in mine]), list(range(per)),
                                   [counts[i] / N for i in mine], P)
            if rank == 0:
                assert _bits(got, exp), P
        # hierarchical cloud formula, one group per rank: bit-identical to the sequential cloud sum
        red = GroupReducer(collective="ordered", chunks=2, local_sum=_oracle_sum)
        got = red.hierarchical([xs[i] for i in mine], [counts[i] for i in mine], N)
        terms = []
        for r in range(world):
            nr = sum(counts[i] for i in ids[r])
            G = orc.weighted_sum([xs[i] for i in ids[r]], 0, [counts[i] / nr for i in ids[r]])
            terms.append(orc.weighted_sum([G], 1, [nr], float(N)))
        if rank == 0:
            assert _bits(got, orc.weighted_sum(terms, 2)), P


def test_ordered_gloo_world3():
    _spawn(_case_ordered_multi, world=3)


def test_ordered_gloo_world4():
    _spawn(_case_ordered_multi, world=4)


def _case_reduce_scatter_out_untouched(rank, world):
    """reduce_scatter stages internally: a caller's ``out`` is never overwritten with partials."""
    from fedml_amd.distributed.group_reduce import GroupReducer
    xs, counts = _clients(2, 4000, seed=3)
    out = torch.full((4000,), 7.0)
    red = GroupReducer(collective="reduce_scatter", chunks=2, local_sum=_oracle_sum)
    shard = red.fedavg([xs[rank]], [0.5], out=out)
    assert torch.equal(out, torch.full((4000,), 7.0))
    assert shard.numel() == 2000


def test_reduce_scatter_out_untouched_gloo_world2():
    _spawn(_case_reduce_scatter_out_untouched)


# ------------------------------------------------------------------------------ PushSum, device weights
def _oracle_pushsum(xs, row_ptr, cols, vals, omega_in, outs, outs2, omega_out):
    """The engine's fa_pushsum restated: omega' = the row's ordered float32 chain, z = x' * fp32(1/omega')."""
    from oracle import orc
    om = omega_in.numpy().astype(np.float32)
    new = []
    for r in range(len(row_ptr) - 1):
        acc = np.float32(-0.0)
        for j in range(row_ptr[r], row_ptr[r + 1]):
            acc = np.float32(acc + np.float32(om[cols[j]] * np.float32(vals[j])))
        new.append(acc)
    post = [float(np.float32(1.0) / a) for a in new]
    o, o2 = orc.mix(xs, row_ptr, cols, vals, post_scale=post)
    for a, b in zip(outs, o):
        a.copy_(b)
    for a, b in zip(outs2, o2):
        a.copy_(b)
    omega_out.copy_(torch.tensor([float(a) for a in new], dtype=torch.float32))


def _case_pushsum_device_omega(rank, world):
    from oracle import orc
    from fedml_amd.core.distributed.topology.topology_manager import SymmetricTopologyManager, gossip_rows
    from fedml_amd.distributed.gossip import DistributedGossip
    n, P = 12, 2001
    m = SymmetricTopologyManager(n, 2)
    m.generate_topology()
    W = m.topology
    xs, _ = _clients(n, P, seed=13)
    om = np.array([1.0 + i / n for i in range(n)], dtype=np.float32)
    # expected: the whole-ring step (host bookkeeping in numpy float32, reference order)
    rp, cs, vs = gossip_rows(W)
    full_om = torch.empty(n, dtype=torch.float32)
    exp_x = [torch.empty(P) for _ in range(n)]
    exp_z = [torch.empty(P) for _ in range(n)]
    _oracle_pushsum(xs, rp, cs, vs, torch.from_numpy(om), exp_x, exp_z, full_om)
    dg = DistributedGossip(W, local_mix=_oracle_mix, local_pushsum=_oracle_pushsum)
    mine = dg.mine
    x, z, om_out = dg.step([xs[i] for i in mine], omega=torch.from_numpy(om[mine].copy()))
    for k, i in enumerate(mine):
        assert _bits(x[k], exp_x[i]) and _bits(z[k], exp_z[i]), i
        assert float(om_out[k]) == float(full_om[i]), i


def test_pushsum_device_omega_gloo_world2():
    _spawn(_case_pushsum_device_omega)


def test_pushsum_device_omega_gloo_world3():
    _spawn(_case_pushsum_device_omega, world=3)


def test_oracle_pushsum_restatement_matches_reference():
    """_oracle_pushsum (the device-weight step's restatement) reproduces the reference's PushSum
    fixture: x', z' bit for bit, omega' equal to the reference's float32 omegas."""
    sys.path[:0] = [os.path.join(ROOT, "tests", "golden")]
    from golden_io import client_dicts, expected_dicts, load_case
    from fedml_amd.core.distributed.topology.topology_manager import gossip_rows
    meta, arr = load_case(os.path.join(ROOT, "tests", "golden", "g8_pushsum_ring_N8.npz"))
    cl = client_dicts(meta, arr)
    exp = expected_dicts(meta, arr)
    rp, cs, vs = gossip_rows(arr["W"])
    n = len(cl)
    for key in meta["keys"]:
        xs = [c[key].reshape(-1).float() for c in cl]
        ox = [torch.empty_like(xs[0]) for _ in range(n)]
        oz = [torch.empty_like(xs[0]) for _ in range(n)]
        om = torch.empty(n, dtype=torch.float32)
        _oracle_pushsum(xs, rp, cs, vs, torch.tensor(meta["omegas_in"], dtype=torch.float32), ox, oz, om)
        assert om.tolist() == meta["omegas_out"]
        for i in range(n):
            assert _bits(oz[i], exp[i][key].reshape(-1).float()), (key, i)


# ------------------------------------------------------------------------------ world 8 (the 8-GPU node's shape)
def test_ordered_gloo_world8():
    """ordered (dst 0 and dst 7) / ordered_all, flat and tiled, and the hierarchical cloud pre-scale
    over 8 groups, with 8 real gloo ranks: 7 owners, every delivery, bit-exact
    (simulation/nccl/base_framework/common.py:196-228)."""
    _spawn(_case_ordered_multi, world=8)


def _case_reduce_scatter_world(rank, world):
    """reduce_scatter at the node's world size: ragged P (shards padded), several chunks, flat and
    tiled; every rank's shard within 1e-6 normwise of the rank-ordered sum (the backend sums in its
    own order) and equal to gloo's own reduce of the same partials."""
    import torch.distributed as dist
    from oracle import orc
    from fedml_amd.distributed.group_reduce import GroupReducer
    per = 2
    K = per * world
    for P in (8 * 1024 * 3 + 517, 1000):
        xs, counts = _clients(K, P, seed=31 + P)
        N = sum(counts)
        ids = [list(range(r * per, (r + 1) * per)) for r in range(world)]
        parts = [orc.weighted_sum([xs[i] for i in ids[r]], 0, [counts[i] / N for i in ids[r]]) for r in range(world)]
        exp = orc.weighted_sum(parts, 2)
        ref = parts[rank].clone()
        dist.all_reduce(ref)  # gloo's own summation of the same partials
        mine = ids[rank]
        for chunks in (1, 5):
            red = GroupReducer(collective="reduce_scatter", chunks=chunks, local_sum=_oracle_sum)
            shard = red.fedavg([xs[i] for i in mine], [counts[i] / N for i in mine])
            S = -(-P // world)
            lo, hi = rank * S, min((rank + 1) * S, P)
            assert shard.numel() == max(0, hi - lo), (P, chunks)
            if hi > lo:
                e = exp[lo:hi].double()
                assert float((shard.double() - e).norm() / e.norm()) <= 1e-6, (P, chunks)
                assert torch.allclose(shard, ref[lo:hi], rtol=0, atol=1e-6)
        if P > 8 * 1024:  # tiled: shards of whole 1024-element tiles
            red = GroupReducer(collective="reduce_scatter", chunks=3, local_sum=_oracle_sum)
            shard = red.fedavg_tiled(_OracleTiledEngine(), _tiled_buf([xs[i] for i in mine]), list(range(per)),
                                     [counts[i] / N for i in mine], P)
            S = -(-P // (world * 1024)) * 1024
            lo, hi = rank * S, min((rank + 1) * S, P)
            assert shard.numel() == max(0, hi - lo)
            if hi > lo:  # the last ranks own nothing when whole-tile shards cover P early
                e = exp[lo:hi].double()
                assert float((shard.double() - e).norm() / e.norm()) <= 1e-6


def test_reduce_scatter_gloo_world8():
    _spawn(_case_reduce_scatter_world, world=8)


def _case_gossip_ring256(rank, world):
    """DistributedGossip on a 256-node ring split 8 ways (32 nodes per rank, a 2-model halo), plain
    DSGD rows and PushSum with the weights on the device: every node bit-identical to the whole-ring
    step (client_dsgd.py:104-122, client_pushsum.py:127-156)."""
    from oracle import orc
    from fedml_amd.core.distributed.topology.topology_manager import SymmetricTopologyManager, gossip_rows
    from fedml_amd.distributed.gossip import DistributedGossip
    n, P = 256, 257
    m = SymmetricTopologyManager(n, 2)
    m.generate_topology()
    W = m.topology
    xs, _ = _clients(n, P, seed=17)
    rp, cs, vs = gossip_rows(W)
    exp_rows, _ = orc.mix(xs, rp, cs, vs)
    dg = DistributedGossip(W, local_mix=_oracle_mix, local_pushsum=_oracle_pushsum)
    mine = dg.mine
    assert mine == list(range(rank * 32, rank * 32 + 32))
    assert sorted(dg.halo_in) == sorted({(rank * 32 - 1) % n, (rank * 32 + 32) % n})
    outs, _ = dg.step([xs[i] for i in mine])
    for k, i in enumerate(mine):
        assert _bits(outs[k], exp_rows[i]), i
    om = np.array([1.0 + (i % 7) / 8 for i in range(n)], dtype=np.float32)
    full_om = torch.empty(n, dtype=torch.float32)
    exp_x = [torch.empty(P) for _ in range(n)]
    exp_z = [torch.empty(P) for _ in range(n)]
    _oracle_pushsum(xs, rp, cs, vs, torch.from_numpy(om), exp_x, exp_z, full_om)
    x, z, om_out = dg.step([xs[i] for i in mine], omega=torch.from_numpy(om[mine].copy()))
    for k, i in enumerate(mine):
        assert _bits(x[k], exp_x[i]) and _bits(z[k], exp_z[i]), i
        assert float(om_out[k]) == float(full_om[i]), i


def test_gossip_ring256_gloo_world8():
    _spawn(_case_gossip_ring256, world=8)


def _case_hier_groups_world(rank, world):
    """cfg4's shape at 8 ranks: 8 groups, one per rank, and 16 groups, two per rank
    (hierarchical_groups): group FedAvg, cloud term (G N_g)/N, ordered sums -> bit-exact on every
    rank (ordered_all) and on dst 7 (ordered)."""
    from oracle import orc
    from fedml_amd.distributed.group_reduce import GroupReducer
    M, P = 3, 3001
    for gpr in (1, 2):
        G = world * gpr
        xs, counts = _clients(G * M, P, seed=40 + gpr)
        N = sum(counts)
        terms = []
        for g in range(G):
            cg = counts[g * M:(g + 1) * M]
            Gj = orc.weighted_sum(xs[g * M:(g + 1) * M], 0, [c / sum(cg) for c in cg])
            terms.append(orc.weighted_sum([Gj], 1, [sum(cg)], float(N)))
        rank_terms = [orc.weighted_sum(terms[r * gpr:(r + 1) * gpr], 2) if gpr > 1 else terms[r] for r in range(world)]
        exp = orc.weighted_sum(rank_terms, 2)
        my_groups = list(range(rank * gpr, (rank + 1) * gpr))
        my_x = [xs[i] for g in my_groups for i in range(g * M, (g + 1) * M)]
        gcounts = [counts[g * M:(g + 1) * M] for g in my_groups]
        for coll, dst in (("ordered_all", 0), ("ordered", world - 1)):
            red = GroupReducer(collective=coll, dst=dst, chunks=3, local_sum=_oracle_sum)
            got = red.hierarchical_groups(my_x, gcounts, N)
            if coll == "ordered_all" or rank == dst:
                assert _bits(got, exp), (gpr, coll)


def test_hier_groups_gloo_world8():
    _spawn(_case_hier_groups_world, world=8)
