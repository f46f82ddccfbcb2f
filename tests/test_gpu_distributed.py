"""The distributed paths with the HIP engine as the local reduction, on the one GPU of the box
(world_size 1 over RCCL: exercises chunked views, out= buffers, the ordered SUM and the gossip
interior/boundary split on device).  The N > 1 exchange logic is covered by the gloo tests."""
from __future__ import annotations

import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def _bits(a, b):
    return torch.equal(a.cpu().view(torch.int32), b.cpu().view(torch.int32))


@pytest.mark.parametrize("collective", ["reduce", "all_reduce", "ordered", "reduce_scatter"])
@pytest.mark.parametrize("chunks", [1, 5])
def test_group_reducer_engine(pg, collective, chunks):
    from oracle import orc
    from fedml_amd.distributed.group_reduce import GroupReducer
    g = torch.Generator().manual_seed(chunks)
    K, P = 9, 300_000
    xs = [torch.randn(P, generator=g) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    N = sum(counts)
    red = GroupReducer(collective=collective, chunks=chunks)
    got = red.fedavg([x.cuda() for x in xs], [c / N for c in counts])
    torch.cuda.synchronize()
    assert _bits(got, orc.weighted_sum(xs, 0, [c / N for c in counts]))
    got = red.hierarchical([x.cuda() for x in xs], counts, 5 * N)
    G = orc.weighted_sum(xs, 0, [c / N for c in counts])
    assert _bits(got, orc.weighted_sum([G], 1, [N], float(5 * N)))


def test_distributed_gossip_engine(pg):
    from oracle import orc
    from fedml_amd.core.distributed.topology.topology_manager import SymmetricTopologyManager, gossip_rows
    from fedml_amd.distributed.gossip import DistributedGossip
    n, P = 16, 100_003
    m = SymmetricTopologyManager(n, 2)
    m.generate_topology()
    g = torch.Generator().manual_seed(1)
    xs = [torch.randn(P, generator=g) for _ in range(n)]
    dg = DistributedGossip(m.topology)
    outs, _ = dg.step([x.cuda() for x in xs])
    exp, _ = orc.mix(xs, *gossip_rows(m.topology))
    for a, b in zip(outs, exp):
        assert _bits(a, b)


@pytest.mark.parametrize("collective", ["reduce", "all_reduce", "ordered", "reduce_scatter"])
def test_group_reducer_tiled_on_cu_masked_stream(pg, collective):
    """The bench's N > 1 local step: tiled arena partials on a CU-masked stream, collectives
    ordered behind them, result handed back to the caller's stream."""
    from oracle import orc
    from fedml_amd.arena import ArenaLayout, ClientArena
    from fedml_amd.distributed.group_reduce import GroupReducer
    from fedml_amd.engine import get_engine
    eng = get_engine(0)
    g = torch.Generator().manual_seed(7)
    K, P = 5, 1024 * 40
    xs = [torch.randn(P, generator=g) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    w = [c / sum(counts) for c in counts]
    arena = ClientArena(ArenaLayout([("w", (P,), torch.float32)]), K, device="cuda:0", tiled=True)
    for i, x in enumerate(xs):
        arena.write(i, {"w": x.cuda()})
    red = GroupReducer(collective=collective, chunks=3, stream=eng.cu_masked_stream(128))
    got = red.fedavg_tiled(eng, arena.bufs[torch.float32], list(range(K)), w, P)
    got = got.clone()  # consumed on the caller's stream
    torch.cuda.synchronize()
    assert _bits(got, orc.weighted_sum(xs, 0, w))


def test_cu_masked_stream_engine(pg):
    from oracle import orc
    from fedml_amd.engine import get_engine
    eng = get_engine(0)
    s = eng.cu_masked_stream(64)
    g = torch.Generator().manual_seed(3)
    xs = [torch.randn(300_001, generator=g) for _ in range(6)]
    ys = [x.cuda() for x in xs]
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        out = eng.weighted_sum(ys, 2)
    s.synchronize()
    assert _bits(out, orc.weighted_sum(xs, 2))


# ----------------------------------------------------------------------------- native exchange (C ABI)
@pytest.mark.parametrize("collective", ["ordered", "ordered_all", "reduce", "all_reduce", "reduce_scatter"])
@pytest.mark.parametrize("chunks", [1, 4])
def test_native_group_reduce_flat_and_grouped(pg, collective, chunks):
    """fa_group_reduce (include/fedagg_comm.h) over libfedagg's own RCCL communicator at world 1:
    the chunked local step through the C ABI, the RCCL collectives (reduce / all_reduce /
    reduce_scatter run through RCCL even at world 1) and the stream ordering, vs the oracle."""
    from oracle import orc
    from fedml_amd.distributed.group_reduce import GroupReducer
    g = torch.Generator().manual_seed(11 + chunks)
    K, P = 7, 250_003
    xs = [torch.randn(P, generator=g) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    N = sum(counts)
    red = GroupReducer(collective=collective, chunks=chunks, native=True, timing=True)
    assert red.native is not None
    got = red.fedavg([x.cuda() for x in xs], [c / N for c in counts])
    torch.cuda.synchronize()
    exp = orc.weighted_sum(xs, 0, [c / N for c in counts])
    assert _bits(got[:P], exp)
    got = red.hierarchical([x.cuda() for x in xs], counts, 3 * N)
    torch.cuda.synchronize()
    G = orc.weighted_sum(xs, 0, [c / N for c in counts])
    assert _bits(got[:P], orc.weighted_sum([G], 1, [N], float(3 * N)))
    ms, launches = red.local_time()
    assert launches >= 2 and ms > 0


@pytest.mark.parametrize("collective", ["ordered", "reduce", "reduce_scatter"])
def test_native_group_reduce_tiled_cu_masked(pg, collective):
    """The bench's N > 1 step through the C ABI: tiled arena partials on a CU-masked stream."""
    from oracle import orc
    from fedml_amd.arena import ArenaLayout, ClientArena
    from fedml_amd.distributed.group_reduce import GroupReducer
    from fedml_amd.engine import get_engine
    eng = get_engine(0)
    g = torch.Generator().manual_seed(5)
    K, P = 6, 1024 * 37 + 11
    xs = [torch.randn(P, generator=g) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    w = [c / sum(counts) for c in counts]
    arena = ClientArena(ArenaLayout([("w", (P,), torch.float32)]), K, device="cuda:0", tiled=True)
    for i, x in enumerate(xs):
        arena.write(i, {"w": x.cuda()})
    red = GroupReducer(collective=collective, chunks=3, stream=eng.cu_masked_stream(128), native=True)
    got = red.fedavg_tiled(eng, arena.bufs[torch.float32], list(range(K)), w, P).clone()
    torch.cuda.synchronize()
    assert _bits(got[:P], orc.weighted_sum(xs, 0, w))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.int64])
def test_native_group_reduce_dtypes(pg, dtype):
    """bf16 partials (per-op bf16 rounding) and int64 SUM (two's-complement wrap) through RCCL."""
    from oracle import orc
    from fedml_amd.distributed.group_reduce import GroupReducer
    g = torch.Generator().manual_seed(9)
    K, P = 5, 70_001
    if dtype == torch.int64:
        xs = [torch.randint(-2**62, 2**62, (P,), generator=g, dtype=torch.int64) for _ in range(K)]
    else:
        xs = [torch.randn(P, generator=g).to(dtype) for _ in range(K)]
    red = GroupReducer(collective="all_reduce", chunks=3, native=True)
    if dtype == torch.int64:
        got = red.sum([x.cuda() for x in xs])
        exp = orc.weighted_sum(xs, 2)
        torch.cuda.synchronize()
        assert torch.equal(got.cpu(), exp)
    else:
        counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
        w = [c / sum(counts) for c in counts]
        got = red.fedavg([x.cuda() for x in xs], w)
        torch.cuda.synchronize()
        exp = orc.weighted_sum(xs, 0, w)
        assert torch.equal(got.cpu().view(torch.int16), exp.view(torch.int16))


def test_native_comm_last_op_and_plan(pg):
    from fedml_amd.distributed.group_reduce import GroupReducer
    red = GroupReducer(collective="reduce", chunks=2, native=True)
    red.fedavg([torch.ones(5000, device="cuda")], [1.0])
    torch.cuda.synchronize()
    assert "ncclReduce" in red.native.comm.last_op()


# ----------------------------------------------------------------------------- loopback: the ordered body on one GPU
def _loop_inputs(dtype, K, P, seed):
    g = torch.Generator().manual_seed(seed)
    if dtype == torch.int64:
        xs = [torch.randint(-2**62, 2**62, (P,), generator=g, dtype=torch.int64) for _ in range(K)]
    else:
        xs = [torch.randn(P, generator=g).to(dtype) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    return xs, counts


def _same_bits(got, exp):
    ib = {4: torch.int32, 2: torch.int16, 8: torch.int64}[exp.element_size()]
    return got.dtype == exp.dtype and torch.equal(got.cpu().view(ib), exp.view(ib))


@pytest.mark.parametrize("collective", ["ordered", "ordered_all"])
@pytest.mark.parametrize("layout", ["flat", "tiled", "grouped"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.int64])
@pytest.mark.parametrize("chunks", [1, 4])
def test_native_loopback_ordered_exchange(pg, collective, layout, dtype, chunks):
    """FA_XCHG_LOOPBACK at world 1: the default N > 1 exchange body (comm.hip ordered(): grouped
    ncclSend / ncclRecv on communicator 1, the after-exchange events, the owner's rank-ordered SUM,
    the delivery on communicator 2's stream) runs through RCCL on one GPU, the own piece going
    through a self send / receive.  Bit-exact vs the oracle; both communicators carried every chunk.
    Reference: python/fedml/simulation/nccl/base_framework/common.py:196-228."""
    from oracle import orc
    from fedml_amd.arena import ArenaLayout, ClientArena
    from fedml_amd.distributed.group_reduce import GroupReducer
    from fedml_amd.engine import get_engine
    if layout == "grouped" and dtype == torch.int64:
        pytest.skip("the grouped (hierarchical) kernel takes float dtypes only (fa_weighted_sum_grouped)")
    K, P = 6, 4096 * 9 + 77
    xs, counts = _loop_inputs(dtype, K, P, seed=31 + chunks)
    N = sum(counts)
    w = [c / N for c in counts]
    red = GroupReducer(collective=collective, chunks=chunks, native=True, loopback=True)
    assert red.native is not None and red.native.loopback
    before = red.native.comm.op_counts()
    if layout == "flat":
        if dtype == torch.int64:
            got, exp = red.sum([x.cuda() for x in xs]), orc.weighted_sum(xs, 2)
        else:
            got, exp = red.fedavg([x.cuda() for x in xs], w), orc.weighted_sum(xs, 0, w)
        align = 256
    elif layout == "tiled":
        arena = ClientArena(ArenaLayout([("w", (P,), dtype)]), K, device="cuda:0", tiled=True)
        for i, x in enumerate(xs):
            arena.write(i, {"w": x.cuda()})
        got = red.fedavg_tiled(get_engine(0), arena.bufs[dtype], list(range(K)), w, P)
        exp = orc.weighted_sum(xs, 0, w)
        align = 4096 // xs[0].element_size()
    else:
        got = red.hierarchical([x.cuda() for x in xs], counts, 3 * N)
        exp = orc.weighted_sum([orc.weighted_sum(xs, 0, w)], 1, [N], float(3 * N))
        align = 256
    torch.cuda.synchronize()
    assert _same_bits(got[:P], exp)
    after = red.native.comm.op_counts()
    C = min(chunks, -(-P // align))
    d = [a - b for a, b in zip(after, before)]
    assert d == [C, C, C, C], f"sends/recvs on c1, c2: {d}"  # one self send + receive per chunk and phase
    assert red.owned == [(0, P)] or sum(hi - lo for lo, hi in red.owned) == P
    assert "delivery" in red.native.comm.last_op()


@pytest.mark.parametrize("chunks", [1, 3])
def test_native_loopback_partial_and_repeat(pg, chunks):
    """A caller's partial (FA_LOCAL_PARTIAL) through the loopback exchange, three calls in a row on
    the same communicators (event pool reuse), the scratch reused across calls."""
    from oracle import orc
    from fedml_amd.distributed.native_exchange import NativeExchange
    from fedml_amd.distributed.group_reduce import GroupReducer
    red = GroupReducer(collective="ordered", chunks=chunks, native=True, loopback=True)
    for it in range(3):
        g = torch.Generator().manual_seed(100 + it)
        x = torch.randn(50_000 + it * 1000, generator=g)
        part = x.cuda()
        got = red.native.run(NativeExchange.partial(part), part.numel(), 256)
        torch.cuda.synchronize()
        assert _same_bits(got, orc.weighted_sum([x], 2))


def test_scratch_bytes_and_reduce_agree_on_loopback(pg):
    """fa_group_reduce_scratch_bytes rejects FA_XCHG_LOOPBACK on the non-ordered exchanges exactly as
    fa_group_reduce does (both FA_ERR_INVALID), and accepts it on the ordered ones."""
    import ctypes
    from fedml_amd import _native as N
    from fedml_amd.distributed.group_reduce import _native_comm
    from fedml_amd.distributed.native_exchange import NativeExchange
    comm = _native_comm(None)
    part = torch.zeros(4096, device="cuda")
    st, _, _ = NativeExchange.partial(part)
    need = ctypes.c_int64()
    L = N.lib()
    for x in (N.XCHG_REDUCE, N.XCHG_ALL_REDUCE, N.XCHG_REDUCE_SCATTER):
        assert L.fa_group_reduce_scratch_bytes(comm.handle, x | N.XCHG_LOOPBACK, ctypes.byref(st), 4096, 2, 256, 0,
                                               ctypes.byref(need)) == N.FA_ERR_INVALID
        assert "LOOPBACK" in L.fa_last_error().decode()
    for x in (N.XCHG_ORDERED, N.XCHG_ORDERED_ALL):
        assert L.fa_group_reduce_scratch_bytes(comm.handle, x | N.XCHG_LOOPBACK, ctypes.byref(st), 4096, 2, 256, 0,
                                               ctypes.byref(need)) == N.FA_OK
    assert L.fa_group_reduce_scratch_bytes(comm.handle, 9, ctypes.byref(st), 4096, 2, 256, 0,
                                           ctypes.byref(need)) == N.FA_ERR_INVALID
