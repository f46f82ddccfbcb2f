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
