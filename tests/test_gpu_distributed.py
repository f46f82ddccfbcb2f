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
