"""Arena groups in physically contiguous device memory (ClientArena._alloc ->
AggEngine.alloc_contiguous -> fa_device_alloc_contiguous, DESIGN A.3 item 11): the same bits as a
caching-allocator arena for every layout and dtype, zeroed padding when asked, the block freed with
its storage (allocating and dropping more than the device holds in total succeeds), and the
`FEDML_AMD_ARENA_ALLOC=torch` switch."""
from __future__ import annotations

import gc
from collections import OrderedDict

import pytest
import torch

from fedml_amd.arena import ArenaLayout, ClientArena
from fedml_amd.engine import SUM

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _dicts(K, seed):
    g = torch.Generator().manual_seed(seed)
    return [OrderedDict([("w", torch.randn(3000, 7, generator=g)), ("b", torch.randn(17, generator=g)),
                         ("h", torch.randn(5000, generator=g).to(torch.bfloat16)),
                         ("n", torch.randint(0, 100, (33,), generator=g))]) for _ in range(K)]


@pytest.mark.parametrize("tiled", [False, True])
def test_contiguous_arena_bits_equal_torch_arena(tiled, monkeypatch):
    cl = _dicts(5, 3)
    monkeypatch.setattr(ClientArena, "CONTIG_MIN_BYTES", 1)
    a = ClientArena.for_model(cl[0], capacity=5, device=DEV, tiled=tiled)
    assert set(a.alloc_kind.values()) == {"contiguous"}
    for buf in a.bufs.values():  # zero=True: padding and unwritten rows are zero
        assert int(torch.count_nonzero(buf)) == 0
    monkeypatch.setenv("FEDML_AMD_ARENA_ALLOC", "torch")
    b = ClientArena.for_model(cl[0], capacity=5, device=DEV, tiled=tiled)
    assert set(b.alloc_kind.values()) == {"torch"}
    for i, d in enumerate(cl):
        a.write(i, OrderedDict((k, v.to(DEV)) for k, v in d.items()))
        b.write(i, OrderedDict((k, v.to(DEV)) for k, v in d.items()))
    counts = [10, 200, 33, 7, 91]
    x, y = a.fedavg(counts), b.fedavg(counts)
    for k in x:
        assert x[k].dtype == y[k].dtype and torch.equal(x[k].contiguous().view(torch.uint8),
                                                        y[k].contiguous().view(torch.uint8)), k
    back = a.read(3)
    for k, v in cl[3].items():
        assert torch.equal(back[k].cpu(), v), k


def test_contiguous_blocks_are_freed():
    """8 x 48 GiB, one at a time: more than the device's 288 GB in total, so each block must be
    returned when its arena goes."""
    lay = ArenaLayout([("w", (12 << 30,), torch.float32)])  # 48 GiB per group
    for _ in range(8):
        a = ClientArena(lay, capacity=1, device=DEV, zero=False, tiled=True)
        assert a.alloc_kind[torch.float32] == "contiguous"
        a.bufs[torch.float32][-1, 0, :4] = 1.0
        del a
        gc.collect()
    torch.cuda.synchronize()


def test_small_groups_stay_on_the_caching_allocator():
    a = ClientArena(ArenaLayout([("w", (1000,), torch.float32)]), capacity=3, device=DEV, tiled=True)
    assert a.alloc_kind[torch.float32] == "torch"


def test_placement_check_keeps_the_best_block(monkeypatch):
    """The placement check (ClientArena._place) on a 16 GiB tiled group: the ratio of every block it
    measured is recorded, at most PLACEMENT_TRIES blocks, the kept one has the smallest ratio; forcing
    a threshold of 0 makes it try all of them; the kept block still aggregates bit-exactly."""
    monkeypatch.setattr(ClientArena, "PLACEMENT_RATIO", 0.0)  # every block "slow": all tries happen
    P = 1 << 25
    lay = ArenaLayout([("w", (P,), torch.float32)])  # 128 MiB per client x 128 clients = 16 GiB
    a = ClientArena(lay, capacity=128, device=DEV, zero=True, tiled=True)
    pl = a.placement[torch.float32]
    assert len(pl["ratios"]) == ClientArena.PLACEMENT_TRIES
    assert pl["ratios"][pl["kept"]] == min(pl["ratios"]) and all(r > 0.5 for r in pl["ratios"])
    for i in (0, 1, 127):
        a.write(i, {"w": torch.full((P,), float(i + 1), device=DEV)})
    got = a.aggregate(SUM, clients=[0, 1, 127])["w"]  # 1 + 2 + 128
    assert float(got.min()) == 131.0 and float(got.max()) == 131.0
    del a, got
    monkeypatch.setenv("FEDML_AMD_ARENA_PLACEMENT", "0")
    b = ClientArena(lay, capacity=128, device=DEV, zero=False, tiled=True)
    assert torch.float32 not in b.placement
