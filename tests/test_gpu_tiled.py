"""GPU parity of the tile-interleaved arena path (fa_weighted_sum_tiled / fa_weighted_sum_grouped_tiled,
ClientArena(tiled=True)): same bits as the flat path and the oracle -- golden fixtures, every dtype x
mode, ragged tails, row subsets, chunked (t0) launches, every kernel variant, host and device ingest."""
from __future__ import annotations

import os
from collections import OrderedDict

import pytest
import torch

from golden_io import aggregation_cases, load_case
from refcases import MUL_N_DIV_N, MUL_W, SUM, bits_equal, check_case

pytestmark = pytest.mark.gpu

E_BYTES = 4096


@pytest.fixture(scope="module")
def eng():
    from fedml_amd.engine import get_engine
    return get_engine(0)


def tiled_buf(xs, capacity=None, rows=None, pad_value=0):
    """Pack flat CPU tensors into a [tiles, capacity, E] device buffer; client j -> row rows[j]."""
    dt = xs[0].dtype
    E = E_BYTES // xs[0].element_size()
    n = xs[0].numel()
    nt = max(1, -(-n // E))
    cap = capacity or len(xs)
    rows = rows or list(range(len(xs)))
    buf = torch.full((nt, cap, E), pad_value, dtype=dt)
    for j, x in enumerate(xs):
        flat = torch.full((nt * E,), pad_value, dtype=dt)
        flat[:n] = x.reshape(-1)
        buf[:, rows[j], :] = flat.view(nt, E)
    return buf.to("cuda:0")


class TiledEngine:
    """refcases engine adapter routing weighted sums through the tiled kernels."""

    def __init__(self, eng):
        self.eng = eng

    def weighted_sum(self, xs, mode, coef=None, divisor=1.0):
        shape = xs[0].shape
        # spread the clients over a larger arena, in reverse row order: rows are addressed, not assumed
        k = len(xs)
        rows = [2 * (k - 1 - j) + 1 for j in range(k)]
        buf = tiled_buf(xs, capacity=2 * k + 1, rows=rows)
        out = self.eng.weighted_sum_tiled(buf, rows, mode, coef, divisor, n=xs[0].numel())
        return out.cpu().view(shape)

    def mix(self, xs, row_ptr, cols, vals, post_scale=None):
        ys = [x.to("cuda:0") for x in xs]
        o, o2 = self.eng.mix(ys, row_ptr, cols, vals, post_scale)
        return [t.cpu() for t in o], ([t.cpu() for t in o2] if o2 is not None else None)


@pytest.mark.parametrize("path", aggregation_cases(), ids=lambda p: os.path.basename(p)[:-4])
def test_tiled_engine_matches_golden(eng, path):
    meta, arrays = load_case(path)
    check_case(TiledEngine(eng), meta, arrays, "hip-tiled:")


DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64]


def _inputs(dt, K, n, seed):
    g = torch.Generator().manual_seed(seed)
    if dt == torch.int64:
        return [torch.randint(-1000, 1000, (n,), generator=g, dtype=dt) for _ in range(K)]
    return [torch.randn(n, generator=g).to(dt) for _ in range(K)]


@pytest.mark.parametrize("dt", DTYPES, ids=str)
@pytest.mark.parametrize("mode", [MUL_W, MUL_N_DIV_N, SUM])
@pytest.mark.parametrize("K,n", [(1, 1), (3, 1023), (7, 4096 * 3 + 5), (33, 70_001), (128, 9000)])
def test_tiled_matches_flat(eng, dt, mode, K, n):
    xs = _inputs(dt, K, n, K * 1000 + n)
    counts = [50 + 7 * i for i in range(K)]
    coef = None if mode == SUM else ([c / sum(counts) for c in counts] if mode == MUL_W else counts)
    div = float(sum(counts)) if mode == MUL_N_DIV_N else 1.0
    flat = eng.weighted_sum([x.cuda() for x in xs], mode, coef, div).cpu()
    buf = tiled_buf(xs)
    got = eng.weighted_sum_tiled(buf, list(range(K)), mode, coef, div, n=n).cpu()
    assert bits_equal(got, flat)


@pytest.mark.parametrize("variant", range(9))
def test_tiled_all_variants(eng, variant):
    K, n = 19, 4096 * 9 + 777
    xs = _inputs(torch.float32, K, n, 5)
    w = [1.0 / (i + 2) for i in range(K)]
    flat = eng.weighted_sum([x.cuda() for x in xs], MUL_W, w).cpu()
    buf = tiled_buf(xs)
    try:
        eng.set_variant(variant)
        got = eng.weighted_sum_tiled(buf, list(range(K)), MUL_W, w, n=n).cpu()
    finally:
        eng.set_variant(0)
    assert bits_equal(got, flat)


def test_tiled_chunks_and_row_subset(eng):
    """Chunked launches (t0 > 0) over a subset of rows reproduce the whole reduction."""
    cap, n = 12, 1024 * 37 + 100
    xs = _inputs(torch.float32, cap, n, 9)
    buf = tiled_buf(xs)
    rows = [11, 0, 5, 3, 7]
    w = [0.1, 0.2, 0.3, 0.15, 0.25]
    whole = eng.weighted_sum_tiled(buf, rows, MUL_W, w, n=n).cpu()
    exp = eng.weighted_sum([xs[r].cuda() for r in rows], MUL_W, w).cpu()
    assert bits_equal(whole, exp)
    E = 1024
    out = torch.empty(n, device="cuda:0")
    bounds = [0, 5 * E, 6 * E, 30 * E, n]
    for a, b in zip(bounds[:-1], bounds[1:]):
        eng.weighted_sum_tiled(buf, rows, MUL_W, w, n=b - a, t0=a // E, out=out[a:b])
    assert bits_equal(out.cpu(), exp)


@pytest.mark.parametrize("variant", [0, 4, 6])
def test_tiled_multi_ranges_one_launch(eng, variant):
    """fa_weighted_sum_tiled_multi: several tile-aligned ranges (a reduce-scatter chunk's per-rank
    slices, the last one ragged) in one launch == the whole reduction, every kernel variant."""
    cap, n = 9, 1024 * 50 + 333
    xs = _inputs(torch.float32, cap, n, 21)
    buf = tiled_buf(xs)
    rows = [8, 2, 4, 0]
    w = [0.4, 0.1, 0.3, 0.2]
    exp = eng.weighted_sum([xs[r].cuda() for r in rows], MUL_W, w).cpu()
    ranges = [(0, 7 * 1024), (13 * 1024, 20 * 1024 + 5), (26 * 1024, n), (7 * 1024, 13 * 1024)]
    outs = [torch.empty(hi - lo, device="cuda:0") for lo, hi in ranges]
    try:
        eng.set_variant(variant)
        eng.weighted_sum_tiled_multi(buf, rows, MUL_W, w, 1.0, ranges, outs)
    finally:
        eng.set_variant(0)
    for (lo, hi), o in zip(ranges, outs):
        assert bits_equal(o.cpu(), exp[lo:hi]), (lo, hi)


def test_tiled_rejects_bad_arguments(eng):
    from fedml_amd import _native as N
    buf = torch.zeros(4, 3, 1024, device="cuda:0")
    with pytest.raises(IndexError):
        eng.weighted_sum_tiled(buf, [3], SUM)
    with pytest.raises(ValueError):
        eng.weighted_sum_tiled(buf, [0], SUM, n=5 * 1024)
    with pytest.raises(ValueError):
        eng.weighted_sum_tiled(torch.zeros(4, 3, 1000, device="cuda:0"), [0], SUM)
    L = N.lib()
    p = N.ptr_array([buf.data_ptr()])
    out = torch.empty(1024, device="cuda:0")
    rc = L.fa_weighted_sum_tiled(eng._ctx, N.F32, N.SUM, 1024, 1, p, 1000, None, 1.0, out.data_ptr(), None)
    assert rc == N.FA_ERR_INVALID and b"tile_stride" in L.fa_last_error()
    p = N.ptr_array([buf.data_ptr() + 4])
    rc = L.fa_weighted_sum_tiled(eng._ctx, N.F32, N.SUM, 1024, 1, p, 4096, None, 1.0, out.data_ptr(), None)
    assert rc == N.FA_ERR_INVALID and b"aligned" in L.fa_last_error()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float64], ids=str)
@pytest.mark.parametrize("gmode", [MUL_W, MUL_N_DIV_N, SUM])
def test_grouped_tiled_matches_grouped(eng, dt, gmode):
    K, n = 24, 4096 + 2049
    xs = _inputs(dt, K, n, 3)
    gptr = [0, 5, 6, 17, 24]
    counts = [60 + i for i in range(K)]
    w = []
    gn = []
    for g in range(4):
        cs = counts[gptr[g]:gptr[g + 1]]
        gn.append(sum(cs))
        w += [c / sum(cs) for c in cs]
    gc = None if gmode == SUM else ([x / sum(gn) for x in gn] if gmode == MUL_W else gn)
    gd = [float(sum(gn))] * 4 if gmode == MUL_N_DIV_N else None
    exp = eng.weighted_sum_grouped([x.cuda() for x in xs], MUL_W, w, 1.0, gptr, gmode, gc, gd).cpu()
    buf = tiled_buf(xs)
    got = eng.weighted_sum_grouped_tiled(buf, list(range(K)), MUL_W, w, 1.0, gptr, gmode, gc, gd, n=n).cpu()
    assert bits_equal(got, exp)


def _model_dicts(K, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(K):
        out.append(OrderedDict([
            ("conv.weight", torch.randn(64, 3, 7, 7, generator=g)),
            ("bn.running_mean", torch.randn(64, generator=g)),
            ("bn.num_batches_tracked", torch.randint(0, 100, (), generator=g)),
            ("fc.weight", torch.randn(10, 3000, generator=g)),
            ("emb", torch.randn(333, 17, generator=g).to(torch.bfloat16)),
        ]))
    return out


@pytest.mark.parametrize("source", ["host", "pinned", "device"])
def test_tiled_arena_matches_flat_arena(eng, source):
    from fedml_amd.arena import ClientArena
    cl = _model_dicts(6, 1)
    flat = ClientArena.for_model(cl[0], capacity=6, device="cuda:0")
    tiled = ClientArena.for_model(cl[0], capacity=6, device="cuda:0", tiled=True)
    for i, d in enumerate(cl):
        flat.write(i, OrderedDict((k, v.cuda()) for k, v in d.items()))
        if source == "device":
            d = OrderedDict((k, v.cuda()) for k, v in d.items())
        elif source == "pinned":
            d = OrderedDict((k, v.pin_memory()) for k, v in d.items())
        tiled.write(i, d)
    for i in (0, 5):  # read-back round trip
        back = tiled.read(i)
        for k, v in cl[i].items():
            assert bits_equal(back[k].cpu(), v), k
    counts = [100, 7, 250, 33, 61, 9]
    a = flat.fedavg(counts)
    b = tiled.fedavg(counts)
    for k in a:
        assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape
        assert bits_equal(a[k].cpu(), b[k].cpu()), k
    sub = [4, 1, 2]
    a = flat.aggregate(SUM, clients=sub)
    b = tiled.aggregate(SUM, clients=sub)
    for k in a:
        assert bits_equal(a[k].cpu(), b[k].cpu()), k
    with pytest.raises(TypeError):
        tiled.slot(0)


def test_tiled_arena_hierarchical(eng):
    from fedml_amd.arena import ArenaLayout, ClientArena
    lay = ArenaLayout([("a", (1000, 9), torch.float32), ("b", (77,), torch.float32)])
    g = torch.Generator().manual_seed(4)
    cl = [OrderedDict([("a", torch.randn(1000, 9, generator=g)), ("b", torch.randn(77, generator=g))])
          for _ in range(7)]
    flat = ClientArena(lay, 7, device="cuda:0")
    tiled = ClientArena(lay, 7, device="cuda:0", tiled=True)
    for i, d in enumerate(cl):
        flat.write(i, d)
        tiled.write(i, d)
    counts = [5, 9, 100, 3, 44, 2, 61]
    for formula in ("sp", "cloud"):
        a = flat.hierarchical([[0, 1], [2, 3, 4], [5, 6]], counts, formula)
        b = tiled.hierarchical([[0, 1], [2, 3, 4], [5, 6]], counts, formula)
        for k in a:
            assert bits_equal(a[k].cpu(), b[k].cpu()), (formula, k)


@pytest.mark.parametrize("momentum,nesterov,wd", [(0.0, False, 0.0), (0.9, False, 0.0), (0.9, True, 1e-4)])
def test_fedavg_sgd_tiled_matches_flat(eng, momentum, nesterov, wd):
    K, n = 9, 1024 * 21 + 13
    xs = _inputs(torch.float32, K, n, 17)
    w = [(i + 1) / 45 for i in range(K)]
    g = torch.Generator().manual_seed(2)
    p0 = torch.randn(n, generator=g)
    pa, pb = p0.cuda(), p0.cuda()
    ba, bb = torch.zeros(n, device="cuda:0"), torch.zeros(n, device="cuda:0")
    buf = tiled_buf(xs, capacity=K + 2, rows=[K + 1 - j for j in range(K)])
    rows = [K + 1 - j for j in range(K)]
    for first in (True, False, False):
        eng.fedavg_sgd([[x.cuda() for x in xs]], w, [pa], [ba] if momentum else None, 0.5, momentum,
                       weight_decay=wd, nesterov=nesterov, first_step=first)
        eng.fedavg_sgd_tiled(buf, rows, w, pb, bb if momentum else None, 0.5, momentum, weight_decay=wd,
                             nesterov=nesterov, first_step=first)
    assert bits_equal(pa.cpu(), pb.cpu())
    if momentum:
        assert bits_equal(ba.cpu(), bb.cpu())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16], ids=str)
@pytest.mark.parametrize("topo", ["ring", "dense", "pushsum"])
def test_mix_tiled_matches_flat(eng, dt, topo):
    from fedml_amd.core.distributed.topology.topology_manager import SymmetricTopologyManager, gossip_rows
    n, P = 10, 1024 * 7 + 300
    if topo == "dense":
        import numpy as np
        W = np.full((n, n), 1.0 / n, dtype=np.float32)
        rp, cs, vs = gossip_rows(W)
    else:
        m = SymmetricTopologyManager(n, 2)
        m.generate_topology()
        rp, cs, vs = gossip_rows(m.topology)
    post = [1.0 / (i + 1.5) for i in range(n)] if topo == "pushsum" else None
    xs = _inputs(dt, n, P, 31)
    fo, fo2 = eng.mix([x.cuda() for x in xs], rp, cs, vs, post)
    cap = n + 3
    in_rows = [(3 * j + 1) % cap for j in range(n)]
    out_rows = [(5 * r + 2) % cap for r in range(n)]
    buf = tiled_buf(xs, capacity=cap, rows=in_rows)
    obuf = torch.zeros_like(buf)
    obuf2 = torch.zeros_like(buf) if post else None
    eng.mix_tiled(buf, in_rows, rp, cs, vs, obuf, out_rows, post, obuf2, n=P)
    E = buf.shape[2]
    for r in range(n):
        got = obuf[:, out_rows[r], :].reshape(-1)[:P].cpu()
        assert bits_equal(got, fo[r].cpu()), r
        if post:
            assert bits_equal(obuf2[:, out_rows[r], :].reshape(-1)[:P].cpu(), fo2[r].cpu()), r
