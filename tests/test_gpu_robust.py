"""GPU parity of the robust-aggregation kernels: coordinate-wise median bit-for-bit against the
reference fixtures (g16) and the C oracle (every K bucket, NaN / +-0 / ties, all dtypes,
multi-segment), Krum's pairwise distances against the exact float64 oracle (rtol 1e-6) and the
Krum / multi-Krum selection against the reference (g18)."""
from __future__ import annotations

import os
import types
from collections import OrderedDict

import numpy as np
import pytest
import torch

from golden_io import ROBUST_PREFIXES, client_dicts, expected_dicts, list_cases, load_case
from refcases import assert_dict_bits, bits_equal

pytestmark = pytest.mark.gpu

CASES = list_cases()
ROB = {kind: [p for p in CASES if os.path.basename(p).startswith(kind)] for kind in ROBUST_PREFIXES}
ids = lambda p: os.path.basename(p)[:-4]  # noqa: E731
DEV = "cuda:0"
WEIGHT = lambda k: "running_mean" not in k and "running_var" not in k and "num_batches_tracked" not in k  # noqa: E731


@pytest.fixture(scope="module")
def eng():
    from fedml_amd.engine import get_engine
    return get_engine(0)


@pytest.mark.parametrize("path", ROB["g16_"], ids=ids)
@pytest.mark.parametrize("where", ["cpu", "cuda"])
def test_median_defense_golden(path, where):
    from fedml_amd.core.security.defense.coordinate_wise_median_defense import CoordinateWiseMedianDefense
    meta, arrays = load_case(path)
    cl = client_dicts(meta, arrays)
    if where == "cuda":
        cl = [OrderedDict((k, v.to(DEV)) for k, v in c.items()) for c in cl]
    raw = list(zip(meta["n"], cl))
    d = CoordinateWiseMedianDefense(types.SimpleNamespace())
    if meta.get("error"):
        with pytest.raises(RuntimeError) as ei:
            d.defend_on_aggregation(raw)
        assert str(ei.value) == meta["error"][1]
        return
    out = d.defend_on_aggregation(raw)
    assert out is cl[0]  # client 0's dict, modified in place (reference :36-44)
    assert_dict_bits(OrderedDict((k, v.cpu()) for k, v in out.items()), expected_dicts(meta, arrays)[0], meta["name"])


def _column_data(g, k, n, dtype, zeros=0.05):
    xs = []
    for i in range(k):
        v = torch.randn(n, generator=g, dtype=torch.float64)
        u = torch.rand(n, generator=g)
        v = torch.where(u < zeros, torch.zeros_like(v), v)
        v = torch.where((u >= zeros) & (u < 2 * zeros), -torch.zeros_like(v), v)
        v = torch.where((u >= 0.5) & (u < 0.52), torch.round(v * 2) / 2, v)  # ties
        v = torch.where((u >= 0.9) & (u < 0.901), torch.full_like(v, float("nan")), v)
        v = torch.where((u >= 0.95) & (u < 0.96), torch.full_like(v, float("inf")) * torch.sign(v - 0.1), v)
        xs.append(v.to(dtype))
    return xs


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 7, 8, 9, 16, 17, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 150])
def test_median_vs_oracle_f32(eng, k):
    from oracle import orc
    g = torch.Generator().manual_seed(k)
    n = 3000 if k > 128 else 20001
    xs = _column_data(g, k, n, torch.float32)
    got = eng.coord_median([[x.to(DEV) for x in xs]])[0].cpu()
    assert bits_equal(got, orc.coord_median(xs))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float64])
@pytest.mark.parametrize("k", [3, 6, 32, 40, 96])
def test_median_vs_oracle_dtypes(eng, dtype, k):
    from oracle import orc
    g = torch.Generator().manual_seed(100 + k)
    xs = _column_data(g, k, 5003, dtype, zeros=0.2)
    got = eng.coord_median([[x.to(DEV) for x in xs]])[0].cpu()
    assert bits_equal(got, orc.coord_median(xs))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("k", [1, 2, 8, 9, 17, 33, 63, 64, 65])
@pytest.mark.parametrize("off", [0, 1])
def test_median_16bit_packed_and_unaligned(eng, dtype, k, off):
    """bf16 / f16: 4-byte aligned columns take the two-coordinates-per-lane kernel (K <= 64), views
    at a 2-byte offset the one-per-lane kernel; odd / tiny segment lengths (the last coordinate of an
    odd segment alone), NaN, +-0, ties, +-Inf -- bit-exact either way."""
    from oracle import orc
    g = torch.Generator().manual_seed(7 * k + off)
    sizes = [1, 2, 3, 257, 4096, 3001]
    cols = [_column_data(g, k, n, dtype, zeros=0.15) for n in sizes]
    segs = []
    for c in cols:
        views = []
        for x in c:
            buf = torch.zeros(x.numel() + off + 3, dtype=dtype, device=DEV)
            buf[off:off + x.numel()] = x.to(DEV)
            views.append(buf[off:off + x.numel()])
        segs.append(views)
    outs = eng.coord_median(segs)
    for c, o in zip(cols, outs):
        exp = orc.coord_median(c)
        assert torch.equal(o.cpu().view(torch.int16), exp.view(torch.int16))


@pytest.mark.parametrize("k", [1, 2, 5, 8, 17, 32, 33])
@pytest.mark.parametrize("off", [0, 1])
def test_median_f32_ragged_and_unaligned(eng, k, off):
    """fp32 columns at 8-byte and 4-byte offsets, odd / tiny segment lengths, NaN, +-0, ties, +-Inf,
    K across the network buckets -- bit-exact."""
    from oracle import orc
    g = torch.Generator().manual_seed(11 * k + off)
    sizes = [1, 2, 3, 257, 4096, 3001]
    cols = [_column_data(g, k, n, torch.float32, zeros=0.15) for n in sizes]
    segs = []
    for c in cols:
        views = []
        for x in c:
            buf = torch.zeros(x.numel() + off + 3, dtype=torch.float32, device=DEV)
            buf[off:off + x.numel()] = x.to(DEV)
            views.append(buf[off:off + x.numel()])
        segs.append(views)
    outs = eng.coord_median(segs)
    for c, o in zip(cols, outs):
        exp = orc.coord_median(c)
        assert torch.equal(o.cpu().view(torch.int32), exp.view(torch.int32))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("k", [65, 72, 73, 88, 96, 97, 100, 113, 120, 121, 127, 128])
def test_median_two_lanes_per_column(eng, dtype, k):
    """K in (64, 128] (k_median_2l where the dispatch picks it: two lanes of different waves per
    column, sorted halves merged
    through LDS, +-inf-key sentinels) -- ragged segments around the 128-column tile, NaN (first NaN
    wins, also when only the upper half holds it), +-0 ranks, ties, +-Inf; bit-exact to the oracle."""
    from oracle import orc
    g = torch.Generator().manual_seed(31 * k + (0 if dtype == torch.float32 else 1 if dtype == torch.bfloat16 else 2))
    sizes = [1, 127, 128, 129, 3001]
    cols = [_column_data(g, k, n, dtype, zeros=0.15) for n in sizes]
    cols[4][k - 1][5] = float("nan")   # a NaN only in the upper half's clients
    cols[4][k // 2 + 3][9] = float("-inf")  # a real -inf next to the low sentinels
    cols[4][k - 2][9] = float("-inf")
    outs = eng.coord_median([[x.to(DEV) for x in c] for c in cols])
    for c, o in zip(cols, outs):
        exp = orc.coord_median(c)
        iv = torch.int32 if dtype == torch.float32 else torch.int16
        assert torch.equal(o.cpu().view(iv), exp.view(iv))


def _special_columns(g, k, n, dtype):
    """Columns mixing normal values with the bit patterns a float-key network could mishandle:
    subnormals of both signs (denormal flushing would change the selected bits), signalling and
    negative / payload NaNs, +-0, +-inf and the largest finite values."""
    fb = dtype
    if dtype == torch.float32:
        pats = [0x00000001, 0x007FFFFF, 0x80000001, 0x807FFFFF, 0x00400000, 0x80400000, 0x7F800001, 0xFFC00000,
                0x7FC12345, 0x00000000, 0x80000000, 0x7F800000, 0xFF800000, 0x7F7FFFFF, 0xFF7FFFFF]
    elif dtype == torch.bfloat16:
        pats = [0x0001, 0x007F, 0x8001, 0x807F, 0x0040, 0x7F81, 0xFFC0, 0x0000, 0x8000, 0x7F80, 0xFF80, 0x7F7F, 0xFF7F]
    else:
        pats = [0x0001, 0x03FF, 0x8001, 0x83FF, 0x0200, 0x7C01, 0xFE00, 0x0000, 0x8000, 0x7C00, 0xFC00, 0x7BFF, 0xFBFF]
    w = (np.uint32, np.int32) if dtype == torch.float32 else (np.uint16, np.int16)
    pats = torch.from_numpy(np.array(pats, dtype=w[0]).view(w[1]))
    xs = []
    for i in range(k):
        v = (torch.randn(n, generator=g) * 1e-3).to(fb)
        u = torch.rand(n, generator=g)
        # most columns: subnormals / extremes only (no NaN) so the network, not the rescan, selects
        sel = torch.randint(0, len(pats), (n,), generator=g)
        special = pats[sel].view(fb)
        nan = (special != special)
        pick = (u < 0.6) & ~nan | (u < 0.002)
        xs.append(torch.where(pick, special, v))
    return xs


@pytest.mark.parametrize("layout", ["lanes1", "lanes2", "packed"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("k", [7, 8, 32, 33, 64, 72, 100, 127, 128])
def test_median_special_values_float_keys(eng, dtype, k, layout, monkeypatch):
    """The float-key networks (IEEE minimum / maximum, NaN-propagating; k_median_off, k_median_2l)
    select the same bits as the oracle on subnormals of both signs (a flushing min / max would
    change them), signalling / negative / payload NaNs, +-0, +-inf and +-max, one and two lanes per
    column; "packed": 4-byte aligned 16-bit columns, two per lane on uint16 keys (k_median_pk, K <= 64)."""
    from oracle import orc
    if layout == "packed" and dtype == torch.float32:
        pytest.skip("no packed form for float32")
    monkeypatch.setenv("FA_MEDIAN_LANES", "2" if layout == "lanes2" else "1")
    g = torch.Generator().manual_seed(1000 + k)
    xs = _special_columns(g, k, 4099, dtype)
    off = torch.zeros(1, dtype=dtype, device=DEV)  # 2-byte views: 16-bit types take the one-per-lane kernels
    segs = [torch.cat([off, x.to(DEV)])[1:] if dtype != torch.float32 and layout != "packed" else x.to(DEV)
            for x in xs]
    got = eng.coord_median([segs])[0].cpu()
    iv = torch.int32 if dtype == torch.float32 else torch.int16
    assert torch.equal(got.view(iv), orc.coord_median(xs).view(iv))


def test_median_all_zero_columns(eng):
    """Columns of only +-0 in every sign pattern: ATen returns the zero of rank (K-1)/2 by index."""
    from oracle import orc
    k = 5
    pats = torch.arange(2 ** k)
    xs = [torch.where((pats >> i) & 1 == 1, -torch.zeros(2 ** k), torch.zeros(2 ** k)) for i in range(k)]
    got = eng.coord_median([[x.to(DEV) for x in xs]])[0].cpu()
    assert bits_equal(got, orc.coord_median(xs))
    assert torch.equal(got.view(torch.int32), orc.coord_median(xs).view(torch.int32))


def test_median_multi_segment(eng):
    from oracle import orc
    g = torch.Generator().manual_seed(7)
    k, sizes = 24, [1, 255, 256, 257, 1000, 0, 13]
    cols = [_column_data(g, k, s, torch.float32) for s in sizes]
    outs = eng.coord_median([[x.to(DEV) for x in c] for c in cols])
    for c, o in zip(cols, outs):
        assert bits_equal(o.cpu(), orc.coord_median(c) if c[0].numel() else torch.empty(0))


@pytest.mark.parametrize("k", [2, 3, 5, 8, 15, 16, 17, 24, 31, 32, 33, 48, 64, 80, 97, 100, 128])
def test_pairwise_sqdist_vs_oracle(eng, k):
    from oracle import orc
    g = torch.Generator().manual_seed(k)
    sizes = [70001, 5, 64, 1000]
    xs = [[torch.randn(s, generator=g) * (1 + (i % 3)) for s in sizes] for i in range(k)]
    D = eng.pairwise_sqdist([[xs[i][s].to(DEV) for i in range(k)] for s in range(len(sizes))]).cpu()
    ref = orc.pairwise_sqdist([torch.cat(x) for x in xs])
    assert torch.equal(D, D.T) and torch.all(D.diag() == 0)
    np.testing.assert_allclose(D.numpy(), ref.numpy(), rtol=1e-6)


@pytest.mark.parametrize("k,off", [(4, 1), (8, 3), (20, 2), (32, 1), (33, 1), (100, 2), (128, 1)])
def test_pairwise_sqdist_unaligned_views(eng, k, off):
    """Client vectors at 4-byte (not 16-byte) offsets take the scalar staging loads; one segment
    whose length ends mid-chunk, another spanning many chunks (double-buffered pipeline)."""
    from oracle import orc
    g = torch.Generator().manual_seed(100 + k)
    sizes = [4099, 123_457]
    xs = [[torch.randn(s, generator=g) for s in sizes] for _ in range(k)]
    segs = []
    for s in range(len(sizes)):
        views = []
        for i in range(k):
            buf = torch.zeros(sizes[s] + off + 5, device=DEV)
            buf[off:off + sizes[s]] = xs[i][s].to(DEV)
            views.append(buf[off:off + sizes[s]])
        segs.append(views)
    D = eng.pairwise_sqdist(segs).cpu()
    ref = orc.pairwise_sqdist([torch.cat(x) for x in xs])
    assert torch.equal(D, D.T) and torch.all(D.diag() == 0)
    np.testing.assert_allclose(D.numpy(), ref.numpy(), rtol=1e-6)


@pytest.mark.parametrize("k", [2, 3, 4, 5, 8, 31, 32, 33, 63, 64, 65, 96, 97, 128])
@pytest.mark.parametrize("form", ["gram", "direct"])
def test_pairwise_forms_vs_oracle(eng, k, form):
    """Both forms of fa_pairwise_sqdist for float32 models, forced: the Gram form on the matrix cores
    (fa_pairwise_sqdist_gram: every 32-client tile count, padding clients, ragged segments, a
    multi-chunk segment) and the direct kernel, each within 1e-6 relative of the float64 oracle on
    clients spread around a common model (kappa small), with the Gram form's kappa reported."""
    from oracle import orc
    g = torch.Generator().manual_seed(1000 + k)
    sizes = [9001, 3, 64, 130]
    base = [torch.randn(s, generator=g) for s in sizes]
    xs = [[b + 0.3 * torch.randn(s, generator=g) * (1 + (i % 3)) for b, s in zip(base, sizes)] for i in range(k)]
    D = eng._pairwise_launch([[xs[i][s].to(DEV) for i in range(k)] for s in range(len(sizes))], form=form).cpu()
    assert eng.last_pair_form == form
    if form == "gram":
        assert 0.5 <= eng.last_kappa_max <= eng.KAPPA_MAX, eng.last_kappa_max
    ref = orc.pairwise_sqdist([torch.cat(x) for x in xs])
    assert torch.equal(D, D.T) and torch.all(D.diag() == 0)
    np.testing.assert_allclose(D.numpy(), ref.numpy(), rtol=1e-6)


@pytest.mark.parametrize("k", [5, 16, 17, 32])
@pytest.mark.parametrize("sizes", [(3, 9001, 64), (64, 3, 129, 128), (256,), (127,)])
def test_pairwise_ring_segment_orders(eng, k, sizes):
    """K <= 32's LDS-DMA ring kernel (k_pair_gram_ring): segments without a full 128-coordinate chunk
    before, between and after full ones (the ring's full-chunk index and its fill loads of chunk 0),
    exact multiples of the chunk, and a lone partial chunk; within 1e-6 of the float64 oracle."""
    from oracle import orc
    g = torch.Generator().manual_seed(31 * k + len(sizes))
    base = [torch.randn(s, generator=g) for s in sizes]
    xs = [[b + 0.3 * torch.randn(s, generator=g) for b, s in zip(base, sizes)] for _ in range(k)]
    D = eng._pairwise_launch([[xs[i][s].to(DEV) for i in range(k)] for s in range(len(sizes))], form="gram").cpu()
    ref = orc.pairwise_sqdist([torch.cat(x) for x in xs])
    assert torch.equal(D, D.T) and torch.all(D.diag() == 0)
    np.testing.assert_allclose(D.numpy(), ref.numpy(), rtol=1e-6)


@pytest.mark.parametrize("k", [8, 40, 128])
def test_pairwise_gram_falls_back_when_ill_conditioned(eng, k):
    """Clients 0..4 (the Gram form's centre) far from a tight honest cluster: the honest pairs cancel
    (kappa >> 16), so the default path reruns the direct kernel -- same bits as the direct form; and
    a non-finite input or two identical clients (D = 0) also report kappa = inf and fall back."""
    g = torch.Generator().manual_seed(7 * k)
    P = 20000
    honest = torch.randn(P, generator=g)
    xs = [honest + 1e-3 * torch.randn(P, generator=g) for _ in range(k)]
    for i in range(5):
        xs[i] = xs[i] + 50.0 + torch.randn(P, generator=g)
    segs = [[x.to(DEV) for x in xs]]
    direct = eng._pairwise_launch(segs, form="direct").cpu()
    auto = eng.pairwise_sqdist(segs).cpu()
    assert eng.last_pair_form == "direct" and eng.last_kappa_max > eng.KAPPA_MAX
    assert torch.equal(auto, direct)
    for bad in ("nan", "dup"):
        ys = [x.clone() for x in xs[5:]] + [torch.randn(P, generator=g) for _ in range(5)]
        if bad == "nan":
            ys[3][17] = float("nan")
        else:
            ys[2] = ys[1].clone()
        segs = [[y.to(DEV) for y in ys]]
        auto = eng.pairwise_sqdist(segs).cpu()
        assert eng.last_pair_form == "direct", bad
        direct = eng._pairwise_launch(segs, form="direct").cpu()
        if bad == "dup":
            assert torch.equal(auto, direct) and float(auto[1, 2]) == 0.0
        else:  # the NaN client's row and column are NaN, the rest as the direct kernel
            assert torch.isnan(auto[3]).sum() == k - 1 and torch.equal(auto[:3, :3], direct[:3, :3])


@pytest.mark.parametrize("path", ROB["g18_"], ids=ids)
@pytest.mark.parametrize("where", ["cpu", "cuda"])
def test_krum_defense_golden(path, where):
    from fedml_amd.core.security.defense.krum_defense import KrumDefense
    meta, arrays = load_case(path)
    cl = client_dicts(meta, arrays)
    if where == "cuda":
        cl = [OrderedDict((k, v.to(DEV)) for k, v in c.items()) for c in cl]
    raw = list(zip(meta["n"], cl))
    d = KrumDefense(types.SimpleNamespace(byzantine_client_num=meta["byzantine_client_num"],
                                          krum_param_m=meta["krum_param_m"]))
    sel = d.defend_before_aggregation(raw)
    assert [next(i for i, (_, c) in enumerate(raw) if c is sc) for _, sc in sel] == meta["selected"]
    np.testing.assert_allclose(d._compute_krum_score(cl), meta["scores"], rtol=1e-5)


@pytest.mark.parametrize("path", [p for p in ROB["g18_"] if "f16" in os.path.basename(p)], ids=ids)
def test_pairwise_half_models_vs_reference(eng, path):
    """bf16 / f16 models through fa_pairwise_sqdist_rt: within 1e-6 relative of the oracle's exact
    sums of dtype-rounded differences, and after the mirror's norm rounding equal to every distance
    the reference recorded (compute_euclidean_distance(v_i, v_j).item() ** 2, inf included)."""
    from oracle import orc
    from fedml_amd.core.security.defense.krum_defense import KrumDefense
    meta, arrays = load_case(path)
    cl = client_dicts(meta, arrays)
    vdt = KrumDefense.vector_dtype(cl)
    keys = [k for k in meta["keys"] if WEIGHT(k)]
    segs = [[c[k].to(DEV).float().reshape(-1) for c in cl] for k in keys]
    D = eng.pairwise_sqdist(segs, diff_dtype=vdt).cpu()
    ref = orc.pairwise_sqdist_rt([torch.cat([c[k].float().reshape(-1) for k in keys]) for c in cl], vdt)
    fin = torch.isfinite(ref)
    assert torch.equal(torch.isfinite(D), fin)
    off = fin & ~torch.eye(len(cl), dtype=torch.bool)
    assert float(((D - ref).abs()[off] / ref[off]).max()) <= 1e-6
    got = torch.sqrt(D).to(torch.float32).to(vdt).to(torch.float64).numpy() ** 2
    np.testing.assert_array_equal(got, np.array(meta["dists"]))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K", [8, 40, 100])
def test_pairwise_half_rounding_random(eng, dt, K):
    """The rounding variant over both kernels (lane staging K <= 32, strided staging above) and a
    ragged multi-segment layout, against the oracle restatement; float16 differences that overflow
    give inf exactly where the oracle's do."""
    from oracle import orc
    g = torch.Generator().manual_seed(K)
    sizes = [1000, 3, 4097]
    xs = [[(torch.randn(n, generator=g) * (1 + i % 5) * (3e4 if dt == torch.float16 and i == 1 else 1)).to(dt)
           for n in sizes] for i in range(K)]
    segs = [[xs[i][s].to(DEV).float() for i in range(K)] for s in range(len(sizes))]
    D = eng.pairwise_sqdist(segs, diff_dtype=dt).cpu()
    ref = orc.pairwise_sqdist_rt([torch.cat(x) for x in xs], dt)
    fin = torch.isfinite(ref)
    assert torch.equal(torch.isfinite(D), fin)
    off = fin & ~torch.eye(K, dtype=torch.bool)
    assert float(((D - ref).abs()[off] / ref[off]).max()) <= 1e-6
    if dt == torch.float16:
        assert not bool(fin.all())


def test_robust_errors(eng):
    x = torch.zeros(10, device=DEV)
    with pytest.raises(ValueError):
        eng.pairwise_sqdist([[x]])
    with pytest.raises(TypeError):
        eng.coord_median([[x.long()]])


@pytest.mark.parametrize("K", [129, 200, 256])
def test_pairwise_more_than_128_clients(eng, K):
    """K > 128: blocks of 64 clients, one launch per block pair; every distance within
    1e-6 relative of the exact float64 oracle, symmetric, zero diagonal; Krum selects as the
    reference's rule on those distances."""
    from oracle import orc
    g = torch.Generator().manual_seed(K)
    xs = [torch.randn(5003, generator=g) * (1 + (i % 7)) for i in range(K)]
    d = eng.pairwise_sqdist([[x.to(DEV) for x in xs]]).cpu()
    ref = orc.pairwise_sqdist(xs)
    off = ~torch.eye(K, dtype=torch.bool)
    assert float(((d - ref).abs()[off] / ref[off]).max()) <= 1e-6
    assert torch.equal(d, d.t()) and float(d.diagonal().abs().max()) == 0.0
    from fedml_amd.core.security.defense.krum_defense import KrumDefense
    raw = [(10, OrderedDict(w=x.to(DEV))) for x in xs]
    dfn = KrumDefense(types.SimpleNamespace(byzantine_client_num=3, krum_param_m=4))
    sel = dfn.defend_before_aggregation(raw)
    # the reference's scores on the exact distances (krum_defense.py:52-66), float32 norms squared
    exact = []
    for i in range(K):
        ds = sorted(float(np.float32(np.sqrt(ref[i, j].item()))) ** 2 for j in range(K) if j != i)
        exact.append(sum(ds[:K - 3 - 2]))
    want = torch.argsort(torch.Tensor(exact)).tolist()[:4]
    assert [next(i for i, (_, c) in enumerate(raw) if c is sc) for _, sc in sel] == want


def _reset_defender():
    from fedml_amd.core.security.fedml_defender import FedMLDefender
    FedMLDefender.get_instance().init(types.SimpleNamespace())


@pytest.mark.parametrize("path", [p for p in ROB["g16_"] if "error" not in p and "mixed" not in p][:6],
                         ids=ids)
def test_wise_median_through_server_aggregator(path):
    """ServerAggregator.aggregate with defense_type=wise_median == the reference's defended aggregate."""
    from fedml_amd.ml.aggregator.default_aggregator import DefaultServerAggregator
    meta, arrays = load_case(path)
    cl = client_dicts(meta, arrays)
    try:
        agg = DefaultServerAggregator(torch.nn.Linear(50, 10), types.SimpleNamespace(
            enable_defense=True, defense_type="wise_median", federated_optimizer="FedAvg"))
        out = agg.aggregate(list(zip(meta["n"], cl)))
    finally:
        _reset_defender()
    assert_dict_bits(OrderedDict((k, v.cpu()) for k, v in out.items()), expected_dicts(meta, arrays)[0], meta["name"])


@pytest.mark.parametrize("path", ROB["g18_"], ids=ids)
def test_krum_through_server_aggregator(path):
    """on_before_aggregation (krum / multikrum) keeps the reference's clients; aggregate then
    averages them on the engine exactly as FedMLAggOperator.agg would."""
    from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator
    from fedml_amd.ml.aggregator.default_aggregator import DefaultServerAggregator
    meta, arrays = load_case(path)
    cl = client_dicts(meta, arrays)
    raw = list(zip(meta["n"], cl))
    dt = "multikrum" if meta["krum_param_m"] > 1 else "krum"
    args = types.SimpleNamespace(enable_defense=True, defense_type=dt, federated_optimizer="FedAvg",
                                 byzantine_client_num=meta["byzantine_client_num"], krum_param_m=meta["krum_param_m"])
    try:
        agg = DefaultServerAggregator(torch.nn.Linear(50, 10), args)
        kept, _ = agg.on_before_aggregation(raw)
        out = agg.aggregate(kept)
    finally:
        _reset_defender()
    assert [next(i for i, (_, c) in enumerate(raw) if c is sc) for _, sc in kept] == meta["selected"]
    ref = FedMLAggOperator.agg(types.SimpleNamespace(federated_optimizer="FedAvg"), kept)
    assert_dict_bits(OrderedDict((k, v.cpu()) for k, v in out.items()),
                     OrderedDict((k, v.cpu()) for k, v in ref.items()), "krum+fedavg")


@pytest.mark.parametrize("path", [p for p in ROB["g18_"] if "f64" in os.path.basename(p)], ids=ids)
def test_pairwise_f64_models_vs_reference(eng, path):
    """float64 models through fa_pairwise_sqdist_rt(FA_DTYPE_F64): every squared distance within
    1e-12 relative of the reference's float64 `compute_euclidean_distance(v_i, v_j).item() ** 2`, and
    the selection (near-ties that float32 distances would flip included) equal to the reference's."""
    from fedml_amd.core.security.defense.krum_defense import KrumDefense
    meta, arrays = load_case(path)
    cl = [OrderedDict((k, v.to(DEV)) for k, v in c.items()) for c in client_dicts(meta, arrays)]
    keys = [k for k in meta["keys"] if WEIGHT(k)]
    D = eng.pairwise_sqdist([[c[k].reshape(-1) for c in cl] for k in keys], diff_dtype=torch.float64).cpu().numpy()
    ref = np.array(meta["dists"])
    off = ~np.eye(len(cl), dtype=bool)
    assert float((np.abs(D - ref)[off] / ref[off]).max()) <= 1e-12
    d = KrumDefense(types.SimpleNamespace(byzantine_client_num=meta["byzantine_client_num"],
                                          krum_param_m=meta["krum_param_m"]))
    raw = list(zip(meta["n"], cl))
    sel = d.defend_before_aggregation(raw)
    assert [next(i for i, (_, c) in enumerate(raw) if c is sc) for _, sc in sel] == meta["selected"]


# ----------------------------------------------------------------------------- median over the tiled arena
def _tiled_rows(xs, dtype, cap_extra=2):
    """The clients as rows of a tile-interleaved ClientArena group (fedml_amd/arena.py tiled=True),
    with spare rows so the row pointers are not the first ``K`` of the capacity."""
    from fedml_amd.arena import ArenaLayout, ClientArena
    n = xs[0].numel()
    arena = ClientArena(ArenaLayout([("w", (n,), dtype)]), len(xs) + cap_extra, device=DEV, tiled=True)
    rows = list(range(cap_extra, cap_extra + len(xs)))
    for r, x in zip(rows, xs):
        arena.write(r, {"w": x.to(DEV)})
    return arena, rows


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
@pytest.mark.parametrize("k", [1, 2, 5, 8, 32, 33, 64, 65, 100, 128, 129])
def test_median_tiled_vs_oracle(eng, dtype, k):
    """fa_coord_median_tiled over tile-interleaved arena rows: every kernel form (one lane, two lanes,
    packed 16-bit, rank counting for float64 and K > 128) addresses element e of a row at
    (e / E) * tile_stride + (e % E) * size -- bit-exact to the oracle, NaN / +-0 / ties / +-inf included,
    with lengths that end inside a tile and a workgroup."""
    from oracle import orc
    g = torch.Generator().manual_seed(500 + k)
    n = 3 * 4096 // (8 if dtype == torch.float64 else 4) + 777 if k <= 128 else 2100
    xs = _column_data(g, k, n, dtype, zeros=0.15)
    arena, rows = _tiled_rows(xs, dtype)
    got = eng.coord_median_tiled(arena.bufs[dtype], rows, n=n).cpu()
    exp = orc.coord_median(xs)
    iv = {8: torch.int64, 4: torch.int32, 2: torch.int16}[exp.element_size()]
    assert torch.equal(got.view(iv), exp.view(iv))


@pytest.mark.parametrize("layout", ["lanes1", "lanes2"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("k", [7, 32, 64, 72, 100, 128])
def test_median_tiled_special_values(eng, dtype, k, layout, monkeypatch):
    """The tiled addressing on the float-key networks' hard cases (subnormals, NaN payloads, +-0,
    +-inf, +-max) and through the rare-case rescan (which re-reads the column in the tiled layout)."""
    from oracle import orc
    monkeypatch.setenv("FA_MEDIAN_LANES", "2" if layout == "lanes2" else "1")
    g = torch.Generator().manual_seed(2000 + k)
    xs = _special_columns(g, k, 5000, dtype)
    arena, rows = _tiled_rows(xs, dtype, cap_extra=1)
    got = eng.coord_median_tiled(arena.bufs[dtype], rows, n=5000).cpu()
    iv = torch.int32 if dtype == torch.float32 else torch.int16
    assert torch.equal(got.view(iv), orc.coord_median(xs).view(iv))


def test_median_tiled_equals_flat_large(eng):
    """A model-sized case (K = 40, 3.1 M coordinates): tiled and flat inputs give the same bits."""
    g = torch.Generator(device=DEV).manual_seed(3)
    n = 3_100_003
    xs = [torch.randn(n, generator=g, device=DEV) for _ in range(40)]
    arena, rows = _tiled_rows(xs, torch.float32, cap_extra=0)
    a = eng.coord_median_tiled(arena.bufs[torch.float32], rows, n=n)
    b = eng.coord_median([xs])[0]
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))


@pytest.mark.parametrize("tiled", [False, True])
def test_arena_median_per_key(eng, tiled):
    """ClientArena.median: one launch per dtype group over the rows (tiled: fa_coord_median_tiled),
    per-key views equal to the oracle's median of each key."""
    from oracle import orc
    from fedml_amd.arena import ArenaLayout, ClientArena
    g = torch.Generator().manual_seed(12)
    shapes = [("conv.weight", (16, 3, 3, 3)), ("conv.bias", (16,)), ("fc.weight", (10, 300)), ("fc.bias", (10,))]
    K = 9
    ds = [OrderedDict((k, _column_data(g, 1, int(np.prod(s)), torch.float32)[0].view(s)) for k, s in shapes)
          for _ in range(K)]
    arena = ClientArena(ArenaLayout([(k, s, torch.float32) for k, s in shapes]), K + 1, device=DEV, tiled=tiled)
    for i, d in enumerate(ds):
        arena.write(i + 1, OrderedDict((k, v.to(DEV)) for k, v in d.items()))
    med = arena.median(list(range(1, K + 1)))
    for k, _ in shapes:
        exp = orc.coord_median([d[k].reshape(-1) for d in ds])
        assert torch.equal(med[k].cpu().reshape(-1).view(torch.int32), exp.view(torch.int32)), k


def test_median_defense_on_adopted_rows(eng):
    """The defense on updates adopted into arena rows (what the round drivers hold) takes the
    arena path and returns the same bits as on separate tensors."""
    from fedml_amd.arena import ClientArena, resident_rows
    from fedml_amd.core.security.defense.coordinate_wise_median_defense import CoordinateWiseMedianDefense
    g = torch.Generator().manual_seed(13)
    K = 11
    mk = lambda: OrderedDict(w=torch.randn(40, 30, generator=g), b=torch.randn(30, generator=g))  # noqa: E731
    ds = [mk() for _ in range(K)]
    sep = [OrderedDict((k, v.to(DEV)) for k, v in d.items()) for d in ds]
    adopted = [OrderedDict((k, v.to(DEV)) for k, v in d.items()) for d in ds]
    arena = ClientArena.for_model(adopted[0], K, device=DEV)
    for i, d in enumerate(adopted):
        arena.adopt(i, d)
    assert resident_rows(adopted) is not None
    d = CoordinateWiseMedianDefense(types.SimpleNamespace())
    a = d.defend_on_aggregation([(1.0, x) for x in adopted])
    b = d.defend_on_aggregation([(1.0, x) for x in sep])
    for k in a:
        assert torch.equal(a[k].cpu().view(torch.int32), b[k].cpu().view(torch.int32)), k
