"""GPU parity: the HIP engine reproduces the reference bit-for-bit (golden fixtures) and matches the
C oracle on larger seeded inputs, every dtype / mode, ragged and misaligned shapes."""
from __future__ import annotations

import os
from collections import OrderedDict

import numpy as np
import pytest
import torch

from golden_io import aggregation_cases, client_dicts, expected_dicts, list_cases, load_case
from refcases import MUL_N_DIV_N, MUL_W, SUM, assert_dict_bits, bits_equal, check_case

pytestmark = pytest.mark.gpu

CASES = aggregation_cases()


@pytest.fixture(scope="module")
def eng():
    from fedml_amd.engine import get_engine
    return get_engine(0)


class HipEngine:
    """refcases engine adapter: CPU tensors in, CPU tensors out, HIP kernels in between."""

    def __init__(self, eng):
        self.eng = eng

    def weighted_sum(self, xs, mode, coef=None, divisor=1.0):
        ys = [x.to("cuda:0") for x in xs]
        out = self.eng.weighted_sum(ys, mode, coef, divisor)
        return out.cpu()

    def mix(self, xs, row_ptr, cols, vals, post_scale=None):
        ys = [x.to("cuda:0") for x in xs]
        o, o2 = self.eng.mix(ys, row_ptr, cols, vals, post_scale)
        return [t.cpu() for t in o], ([t.cpu() for t in o2] if o2 is not None else None)


@pytest.mark.parametrize("path", CASES, ids=lambda p: os.path.basename(p)[:-4])
def test_engine_matches_golden(eng, path):
    meta, arrays = load_case(path)
    check_case(HipEngine(eng), meta, arrays, "hip:")


class Args:
    def __init__(self, **kw):
        self.__dict__.update(kw)


@pytest.mark.parametrize("path", [p for p in CASES if os.path.basename(p).startswith(("g1_fedavg", "g1_fedprox",
                                                                                    "g2_", "g3_", "g5_", "g9_e",
                                                                                    "g9_i"))],
                         ids=lambda p: os.path.basename(p)[:-4])
@pytest.mark.parametrize("where", ["cpu", "cuda"])
def test_dropin_agg_matches_golden(path, where):
    """fedml_amd's FedMLAggOperator.agg == the reference's FedMLAggOperator.agg, same inputs."""
    from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator
    meta, arrays = load_case(path)
    cl = client_dicts(meta, arrays)
    if where == "cuda":
        cl = [OrderedDict((k, v.to("cuda:0")) for k, v in c.items()) for c in cl]
    n = meta["n"]
    opt = meta["optimizer"]
    args = Args(federated_optimizer=opt, client_num_in_total=meta.get("client_num_in_total"),
                client_num_per_round=meta.get("client_num_per_round"))
    if opt in ("SCAFFOLD", "Mime"):
        cs = [OrderedDict((k, torch.from_numpy(arrays[f"c{i}__{k}"].copy()).to(where if where == "cpu" else "cuda:0"))
                          for k in meta["keys"]) for i in range(len(cl))]
        got = list(FedMLAggOperator.agg(args, [(n[i], cl[i], cs[i]) for i in range(len(cl))]))
    else:
        before = [OrderedDict((k, v.clone()) for k, v in c.items()) for c in cl]
        got = [FedMLAggOperator.agg(args=args, raw_grad_list=list(zip(n, cl)))]
        for a, b in zip(cl, before):  # inputs untouched
            assert_dict_bits(a, b, "inputs")
    exp = expected_dicts(meta, arrays)
    for g, e in zip(got, exp):
        for k in g:
            assert g[k].device.type == where.split(":")[0]
        assert_dict_bits(OrderedDict((k, v.cpu()) for k, v in g.items()), e, f"dropin:{meta['name']}")


# ---------------------------------------------------------------- oracle-checked random cases
DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64]


def _rand(shape, dtype, g):
    if dtype == torch.int64:
        return torch.randint(-1000, 1000, shape, generator=g, dtype=torch.int64)
    return torch.randn(shape, generator=g, dtype=torch.float64).to(dtype)


@pytest.mark.parametrize("dtype", DTYPES, ids=str)
@pytest.mark.parametrize("mode", [MUL_W, MUL_N_DIV_N, SUM])
@pytest.mark.parametrize("K,P", [(1, 1), (3, 1023), (5, 4096 * 8 + 3), (33, 100_003), (128, 262_144)])
def test_engine_vs_oracle_random(eng, dtype, mode, K, P):
    from oracle import orc
    g = torch.Generator().manual_seed(K * 1000 + P)
    xs = [_rand((P,), dtype, g) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    N = sum(counts)
    coef = [c / N for c in counts] if mode == MUL_W else counts
    div = float(N)
    exp = orc.weighted_sum(xs, mode, coef, div)
    got = eng.weighted_sum([x.cuda() for x in xs], mode, coef, div).cpu()
    assert bits_equal(got, exp), (dtype, mode, K, P)


@pytest.mark.parametrize("offset", [1, 2, 3, 5])
def test_engine_misaligned_views(eng, offset):
    """Views whose data pointers are not 16-byte aligned take the scalar path, same results."""
    from oracle import orc
    g = torch.Generator().manual_seed(offset)
    K, P = 7, 50_001
    base = [torch.randn(P + 8, generator=g) for _ in range(K)]
    xs = [b[offset:offset + P] for b in base]
    coef = [0.1 * (i + 1) for i in range(K)]
    exp = orc.weighted_sum([x.contiguous() for x in xs], MUL_W, coef)
    got = eng.weighted_sum([b.cuda()[offset:offset + P] for b in base], MUL_W, coef).cpu()
    assert bits_equal(got, exp)


def test_engine_multi_segment_layout(eng):
    """A ResNet-18-GN-shaped state_dict (122 keys, fp32 + int64) in one call per dtype group."""
    import json
    from oracle import orc
    from fedml_amd.ml.aggregator.state_dict_agg import fedavg
    lay = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "layouts.json")))["resnet18_gn"]
    K = 4
    g = torch.Generator().manual_seed(7)
    dicts = []
    for _ in range(K):
        d = OrderedDict()
        for name, shape, dt in lay:
            d[name] = _rand(tuple(shape), getattr(torch, dt), g).cuda()
        dicts.append(d)
    counts = [100, 250, 75, 313]
    out = fedavg(dicts, counts)
    N = sum(counts)
    for name, shape, dt in lay:
        exp = orc.weighted_sum([d[name].cpu().reshape(-1) for d in dicts], MUL_W, [c / N for c in counts])
        assert bits_equal(out[name].cpu().reshape(-1), exp), name
        assert out[name].dtype == (torch.float32 if dt == "int64" else getattr(torch, dt))


def test_engine_empty_and_error_paths(eng):
    from fedml_amd import _native as N
    x = torch.empty(0, device="cuda")
    assert eng.weighted_sum([x, x], MUL_W, [0.5, 0.5]).numel() == 0
    with pytest.raises(ValueError):
        eng.weighted_sum([], MUL_W, [])
    with pytest.raises(RuntimeError):
        eng.weighted_sum([torch.ones(3, device="cuda"), torch.ones(4, device="cuda")], MUL_W, [0.5, 0.5])
    with pytest.raises(TypeError):
        eng.weighted_sum([torch.ones(3, device="cuda", dtype=torch.complex64)], MUL_W, [1.0])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16], ids=str)
def test_mix_vs_oracle_ring(eng, dtype):
    from oracle import orc
    from refcases import dense_csr, dsgd_csr
    g = torch.Generator().manual_seed(3)
    n = 16
    W = np.zeros((n, n), dtype=np.float32)
    for i in range(n):
        for j in (i - 1, i, i + 1):
            W[i, j % n] = np.float32(1 / 3)
    xs = [_rand((70_001,), dtype, g) for _ in range(n)]
    for csr in (dense_csr(W), dsgd_csr(W)):
        scale = [1.0 / (1 + 0.25 * i) for i in range(n)]
        eo, eo2 = orc.mix(xs, *csr, post_scale=scale)
        go, go2 = eng.mix([x.cuda() for x in xs], *csr, post_scale=scale)
        for a, b in zip(go + go2, eo + eo2):
            assert bits_equal(a.cpu(), b)


@pytest.mark.parametrize("variant", list(range(9)))
@pytest.mark.parametrize("dtype,mode", [(torch.float32, MUL_W), (torch.bfloat16, MUL_W), (torch.float16, MUL_N_DIV_N),
                                        (torch.float64, MUL_W), (torch.int64, SUM), (torch.int64, MUL_N_DIV_N)],
                         ids=str)
def test_all_kernel_variants_identical(variant, dtype, mode):
    """Every tuning variant computes the same bits (incl. ragged tails and K not a multiple of U)."""
    from oracle import orc
    from fedml_amd.engine import AggEngine
    eng = AggEngine(0)
    try:
        eng.set_variant(variant)
        g = torch.Generator().manual_seed(variant)
        for K, P in ((1, 70_001), (13, 262_144 + 77), (37, 33_333)):
            xs = [_rand((P,), dtype, g) for _ in range(K)]
            counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
            N = sum(counts)
            coef = [c / N for c in counts] if mode == MUL_W else counts
            exp = orc.weighted_sum(xs, mode, coef, float(N))
            got = eng.weighted_sum([x.cuda() for x in xs], mode, coef, float(N)).cpu()
            assert bits_equal(got, exp), (variant, dtype, mode, K, P)
    finally:
        eng.close()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64], ids=str)
@pytest.mark.parametrize("mode,gmode", [(MUL_W, MUL_W), (MUL_W, MUL_N_DIV_N), (MUL_W, SUM), (SUM, SUM),
                                        (MUL_N_DIV_N, MUL_N_DIV_N)])
@pytest.mark.parametrize("P", [1, 2049, 300_001])
def test_grouped_two_level_vs_oracle(eng, dtype, mode, gmode, P):
    """fa_weighted_sum_grouped == the levels run as separate ordered reductions (C oracle)."""
    from oracle import orc
    g = torch.Generator().manual_seed(P + mode * 10 + gmode)
    gptr = [0, 4, 5, 13, 20]
    K = gptr[-1]
    xs = [_rand((P,), dtype, g) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    coef = [c / sum(counts) for c in counts] if mode == MUL_W else counts
    div = float(sum(counts))
    gcoef = [0.3, 1.7, 2.0, 0.01] if gmode == MUL_W else [11, 7, 3, 5]
    gdiv = [26.0, 26.0, 13.0, 7.0]
    terms = []
    for j in range(len(gptr) - 1):
        Gj = orc.weighted_sum(xs[gptr[j]:gptr[j + 1]], mode, coef[gptr[j]:gptr[j + 1]], div)
        if gmode == SUM:
            terms.append(Gj)
        elif gmode == MUL_W:
            terms.append(orc.weighted_sum([Gj], MUL_W, [gcoef[j]]))
        else:
            terms.append(orc.weighted_sum([Gj], MUL_N_DIV_N, [gcoef[j]], gdiv[j]))
    exp = orc.weighted_sum(terms, SUM)
    got = eng.weighted_sum_grouped([x.cuda() for x in xs], mode, coef, div, gptr, gmode,
                                   gcoef if gmode != SUM else None, gdiv if gmode == MUL_N_DIV_N else None)
    assert bits_equal(got.cpu(), exp)


@pytest.mark.parametrize("mode,gmode", [(MUL_W, MUL_W), (SUM, SUM), (MUL_N_DIV_N, MUL_N_DIV_N)])
@pytest.mark.parametrize("P", [3_122_193, 2_400_000])
def test_grouped_multi_round_vs_oracle(eng, mode, gmode, P):
    """More than one round of resident workgroups (> 8 x CUs tiles of 1,024 floats), a partial last
    round and a ragged last tile, which workgroup 0 takes (r04): fa_weighted_sum_grouped bit-identical
    to the levels as separate ordered reductions over the WHOLE output."""
    from oracle import orc
    g = torch.Generator().manual_seed(P + mode)
    gptr = [0, 3, 8, 9, 16]
    K = gptr[-1]
    xs = [torch.randn(P, generator=g) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    coef = [c / sum(counts) for c in counts] if mode == MUL_W else counts
    div = float(sum(counts))
    gcoef = [0.3, 1.7, 2.0, 0.01] if gmode == MUL_W else [11, 7, 3, 5]
    gdiv = [26.0, 26.0, 13.0, 7.0]
    terms = []
    for j in range(len(gptr) - 1):
        Gj = orc.weighted_sum(xs[gptr[j]:gptr[j + 1]], mode, coef[gptr[j]:gptr[j + 1]], div)
        if gmode == SUM:
            terms.append(Gj)
        elif gmode == MUL_W:
            terms.append(orc.weighted_sum([Gj], MUL_W, [gcoef[j]]))
        else:
            terms.append(orc.weighted_sum([Gj], MUL_N_DIV_N, [gcoef[j]], gdiv[j]))
    exp = orc.weighted_sum(terms, SUM)
    got = eng.weighted_sum_grouped([x.cuda() for x in xs], mode, coef, div, gptr, gmode,
                                   gcoef if gmode != SUM else None, gdiv if gmode == MUL_N_DIV_N else None)
    assert bits_equal(got.cpu(), exp)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16], ids=str)
@pytest.mark.parametrize("layout", ["ring", "halo"])
def test_banded_mix_kernel_equals_general(dtype, layout):
    """The sliding-window (banded) mixing kernel == the general CSR kernel == the oracle."""
    from oracle import orc
    from fedml_amd.engine import AggEngine
    from fedml_amd.core.distributed.topology.topology_manager import SymmetricTopologyManager, gossip_rows
    n = 37
    m = SymmetricTopologyManager(n, 2)
    m.generate_topology()
    g = torch.Generator().manual_seed(11)
    xs = [_rand((50_003,), dtype, g) for _ in range(n)]
    rp, cs, vs = gossip_rows(m.topology)
    if layout == "halo":  # rows 5..20 with inputs ordered [left halo, own, right halo] (distributed)
        rows = list(range(5, 21))
        rp, cs, vs = gossip_rows(m.topology, rows)
        order = list(range(4, 22))
        pos = {v: k for k, v in enumerate(order)}
        cs = [pos[c] for c in cs]
        xs = [xs[v] for v in order]
    scale = [1.0 + 0.5 * i for i in range(len(rp) - 1)]
    exp, exp2 = orc.mix(xs, rp, cs, vs, post_scale=scale)
    outs = {}
    for band in (True, False):
        eng = AggEngine(0)
        try:
            eng.set_mix_band(band)
            o, o2 = eng.mix([x.cuda() for x in xs], rp, cs, vs, post_scale=scale)
            outs[band] = ([t.cpu() for t in o], [t.cpu() for t in o2])
        finally:
            eng.close()
    for band in (True, False):
        for a, b in zip(outs[band][0] + outs[band][1], exp + exp2):
            assert bits_equal(a, b), band


@pytest.mark.parametrize("momentum,dampening,wd,nesterov", [(0.9, 0.0, 0.0, False), (0.0, 0.0, 0.0, False),
                                                            (0.5, 0.1, 0.01, False), (0.9, 0.0, 0.001, True)])
@pytest.mark.parametrize("P", [7, 4099, 262_147])
def test_fedavg_sgd_fused_vs_oracle(eng, momentum, dampening, wd, nesterov, P):
    """fa_fedavg_sgd == FedAvg then the oracle's torch.optim.SGD step, two consecutive steps."""
    from oracle import orc
    g = torch.Generator().manual_seed(P)
    K = 9
    xs = [torch.randn(P, generator=g) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    w = [c / sum(counts) for c in counts]
    p_ref = torch.randn(P, generator=g)
    b_ref = torch.zeros(P)
    p_gpu, b_gpu = p_ref.cuda(), torch.zeros(P, device="cuda")
    for step in range(2):
        avg = orc.weighted_sum(xs, MUL_W, w)
        orc.sgd_apply(avg, p_ref, b_ref if momentum else None, 0.3, momentum, dampening, wd, nesterov, step == 0)
        eng.fedavg_sgd([[x.cuda() for x in xs]], w, [p_gpu], [b_gpu] if momentum else None, 0.3, momentum,
                       dampening, wd, nesterov, first_step=(step == 0))
        assert bits_equal(p_gpu.cpu(), p_ref), step
        if momentum:
            assert bits_equal(b_gpu.cpu(), b_ref), step


def test_more_than_2g_elements(eng):
    """Maximum-size edge: P > 2^31 elements per client (64-bit element indexing in every tile and
    the scalar tail); checked on samples at the start, across the 2^31 boundary and at the end."""
    from oracle import orc
    P = 2 ** 31 + 1029  # ragged tail tile too
    g = torch.Generator(device="cuda").manual_seed(5)
    xs = [torch.randn(P, generator=g, device="cuda") for _ in range(2)]
    w = [0.3, 0.7]
    out = eng.weighted_sum(xs, MUL_W, w)
    # contiguous slices (plain copies): torch's index_select/gather kernels fault on tensors of
    # more than 2^31 elements on this ROCm build (diagnosed with tools/diag_large.py)
    spans = [(0, 4096), (2 ** 31 - 4096, 2 ** 31 + 4096), (P - 4096, P)]
    pick = lambda t: torch.cat([t[a:b].cpu() for a, b in spans])  # noqa: E731
    exp = orc.weighted_sum([pick(x) for x in xs], MUL_W, w)
    assert bits_equal(pick(out), exp)
    del xs, out
    torch.cuda.empty_cache()
