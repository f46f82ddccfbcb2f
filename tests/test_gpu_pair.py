"""GPU parity of fa_weighted_sum_pair: a float group and the int64 (BatchNorm counter) group of the
same clients in ONE launch -- bit-identical to the two separate launches for every float dtype x
mode x layout (row-major / tiled) x kernel shape (K <= 16 and K > 16), ragged lengths, row subsets,
and through ClientArena on the reference's mixed-dtype golden fixtures (agg_operator.py:37-44 with
int64 -> float32 promotion; FedAVGAggregator.py:99-116 for (x*n)/N)."""
from __future__ import annotations

import os
from collections import OrderedDict

import pytest
import torch

from golden_io import GOLDEN_DIR, client_dicts, expected_dicts, load_case
from refcases import MUL_N_DIV_N, MUL_W, SUM, assert_dict_bits, bits_equal

pytestmark = pytest.mark.gpu

E_BYTES = 4096


@pytest.fixture(scope="module")
def eng():
    from fedml_amd.engine import get_engine
    return get_engine(0)


def _tiled(rows2d, cap_rows):
    """[cap, n] CPU rows -> [tiles, cap, E] device buffer (zero padded)."""
    cap, n = rows2d.shape
    E = E_BYTES // rows2d.element_size()
    nt = max(1, -(-n // E))
    flat = torch.zeros((cap, nt * E), dtype=rows2d.dtype)
    flat[:, :n] = rows2d
    return flat.view(cap, nt, E).transpose(0, 1).contiguous().to("cuda:0")


def _data(dt, cap, n, n64, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(cap, n, generator=g, dtype=torch.float64).mul_(3).to(dt)
    c = torch.randint(0, 1 << 40, (cap, n64), generator=g, dtype=torch.int64)
    c[:, :3] = torch.tensor([0, 1, -7])  # small counters as BatchNorm holds them
    return x, c


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
@pytest.mark.parametrize("mode", [MUL_W, MUL_N_DIV_N, SUM])
@pytest.mark.parametrize("k", [5, 20, 33])
@pytest.mark.parametrize("layout", ["rows", "tiled"])
def test_pair_matches_separate_launches(eng, dt, mode, k, layout):
    cap = k + 3
    n, n64 = 3 * 1024 * 8 + 77, 1029  # ragged: a partial tail tile in both groups
    x, c = _data(dt, cap, n, n64, seed=k * 31 + mode)
    rows = [cap - 1 - 2 * j if j < 2 else j - 2 for j in range(k)]  # out of order, not the first k rows
    counts = [50 + 13 * j for j in range(k)]
    N = sum(counts)
    coef = None if mode == SUM else ([ci / N for ci in counts] if mode == MUL_W else [float(ci) for ci in counts])
    div = float(N) if mode == MUL_N_DIV_N else 1.0
    if layout == "rows":
        bx, bc = x.to("cuda:0"), c.to("cuda:0")
        ref_x = eng.weighted_sum_rows(bx, rows, mode, coef, div)
        ref_c = eng.weighted_sum_rows(bc, rows, mode, coef, div)
        got_x, got_c = eng.weighted_sum_pair(bx, bc, rows, mode, coef, div)
    else:
        bx, bc = _tiled(x, cap), _tiled(c, cap)
        ref_x = eng.weighted_sum_tiled(bx, rows, mode, coef, div, n=n)
        ref_c = eng.weighted_sum_tiled(bc, rows, mode, coef, div, n=n64)
        got_x, got_c = eng.weighted_sum_pair(bx, bc, rows, mode, coef, div, n=n, n_i64=n64)
    assert got_x.dtype == ref_x.dtype and got_c.dtype == ref_c.dtype
    assert got_c.dtype == (torch.int64 if mode == SUM else torch.float32)
    assert bits_equal(got_x.cpu(), ref_x.cpu())
    assert bits_equal(got_c.cpu(), ref_c.cpu())


def test_pair_rejects_bad_groups(eng):
    a = torch.zeros(4, 100, device="cuda:0")
    c = torch.zeros(4, 10, dtype=torch.int64, device="cuda:0")
    with pytest.raises(TypeError):
        eng.weighted_sum_pair(a, a, [0, 1], SUM)
    with pytest.raises(ValueError):
        eng.weighted_sum_pair(a, c.view(4, 10, 1), [0, 1], SUM)
    with pytest.raises(ValueError):
        eng.weighted_sum_pair(a, c, [0, 1], MUL_W, [0.5])
    with pytest.raises(ValueError):  # the int64 group's SUM output is int64
        eng.weighted_sum_pair(a, c, [0, 1], SUM, out_i64=torch.empty(10, device="cuda:0"))


@pytest.mark.parametrize("name", ["g3_fedavg_mixed_K5", "g3_fedavg_mixed_K2", "g4_mpi_xn_div_N_int64_K5"])
@pytest.mark.parametrize("tiled", [False, True])
def test_arena_pair_golden(eng, name, tiled):
    """ClientArena with one float + one int64 group aggregates in one pair launch; same bits as the
    reference on its fixtures (FedAvg x*w and the MPI (x*n)/N)."""
    from fedml_amd.arena import ClientArena
    meta, arr = load_case(os.path.join(GOLDEN_DIR, name + ".npz"))
    cl = client_dicts(meta, arr)
    arena = ClientArena.for_model(cl[0], capacity=len(cl) + 2, device="cuda:0", tiled=tiled)
    assert arena._pair_groups() == torch.float32
    for i, d in enumerate(cl):
        arena.write(i + 1, d)
    rows = list(range(1, len(cl) + 1))
    n = meta["n"]
    if name.startswith("g4"):
        got = arena.aggregate(MUL_N_DIV_N, [float(v) for v in n], float(sum(n)), clients=rows)
    else:
        got = arena.fedavg(n, clients=rows)
    assert_dict_bits(OrderedDict((k, v.cpu()) for k, v in got.items()), expected_dicts(meta, arr)[0], name)


_INLINE_SCRIPT = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from fedml_amd.engine import get_engine
eng = get_engine(0)
g = torch.Generator().manual_seed(5)
outs = []
for k in (3, 16, 40, 128):
    x = torch.randn(k, 20000 + k, generator=g).cuda()
    c = torch.randint(0, 1000, (k, 37), generator=g).cuda()
    w = [1.0 / (i + 2) for i in range(k)]
    outs.append(eng.weighted_sum_rows(x, list(range(k)), 0, w))
    outs.extend(eng.weighted_sum_pair(x, c, list(range(k))[::-1], 1, [float(i + 1) for i in range(k)], 7.0))
    segs = [[x[i, :5000] for i in range(k)], [x[i, 5000:] for i in range(k)]]
    params = [torch.randn(5000, generator=g).cuda(), torch.randn(x.shape[1] - 5000, generator=g).cuda()]
    bufs = [torch.randn(p.numel(), generator=g).cuda() for p in params]
    sq = [torch.rand(p.numel(), generator=g).cuda() for p in params]
    eng.fedavg_sgd(segs, w, params, bufs, 0.5, momentum=0.9, first_step=False)
    eng.fedavg_rmsprop(segs, w, [p.clone() for p in params], sq, None, 0.01)
    outs.extend(params + bufs + sq)
torch.save([o.cpu() for o in outs], sys.argv[2])
"""


def test_inline_descriptors_match_staged(tmp_path):
    """Tables passed as the kernel argument (default for small tables) and staged through a device
    copy (FA_INLINE_DESC=0) give the same bits: weighted sums, the pair launch, fused FedOpt SGD and
    RMSprop steps."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for flag in ("1", "0"):
        path = str(tmp_path / f"out{flag}.pt")
        env = dict(os.environ, FA_INLINE_DESC=flag)
        subprocess.run([sys.executable, "-c", _INLINE_SCRIPT, root, path], env=env, check=True, timeout=120)
        res[flag] = torch.load(path, weights_only=True)
    assert len(res["1"]) == len(res["0"]) == 36
    for a, b in zip(res["1"], res["0"]):
        assert bits_equal(a, b)


@pytest.mark.parametrize("fdt", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
@pytest.mark.parametrize("mode", [MUL_W, MUL_N_DIV_N, SUM])
@pytest.mark.parametrize("k", [3, 17, 40])
def test_state_dict_pair_multi_vs_oracle(fdt, mode, k):
    """Device state_dicts with BatchNorm counters (the drop-in agg() path): the float keys and the
    int64 keys aggregate in one fa_weighted_sum_pair_multi launch; every key equals the oracle."""
    from oracle import orc
    from fedml_amd.ml.aggregator.state_dict_agg import aggregate
    g = torch.Generator().manual_seed(k + 7 * mode)
    spec = [("conv.w", (16, 3, 3, 3)), ("bn.w", (16,)), ("bn.n", ()), ("fc.w", (10, 1000)), ("bn2.n", ()),
            ("big", (70001,)), ("cnt", (5,)), ("tail", (3,))]
    dicts = []
    for _ in range(k):
        d = OrderedDict()
        for name, shape in spec:
            if name.endswith(".n") or name == "cnt":
                d[name] = torch.randint(0, 5000, shape, generator=g, dtype=torch.int64).cuda()
            else:
                d[name] = torch.randn(shape, generator=g, dtype=torch.float64).to(fdt).cuda()
        dicts.append(d)
    counts = [60 + 31 * i for i in range(k)]
    N = sum(counts)
    coef = None if mode == SUM else ([c / N for c in counts] if mode == MUL_W else [float(c) for c in counts])
    div = float(N) if mode == MUL_N_DIV_N else 1.0
    got = aggregate(dicts, mode, coef, div)
    assert list(got) == [n for n, _ in spec]
    for name, shape in spec:
        exp = orc.weighted_sum([d[name].cpu() for d in dicts], mode, coef, div)
        assert got[name].shape == torch.Size(shape) and got[name].dtype == exp.dtype, name
        assert bits_equal(got[name].cpu(), exp), name


def test_staged_table_reuse_across_calls(monkeypatch):
    """r04: a read-only descriptor table identical to the one a staging slot already holds is not
    copied again (fa_detail::stage reuse).  Interleave rounds over two sets of separate-tensor dicts
    (same table -> reuse; other table -> copy), in-place updates of the same tensors between calls
    (same pointers, new data), and a PushSum mix (its kernel writes its staged table: no reuse after
    it) -- every result bit-exact to the oracle, with reuse on and off."""
    from collections import OrderedDict as OD
    from oracle import orc
    from fedml_amd.engine import get_engine
    from fedml_amd.ml.aggregator.state_dict_agg import MUL_W, aggregate
    eng = get_engine(0)
    g = torch.Generator().manual_seed(77)
    shapes = [("a", (300, 7)), ("b", (64,)), ("c", (5, 5, 3)), ("n", (1,))]
    K = 9

    def mk():
        return [OD((k, (torch.randint(0, 50, s, generator=g) if k == "n" else torch.randn(s, generator=g)).cuda())
                   for k, s in shapes) for _ in range(K)]
    for reuse in ("1", "0"):
        monkeypatch.setenv("FA_STAGE_REUSE", reuse)
        A, B = mk(), mk()
        w = [1.0 / K] * K
        for it in range(12):
            ds = A if it % 3 else B
            if it == 5:
                for d in A:  # same pointers, new values
                    d["a"].add_(1.0)
            if it == 7:
                xs = [torch.randn(4099, generator=g).cuda() for _ in range(3)]
                eng.pushsum(xs, [0, 2, 4, 6], [0, 1, 1, 2, 0, 2], [0.5] * 6, torch.ones(3, device="cuda"))
            out = aggregate(ds, MUL_W, w)
            torch.cuda.synchronize()
            for k, _ in shapes:
                exp = orc.weighted_sum([d[k].cpu().reshape(-1) for d in ds], MUL_W, w)
                got = out[k].cpu().reshape(-1)
                ib = {4: torch.int32, 8: torch.int64}[got.element_size()]
                assert torch.equal(got.view(ib), exp.view(ib)), (reuse, it, k)
