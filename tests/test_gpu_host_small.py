"""Small host-resident rounds (cfg1, the reference's quick_start: CPU state_dicts in, CPU tensors out):
the one-call C++ path (_host.small_host_round -> fa_weighted_sum_host -> the one-workgroup kernel
k_wsum_host1 + completion word) against the C oracle bit for bit -- ragged sizes, many keys, K past
one client group, every dtype, int64 BatchNorm counters (float32 under the weighted modes), mixed
dtype groups, each mode -- and against the larger-round form of the same C-ABI call.
Reference op sequence: python/fedml/ml/aggregator/agg_operator.py:35-63."""
from __future__ import annotations

import os
import subprocess
import sys
import zlib
from collections import OrderedDict

import pytest
import torch

from refcases import MUL_N_DIV_N, MUL_W, SUM, bits_equal

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dicts(g, K, layout):
    out = []
    for i in range(K):
        d = OrderedDict()
        for name, shape, dt in layout:
            if dt == torch.int64:
                d[name] = torch.randint(-1000, 1000, shape, generator=g, dtype=torch.int64)
            else:
                d[name] = torch.randn(shape, generator=g).to(dt)
        out.append(d)
    return out


def _expect(dicts, mode, coef, divisor):
    from oracle import orc
    return OrderedDict((k, orc.weighted_sum([d[k].reshape(-1) for d in dicts], mode, coef, divisor)
                        .reshape(dicts[0][k].shape)) for k in dicts[0])


LAYOUTS = {
    "lr_mnist": [("linear.weight", (10, 784), torch.float32), ("linear.bias", (10,), torch.float32)],
    "ragged": [("a", (1,), torch.float32), ("b", (3, 5), torch.float32), ("c", (4097,), torch.float32),
               ("d", (2, 3, 3), torch.float32)],
    "bn": [("conv.weight", (16, 3, 3, 3), torch.float32), ("bn.weight", (16,), torch.float32),
           ("bn.num_batches_tracked", (), torch.int64), ("fc.weight", (10, 37), torch.float32)],
    "bf16": [("w", (333,), torch.bfloat16), ("b", (7,), torch.bfloat16)],
    "f16": [("w", (1023,), torch.float16), ("b", (9,), torch.float16)],
    "f64": [("w", (513,), torch.float64), ("b", (3,), torch.float64)],
    "mixed": [("w", (257,), torch.float32), ("h", (131,), torch.bfloat16), ("d", (65,), torch.float64),
              ("n", (5,), torch.int64)],
    "many_keys": [(f"k{t}", (t % 7 + 1,), torch.float32) for t in range(40)],
}


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 2, 5, 9])
@pytest.mark.parametrize("name", sorted(LAYOUTS))
@pytest.mark.parametrize("mode", [MUL_W, MUL_N_DIV_N, SUM])
def test_small_host_round_vs_oracle(name, K, mode):
    from fedml_amd import _host
    from fedml_amd.ml.aggregator import state_dict_agg as sda
    g = torch.Generator().manual_seed(zlib.crc32(f"{name}/{K}/{mode}".encode()))
    dicts = _dicts(g, K, LAYOUTS[name])
    counts = [int(c) for c in torch.randint(10, 900, (K,), generator=g)]
    if mode == MUL_W:
        coef, div = [c / sum(counts) for c in counts], 1.0
    elif mode == MUL_N_DIV_N:
        coef, div = [float(c) for c in counts], float(sum(counts))
    else:
        coef, div = None, 1.0
    eng = sda.get_engine(None)
    fn, err, ctx = eng.host_round_abi()
    with eng.lock:
        got = _host.small_host_round(dicts, list(dicts[0]), mode, coef, div, fn, err, ctx, 0, 4 << 20)
    assert got is not None and list(got) == list(dicts[0])
    exp = _expect(dicts, mode, coef, div)
    for k in exp:
        assert got[k].device.type == "cpu" and got[k].dtype == exp[k].dtype and got[k].shape == exp[k].shape, k
        assert bits_equal(got[k].reshape(-1), exp[k].reshape(-1)), f"{name} K={K} mode={mode} key {k}"
    # the drop-in entry takes the same path and returns the same bits
    via = sda.aggregate(dicts, mode, coef, div)
    for k in exp:
        assert bits_equal(via[k].reshape(-1), exp[k].reshape(-1)), k


@pytest.mark.gpu
def test_small_host_results_are_owned_across_rounds():
    """Every call returns fresh CPU tensors: round r's result survives rounds r+1 and r+2."""
    from fedml_amd.ml.aggregator.agg_operator import FedMLAggOperator
    g = torch.Generator().manual_seed(5)
    A = type("Args", (), {"federated_optimizer": "FedAvg"})()
    rounds = [_dicts(g, 2, LAYOUTS["lr_mnist"]) for _ in range(3)]
    outs = [FedMLAggOperator.agg(A, [(300, d[0]), (500, d[1])]) for d in rounds]
    for d, o in zip(rounds, outs):
        exp = _expect(d, MUL_W, [300 / 800, 500 / 800], 1.0)
        for k in exp:
            assert bits_equal(o[k].reshape(-1), exp[k].reshape(-1))


@pytest.mark.gpu
def test_one_workgroup_path_equals_event_path():
    """FA_HOST1=0 (the device kernel + event wait) and the one-workgroup path give the same bits."""
    code = ("import sys, torch; sys.path[:0] = [%r, %r, %r]\n"
            "from test_gpu_host_small import _dicts, LAYOUTS\n"
            "from fedml_amd.ml.aggregator import state_dict_agg as sda\n"
            "g = torch.Generator().manual_seed(11)\n"
            "d = _dicts(g, 3, LAYOUTS['bn'] + LAYOUTS['ragged'])\n"
            "o = sda.aggregate(d, 0, [0.2, 0.3, 0.5])\n"
            "torch.save({k: v for k, v in o.items()}, sys.argv[1])\n") % (ROOT, os.path.join(ROOT, "tests"),
                                                                         os.path.join(ROOT, "tests", "golden"))
    outs = []
    for flag in ("1", "0"):
        path = os.path.join(ROOT, "gpurun_out", f"host1_{flag}.pt")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        env = dict(os.environ, FA_HOST1=flag)
        subprocess.run([sys.executable, "-c", code, path], check=True, env=env, timeout=120)
        outs.append(torch.load(path, weights_only=True))
    for k in outs[0]:
        assert torch.equal(outs[0][k].view(-1).view(torch.uint8), outs[1][k].view(-1).view(torch.uint8)), k


def test_small_host_round_declines_without_calling():
    """Rounds the one-call path does not take return None before any native call (fn = 0 here)."""
    from fedml_amd import _host
    g = torch.Generator().manual_seed(1)
    base = _dicts(g, 2, LAYOUTS["lr_mnist"])
    keys = list(base[0])

    def run(dicts, mode=MUL_W, coef=(0.5, 0.5), max_bytes=4 << 20, ks=None):
        return _host.small_host_round(dicts, ks or keys, mode, list(coef) if coef else None, 1.0, 0, 0, 0, 0,
                                      max_bytes)

    assert run(base, max_bytes=1000) is None                                    # above the size limit
    nc = [OrderedDict(d) for d in base]
    nc[1]["linear.weight"] = torch.randn(784, 10).t()                          # non-contiguous
    assert run(nc) is None
    dt = [OrderedDict(d) for d in base]
    dt[1]["linear.bias"] = dt[1]["linear.bias"].double()                       # clients disagree on a dtype
    assert run(dt) is None
    sh = [OrderedDict(d) for d in base]
    sh[1]["linear.bias"] = torch.randn(11)                                     # shape mismatch
    assert run(sh) is None
    bl = [OrderedDict([("m", torch.ones(3, dtype=torch.bool))]) for _ in range(2)]  # not a C-ABI dtype
    assert run(bl, ks=["m"]) is None
    ro = [base[0], OrderedDict(reversed(list(base[1].items())))]               # other key order
    assert run(ro) is None
    assert run(base, coef=(1.0,)) is None                                      # one coefficient short
    assert run(base[:1] * 4097, coef=[1.0] * 4097) is None                      # K above the table limit
