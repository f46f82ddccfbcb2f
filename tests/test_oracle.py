"""Pin the oracle: both CPU restatements reproduce every golden fixture bit-for-bit (CPU only)."""
from __future__ import annotations

import os
import re
from collections import OrderedDict

import numpy as np
import pytest
import torch

from golden_io import aggregation_cases, client_dicts, expected_dicts, list_cases, load_case
from refcases import assert_dict_bits, check_case, dsgd_csr

from oracle import orc, torch_port

CASES = list_cases()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fixture_inventory():
    names = {os.path.basename(p)[:-4] for p in CASES}
    # every survey fixture family G1..G9 is present
    for g in ("g1_", "g2_", "g3_", "g4_", "g5_", "g6_", "g7_", "g8_", "g9_"):
        assert any(n.startswith(g) for n in names), g
    assert "topologies" in names
    assert sum(os.path.getsize(p) for p in CASES) < 5.5e6  # r06: + the Krum kappa-band fixtures (g18_krum_band_*)


class _Orc:
    weighted_sum = staticmethod(orc.weighted_sum)
    mix = staticmethod(orc.mix)


GENERIC = aggregation_cases()
FEDOPT = [p for p in CASES if "fedopt_sgd" in p]  # the C oracle restates SGD (RMSprop: GPU test, 1e-6)


@pytest.mark.parametrize("path", GENERIC, ids=lambda p: os.path.basename(p)[:-4])
def test_c_oracle_matches_golden(path):
    meta, arrays = load_case(path)
    check_case(_Orc, meta, arrays, "c-oracle:")


def _port_replay(meta, arrays):
    kind = meta["kind"]
    cl = client_dicts(meta, arrays)
    n = meta.get("n")
    if kind == "agg":
        opt = meta["optimizer"]
        if opt in ("SCAFFOLD", "Mime"):
            cs = []
            for i in range(meta["num_clients"]):
                cs.append(OrderedDict((k, torch.from_numpy(arrays[f"c{i}__{k}"].copy())) for k in meta["keys"]))
            out = torch_port.agg(opt, [(n[i], cl[i], cs[i]) for i in range(len(cl))],
                                 client_num_in_total=meta.get("client_num_in_total"),
                                 client_num_per_round=meta.get("client_num_per_round"))
            return list(out)
        return [torch_port.agg(opt, list(zip(n, cl)))]
    if kind == "sp_aggregate":
        return [torch_port.sp_aggregate(list(zip(n, cl)))]
    if kind == "mpi_fedavg":
        return [torch_port.mpi_fedavg(list(zip(n, cl)))]
    if kind == "fedavg_seq":
        w = torch_port.fedavg_seq_weights(n)
        partials = []
        for wk in meta["schedule"]:
            acc = {}
            for i in wk:
                torch_port.fedavg_seq_worker(acc, cl[i], w[i])
            partials.append(acc)
        return [torch_port.fedavg_seq_server(partials)]
    if kind == "hier_sp":
        groups = [(sum(n[i] for i in g), torch_port.sp_aggregate([(n[i], cl[i]) for i in g]))
                  for g in meta["groups"]]
        return [torch_port.sp_aggregate(groups)]
    E, R = meta.get("edges"), meta.get("group_comm_round")
    if kind == "hier_cloud":
        snd = {e: meta["edge_counts"][e] for e in range(E)}
        md = {e: [(r, cl[e * R + r]) for r in range(R)] for e in range(E)}
        return [torch_port.cloud_aggregate(snd, md, E)]
    if kind == "hier_mix":
        snd = {e: meta["edge_counts"][e] for e in range(E)}
        md = {e: [(r, cl[e * R + r]) for r in range(R)] for e in range(E)}
        return torch_port.cloud_mix(snd, md, E, arrays["W"])
    if kind == "mix_rows":
        W = arrays["W"]
        return [torch_port.pfedavg_mixing([(1, c) for c in cl], W[i]) for i in range(W.shape[0])]
    if kind in ("dsgd", "pushsum"):
        W = arrays["W"]
        outs = []
        for i in range(W.shape[0]):
            neigh = [([cl[j][k] for k in meta["keys"]], W[j][i]) for j in range(W.shape[0])
                     if j != i and W[j][i] != 0]
            if kind == "dsgd":
                x = torch_port.dsgd_update([cl[i][k] for k in meta["keys"]], W[i][i], neigh)
            else:
                omg = [meta["omegas_in"][j] * W[j][i] for j in range(W.shape[0]) if j != i and W[j][i] != 0]
                _, x, om = torch_port.pushsum_update([cl[i][k] for k in meta["keys"]], W[i][i], neigh,
                                                     meta["omegas_in"][i], omg)
                assert om == meta["omegas_out"][i]
            outs.append(OrderedDict(zip(meta["keys"], x)))
        return outs
    raise ValueError(kind)


@pytest.mark.parametrize("path", GENERIC, ids=lambda p: os.path.basename(p)[:-4])
def test_torch_port_matches_golden(path):
    meta, arrays = load_case(path)
    got = _port_replay(meta, arrays)
    exp = expected_dicts(meta, arrays)
    assert len(got) == len(exp)
    for j, (g, e) in enumerate(zip(got, exp)):
        assert_dict_bits(g, e, f"torch-port:{meta['name']}[{j}]")


def test_port_inputs_untouched():
    meta, arrays = load_case(os.path.join(ROOT, "tests", "golden", "g5_fedavg_seq_sum_K6.npz"))
    cl = client_dicts(meta, arrays)
    before = [OrderedDict((k, v.clone()) for k, v in c.items()) for c in cl]
    torch_port.agg("FedAvg_seq", list(zip(meta["n"], cl)))
    for a, b in zip(cl, before):
        assert_dict_bits(a, b, "inputs")


def test_codes_match_public_header():
    hdr = open(os.path.join(ROOT, "include", "fedagg.h")).read()
    want = {"FA_DTYPE_F32": orc.F32, "FA_DTYPE_BF16": orc.BF16, "FA_DTYPE_F16": orc.F16,
            "FA_DTYPE_F64": orc.F64, "FA_DTYPE_I64": orc.I64, "FA_MODE_MUL_W": orc.MUL_W,
            "FA_MODE_MUL_N_DIV_N": orc.MUL_N_DIV_N, "FA_MODE_SUM": orc.SUM}
    for name, v in want.items():
        m = re.search(rf"\b{name}\s*=\s*(\d+)", hdr)
        assert m and int(m.group(1)) == v, name


@pytest.mark.parametrize("seed", [0, 1])
def test_rounding_helpers_match_torch(seed):
    """bf16/fp16 RNE conversions of the C oracle vs torch's, on random + special bit patterns."""
    L = orc.lib()
    g = np.random.default_rng(seed)
    bits = g.integers(0, 2 ** 32, size=20000, dtype=np.uint64).astype(np.uint32)
    specials = np.array([0, 0x80000000, 0x7F800000, 0xFF800000, 0x00000001, 0x477FE000, 0x477FF000,
                         0x477FEFFF, 0x33000000, 0x33000001, 0x387FC000, 0x38800000, 0x7F7FFFFF],
                        dtype=np.uint32)
    bits = np.concatenate([bits, specials])
    f = torch.from_numpy(bits.view(np.float32).copy())
    ok_bf = torch.from_numpy(np.array([L.orc_f32_to_bf16(float(v)) for v in f.tolist()], dtype=np.uint16))
    ok_h = torch.from_numpy(np.array([L.orc_f32_to_f16(float(v)) for v in f.tolist()], dtype=np.uint16))
    tb = f.to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    th = f.to(torch.float16).view(torch.int16).numpy().view(np.uint16)
    nan = torch.isnan(f).numpy()
    assert np.array_equal(ok_bf.numpy()[~nan], tb[~nan])
    assert np.array_equal(ok_h.numpy()[~nan], th[~nan])


def test_topologies_fixture_shapes():
    from golden_io import GOLDEN_DIR
    with np.load(os.path.join(GOLDEN_DIR, "topologies.npz"), allow_pickle=False) as z:
        W = z["W_ring_256"]
        assert W.shape == (256, 256) and W.dtype == np.float32
        assert np.all(W.sum(1) > 0.99)
        assert W[0, 0] == np.float32(1 / 3) and W[0, 255] == np.float32(1 / 3)


@pytest.mark.parametrize("path", FEDOPT, ids=lambda p: os.path.basename(p)[:-4])
def test_c_oracle_fedopt_matches_golden(path):
    """FedAvg + torch.optim.SGD server step (FedOptAggregator.py:104-131), three rounds."""
    from refcases import fedopt_expected, fedopt_replay
    meta, arrays = load_case(path)
    got = fedopt_replay(meta, arrays, orc.weighted_sum, orc.sgd_apply)
    for r, (g, e) in enumerate(zip(got, fedopt_expected(meta, arrays))):
        assert_dict_bits(g, e, f"fedopt round {r}")
