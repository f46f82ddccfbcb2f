"""Pin the robust-aggregation oracle (oracle/robust_oracle.c) and the host-side logic of the
robust mirrors to the reference's fixtures g16-g18 (CPU only)."""
from __future__ import annotations

import json
import os
import types
from collections import OrderedDict

import numpy as np
import pytest
import torch

from golden_io import GOLDEN_DIR, ROBUST_PREFIXES, client_dicts, expected_dicts, list_cases, load_case
from refcases import assert_dict_bits, bits_equal

from oracle import orc

CASES = list_cases()
ROB = {kind: [p for p in CASES if os.path.basename(p).startswith(kind)] for kind in ROBUST_PREFIXES}
ids = lambda p: os.path.basename(p)[:-4]  # noqa: E731
WEIGHT = lambda k: "running_mean" not in k and "running_var" not in k and "num_batches_tracked" not in k  # noqa: E731


def oracle_median_defense(meta, arrays):
    """The reference's defend_on_aggregation with the C oracle as the median (write-back walk incl.)."""
    cl = client_dicts(meta, arrays)
    keys = [k for k in meta["keys"] if WEIGHT(k)]
    dt = cl[0][keys[0]].dtype
    for k in keys[1:]:
        dt = torch.promote_types(dt, cl[0][k].dtype)
    vec = torch.cat([orc.coord_median([c[k].to(dt).reshape(-1) for c in cl]) for k in keys])
    out, index = OrderedDict(cl[0]), 0
    for k, params in cl[0].items():
        out[k] = vec[index: index + params.numel()].view(params.size())
        index += params.numel()
    return out


def test_inventory():
    assert len(ROB["g16_"]) >= 20 and len(ROB["g17_"]) >= 5 and len(ROB["g18_"]) >= 4
    assert sum(os.path.getsize(p) for p in CASES) < 5.5e6  # r06: + the Krum kappa-band fixtures


@pytest.mark.parametrize("path", ROB["g16_"], ids=ids)
def test_median_matches_golden(path):
    meta, arrays = load_case(path)
    if meta.get("error"):
        with pytest.raises(RuntimeError) as ei:
            oracle_median_defense(meta, arrays)
        assert str(ei.value) == meta["error"][1]
        return
    assert_dict_bits(oracle_median_defense(meta, arrays), expected_dicts(meta, arrays)[0], meta["name"])


@pytest.mark.parametrize("path", ROB["g17_"], ids=ids)
def test_trimmed_mean_selection_matches_golden(path):
    from fedml_amd.core.security.defense.coordinate_wise_trimmed_mean_defense import CoordinateWiseTrimmedMeanDefense
    meta, arrays = load_case(path)
    cl = client_dicts(meta, arrays)
    raw = list(zip(meta["n"], cl))
    sel = CoordinateWiseTrimmedMeanDefense(types.SimpleNamespace(beta=meta["beta"])).defend_before_aggregation(raw)
    assert [next(i for i, (_, c) in enumerate(raw) if c is sc) for _, sc in sel] == meta["selected"]


def test_trimmed_mean_beta_bound():
    from fedml_amd.core.security.defense.coordinate_wise_trimmed_mean_defense import CoordinateWiseTrimmedMeanDefense
    with pytest.raises(ValueError):
        CoordinateWiseTrimmedMeanDefense(types.SimpleNamespace(beta=0.6)).defend_before_aggregation([])


@pytest.mark.parametrize("path", ROB["g18_"], ids=ids)
def test_krum_selection_with_oracle_distances(path, monkeypatch):
    """The mirror's score bookkeeping over exact distances picks the reference's clients and
    reproduces its float32-norm scores to 1e-5."""
    from fedml_amd.core.security.defense.krum_defense import KrumDefense
    meta, arrays = load_case(path)
    cl = client_dicts(meta, arrays)
    keys = [k for k in meta["keys"] if WEIGHT(k)]
    vdt = KrumDefense.vector_dtype(cl)
    if vdt == torch.float64:  # float64 models: float64 differences and sums (numpy), as the reference
        X = np.stack([torch.cat([c[k].reshape(-1) for k in keys]).numpy() for c in cl])
        D = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    else:
        vecs = [torch.cat([c[k].float().reshape(-1) for k in keys]) for c in cl]
        D = (orc.pairwise_sqdist_rt(vecs, vdt) if vdt in (torch.bfloat16, torch.float16)
             else orc.pairwise_sqdist(vecs)).numpy()
    d = KrumDefense(types.SimpleNamespace(byzantine_client_num=meta["byzantine_client_num"],
                                          krum_param_m=meta["krum_param_m"]))
    monkeypatch.setattr(d, "pairwise_sq_distances", lambda grads: D)
    raw = list(zip(meta["n"], cl))
    sel = d.defend_before_aggregation(raw)
    assert [next(i for i, (_, c) in enumerate(raw) if c is sc) for _, sc in sel] == meta["selected"]
    np.testing.assert_allclose(d._compute_krum_score(cl), meta["scores"], rtol=1e-5)


@pytest.mark.parametrize("path", [p for p in ROB["g18_"] if "f16" in os.path.basename(p)], ids=ids)
def test_krum_half_oracle_distances_match_reference(path):
    """bf16 / f16 models: the oracle's squared distances (differences rounded to the model dtype,
    exact sums), with the norm rounded to that dtype and squared as the mirror does, equal every
    `compute_euclidean_distance(v_i, v_j).item() ** 2` the reference recorded (inf included)."""
    from fedml_amd.core.security.defense.krum_defense import KrumDefense
    meta, arrays = load_case(path)
    cl = client_dicts(meta, arrays)
    vdt = KrumDefense.vector_dtype(cl)
    assert str(vdt).replace("torch.", "") == meta["vector_dtype"]
    keys = [k for k in meta["keys"] if WEIGHT(k)]
    D = orc.pairwise_sqdist_rt([torch.cat([c[k].float().reshape(-1) for k in keys]) for c in cl], vdt)
    got = torch.sqrt(D).to(torch.float32).to(vdt).to(torch.float64).numpy() ** 2
    np.testing.assert_array_equal(got, np.array(meta["dists"]))


def test_krum_requirement_error_matches_reference():
    from fedml_amd.core.security.defense.krum_defense import KrumDefense
    err = json.load(open(os.path.join(GOLDEN_DIR, "g18_krum_errors.json")))["K9_f4_m1"]
    with pytest.raises(ValueError) as ei:
        KrumDefense(types.SimpleNamespace(byzantine_client_num=4, krum_param_m=1)).defend_before_aggregation(
            [(1, {})] * 9)
    assert str(ei.value) == err[1]


def test_pairwise_oracle_matches_numpy():
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(1000, generator=g) for _ in range(5)]
    D = orc.pairwise_sqdist(xs).numpy()
    X = torch.stack(xs).double().numpy()
    ref = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    np.testing.assert_allclose(D, ref, rtol=1e-12)


def test_krum_f64_fixtures_present_and_float64():
    """g18_krum_f64_*: float64 models, including near-ties a float32 measurement would order
    differently (make_golden.py cases_krum_f64 asserts that when it writes them)."""
    from fedml_amd.core.security.defense.krum_defense import KrumDefense
    paths = [p for p in ROB["g18_"] if "f64" in os.path.basename(p)]
    assert len(paths) >= 4 and any("near_tie" in p for p in paths)
    for p in paths:
        meta, arrays = load_case(p)
        assert KrumDefense.vector_dtype(client_dicts(meta, arrays)) == torch.float64
