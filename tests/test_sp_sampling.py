"""The SP round driver samples clients as the reference does (simulation/sp/fedavg/fedavg_api.py:
127-135), pinned by tests/golden/g20_sp_sampling.json (generated from the reference itself by
tests/golden/make_golden.py sp_sampling).  CPU only: the sampling is host logic."""
import json
import os

from conftest import ROOT


def test_client_sampling_matches_reference_fixture():
    from fedml_amd.simulation.sp.fedavg_api import FedAvgAPI
    with open(os.path.join(ROOT, "tests", "golden", "g20_sp_sampling.json")) as f:
        fx = json.load(f)
    api = FedAvgAPI(None, "cpu", None)
    for key, per_round in fx["cases"].items():
        total, per = (int(v) for v in key.split("_"))
        for r, exp in enumerate(per_round):
            got = [int(v) for v in api._client_sampling(r, total, per)]
            assert got == exp, (key, r)
