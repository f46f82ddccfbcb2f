"""The bench's own 8-rank chain on the CPU: ``python bench.py --gpus 8`` (no outer launcher) starts
torch.distributed.run, which starts 8 ranks over gloo; every rank runs the metric / hier / gossip
N > 1 code path (GroupReducer, DistributedGossip) with tests/rehearsal_engine.py's oracle local
reductions, and the line's parity covers the WHOLE global model on rank 0 (or every rank's shard,
every gossip node).  What the driver's 8-GPU scaling run executes, minus RCCL and the kernels
(reference: simulation/nccl/base_framework/common.py:196-228, sp/decentralized/client_dsgd.py:104-122).
tools/rehearsal_n8.py runs the full set and records profiles/r05/rehearsal_n8.jsonl."""
from __future__ import annotations

import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool():
    spec = importlib.util.spec_from_file_location("rehearsal_n8", os.path.join(ROOT, "tools", "rehearsal_n8.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("extra,exact", [
    (["--config", "metric", "--clients", "128", "--params", "40000"], True),
    (["--config", "metric", "--clients", "128", "--params", "40000", "--collective", "reduce_scatter"], False),
    (["--config", "hier", "--clients", "64", "--params", "8000", "--collective", "ordered_all"], True),
    (["--config", "gossip", "--clients", "256", "--params", "3000"], True),
], ids=["metric-ordered", "metric-reduce_scatter", "hier-ordered_all", "gossip"])
def test_bench_chain_world8_cpu(extra, exact):
    d = _tool().run(extra, gpus=8)
    assert d["n_gpus"] == 8 and "rehearsal" in d
    assert "gloo (CPU rehearsal" in d["config"]["parallelism"] or extra[1] == "gossip"
    if exact:
        assert d["parity"].startswith("bit-exact"), d["parity"]
    else:  # the backend's own summation order: 1e-6 normwise, every shard checked
        assert d["parity"].startswith(("bit-exact", "within 1e-6")), d["parity"]
    if extra[1] == "metric" and exact:
        assert "40000 sampled elements of the whole global model on rank 0" in d["parity"]
    if extra[1] == "gossip":
        assert "over all 256 nodes (8 ranks" in d["parity"]


def test_cpu_rehearsal_refuses_without_injected_engine():
    """The product engine is HIP-only: the CPU mode never falls back to a CPU reduction of its own."""
    import subprocess
    import sys
    env = dict(os.environ, FEDML_AMD_BENCH_REHEARSAL="cpu", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    env.pop("FEDML_AMD_BENCH_ENGINE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "metric", "--params", "1000",
                        "--clients", "4", "--steps", "1", "--warmup", "0"], env=env, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode != 0 and "FEDML_AMD_BENCH_ENGINE" in p.stderr
