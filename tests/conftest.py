import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_sessionstart(session):
    """Build the native pieces if a fresh checkout lacks them (they are git-ignored artefacts)."""
    import glob
    need = [os.path.join(ROOT, "fedml_amd", "libfedagg.so"), os.path.join(ROOT, "oracle", "_build", "liborc.so")]
    if any(not os.path.exists(p) for p in need) or not glob.glob(os.path.join(ROOT, "fedml_amd", "_host*.so")):
        import __graft_entry__
        __graft_entry__.build()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: multi-process or large CPU test")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
