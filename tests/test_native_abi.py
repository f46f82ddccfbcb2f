"""CPU-side checks of the C ABI boundary: the library loads, exports every declared symbol, and
fails with error codes (never aborts) when no device is usable."""
from __future__ import annotations

import ctypes
import os
import re

import pytest
import torch

from conftest import ROOT, gpu_available
from fedml_amd import _native as N

HDRS = [os.path.join(ROOT, "include", h) for h in ("fedagg.h", "fedagg_finite.h", "fedagg_robust.h")]


def declared_functions():
    fns = set()
    for h in HDRS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        fns |= set(re.findall(r"\b(fa_[a-z_]+)\s*\(", src))
    return sorted(fns)


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    assert set(fns) == set(N.EXPORTED_SYMBOLS), fns


def test_library_exports_every_declared_symbol():
    L = N.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert L.fa_abi_version() == N.ABI_VERSION


def test_library_is_a_gfx950_code_object():
    data = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_strerror_names():
    L = N.lib()
    for code, name in [(0, b"FA_OK"), (-1, b"FA_ERR_INVALID"), (-2, b"FA_ERR_DTYPE"), (-3, b"FA_ERR_HIP"),
                       (-4, b"FA_ERR_NOMEM"), (-99, b"FA_ERR_UNKNOWN")]:
        assert L.fa_strerror(code) == name


def test_invalid_arguments_return_codes_without_device():
    L = N.lib()
    # NULL context and bad arguments are rejected before any HIP call
    rc = L.fa_weighted_sum(None, N.F32, N.MUL_W, 10, 2, None, None, 1.0, None, None)
    assert rc == N.FA_ERR_INVALID
    assert b"ctx" in L.fa_last_error()
    rc = L.fa_ctx_create(0, None)
    assert rc == N.FA_ERR_INVALID
    rc = L.fa_mix(None, N.F32, 10, 1, None, None, None, 1, None, None, None, None, None)
    assert rc == N.FA_ERR_INVALID
    rc = L.fa_finite_sum(None, 1, None, 1, None, None, 7, 0, None, 0, 1.0, None, None)
    assert rc == N.FA_ERR_INVALID
    rc = L.fa_finite_quantize(None, N.F32, 1, None, None, None, 7, 8, None, None)
    assert rc == N.FA_ERR_INVALID
    rc = L.fa_lcc_decode(None, 1, 1, 1, None, None, 7, 1, None, None)
    assert rc == N.FA_ERR_INVALID
    rc = L.fa_weighted_sum_pair(None, N.F32, N.MUL_W, 10, 1, 2, None, None, 0, 0, None, 1.0, None, None, None)
    assert rc == N.FA_ERR_INVALID and b"ctx" in L.fa_last_error()


@pytest.mark.skipif(gpu_available(), reason="checks the no-device error path")
def test_ctx_create_without_gpu_fails_cleanly():
    L = N.lib()
    h = ctypes.c_void_p()
    rc = L.fa_ctx_create(0, ctypes.byref(h))
    assert rc in (N.FA_ERR_HIP, N.FA_ERR_INVALID)
    assert not h.value


@pytest.mark.skipif(gpu_available(), reason="checks the no-device error path")
def test_product_path_fails_loudly_without_gpu():
    from fedml_amd.engine import AggEngine
    with pytest.raises(N.FedAggNativeError):
        AggEngine()


def test_product_does_not_import_oracle():
    """The product package never imports or links the test oracle (no CPU fallback)."""
    pkg = os.path.join(ROOT, "fedml_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".cpp", ".h", "Makefile")):
                src = open(os.path.join(dp, f)).read()
                for bad in ("from oracle", "import oracle", "liborc", "torch_port"):
                    assert bad not in src, (f, bad)
