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

HDRS = [os.path.join(ROOT, "include", h) for h in ("fedagg.h", "fedagg_finite.h", "fedagg_robust.h", "fedagg_comm.h")]


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
                       (-4, b"FA_ERR_NOMEM"), (-5, b"FA_ERR_COMM"), (-99, b"FA_ERR_UNKNOWN")]:
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


def test_library_links_rccl():
    """The multi-GPU entry (include/fedagg_comm.h) calls RCCL directly: librccl is a dependency of the
    library (resolved to the RCCL torch already loaded, same soname)."""
    import subprocess
    out = subprocess.run(["readelf", "-d", N.LIB_PATH], capture_output=True, text=True).stdout
    assert "librccl.so" in out


def test_comm_entries_reject_invalid_arguments_without_device():
    L = N.lib()
    assert L.fa_comm_unique_id(None, 128) == N.FA_ERR_INVALID
    assert L.fa_comm_init(0, 2, 0, None, None) == N.FA_ERR_INVALID
    h = ctypes.c_void_p()
    assert L.fa_comm_init(0, 2, 5, (ctypes.c_uint8 * 128)(), ctypes.byref(h)) == N.FA_ERR_INVALID  # rank >= world
    assert L.fa_comm_wrap(0, None, None, ctypes.byref(h)) == N.FA_ERR_INVALID
    assert L.fa_comm_size(None, None, None) == N.FA_ERR_INVALID
    assert L.fa_comm_destroy(None) == N.FA_OK
    st = N.LocalStep(kind=N.LOCAL_FLAT, dtype=N.F32, mode=N.MUL_W, k=0)
    assert L.fa_group_reduce(None, None, 0, ctypes.byref(st), 10, 2, 1, 0, None, None, 0, None) == N.FA_ERR_INVALID
    need = ctypes.c_int64()
    assert L.fa_group_reduce_scratch_bytes(None, 0, ctypes.byref(st), 10, 2, 1, 0, ctypes.byref(need)) == \
        N.FA_ERR_INVALID
    assert L.fa_comm_set_timing(None, 1) == N.FA_ERR_INVALID
    assert L.fa_comm_local_time(None, 1, None, None) == N.FA_ERR_INVALID
    assert L.fa_local_out_dtype(N.I64, N.MUL_W) == N.F32 and L.fa_local_out_dtype(N.I64, N.SUM) == N.I64
    assert L.fa_local_out_dtype(N.BF16, N.MUL_W) == N.BF16
    assert L.fa_group_plan(-1, 1, 1, 2, 0, 4, None, None, None, None) == N.FA_ERR_INVALID


def test_local_step_struct_layout():
    """ctypes' fa_local_step matches the C struct's field offsets (x86-64 SysV)."""
    f = {name: getattr(N.LocalStep, name).offset for name, _ in N.LocalStep._fields_}
    assert (f["d_in"], f["tile_stride"], f["coef"], f["divisor"], f["num_groups"], f["group_ptr"],
            f["group_divisor"], f["d_partial"]) == (16, 24, 32, 40, 48, 56, 72, 80)
    assert ctypes.sizeof(N.LocalStep) == 88


@pytest.mark.parametrize("n,chunks,align,world,root", [
    (125_000_000, 8, 1024, 8, 0), (125_000_000, 8, 1024, 2, 0), (1000, 3, 1, 4, 2), (7, 8, 1, 3, 0),
    (0, 4, 256, 4, 0), (4099, 5, 256, 5, 4), (1 << 20, 1, 1024, 1, 0), (10, 64, 4, 8, 7)])
def test_native_plan_matches_the_python_exchange(n, chunks, align, world, root):
    """fa_group_plan (the C pipeline's chunks and owner pieces) is the plan of group_reduce.py's
    torch.distributed form (the one the gloo tests run), so both deliver the same pieces."""
    from fedml_amd.distributed.group_reduce import chunk_bounds, split_bounds
    from fedml_amd.distributed.native_exchange import group_plan
    plan = group_plan(n, chunks, align, world, root)
    exp = chunk_bounds(n, chunks, align)
    assert [(lo, hi) for lo, hi, _ in plan] == exp
    owners = [r for r in range(world) if r != root]
    for (a, b, pieces) in plan:
        assert pieces[root] == (a, 0) or world == 1
        if world == 1:
            continue
        for o, (lo, hi) in zip(owners, split_bounds(b - a, len(owners), align)):
            assert pieces[o] == (a + lo, hi - lo)


def test_match_rows_checks_dtype_and_shape():
    """The arena fast path's C++ check (fedml_amd._host.match_rows) accepts only the layout's own
    views: a same-address re-view with another dtype or shape is rejected."""
    from fedml_amd import _host
    buf = torch.zeros(2, 16)
    base = torch.tensor([buf.data_ptr(), buf.data_ptr() + 12 * 4], dtype=torch.int64)
    stride = torch.tensor([16 * 4, 16 * 4], dtype=torch.int64)
    meta = torch.tensor([6, 2, 3, 4, 6, 1, 4], dtype=torch.int64)  # float32 (3, 4); float32 (4,)
    moff = torch.tensor([0, 4], dtype=torch.int64)
    ok = {"w": buf[1, :12].view(3, 4), "b": buf[1, 12:16]}
    assert _host.match_rows([ok], ["w", "b"], base, stride, [1], meta, moff)
    assert not _host.match_rows([{"w": buf[1, :12].view(4, 3), "b": buf[1, 12:16]}], ["w", "b"], base, stride, [1],
                                meta, moff)
    assert not _host.match_rows([{"w": buf[1, :12].view(3, 4).view(torch.int32), "b": buf[1, 12:16]}], ["w", "b"],
                                base, stride, [1], meta, moff)
    assert not _host.match_rows([ok], ["w", "b"], base, stride, [0], meta, moff)


def test_storage_held_counts_derived_views():
    """ingest._storage_held: a buffer is held while ANY tensor on its storage lives outside it --
    the handed-out view, or one derived from it after the original is gone."""
    import torch
    from fedml_amd.ml.aggregator.ingest import _storage_held
    buf = torch.zeros(100)
    assert not _storage_held([buf])
    v = buf[10:20].view(2, 5)
    assert _storage_held([buf])
    d = v.reshape(-1)[3:].T if v.dim() == 1 else v.reshape(-1)[3:]
    del v
    assert _storage_held([buf])  # only the derived view remains
    del d
    assert not _storage_held([buf])
