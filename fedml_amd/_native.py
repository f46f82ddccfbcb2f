"""ctypes binding of libfedagg.so (the C ABI in include/fedagg.h).

The library is built in-tree (``make -C fedml_amd/csrc`` or ``__graft_entry__.build()``) and
loaded from ``fedml_amd/libfedagg.so``.  There is no fallback: if the library is missing or fails
to load, every entry point raises ``FedAggNativeError`` -- the product path never silently
computes on the CPU.

torch is imported first so that the HIP runtime torch ships (soname ``libamdhip64.so.7``) is the
one the library binds to; both then share devices, streams and the caching allocator's memory.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (load torch's HIP runtime before libfedagg.so)

HERE = os.path.dirname(os.path.abspath(__file__))
# FEDML_AMD_LIB: another build of the same ABI (interleaved A/B measurements of a kernel change only)
LIB_PATH = os.environ.get("FEDML_AMD_LIB") or os.path.join(HERE, "libfedagg.so")
ABI_VERSION = 3
TILE_BYTES = 4096  # FA_TILE_BYTES

F32, BF16, F16, F64, I64 = 0, 1, 2, 3, 4
MUL_W, MUL_N_DIV_N, SUM = 0, 1, 2

FA_OK, FA_ERR_INVALID, FA_ERR_DTYPE, FA_ERR_HIP, FA_ERR_NOMEM, FA_ERR_COMM = 0, -1, -2, -3, -4, -5

EXPORTED_SYMBOLS = (
    "fa_abi_version", "fa_ctx_create", "fa_ctx_destroy", "fa_weighted_sum",
    "fa_weighted_sum_multi", "fa_weighted_sum_tiled", "fa_weighted_sum_tiled_multi", "fa_weighted_sum_pair", "fa_weighted_sum_pair_multi", "fa_weighted_sum_grouped", "fa_weighted_sum_grouped_tiled",
    "fa_fedavg_sgd", "fa_fedavg_sgd_tiled", "fa_fedavg_rmsprop", "fa_mix", "fa_mix_tiled", "fa_ctx_set_variant",
    "fa_ctx_set_mix_band", "fa_stream_create_cu_masked", "fa_stream_destroy", "fa_strerror", "fa_last_error",
    "fa_promote_add", "fa_weighted_sum_host", "fa_pushsum", "fa_read_probe",
    "fa_device_alloc_contiguous", "fa_device_free",
    # include/fedagg_finite.h
    "fa_finite_sum", "fa_finite_sum_tiled", "fa_finite_quantize", "fa_lcc_decode", "fa_mt_randint_sum",
    "fa_mt_randint_sum_scratch_bytes",
    # include/fedagg_robust.h
    "fa_coord_median", "fa_coord_median_tiled", "fa_pairwise_sqdist", "fa_pairwise_sqdist_rt", "fa_pairwise_sqdist_scratch_bytes",
    "fa_pairwise_sqdist_gram", "fa_pairwise_sqdist_gram_scratch_bytes", "fa_pairwise_sqdist_gram_limit",
    # include/fedagg_comm.h
    "fa_comm_unique_id", "fa_comm_init", "fa_comm_wrap", "fa_comm_destroy", "fa_comm_size", "fa_local_out_dtype",
    "fa_group_plan", "fa_group_ops", "fa_group_reduce_scratch_bytes", "fa_group_reduce", "fa_comm_set_timing", "fa_comm_local_time",
    "fa_comm_last_op", "fa_group_plan_ex", "fa_group_ops_ex", "fa_comm_op_counts",
)

# enum fa_exchange / fa_local_kind (include/fedagg_comm.h)
XCHG_ORDERED, XCHG_ORDERED_ALL, XCHG_REDUCE, XCHG_ALL_REDUCE, XCHG_REDUCE_SCATTER = 0, 1, 2, 3, 4
XCHG_LOOPBACK = 0x100                    # OR'ed into an ordered exchange
XFLAG_DELIVER_ALL, XFLAG_LOOPBACK = 1, 2  # fa_group_plan_ex / fa_group_ops_ex flags
LOCAL_FLAT, LOCAL_TILED, LOCAL_GROUPED, LOCAL_GROUPED_TILED, LOCAL_PARTIAL = 0, 1, 2, 3, 4
COMM_ID_BYTES = 128


class LocalStep(ctypes.Structure):
    """struct fa_local_step (include/fedagg_comm.h)."""
    _fields_ = [("kind", ctypes.c_int32), ("dtype", ctypes.c_int32), ("mode", ctypes.c_int32), ("k", ctypes.c_int32),
                ("d_in", ctypes.POINTER(ctypes.c_void_p)), ("tile_stride", ctypes.c_int64),
                ("coef", ctypes.POINTER(ctypes.c_double)), ("divisor", ctypes.c_double),
                ("num_groups", ctypes.c_int32), ("group_mode", ctypes.c_int32),
                ("group_ptr", ctypes.POINTER(ctypes.c_int32)), ("group_coef", ctypes.POINTER(ctypes.c_double)),
                ("group_divisor", ctypes.POINTER(ctypes.c_double)), ("d_partial", ctypes.c_void_p)]

MOD_FIRST, MOD_EACH, MOD_END, REAL_F64 = 1, 2, 4, 8  # enum fa_finite_flags


class FedAggNativeError(RuntimeError):
    """The HIP library is unavailable or a native call failed."""


_lib = None
_lock = threading.Lock()

_vp = ctypes.c_void_p
_P_vp = ctypes.POINTER(ctypes.c_void_p)
_P_d = ctypes.POINTER(ctypes.c_double)
_P_i64 = ctypes.POINTER(ctypes.c_int64)
_P_i32 = ctypes.POINTER(ctypes.c_int32)


def _declare(L):
    L.fa_abi_version.restype = ctypes.c_int
    L.fa_abi_version.argtypes = []
    L.fa_ctx_create.restype = ctypes.c_int
    L.fa_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.fa_ctx_destroy.restype = ctypes.c_int
    L.fa_ctx_destroy.argtypes = [_vp]
    L.fa_ctx_set_variant.restype = ctypes.c_int
    L.fa_ctx_set_variant.argtypes = [_vp, ctypes.c_int]
    L.fa_ctx_set_mix_band.restype = ctypes.c_int
    L.fa_ctx_set_mix_band.argtypes = [_vp, ctypes.c_int]
    L.fa_stream_create_cu_masked.restype = ctypes.c_int
    L.fa_stream_create_cu_masked.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.fa_stream_destroy.restype = ctypes.c_int
    L.fa_stream_destroy.argtypes = [_vp]
    L.fa_weighted_sum.restype = ctypes.c_int
    L.fa_weighted_sum.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int32,
                                  _P_vp, _P_d, ctypes.c_double, _vp, _vp]
    L.fa_weighted_sum_multi.restype = ctypes.c_int
    L.fa_weighted_sum_multi.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int32, _P_i64,
                                        ctypes.c_int32, _P_vp, _P_d, ctypes.c_double, _P_vp, _vp]
    L.fa_weighted_sum_tiled.restype = ctypes.c_int
    L.fa_weighted_sum_tiled.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int32, _P_vp,
                                        ctypes.c_int64, _P_d, ctypes.c_double, _vp, _vp]
    L.fa_weighted_sum_tiled_multi.restype = ctypes.c_int
    L.fa_weighted_sum_tiled_multi.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int32, _P_i64, ctypes.c_int32,
                                              _P_vp, ctypes.c_int64, _P_d, ctypes.c_double, _P_vp, _vp]
    L.fa_weighted_sum_pair.restype = ctypes.c_int
    L.fa_weighted_sum_pair.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                       _P_vp, _P_vp, ctypes.c_int64, ctypes.c_int64, _P_d, ctypes.c_double, _vp, _vp,
                                       _vp]
    L.fa_weighted_sum_pair_multi.restype = ctypes.c_int
    L.fa_weighted_sum_pair_multi.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int32, _P_i64, ctypes.c_int32,
                                             _P_i64, ctypes.c_int32, _P_vp, _P_vp, _P_d, ctypes.c_double, _P_vp,
                                             _P_vp, _vp]
    L.fa_weighted_sum_grouped_tiled.restype = ctypes.c_int
    L.fa_weighted_sum_grouped_tiled.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int32,
                                                _P_vp, ctypes.c_int64, _P_d, ctypes.c_double, ctypes.c_int32,
                                                _P_i32, ctypes.c_int, _P_d, _P_d, _vp, _vp]
    L.fa_weighted_sum_grouped.restype = ctypes.c_int
    L.fa_weighted_sum_grouped.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int32,
                                          _P_vp, _P_d, ctypes.c_double, ctypes.c_int32, _P_i32, ctypes.c_int,
                                          _P_d, _P_d, _vp, _vp]
    L.fa_fedavg_sgd.restype = ctypes.c_int
    L.fa_fedavg_sgd.argtypes = [_vp, ctypes.c_int32, _P_i64, ctypes.c_int32, _P_vp, _P_d, _P_vp, _P_vp,
                                ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                ctypes.c_int, ctypes.c_int, _vp]
    L.fa_fedavg_rmsprop.restype = ctypes.c_int
    L.fa_fedavg_rmsprop.argtypes = [_vp, ctypes.c_int32, _P_i64, ctypes.c_int32, _P_vp, _P_d, _P_vp, _P_vp, _P_vp,
                                    ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_int, _vp]
    L.fa_fedavg_sgd_tiled.restype = ctypes.c_int
    L.fa_fedavg_sgd_tiled.argtypes = [_vp, ctypes.c_int64, ctypes.c_int32, _P_vp, ctypes.c_int64, _P_d, _vp, _vp,
                                      ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_int, ctypes.c_int, _vp]
    L.fa_mix.restype = ctypes.c_int
    L.fa_mix.argtypes = [_vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int32, _P_i32, _P_i32, _P_d,
                         ctypes.c_int32, _P_vp, _P_vp, _P_d, _P_vp, _vp]
    L.fa_mix_tiled.restype = ctypes.c_int
    L.fa_mix_tiled.argtypes = [_vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int32, _P_i32, _P_i32, _P_d,
                               ctypes.c_int32, _P_vp, ctypes.c_int64, _P_vp, ctypes.c_int64, _P_d, _P_vp, _vp]
    L.fa_finite_sum.restype = ctypes.c_int
    L.fa_finite_sum.argtypes = [_vp, ctypes.c_int32, _P_i64, ctypes.c_int32, _P_vp, _P_vp, ctypes.c_int64,
                                ctypes.c_int, _P_vp, ctypes.c_int32, ctypes.c_double, _P_vp, _vp]
    L.fa_finite_sum_tiled.restype = ctypes.c_int
    L.fa_finite_sum_tiled.argtypes = [_vp, ctypes.c_int64, ctypes.c_int32, _P_vp, ctypes.c_int64, _vp, ctypes.c_int64,
                                      ctypes.c_int, _vp, ctypes.c_int32, ctypes.c_double, _vp, _vp]
    L.fa_finite_quantize.restype = ctypes.c_int
    L.fa_finite_quantize.argtypes = [_vp, ctypes.c_int, ctypes.c_int32, _P_i64, _P_vp, _P_vp, ctypes.c_int64,
                                     ctypes.c_int32, _P_vp, _vp]
    L.fa_lcc_decode.restype = ctypes.c_int
    L.fa_lcc_decode.argtypes = [_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, _P_i64, _vp, ctypes.c_int64,
                                ctypes.c_int64, _vp, _vp]
    L.fa_mt_randint_sum.restype = ctypes.c_int
    L.fa_mt_randint_sum.argtypes = [_vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int8),
                                    ctypes.c_int64, ctypes.c_int64, _vp, _vp, ctypes.c_size_t, _vp]
    L.fa_mt_randint_sum_scratch_bytes.restype = ctypes.c_size_t
    L.fa_mt_randint_sum_scratch_bytes.argtypes = [ctypes.c_int64]
    L.fa_coord_median.restype = ctypes.c_int
    L.fa_coord_median.argtypes = [_vp, ctypes.c_int, ctypes.c_int32, _P_i64, ctypes.c_int32, _P_vp, _P_vp, _vp]
    L.fa_coord_median_tiled.restype = ctypes.c_int
    L.fa_coord_median_tiled.argtypes = [_vp, ctypes.c_int, ctypes.c_int32, _P_i64, ctypes.c_int32, _P_vp,
                                        ctypes.c_int64, _P_vp, _vp]
    L.fa_pairwise_sqdist.restype = ctypes.c_int
    L.fa_pairwise_sqdist.argtypes = [_vp, ctypes.c_int32, _P_i64, ctypes.c_int32, _P_vp, _vp, _vp, ctypes.c_size_t, _vp]
    L.fa_pairwise_sqdist_rt.restype = ctypes.c_int
    L.fa_pairwise_sqdist_rt.argtypes = [_vp, ctypes.c_int, ctypes.c_int32, _P_i64, ctypes.c_int32, _P_vp, _vp, _vp,
                                        ctypes.c_size_t, _vp]
    L.fa_pairwise_sqdist_scratch_bytes.restype = ctypes.c_size_t
    L.fa_pairwise_sqdist_scratch_bytes.argtypes = [ctypes.c_int32, _P_i64, ctypes.c_int32]
    L.fa_pairwise_sqdist_gram.restype = ctypes.c_int
    L.fa_pairwise_sqdist_gram.argtypes = [_vp, ctypes.c_int32, _P_i64, ctypes.c_int32, _P_vp, _vp, _vp,
                                          ctypes.c_double, _vp, ctypes.c_size_t, _vp]
    L.fa_pairwise_sqdist_gram_scratch_bytes.restype = ctypes.c_size_t
    L.fa_pairwise_sqdist_gram_scratch_bytes.argtypes = [ctypes.c_int32, _P_i64, ctypes.c_int32]
    L.fa_pairwise_sqdist_gram_limit.restype = ctypes.c_double
    L.fa_pairwise_sqdist_gram_limit.argtypes = [ctypes.c_int32, _P_i64, ctypes.c_int32, _P_vp, ctypes.c_double]
    L.fa_weighted_sum_host.restype = ctypes.c_int
    L.fa_weighted_sum_host.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int32, _P_i64, ctypes.c_int32,
                                       _P_vp, _P_d, ctypes.c_double, _P_vp, _vp]
    L.fa_pushsum.restype = ctypes.c_int
    L.fa_pushsum.argtypes = [_vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int32, _P_i32, _P_i32, _P_d, ctypes.c_int32,
                             _P_vp, _vp, _P_vp, _P_vp, _vp, _vp]
    L.fa_read_probe.restype = ctypes.c_int
    L.fa_read_probe.argtypes = [_vp, _vp, ctypes.c_int64, ctypes.c_int32, _vp, _vp]
    L.fa_device_alloc_contiguous.restype = ctypes.c_int
    L.fa_device_alloc_contiguous.argtypes = [_vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]
    L.fa_device_free.restype = ctypes.c_int
    L.fa_device_free.argtypes = [_vp, _vp]
    L.fa_promote_add.restype = ctypes.c_int
    L.fa_promote_add.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64, _vp, _vp, _vp, _vp]
    _P_ls = ctypes.POINTER(LocalStep)
    L.fa_comm_unique_id.restype = ctypes.c_int
    L.fa_comm_unique_id.argtypes = [_vp, ctypes.c_int64]
    L.fa_comm_init.restype = ctypes.c_int
    L.fa_comm_init.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, ctypes.POINTER(ctypes.c_void_p)]
    L.fa_comm_wrap.restype = ctypes.c_int
    L.fa_comm_wrap.argtypes = [ctypes.c_int, _vp, _vp, ctypes.POINTER(ctypes.c_void_p)]
    L.fa_comm_destroy.restype = ctypes.c_int
    L.fa_comm_destroy.argtypes = [_vp]
    L.fa_comm_size.restype = ctypes.c_int
    L.fa_comm_size.argtypes = [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.fa_local_out_dtype.restype = ctypes.c_int
    L.fa_local_out_dtype.argtypes = [ctypes.c_int, ctypes.c_int]
    L.fa_group_plan.restype = ctypes.c_int
    L.fa_group_plan.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                ctypes.c_int32, _P_i64, _P_i64, _P_i64, _P_i64]
    L.fa_group_ops.restype = ctypes.c_int
    L.fa_group_ops.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                               ctypes.c_int32, ctypes.c_int, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P_i32,
                               _P_i32, _P_i32, _P_i64, _P_i64]
    L.fa_group_plan_ex.restype = ctypes.c_int
    L.fa_group_plan_ex.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_int32, ctypes.c_int32, _P_i64, _P_i64, _P_i64, _P_i64]
    L.fa_group_ops_ex.restype = ctypes.c_int
    L.fa_group_ops_ex.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                  ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                  _P_i32, _P_i32, _P_i32, _P_i64, _P_i64]
    L.fa_comm_op_counts.restype = ctypes.c_int
    L.fa_comm_op_counts.argtypes = [_vp, _P_i64]
    L.fa_group_reduce_scratch_bytes.restype = ctypes.c_int
    L.fa_group_reduce_scratch_bytes.argtypes = [_vp, ctypes.c_int, _P_ls, ctypes.c_int64, ctypes.c_int32,
                                                ctypes.c_int32, ctypes.c_int32, _P_i64]
    L.fa_group_reduce.restype = ctypes.c_int
    L.fa_group_reduce.argtypes = [_vp, _vp, ctypes.c_int, _P_ls, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                  ctypes.c_int32, _vp, _vp, ctypes.c_int64, _vp]
    L.fa_comm_set_timing.restype = ctypes.c_int
    L.fa_comm_set_timing.argtypes = [_vp, ctypes.c_int]
    L.fa_comm_local_time.restype = ctypes.c_int
    L.fa_comm_local_time.argtypes = [_vp, ctypes.c_int, _P_d, _P_i64]
    L.fa_comm_last_op.restype = ctypes.c_int
    L.fa_comm_last_op.argtypes = [_vp, ctypes.c_char_p, ctypes.c_int64]
    L.fa_strerror.restype = ctypes.c_char_p
    L.fa_strerror.argtypes = [ctypes.c_int]
    L.fa_last_error.restype = ctypes.c_char_p
    L.fa_last_error.argtypes = []


def lib():
    """Load (once) and return the native library, or raise FedAggNativeError."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise FedAggNativeError(
                f"{LIB_PATH} not found: build it with `make -C fedml_amd/csrc` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise FedAggNativeError(f"cannot load {LIB_PATH}: {e}") from e
        missing = [s for s in EXPORTED_SYMBOLS if not hasattr(L, s)]
        if missing:
            raise FedAggNativeError(f"{LIB_PATH} lacks symbols {missing}")
        _declare(L)
        if L.fa_abi_version() != ABI_VERSION:
            raise FedAggNativeError(f"ABI version {L.fa_abi_version()} != {ABI_VERSION}")
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != FA_OK:
        L = lib()
        raise FedAggNativeError(
            f"{what} failed: {L.fa_strerror(rc).decode()} ({L.fa_last_error().decode()})")


def ptr_array(ptrs):
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


def f64_array(vals):
    return (ctypes.c_double * len(vals))(*[float(v) for v in vals])


def i64_array(vals):
    return (ctypes.c_int64 * len(vals))(*[int(v) for v in vals])


def i32_array(vals):
    return (ctypes.c_int32 * len(vals))(*[int(v) for v in vals])
