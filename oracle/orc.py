"""ctypes wrapper over the C oracle (``fedagg_oracle.c``) -- TEST INFRASTRUCTURE ONLY.

Operates on CPU torch tensors.  Codes follow include/fedagg.h (F32=0, BF16=1, F16=2, F64=3,
I64=4; MUL_W=0, MUL_N_DIV_N=1, SUM=2).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liborc.so")

F32, BF16, F16, F64, I64 = 0, 1, 2, 3, 4
MUL_W, MUL_N_DIV_N, SUM = 0, 1, 2

_DT = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: F16, torch.float64: F64,
       torch.int64: I64}

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_weighted_sum.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_double),
                                       ctypes.c_double, ctypes.c_void_p]
        L.orc_weighted_sum.restype = ctypes.c_int
        L.orc_mix.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int32,
                              ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                              ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_void_p),
                              ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_double),
                              ctypes.POINTER(ctypes.c_void_p)]
        L.orc_mix.restype = ctypes.c_int
        L.orc_sgd_apply.argtypes = [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_int, ctypes.c_int]
        L.orc_sgd_apply.restype = ctypes.c_int
        L.orc_finite_sum.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p,
                                     ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_double,
                                     ctypes.c_void_p]
        L.orc_finite_sum.restype = ctypes.c_int
        L.orc_finite_quantize.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]
        L.orc_finite_quantize.restype = ctypes.c_int
        L.orc_lcc_decode.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
        L.orc_lcc_decode.restype = ctypes.c_int
        L.orc_f32_to_bf16.argtypes = [ctypes.c_float]
        L.orc_f32_to_bf16.restype = ctypes.c_uint16
        L.orc_f32_to_f16.argtypes = [ctypes.c_float]
        L.orc_f32_to_f16.restype = ctypes.c_uint16
        _lib = L
    return _lib


def out_dtype(dtype: torch.dtype, mode: int) -> torch.dtype:
    if dtype == torch.int64 and mode != SUM:
        return torch.float32
    return dtype


def weighted_sum(xs, mode: int, coef=None, divisor: float = 1.0) -> torch.Tensor:
    """Ordered reduction over the list of same-shape CPU tensors ``xs``."""
    xs = [x.contiguous() for x in xs]
    dt = xs[0].dtype
    assert all(x.dtype == dt and x.shape == xs[0].shape for x in xs)
    k = len(xs)
    out = torch.empty(xs[0].shape, dtype=out_dtype(dt, mode))
    ptrs = (ctypes.c_void_p * k)(*[x.data_ptr() for x in xs])
    c = (ctypes.c_double * k)(*([float(v) for v in coef] if coef is not None else [0.0] * k))
    rc = lib().orc_weighted_sum(_DT[dt], mode, xs[0].numel(), k, ptrs, c, float(divisor), out.data_ptr())
    if rc != 0:
        raise RuntimeError(f"orc_weighted_sum failed: {rc}")
    return out


def promote_add(acc, t):
    """acc += t across dtypes with PyTorch's in-place semantics (see orc_promote_add); new tensor."""
    L = lib()
    if not getattr(L, "_promote_declared", False):
        L.orc_promote_add.restype = ctypes.c_int
        L.orc_promote_add.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]
        L._promote_declared = True
    acc, t = acc.contiguous(), t.contiguous()
    out = torch.empty_like(acc)
    rc = L.orc_promote_add(_DT[acc.dtype], _DT[t.dtype], acc.numel(), acc.data_ptr(), t.data_ptr(), out.data_ptr())
    if rc != 0:
        raise RuntimeError(f"orc_promote_add failed: {rc}")
    return out


def mix(xs, row_ptr, cols, vals, post_scale=None):
    """CSR-ordered mixing rows (see orc_mix); returns (outs, outs2 or None)."""
    xs = [x.contiguous() for x in xs]
    rows = len(row_ptr) - 1
    outs = [torch.empty_like(xs[0]) for _ in range(rows)]
    outs2 = [torch.empty_like(xs[0]) for _ in range(rows)] if post_scale is not None else None
    P = ctypes.c_void_p
    rc = lib().orc_mix(
        _DT[xs[0].dtype], xs[0].numel(), rows,
        (ctypes.c_int32 * len(row_ptr))(*row_ptr), (ctypes.c_int32 * len(cols))(*cols),
        (ctypes.c_double * len(vals))(*[float(v) for v in vals]),
        (P * len(xs))(*[x.data_ptr() for x in xs]), (P * rows)(*[o.data_ptr() for o in outs]),
        (ctypes.c_double * rows)(*post_scale) if post_scale is not None else None,
        (P * rows)(*[o.data_ptr() for o in outs2]) if outs2 is not None else None)
    if rc != 0:
        raise RuntimeError(f"orc_mix failed: {rc}")
    return outs, outs2


def sgd_apply(avg, param, buf, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
              first_step=True):
    """In-place FedOpt SGD step on fp32 CPU tensors (see orc_sgd_apply)."""
    for t in (avg, param) + ((buf,) if buf is not None else ()):
        assert t.dtype == torch.float32 and t.is_contiguous()
    rc = lib().orc_sgd_apply(param.numel(), avg.data_ptr(), param.data_ptr(),
                             buf.data_ptr() if buf is not None else None, float(lr), float(momentum),
                             float(dampening), float(weight_decay), int(nesterov), int(first_step))
    if rc != 0:
        raise RuntimeError(f"orc_sgd_apply failed: {rc}")


MOD_FIRST, MOD_EACH, MOD_END, REAL_F64 = 1, 2, 4, 8


def finite_sum(xs, p, flags, mask=None, q_bits=None, scale=1.0):
    """Finite-field client sum (see orc_finite_sum).  Returns (finite int64, real or None); the real
    output (float32 dequantized * fp32(scale), or float64 with REAL_F64) only when q_bits is given."""
    xs = [x.contiguous() for x in xs]
    assert all(x.dtype == torch.int64 and x.numel() == xs[0].numel() for x in xs)
    n = xs[0].numel()
    fin = torch.empty(n, dtype=torch.int64)
    real = torch.empty(n, dtype=torch.float64 if flags & REAL_F64 else torch.float32) if q_bits is not None else None
    m = mask.contiguous() if mask is not None else None
    rc = lib().orc_finite_sum(n, len(xs), (ctypes.c_void_p * len(xs))(*[x.data_ptr() for x in xs]),
                              m.data_ptr() if m is not None else None, int(p), int(flags), fin.data_ptr(),
                              int(q_bits or 0), float(scale), real.data_ptr() if real is not None else None)
    if rc != 0:
        raise RuntimeError(f"orc_finite_sum failed: {rc}")
    return fin, real


def finite_quantize(x, p, q_bits, mask=None):
    """my_q (+ model_masking when mask is given) of a float32 / float64 / int64 CPU tensor."""
    x = x.contiguous()
    out = torch.empty(x.numel(), dtype=torch.int64)
    m = mask.contiguous() if mask is not None else None
    rc = lib().orc_finite_quantize(_DT[x.dtype], x.numel(), x.data_ptr(), m.data_ptr() if m is not None else None,
                                   int(p), int(q_bits), out.data_ptr())
    if rc != 0:
        raise RuntimeError(f"orc_finite_quantize failed: {rc}")
    return out


def lcc_decode(coef, f, p, n_out):
    """np.mod(coef.dot(f), p).reshape(-1)[:n_out] with int64 wrap (coef rows x k, f k x m)."""
    coef = coef.contiguous()
    f = f.contiguous()
    rows, k = coef.shape
    out = torch.empty(n_out, dtype=torch.int64)
    rc = lib().orc_lcc_decode(rows, k, f.shape[1], coef.data_ptr(), f.data_ptr(), int(p), int(n_out), out.data_ptr())
    if rc != 0:
        raise RuntimeError(f"orc_lcc_decode failed: {rc}")
    return out


def coord_median(xs):
    """torch.median over the client axis (see orc_coord_median) of same-shape CPU tensors."""
    xs = [x.contiguous() for x in xs]
    L = lib()
    if not hasattr(L, "_median_declared"):
        L.orc_coord_median.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
        L.orc_coord_median.restype = ctypes.c_int
        L.orc_pairwise_sqdist.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p),
                                          ctypes.c_void_p]
        L.orc_pairwise_sqdist.restype = ctypes.c_int
        L.orc_pairwise_sqdist_rt.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p),
                                             ctypes.c_int, ctypes.c_void_p]
        L.orc_pairwise_sqdist_rt.restype = ctypes.c_int
        L._median_declared = True
    out = torch.empty_like(xs[0])
    rc = L.orc_coord_median(_DT[xs[0].dtype], xs[0].numel(), len(xs),
                            (ctypes.c_void_p * len(xs))(*[x.data_ptr() for x in xs]), out.data_ptr())
    if rc != 0:
        raise RuntimeError(f"orc_coord_median failed: {rc}")
    return out


def pairwise_sqdist(xs):
    """K x K float64 matrix of exact squared Euclidean distances of float32 CPU vectors."""
    coord_median([torch.zeros(1)])  # declares the robust entry points
    xs = [x.contiguous().reshape(-1) for x in xs]
    k = len(xs)
    d = torch.empty((k, k), dtype=torch.float64)
    rc = lib().orc_pairwise_sqdist(xs[0].numel(), k, (ctypes.c_void_p * k)(*[x.data_ptr() for x in xs]), d.data_ptr())
    if rc != 0:
        raise RuntimeError(f"orc_pairwise_sqdist failed: {rc}")
    return d


def pairwise_sqdist_rt(xs, dtype):
    """Squared distances of a bfloat16 / float16 model's vectors as the reference forms them
    (differences rounded to ``dtype``, see orc_pairwise_sqdist_rt); xs: CPU vectors of any float
    dtype holding values of ``dtype``."""
    rt = {torch.bfloat16: 1, torch.float16: 2, torch.float32: 0}[dtype]
    coord_median([torch.zeros(1)])
    xs = [x.to(torch.float32).contiguous().reshape(-1) for x in xs]
    k = len(xs)
    d = torch.empty((k, k), dtype=torch.float64)
    rc = lib().orc_pairwise_sqdist_rt(xs[0].numel(), k, (ctypes.c_void_p * k)(*[x.data_ptr() for x in xs]), rt,
                                      d.data_ptr())
    if rc != 0:
        raise RuntimeError(f"orc_pairwise_sqdist_rt failed: {rc}")
    return d
