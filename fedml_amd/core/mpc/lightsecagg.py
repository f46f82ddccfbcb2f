"""Finite-field secure-aggregation primitives on the HIP engine (drop-in for the reference's
python/fedml/core/mpc/lightsecagg.py; secagg.py shares the same functions).

Same names, arguments and results as the reference, element-for-element (tests/golden/g11-g15):

* ``aggregate_models_in_finite``  (lightsecagg.py:134-145)  -> fa_finite_sum, FA_FINITE_MOD_EACH
* ``my_q`` / ``transform_tensor_to_finite`` (:150-154, :187-192) -> fa_finite_quantize
* ``my_q_inv`` / ``transform_finite_to_tensor`` (:157-185)  -> fa_finite_sum (k = 1) dequantize
* ``model_masking``  (:83-95)                                -> fa_finite_sum (k = 2), MOD_EACH
* ``LCC_decoding_with_points`` (:50-55)                      -> fa_lcc_decode (+ host coefficients)
* ``gen_Lagrange_coeffs`` / ``modular_inv`` / ``divmod`` / ``PI`` (:8-80): the U x U Lagrange
  coefficients, computed on the host (they are O(U^2) scalars) with the reference's int64
  wrap-around reproduced exactly, so that the overflowing large-prime cases match too.

Placement: device tensors in -> device tensors out.  numpy arrays / CPU tensors (what the
reference's transports deliver) are staged to the engine's device and the results come back in
the reference's types: numpy int64 arrays for the finite-field functions, CPU float32 tensors
from ``transform_finite_to_tensor``.  Every element of arithmetic runs in the HIP kernels
(fedml_amd/csrc/finite.hip); there is no CPU fallback.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ... import _native as N
from ...engine import AggEngine, get_engine

MOD_FIRST, MOD_EACH, MOD_END, REAL_F64 = N.MOD_FIRST, N.MOD_EACH, N.MOD_END, N.REAL_F64
_I64 = 1 << 64
_Q_MAX = 62


# ------------------------------------------------------------------------------ host scalars
def _w64(v: int) -> int:
    """Two's-complement wrap of a Python int to int64 (numpy int64 arithmetic)."""
    v &= _I64 - 1
    return v - _I64 if v >= 1 << 63 else v


def _npmod(a: int, p: int) -> int:
    """np.mod on int64 scalars (floor remainder; p > 0)."""
    return a % p


def _npfloordiv(a: int, b: int) -> int:
    return a // b


def modular_inv(a, p):
    """Extended-Euclid inverse as the reference computes it (lightsecagg.py:8-22), int64 wrap."""
    a, p = int(a), int(p)
    x, y, m = 1, 0, p
    while a > 1:
        q = _npfloordiv(a, m)
        t = m
        m = _npmod(a, m)
        a = t
        t = y
        y, x = _w64(x - _w64(q * y)), t
        if x < 0:
            x = _npmod(x, p)
    return _npmod(x, p)


def divmod(_num, _den, _p):  # noqa: A001  (the reference's name)
    _num = _npmod(int(_num), _p)
    _den = _npmod(int(_den), _p)
    _inv = modular_inv(_den, _p)
    return _npmod(_w64(_num * _inv), _p)


def PI(vals, p):  # noqa: N802
    accum = 1
    for v in vals:
        tmp = _npmod(int(v), p)
        accum = _npmod(_w64(accum * tmp), p)
    return accum


def gen_Lagrange_coeffs(alpha_s, beta_s, p, is_K1=0):  # noqa: N802
    """U[i][j] (num_alpha x len(beta_s)) exactly as lightsecagg.py:59-80 (int64 results)."""
    p = int(p)
    alpha_s = [_w64(int(v)) for v in alpha_s]
    beta_s = [_w64(int(v)) for v in beta_s]
    num_alpha = 1 if is_K1 == 1 else len(alpha_s)
    w = [PI([_w64(cb - o) for o in beta_s if cb != o], p) for cb in beta_s]
    lv = [PI([_w64(alpha_s[i] - o) for o in beta_s], p) for i in range(num_alpha)]
    U = np.zeros((num_alpha, len(beta_s)), dtype=np.int64)
    for j in range(len(beta_s)):
        for i in range(num_alpha):
            den = _npmod(_w64(_npmod(_w64(alpha_s[i] - beta_s[j]), p) * w[j]), p)
            U[i][j] = divmod(lv[i], den, p)
    return U


# ------------------------------------------------------------------------------ placement
def _is_device(v) -> bool:
    return isinstance(v, torch.Tensor) and v.is_cuda


def _engine(values) -> AggEngine:
    for v in values:
        if _is_device(v):
            return get_engine(v.device.index)
    return get_engine(None)


def _dev(v, eng: AggEngine, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """numpy array / numpy scalar / Python number / tensor -> contiguous tensor on the engine."""
    if isinstance(v, torch.Tensor):
        t = v
    else:
        a = np.asarray(v)
        if a.dtype == np.float16 or a.dtype.kind not in "fiub":
            raise TypeError(f"unsupported array dtype {a.dtype}")
        t = torch.from_numpy(np.ascontiguousarray(a).reshape(a.shape))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    if t.device != eng.device:
        t = t.to(eng.device)
    return t if t.is_contiguous() else t.contiguous()


def _to_numpy(t: torch.Tensor):
    a = t.cpu().numpy()
    return a if a.ndim else a[()]  # the reference's 0-d results are numpy scalars


def _check_q(q_bits):
    q = int(q_bits)
    if not 0 <= q <= _Q_MAX:
        raise ValueError(f"q_bits must be in [0, {_Q_MAX}] (got {q_bits})")
    return q


# ------------------------------------------------------------------------------ field ops
def aggregate_models_in_finite(weights_finite, prime_number):
    """Sum of the clients' finite models, reduced mod p after every add (lightsecagg.py:134-145):
    w = x_0; w = mod(w + x_i, p) for i >= 1 (client 0 alone is returned unreduced)."""
    if len(weights_finite) == 0:
        raise IndexError("list index out of range")
    keys = list(weights_finite[0].keys())
    on_device = all(_is_device(w[k]) for w in weights_finite for k in keys)
    eng = _engine([w[k] for w in weights_finite for k in keys])
    segs, shapes = [], []
    for k in keys:
        col = [_dev(w[k], eng, torch.int64) for w in weights_finite]
        segs.append(col)
        shapes.append(col[0].shape)
    if not segs:
        return OrderedDict()
    fin, _ = eng.finite_sum(segs, int(prime_number), MOD_EACH)
    out = OrderedDict()
    for k, t in zip(keys, fin):
        out[k] = t if on_device else _to_numpy(t)
    return out


def my_q(X, q_bit, p):
    """Fixed-point quantisation into Z_p (lightsecagg.py:150-154) of one array / tensor."""
    eng = _engine([X])
    t = _dev(X, eng)
    if t.dtype not in (torch.float32, torch.float64, torch.int64):
        raise TypeError(f"my_q: unsupported dtype {t.dtype}")
    out = eng.finite_quantize([t], int(p), _check_q(q_bit))[0]
    return out if _is_device(X) else _to_numpy(out)


def my_q_inv(X_q, q_bit, p):  # noqa: N803
    """Back to reals (lightsecagg.py:157-161): float64, as numpy evaluates it."""
    eng = _engine([X_q])
    t = _dev(X_q, eng, torch.int64)
    _, real = eng.finite_sum([[t]], int(p), REAL_F64, finite=False, q_bits=_check_q(q_bit))
    return real[0] if _is_device(X_q) else _to_numpy(real[0])


def transform_tensor_to_finite(model_params, p, q_bits):
    """my_q of every key, in place in the dict like the reference (lightsecagg.py:187-192); keys of
    one dtype go to the device in one launch."""
    q = _check_q(q_bits)
    keys = list(model_params.keys())
    on_device = all(_is_device(model_params[k]) for k in keys)
    eng = _engine([model_params[k] for k in keys])
    groups: Dict[torch.dtype, List[str]] = {}
    tens = {}
    for k in keys:
        t = _dev(model_params[k], eng)
        if t.dtype in (torch.int32, torch.int16, torch.int8, torch.uint8):
            t = t.to(torch.int64)  # numpy promotes small ints with the Python-int 2**q to int64
        if t.dtype not in (torch.float32, torch.float64, torch.int64):
            raise TypeError(f"transform_tensor_to_finite: key {k!r} has unsupported dtype {t.dtype}")
        tens[k] = t
        groups.setdefault(t.dtype, []).append(k)
    for dt, ks in groups.items():
        outs = eng.finite_quantize([tens[k] for k in ks], int(p), q)
        for k, o in zip(ks, outs):
            model_params[k] = o if on_device else _to_numpy(o)
    return model_params


def transform_finite_to_tensor(model_params, p, q_bits):
    """my_q_inv of every key into float32 tensors, in place (lightsecagg.py:164-185); a 0-d key
    becomes shape [1], as the reference's ``torch.Tensor([numpy scalar])``."""
    q = _check_q(q_bits)
    keys = list(model_params.keys())
    on_device = all(_is_device(model_params[k]) for k in keys)
    eng = _engine([model_params[k] for k in keys])
    segs = [[_dev(model_params[k], eng, torch.int64)] for k in keys]
    if not segs:
        return model_params
    _, real = eng.finite_sum(segs, int(p), 0, finite=False, q_bits=q, scale=1.0)
    for k, r in zip(keys, real):
        r = r.reshape(1) if r.dim() == 0 else r
        model_params[k] = r if on_device else r.cpu()
    return model_params


def model_masking(weights_finite, dimensions, local_mask, prime_number):
    """w_k = mod(w_k + mask[pos:pos+d_k], p) per key, in place (lightsecagg.py:83-95)."""
    keys = list(weights_finite.keys())
    on_device = all(_is_device(weights_finite[k]) for k in keys) and _is_device(local_mask)
    eng = _engine([weights_finite[k] for k in keys] + [local_mask])
    mask = _dev(local_mask, eng, torch.int64).reshape(-1)
    segs, pos = [], 0
    for i, k in enumerate(keys):
        w = _dev(weights_finite[k], eng, torch.int64)
        d = int(dimensions[i])
        if d != w.numel():
            raise ValueError(f"cannot reshape array of size {d} into shape {tuple(w.shape)}")
        segs.append([w, mask[pos:pos + d].reshape(w.shape)])
        pos += d
    fin, _ = eng.finite_sum(segs, int(prime_number), MOD_EACH)
    for k, t in zip(keys, fin):
        weights_finite[k] = t if on_device else _to_numpy(t)
    return weights_finite


def LCC_decoding_with_points(f_eval, eval_points, target_points, p, n_out: Optional[int] = None):  # noqa: N802
    """np.mod(U_dec.dot(f_eval), p) with U_dec = gen_Lagrange_coeffs(target, eval) (lightsecagg.py:
    50-55).  Returns the (len(target), m) matrix, or its first ``n_out`` row-major entries."""
    U_dec = gen_Lagrange_coeffs(target_points, eval_points, p)
    eng = _engine([f_eval])
    f = _dev(f_eval, eng, torch.int64)
    if f.dim() != 2 or f.shape[0] != U_dec.shape[1]:
        raise ValueError(f"shapes {U_dec.shape} and {tuple(f.shape)} not aligned")
    rows, m = U_dec.shape[0], f.shape[1]
    total = rows * m if n_out is None else int(n_out)
    out = eng.lcc_decode(U_dec.tolist(), f, int(p), total)
    if n_out is None:
        out = out.reshape(rows, m)
    return out if _is_device(f_eval) else _to_numpy(out)


def model_dimension(weights):
    """Per-key element counts and their total (lightsecagg.py:195-205)."""
    dims = []
    for k in weights.keys():
        shape = tuple(weights[k].shape)
        d = 1
        for s in shape:
            d *= int(s)
        dims.append(d)
    return dims, int(np.sum(dims)) if dims else 0
