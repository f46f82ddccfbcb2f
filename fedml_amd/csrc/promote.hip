// promote.hip -- the reference's per-key accumulation step when clients disagree on a key's dtype.
//
// The reference's FedAvg loop (python/fedml/ml/aggregator/agg_operator.py:37-44) is, per key,
//   avg = x_0 * w_0;   avg += x_i * w_i  (i = 1..K-1)
// and its plain-sum branch (:55-63) avg = x_0; avg += x_i.  When client i's tensor has another
// dtype than avg, `avg += t` is PyTorch's in-place add across dtypes: both operands are cast to the
// promoted type C = promote_types(avg, t), added in C (C's op-math: float for bf16/f16/f32,
// double for f64), and the sum is cast back to avg's dtype.  The casts are c10's: int64 -> float
// types and f64 -> bf16/f16 go THROUGH float32 (two roundings), which tests/golden/g19_* (made by
// the reference itself) pin.  The terms t_i = x_i * w_i are the engine's ordinary K = 1 weighted
// sums (same kernels, same bits as the reference's `x * w` in x's dtype); this kernel is only the
// cross-dtype `avg += t`, one element per lane, HBM-bound (read avg and t, write avg).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "fa_internal.h"

using namespace fa_detail;

namespace {

__device__ __forceinline__ float pin(float x) {  // keep the f32 intermediate (no fused f32->f16 paths)
  asm("" : "+v"(x));
  return x;
}
__device__ __forceinline__ float rnd_bf16(float x) { return (float)(__bf16)pin(x); }
__device__ __forceinline__ float rnd_f16(float x) { return (float)(_Float16)pin(x); }

// value of element e of a tensor of dtype DT, widened exactly (float for f32/bf16/f16, double for
// f64, int64 as is)
template <int DT> struct Ld;
template <> struct Ld<FA_DTYPE_F32> { using T = float; __device__ static T get(const void* p, int64_t e) { return ((const float*)p)[e]; } };
template <> struct Ld<FA_DTYPE_F64> { using T = double; __device__ static T get(const void* p, int64_t e) { return ((const double*)p)[e]; } };
template <> struct Ld<FA_DTYPE_I64> { using T = long long; __device__ static T get(const void* p, int64_t e) { return ((const long long*)p)[e]; } };
template <> struct Ld<FA_DTYPE_BF16> {
  using T = float;
  __device__ static T get(const void* p, int64_t e) { return __uint_as_float((unsigned)((const unsigned short*)p)[e] << 16); }
};
template <> struct Ld<FA_DTYPE_F16> {
  using T = float;
  __device__ static T get(const void* p, int64_t e) { return (float)__builtin_bit_cast(_Float16, ((const unsigned short*)p)[e]); }
};

// PyTorch's promote_types for the pairs that reach this kernel (acc a float dtype)
template <int A, int B>
constexpr int promoted() {
  if (B == FA_DTYPE_I64 || A == B) return A;
  if (A == FA_DTYPE_F64 || B == FA_DTYPE_F64) return FA_DTYPE_F64;
  return FA_DTYPE_F32;  // f32 with anything below it, and bf16 with f16
}

// c10 cast of an exactly-widened value to dtype C (returned in C's op-math type)
template <int C, class V>
__device__ __forceinline__ auto to_common(V v) {
  if constexpr (C == FA_DTYPE_F64) {
    return (double)v;  // float -> double exact; int64 -> double correctly rounded
  } else {
    const float f = (float)v;  // float types exact; int64 -> float correctly rounded; (no f64 here)
    if constexpr (C == FA_DTYPE_BF16) return rnd_bf16(f);
    else if constexpr (C == FA_DTYPE_F16) return rnd_f16(f);
    else return f;
  }
}

// C's add, rounded to C
template <int C, class V>
__device__ __forceinline__ V add_in(V a, V b) {
  if constexpr (C == FA_DTYPE_F64) return __dadd_rn(a, b);
  else if constexpr (C == FA_DTYPE_BF16) return rnd_bf16(__fadd_rn(a, b));
  else if constexpr (C == FA_DTYPE_F16) return rnd_f16(__fadd_rn(a, b));
  else return __fadd_rn(a, b);
}

// c10 cast of a C value to the accumulator dtype A, stored
template <int A, class V>
__device__ __forceinline__ void store(void* p, int64_t e, V v) {
  if constexpr (A == FA_DTYPE_F64) {
    ((double*)p)[e] = (double)v;
  } else {
    const float f = (float)v;  // double -> float (round), float -> float
    if constexpr (A == FA_DTYPE_F32) ((float*)p)[e] = f;
    else if constexpr (A == FA_DTYPE_BF16) ((unsigned short*)p)[e] = __builtin_bit_cast(unsigned short, (__bf16)pin(f));
    else ((unsigned short*)p)[e] = __builtin_bit_cast(unsigned short, (_Float16)pin(f));
  }
}

template <int A, int B>
__global__ void __launch_bounds__(kBlock) k_promote_add(const void* __restrict__ acc, const void* __restrict__ t,
                                                        void* out, int64_t n) {
  constexpr int C = promoted<A, B>();
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride) {
    const auto a = to_common<C>(Ld<A>::get(acc, e));
    const auto b = to_common<C>(Ld<B>::get(t, e));
    store<A>(out, e, add_in<C>(a, b));
  }
}

template <int A, int B>
void launch(const void* acc, const void* t, void* out, int64_t n, hipStream_t st) {
  const int64_t blocks = std::min<int64_t>((n + kBlock - 1) / kBlock, 65536);
  hipLaunchKernelGGL((k_promote_add<A, B>), dim3((unsigned)blocks), dim3(kBlock), 0, st, acc, t, out, n);
}

template <int A>
int dispatch_t(int t_dtype, const void* acc, const void* t, void* out, int64_t n, hipStream_t st) {
  switch (t_dtype) {
    case FA_DTYPE_F32: launch<A, FA_DTYPE_F32>(acc, t, out, n, st); return FA_OK;
    case FA_DTYPE_BF16: launch<A, FA_DTYPE_BF16>(acc, t, out, n, st); return FA_OK;
    case FA_DTYPE_F16: launch<A, FA_DTYPE_F16>(acc, t, out, n, st); return FA_OK;
    case FA_DTYPE_F64: launch<A, FA_DTYPE_F64>(acc, t, out, n, st); return FA_OK;
    case FA_DTYPE_I64: launch<A, FA_DTYPE_I64>(acc, t, out, n, st); return FA_OK;
    default: return fail(FA_ERR_DTYPE, "fa_promote_add: term dtype %d not supported", t_dtype);
  }
}

}  // namespace

extern "C" int fa_promote_add(fa_ctx* ctx, int acc_dtype, int t_dtype, int64_t n, const void* d_acc,
                              const void* d_t, void* d_out, void* hip_stream) {
  if (!ctx || n < 0 || (n > 0 && (!d_acc || !d_t || !d_out)))
    return fail(FA_ERR_INVALID, "fa_promote_add: invalid arguments");
  if (n == 0) return FA_OK;
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "fa_promote_add: hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  int rc;
  switch (acc_dtype) {
    case FA_DTYPE_F32: rc = dispatch_t<FA_DTYPE_F32>(t_dtype, d_acc, d_t, d_out, n, st); break;
    case FA_DTYPE_BF16: rc = dispatch_t<FA_DTYPE_BF16>(t_dtype, d_acc, d_t, d_out, n, st); break;
    case FA_DTYPE_F16: rc = dispatch_t<FA_DTYPE_F16>(t_dtype, d_acc, d_t, d_out, n, st); break;
    case FA_DTYPE_F64: rc = dispatch_t<FA_DTYPE_F64>(t_dtype, d_acc, d_t, d_out, n, st); break;
    default: return fail(FA_ERR_DTYPE, "fa_promote_add: accumulator dtype %d must be a float type", acc_dtype);
  }
  if (rc != FA_OK) return rc;
  FA_HIP(hipGetLastError());
  return FA_OK;
}
