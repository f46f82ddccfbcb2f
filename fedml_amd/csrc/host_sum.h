// host_sum.h -- the ordered weighted sum for SMALL HOST-RESIDENT rounds, on the CPU that already holds
// the data (BASELINE configs[0]: the reference's quick_start, LR-MNIST, K = 2 clients of 63 KB, "MPI
// simulation on CPU").  A device round trip for such a round costs at least the PCIe doorbell floor
// (13.7 us measured) while the reference's CPU loop takes 10.9 us, so below a measured
// break-even size the engine sums host-resident rounds here instead of shipping them to the GPU;
// device-resident rounds, and every host round above the threshold, keep the HIP kernels.
//
// Same per-element contract as the kernels (fedagg.hip term()/accum(), include/fedagg.h):
//   acc = -0 (the exact identity of IEEE addition), then for i = 0..K-1 IN ORDER acc = op(acc + t_i),
//   t_i = x_i * c_i (MUL_W), (x_i * c_i) / d (MUL_N_DIV_N), x_i (SUM); every op one IEEE rounding to
//   the storage type (bf16 / f16: through float32, as PyTorch-CPU computes a reduced-precision op);
//   int64 inputs under the weighted modes promote to float32 (MUL_N_DIV_N: int64 x int64 wrapping
//   product first), under SUM wrap in int64.  Compiled with -ffp-contract=off: no FMA anywhere.
// Reference: python/fedml/ml/aggregator/agg_operator.py:35-63, simulation/mpi/fedavg/FedAVGAggregator.py:99-116.
#pragma once

#include <cstdint>
#include <cstring>

namespace fa_host {

enum { MUL_W = 0, MUL_N_DIV_N = 1, SUM = 2 };
enum { F32 = 0, BF16 = 1, F16 = 2, F64 = 3, I64 = 4 };

inline uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float fromb(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

// float32 -> bfloat16, round to nearest even (c10::BFloat16's rule; a NaN becomes the quiet 0x7FC0)
inline uint16_t bf16_bits(float f) {
  const uint32_t u = fbits(f);
  if ((u & 0x7FFFFFFFu) > 0x7F800000u) return 0x7FC0;
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
inline float bf16_float(uint16_t b) { return fromb((uint32_t)b << 16); }
inline float bf16_round(float f) { return bf16_float(bf16_bits(f)); }

// float32 -> IEEE half, round to nearest even incl. subnormals and overflow to inf (the branch-free
// scaling construction PyTorch's c10::Half uses; needs RNE float arithmetic and no FMA contraction)
inline uint16_t f16_bits(float f) {
  const float to_inf = fromb(0x77800000u), to_zero = fromb(0x08800000u);  // 2^112, 2^-110
  float base = (__builtin_fabsf(f) * to_inf) * to_zero;
  const uint32_t w = fbits(f), shl1 = w + w, sign = w & 0x80000000u;
  uint32_t bias = shl1 & 0xFF000000u;
  if (bias < 0x71000000u) bias = 0x71000000u;
  base = fromb((bias >> 1) + 0x07800000u) + base;
  const uint32_t b = fbits(base);
  const uint32_t nonsign = ((b >> 13) & 0x7C00u) + (b & 0x0FFFu);
  return (uint16_t)((sign >> 16) | (shl1 > 0xFF000000u ? 0x7E00u : nonsign));
}
// IEEE half -> float32 (exact)
inline float f16_float(uint16_t h) {
  const uint32_t w = (uint32_t)h << 16, sign = w & 0x80000000u, two_w = w + w;
  const float exp_scale = fromb(0x07800000u);  // 2^-112
  const float normalized = fromb((two_w >> 4) + 0x70000000u) * exp_scale;
  const float denormalized = fromb((two_w >> 17) | 0x3F000000u) - 0.5f;
  const uint32_t r = sign | (two_w < 0x08000000u ? fbits(denormalized) : fbits(normalized));
  return fromb(r);
}
inline float f16_round(float f) { return f16_float(f16_bits(f)); }

constexpr int64_t kBlock = 1024;  // elements per accumulator block (stays in L1)

// One key: out[0..n) = ordered reduction of the k inputs in[i][0..n).
template <int DT, int MODE>
void sum_key(int64_t n, int k, const void* const* in, const double* coef, double divisor, void* out) {
  for (int64_t e0 = 0; e0 < n; e0 += kBlock) {
    const int64_t m = n - e0 < kBlock ? n - e0 : kBlock;
    if constexpr (DT == F64) {
      double acc[kBlock];
      for (int64_t j = 0; j < m; ++j) acc[j] = -0.0;
      const double d = divisor;
      for (int i = 0; i < k; ++i) {
        const double* x = (const double*)in[i] + e0;
        const double c = coef ? coef[i] : 0.0;
        for (int64_t j = 0; j < m; ++j) {
          double t = MODE == SUM ? x[j] : x[j] * c;
          if (MODE == MUL_N_DIV_N) t = t / d;
          acc[j] = acc[j] + t;
        }
      }
      std::memcpy((double*)out + e0, acc, m * sizeof(double));
    } else if constexpr (DT == I64 && MODE == SUM) {
      uint64_t acc[kBlock];
      for (int64_t j = 0; j < m; ++j) acc[j] = 0;
      for (int i = 0; i < k; ++i) {
        const uint64_t* x = (const uint64_t*)in[i] + e0;
        for (int64_t j = 0; j < m; ++j) acc[j] += x[j];
      }
      std::memcpy((uint64_t*)out + e0, acc, m * sizeof(uint64_t));
    } else {
      float acc[kBlock];
      for (int64_t j = 0; j < m; ++j) acc[j] = -0.0f;
      const float d = (float)divisor;
      for (int i = 0; i < k; ++i) {
        const float c = coef ? (float)coef[i] : 0.0f;
        if constexpr (DT == F32) {
          const float* x = (const float*)in[i] + e0;
          for (int64_t j = 0; j < m; ++j) {
            float t = MODE == SUM ? x[j] : x[j] * c;
            if (MODE == MUL_N_DIV_N) t = t / d;
            acc[j] = acc[j] + t;
          }
        } else if constexpr (DT == BF16 || DT == F16) {
          const uint16_t* x = (const uint16_t*)in[i] + e0;
          for (int64_t j = 0; j < m; ++j) {
            const float v = DT == BF16 ? bf16_float(x[j]) : f16_float(x[j]);
            float t = v;
            if (MODE != SUM) {
              t = v * c;
              t = DT == BF16 ? bf16_round(t) : f16_round(t);
              if (MODE == MUL_N_DIV_N) {
                t = t / d;
                t = DT == BF16 ? bf16_round(t) : f16_round(t);
              }
            }
            const float s = acc[j] + t;
            acc[j] = DT == BF16 ? bf16_round(s) : f16_round(s);
          }
        } else {  // int64, weighted: float32 output
          const int64_t* x = (const int64_t*)in[i] + e0;
          const int64_t cn = coef ? (int64_t)coef[i] : 0;
          for (int64_t j = 0; j < m; ++j) {
            float t;
            if (MODE == MUL_W) {
              t = (float)x[j] * c;
            } else {  // int64 * int64 (wrapping), then true division in float32
              t = (float)(int64_t)((uint64_t)x[j] * (uint64_t)cn) / d;
            }
            acc[j] = acc[j] + t;
          }
        }
      }
      if constexpr (DT == F32 || DT == I64) {
        std::memcpy((float*)out + e0, acc, m * sizeof(float));
      } else {
        uint16_t* o = (uint16_t*)out + e0;
        for (int64_t j = 0; j < m; ++j) o[j] = DT == BF16 ? bf16_bits(acc[j]) : f16_bits(acc[j]);
      }
    }
  }
}

template <int DT>
inline void sum_key_dt(int mode, int64_t n, int k, const void* const* in, const double* coef, double divisor,
                       void* out) {
  switch (mode) {
    case MUL_W: sum_key<DT, MUL_W>(n, k, in, coef, divisor, out); break;
    case MUL_N_DIV_N: sum_key<DT, MUL_N_DIV_N>(n, k, in, coef, divisor, out); break;
    default: sum_key<DT, SUM>(n, k, in, nullptr, divisor, out); break;
  }
}

// Returns 0, or -1 for an unknown dtype / mode.
inline int sum_key_any(int dtype, int mode, int64_t n, int k, const void* const* in, const double* coef,
                       double divisor, void* out) {
  if (mode < MUL_W || mode > SUM) return -1;
  switch (dtype) {
    case F32: sum_key_dt<F32>(mode, n, k, in, coef, divisor, out); return 0;
    case BF16: sum_key_dt<BF16>(mode, n, k, in, coef, divisor, out); return 0;
    case F16: sum_key_dt<F16>(mode, n, k, in, coef, divisor, out); return 0;
    case F64: sum_key_dt<F64>(mode, n, k, in, coef, divisor, out); return 0;
    case I64: sum_key_dt<I64>(mode, n, k, in, coef, divisor, out); return 0;
    default: return -1;
  }
}

}  // namespace fa_host
