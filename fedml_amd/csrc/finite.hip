// finite.hip -- MI355X (gfx950) kernels + C ABI of the finite-field secure-aggregation family
// (include/fedagg_finite.h): the server's masked-model reconstruction in Z_p, the fixed-point
// quantisation (my_q / model_masking) and the LCC mask decoding of LightSecAgg.
//
// Design:
//  * Same shape as the weighted sum (fedagg.hip): HBM-bound, one lane = one 16-byte vector of
//    int64 (2 elements) of one tile, the K clients walked in order with U clamped loads in flight,
//    non-temporal loads/stores, one launch per state_dict via the segment table.
//  * The reduction is int64 with the reference's exact numpy semantics: two's-complement wrap on
//    +/-, floor remainder for np.mod.  A 64-bit `%` is a ~100-instruction software routine on the
//    GPU, so mod is layered: in-range operands (the protocol's normal case, values in [0, p))
//    take a compare-and-subtract; |a| < 2^53 takes a float64 reciprocal quotient with a +-1
//    fix-up; only the rest (adversarial / wrapped inputs) pays for the division.  Every layer
//    returns the identical floor remainder, so the layering is invisible in the results.
//  * Dequantisation (my_q_inv) is float64 exactly as numpy evaluates it, then float32 as
//    torch.Tensor(ndarray) converts it, then the float32 "* (1 / len(active))".
//  * LCC decoding is a tiny-K (U x U coefficients) int64 matrix product over m columns: one lane
//    per column keeps RB row accumulators, the column's k inputs stream through (L2-resident when
//    re-read for the next row block); coefficients are wave-uniform scalar loads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <type_traits>

#include "fa_internal.h"
#include "fedagg_finite.h"
#include "mt_poly.h"

using namespace fa_detail;

namespace {

constexpr int kV = 2;                       // int64 elements per 16-byte vector
constexpr int64_t kTile = (int64_t)kBlock * kV;
constexpr int kU = 8;                       // clients per load group

struct FSeg {
  int64_t numel;
  int64_t tile_start;
  int32_t ptr_base;
  int32_t aligned;
  const long long* mask;  // may be null
  long long* out_fin;     // may be null
  void* out_real;         // may be null; float32, or float64 with FA_FINITE_REAL_F64
};
static_assert(sizeof(FSeg) == 48, "FSeg layout");

struct ModP {
  long long p;
  double inv_p;   // RN(1 / p)
  bool small;     // p <= 2^62: in-range sums cannot wrap
};

typedef const __attribute__((address_space(1))) u32x4* gp_u32x4;
typedef __attribute__((address_space(1))) u32x4* gpw_u32x4;

__device__ __forceinline__ long long wadd(long long a, long long b) {
  return (long long)((unsigned long long)a + (unsigned long long)b);
}
__device__ __forceinline__ long long wsub(long long a, long long b) {
  return (long long)((unsigned long long)a - (unsigned long long)b);
}

// np.mod(a, p) for any int64 a, p > 0
__device__ __forceinline__ long long mod_any(long long a, const ModP& m) {
  if ((unsigned long long)a < (unsigned long long)m.p) return a;
  if (a > -(1ll << 53) && a < (1ll << 53)) {
    const double q = floor(__dmul_rn((double)a, m.inv_p));
    long long r = a - (long long)q * m.p;
    if (r < 0) r += m.p;
    else if (r >= m.p) r -= m.p;
    return r;
  }
  const long long r = a % m.p;
  return r < 0 ? r + m.p : r;
}

// np.mod(a, p) for 0 <= a < 2^53 (no division routine)
__device__ __forceinline__ long long mod_nonneg53(long long a, const ModP& m) {
  const double q = floor(__dmul_rn((double)a, m.inv_p));
  long long r = a - (long long)q * m.p;
  if (r < 0) r += m.p;
  else if (r >= m.p) r -= m.p;
  return r;
}
// np.mod(a + b, p) with wrapping a + b
__device__ __forceinline__ long long mod_add(long long a, long long b, const ModP& m) {
  if (m.small && (unsigned long long)a < (unsigned long long)m.p && (unsigned long long)b < (unsigned long long)m.p) {
    const long long s = a + b;
    return s >= m.p ? s - m.p : s;
  }
  return mod_any(wadd(a, b), m);
}
// np.mod(a - b, p) with wrapping a - b
__device__ __forceinline__ long long mod_sub(long long a, long long b, const ModP& m) {
  if ((unsigned long long)a < (unsigned long long)m.p && (unsigned long long)b < (unsigned long long)m.p) {
    const long long d = a - b;
    return d < 0 ? d + m.p : d;
  }
  return mod_any(wsub(a, b), m);
}

struct Dequant {
  double half;       // (p - 1) / 2
  double pd;         // (double)p
  double inv_pow2q;  // 2^-q (exact: x / 2^q == x * 2^-q, no subnormal results for |x| < 2^63)
  float scale;
};

// my_q_inv in float64 (numpy's evaluation)
__device__ __forceinline__ double dequant64(long long v, const Dequant& dq) {
  const double vd = (double)v;
  const double xq = __dsub_rn(vd, dq.half) > 0.0 ? __dsub_rn(vd, dq.pd) : vd;
  return __dmul_rn(xq, dq.inv_pow2q);
}
// ... then torch.Tensor's float32 conversion and the float32 "* scale"
__device__ __forceinline__ float dequant(long long v, const Dequant& dq) {
  return __fmul_rn(__double2float_rn(dequant64(v, dq)), dq.scale);
}

__device__ __forceinline__ long long lo64(u32x4 r) { return __builtin_bit_cast(long long, u32x2{r[0], r[1]}); }
__device__ __forceinline__ long long hi64(u32x4 r) { return __builtin_bit_cast(long long, u32x2{r[2], r[3]}); }
__device__ __forceinline__ u32x4 pack64(long long a, long long b) {
  const u32x2 x = __builtin_bit_cast(u32x2, a), y = __builtin_bit_cast(u32x2, b);
  return u32x4{x[0], x[1], y[0], y[1]};
}

template <bool EACH>
__device__ __forceinline__ long long step(long long acc, long long x, const ModP& m) {
  if constexpr (EACH) return mod_add(acc, x, m);
  else return wadd(acc, x);
}

__device__ __forceinline__ void finish(long long& acc, bool has_mask, long long mk, int flags, const ModP& m) {
  if (has_mask) {
    acc = (flags & FA_FINITE_MOD_END) ? mod_sub(acc, mk, m) : wsub(acc, mk);
  } else if (flags & FA_FINITE_MOD_END) {
    acc = mod_any(acc, m);
  }
}

// ---------------------------------------------------------------------------------- reconstruct
template <bool EACH>
__global__ void __launch_bounds__(kBlock)
k_finite_sum(const FSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k, int flags,
             ModP m, Dequant dq, int64_t sstr) {
  const int64_t tile = blockIdx.x;
  const FSeg sg = segs[nseg > 1 ? find_seg(segs, nseg, tile) : 0];
  const int64_t tl = tile - sg.tile_start;
  const int64_t base = tl * kTile;
  // input tile stride: kTile * 8 bytes (flat) or the arena's tile stride (tile-interleaved inputs)
  const int64_t sst = sstr ? sstr : kTile * 8;
  const void* const* in = ptrs + sg.ptr_base;
  const bool first = flags & FA_FINITE_MOD_FIRST;

  if (sg.aligned && base + kTile <= sg.numel) {
    const int64_t e0 = base + (int64_t)threadIdx.x * kV;
    const int64_t boff = tl * sst + (int64_t)threadIdx.x * kV * 8;
    long long a0 = 0, a1 = 0;
    // the mask is needed only at the end: issue its load first, it lands while the clients stream
    const u32x4 mk = sg.mask ? __builtin_nontemporal_load((gp_u32x4)(sg.mask + e0)) : u32x4{0, 0, 0, 0};
    for (int i0 = 0; i0 < k; i0 += kU) {
      u32x4 r[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int i = min(i0 + u, k - 1);  // clamped: every load unconditional
        r[u] = __builtin_nontemporal_load((gp_u32x4)((const char*)in[i] + boff));
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int i = i0 + u;
        if (i < k) {  // wave-uniform
          const long long x0 = lo64(r[u]), x1 = hi64(r[u]);
          if (i == 0) {
            a0 = first ? mod_any(x0, m) : x0;
            a1 = first ? mod_any(x1, m) : x1;
          } else {
            a0 = step<EACH>(a0, x0, m);
            a1 = step<EACH>(a1, x1, m);
          }
        }
      }
    }
    finish(a0, sg.mask != nullptr, lo64(mk), flags, m);
    finish(a1, sg.mask != nullptr, hi64(mk), flags, m);
    if (sg.out_fin) __builtin_nontemporal_store(pack64(a0, a1), (gpw_u32x4)(sg.out_fin + e0));
    if (sg.out_real) {
      if (flags & FA_FINITE_REAL_F64) {
        const u32x4 w = pack64(__double_as_longlong(dequant64(a0, dq)), __double_as_longlong(dequant64(a1, dq)));
        __builtin_nontemporal_store(w, (gpw_u32x4)((double*)sg.out_real + e0));
      } else {
        *(float2*)((float*)sg.out_real + e0) = make_float2(dequant(a0, dq), dequant(a1, dq));
      }
    }
  } else {
    const int64_t end = min(base + kTile, sg.numel);
    for (int64_t e = base + threadIdx.x; e < end; e += kBlock) {
      const int64_t pe = (e / kTile) * (sst / 8) + e % kTile;
      long long acc = ((const long long*)in[0])[pe];
      if (first) acc = mod_any(acc, m);
      for (int i = 1; i < k; ++i) acc = step<EACH>(acc, ((const long long*)in[i])[pe], m);
      finish(acc, sg.mask != nullptr, sg.mask ? sg.mask[e] : 0, flags, m);
      if (sg.out_fin) sg.out_fin[e] = acc;
      if (sg.out_real) {
        if (flags & FA_FINITE_REAL_F64) ((double*)sg.out_real)[e] = dequant64(acc, dq);
        else ((float*)sg.out_real)[e] = dequant(acc, dq);
      }
    }
  }
}

// ----------------------------------------------------------------------------------- quantise
struct QSeg {
  int64_t numel;
  int64_t tile_start;
  const void* x;
  const long long* mask;  // may be null
  long long* out;
  int64_t aligned;
};
static_assert(sizeof(QSeg) == 48, "QSeg layout");

struct QParams {
  float pow2q_f;   // 2^q
  float pf;        // (float)p
  double pow2q_d;
  double pd;       // (double)p
  int q;
};

__device__ __forceinline__ long long d2i64(double v) {
  // numpy astype(int64) on x86: truncation; NaN / +-Inf / out of range -> INT64_MIN
  if (!(v >= -9223372036854775808.0 && v < 9223372036854775808.0)) return LLONG_MIN;
  return (long long)v;
}

template <int DT>
__device__ __forceinline__ long long quant1(const void* x, int64_t e, const QParams& qp) {
  if constexpr (DT == FA_DTYPE_F32) {
    const float t = rintf(__fmul_rn(((const float*)x)[e], qp.pow2q_f));
    const float o = t < 0.0f ? __fadd_rn(t, qp.pf) : t;  // t + p * is_negative (NaN stays NaN)
    return d2i64((double)o);
  } else if constexpr (DT == FA_DTYPE_F64) {
    const double t = rint(__dmul_rn(((const double*)x)[e], qp.pow2q_d));
    const double o = t < 0.0 ? __dadd_rn(t, qp.pd) : t;
    return d2i64(o);
  } else {
    const long long t = (long long)((unsigned long long)((const long long*)x)[e] << qp.q);
    const double td = (double)t;
    return d2i64(t < 0 ? __dadd_rn(td, qp.pd) : td);
  }
}

template <int DT> struct QElems { static constexpr int V = DT == FA_DTYPE_F32 ? 4 : 2; };

template <int DT, bool MASK>
__global__ void __launch_bounds__(kBlock)
k_finite_quant(const QSeg* __restrict__ segs, int nseg, QParams qp, ModP m) {
  constexpr int V = QElems<DT>::V;
  constexpr int64_t TILE = (int64_t)kBlock * V;
  const int64_t tile = blockIdx.x;
  const QSeg sg = segs[nseg > 1 ? find_seg(segs, nseg, tile) : 0];
  const int64_t base = (tile - sg.tile_start) * TILE;
  const int64_t end = min(base + TILE, sg.numel);
  // element-wise; the per-element loads are coalesced across the wave (V elements per lane)
  const int64_t e0 = base + (int64_t)threadIdx.x * V;
  if (sg.aligned && base + TILE <= sg.numel) {
    long long v[V];
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = quant1<DT>(sg.x, e0 + j, qp);
    if constexpr (MASK) {
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = mod_add(v[j], sg.mask[e0 + j], m);
    }
#pragma unroll
    for (int j = 0; j < V; j += 2)
      __builtin_nontemporal_store(pack64(v[j], v[j + 1]), (gpw_u32x4)(sg.out + e0 + j));
  } else {
    for (int64_t e = base + threadIdx.x; e < end; e += kBlock) {
      long long v = quant1<DT>(sg.x, e, qp);
      if constexpr (MASK) v = mod_add(v, sg.mask[e], m);
      sg.out[e] = v;
    }
  }
}

// ---------------------------------------------------------------------------------- LCC decode
// General path: exact int64 (wrapping) multiply-accumulate, RB output rows per register block.
constexpr int kRB = 8;

__device__ __forceinline__ void lcc_rows_i64(const long long* __restrict__ coef, int j0, int j1, int k, int64_t m_cols,
                                             const long long* __restrict__ f, int64_t c, int64_t cc, bool live,
                                             int64_t n_out, long long* __restrict__ out, const ModP& md) {
  for (; j0 < j1; j0 += kRB) {
    unsigned long long acc[kRB];
#pragma unroll
    for (int r = 0; r < kRB; ++r) acc[r] = 0;
#pragma unroll 4
    for (int i = 0; i < k; ++i) {
      const unsigned long long fv = (unsigned long long)f[(int64_t)i * m_cols + cc];
#pragma unroll
      for (int r = 0; r < kRB; ++r) {
        const int j = min(j0 + r, j1 - 1);  // uniform clamp; extra rows are never stored
        acc[r] += (unsigned long long)coef[(int64_t)j * k + i] * fv;
      }
    }
    if (live) {
#pragma unroll
      for (int r = 0; r < kRB; ++r) {
        const int64_t e = (int64_t)(j0 + r) * m_cols + c;
        if (j0 + r < j1 && e < n_out) out[e] = mod_any((long long)acc[r], md);
      }
    }
  }
}

// redo: when non-null, only the blocks the float64 kernel flagged are (re)computed here.
__global__ void __launch_bounds__(kBlock)
k_lcc_decode(const long long* __restrict__ coef, int rows_needed, int k, int64_t m_cols,
             const long long* __restrict__ f, int64_t n_out, long long* __restrict__ out, ModP md,
             const int* __restrict__ redo) {
  if (redo && !redo[blockIdx.x]) return;
  const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool live = c < m_cols;
  lcc_rows_i64(coef, 0, rows_needed, k, m_cols, f, c, live ? c : m_cols - 1, live, n_out, out, md);
}

// Fast path when every partial sum is an exactly representable double: coefficients in [0, p)
// (checked on the host), (p-1)^2 * k < 2^53 (host) and every f in [0, p) (checked per lane while
// streaming; a block that meets an out-of-range value flags itself in `redo`, and k_lcc_decode,
// launched right after on the same stream, recomputes exactly those blocks on the int64 path).
// Then fma(c, f, acc) is exact integer arithmetic and float64 FMA -- full rate on CDNA4 -- replaces
// the ~6-instruction int64 multiply.  The coefficients of one pass (kRBF rows x up to kLdsI rows of
// f, transposed: [i][r]) are staged once per block in LDS and read as wave-wide broadcasts; the f
// loads run kPF rows ahead in a register ring.
constexpr int kRBF = 32;
constexpr int kLdsI = 128;  // f rows per LDS chunk: 128 x 32 doubles = 32 KiB

__global__ void __launch_bounds__(kBlock)
k_lcc_decode_f64(const double* __restrict__ coefT, int rows_needed, int k, int64_t m_cols,
                 const long long* __restrict__ f, int64_t n_out, long long* __restrict__ out, ModP md,
                 int* __restrict__ redo) {
  __shared__ double cs[kLdsI * kRBF];
  const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool live = c < m_cols;
  const int64_t cc = live ? c : m_cols - 1;  // clamped column: loads stay in bounds
  const unsigned long long up = (unsigned long long)md.p;
  constexpr int kPF = 4;
  bool ok = true;
  for (int j0 = 0; j0 < rows_needed; j0 += kRBF) {
    const double* __restrict__ cT = coefT + (int64_t)(j0 / kRBF) * k * kRBF;
    double acc[kRBF];
#pragma unroll
    for (int r = 0; r < kRBF; ++r) acc[r] = 0.0;
    for (int ib = 0; ib < k; ib += kLdsI) {
      const int ni = min(kLdsI, k - ib);
      __syncthreads();  // previous chunk fully consumed
      for (int t = threadIdx.x; t < ni * kRBF; t += kBlock) cs[t] = cT[(int64_t)ib * kRBF + t];
      __syncthreads();
      unsigned long long ring[kPF];
#pragma unroll
      for (int u = 0; u < kPF; ++u) ring[u] = (unsigned long long)f[(int64_t)(ib + min(u, ni - 1)) * m_cols + cc];
      for (int i0 = 0; i0 < ni; i0 += kPF) {
#pragma unroll
        for (int u = 0; u < kPF; ++u) {
          const int i = i0 + u;
          const unsigned long long fv = ring[u];
          ring[u] = (unsigned long long)f[(int64_t)(ib + min(i + kPF, ni - 1)) * m_cols + cc];
          if (i < ni) {  // wave-uniform
            ok = ok && fv < up;
            const double fd = (double)(unsigned)fv;
#pragma unroll
            for (int r = 0; r < kRBF; ++r) acc[r] = __fma_rn(cs[i * kRBF + r], fd, acc[r]);
          }
        }
      }
    }
    const int j1 = min(j0 + kRBF, rows_needed);
    const bool wave_ok = __ballot(!ok) == 0;  // every lane votes (no short-circuit around the ballot)
    if (live && wave_ok) {
#pragma unroll
      for (int r = 0; r < kRBF; ++r) {
        const int64_t e = (int64_t)(j0 + r) * m_cols + c;
        if (j0 + r < j1 && e < n_out) out[e] = mod_nonneg53((long long)acc[r], md);
      }
    }
  }
  // every wave stays to the end (the block shares LDS and barriers); a wave that saw an
  // out-of-range f hands the block to the int64 kernel
  if (__ballot(!ok) != 0 && threadIdx.x % 64 == 0) redo[blockIdx.x] = 1;
}

ModP make_modp(int64_t p) {
  ModP m;
  m.p = p;
  m.inv_p = 1.0 / (double)p;
  m.small = p <= (1ll << 62);
  return m;
}


// ============================================================================================
// SecAgg mask re-expansion: numpy legacy RandomState(seed).randint(0, p, size=n) per stream, on the
// device.  One wave per stream: the 624-word MT19937 state lives in LDS; each twist regenerates it
// in three dependency-free phases (words [0, 227) read only old words; [227, 454) read the new
// [0, 227); [454, 624) the new [227, 397) and word 0), every lane reading its inputs before any
// lane writes; then each word is tempered, masked and accepted or rejected, and the accepted
// draws are placed in stream order by a ballot prefix count.  The signed values go into a uint64
// accumulator with no-return atomics (streams are batched so that a batch's sum of values in
// [0, p) cannot wrap); a fold kernel reduces each batch mod p into d_out.
constexpr int kMtN = 624, kMtM = 397;
constexpr uint32_t kMtA = 0x9908b0dfu, kMtUp = 0x80000000u, kMtLo = 0x7fffffffu;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t next, uint32_t far) {
  const uint32_t y = (cur & kMtUp) | (next & kMtLo);
  return far ^ (y >> 1) ^ ((y & 1u) ? kMtA : 0u);
}

// numpy mt19937_gen, out of place: B = the generation after A (one wave, lane = 0..63).  Written to
// another buffer, the recurrence needs no read-before-write split: [0, 227) reads A only, [227, 454)
// reads A and B[0, 227), [454, 624) reads A and B[227, 397) and B[0] -- one barrier per range.
__device__ __forceinline__ void mt_next_block(const uint32_t* A, uint32_t* B, int lane) {
  constexpr int a = kMtN - kMtM;  // 227
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = r * 64 + lane;
    if (i < a) B[i] = mt_mix(A[i], A[i + 1], A[i + kMtM]);
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = a + r * 64 + lane;
    if (i < 2 * a) B[i] = mt_mix(A[i], A[i + 1], B[i - a]);
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int i = 2 * a + r * 64 + lane;
    if (i < kMtN) B[i] = mt_mix(A[i], i + 1 < kMtN ? A[i + 1] : B[0], B[i - a]);
  }
  __syncthreads();
}

template <bool WIDE>
__global__ void __launch_bounds__(64)
k_mt_randint(const uint32_t* __restrict__ seeds, const int8_t* __restrict__ signs, uint64_t rng, uint64_t mask,
             uint64_t p, int64_t n, unsigned long long* __restrict__ acc) {
  __shared__ uint32_t mt[2][kMtN];  // the last two generations of the state
  const int lane = threadIdx.x;
  const int s = blockIdx.x;
  const bool neg = signs[s] < 0;
  if (lane == 0) {  // numpy mt19937_seed (init_genrand): a serial recurrence, 624 steps
    uint32_t x = seeds[s];
    for (int i = 0; i < kMtN; ++i) {
      mt[0][i] = x;
      x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)(i + 1);
    }
  }
  __syncthreads();
  int64_t count = 0;  // draws accepted so far (wave-uniform)
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  constexpr int kVals = WIDE ? kMtN / 2 : kMtN;  // candidate values per generation (64-bit: word pairs)
  constexpr int kRounds = (kVals + 63) / 64;
  int cur = 0;
  while (count < n) {
    mt_next_block(mt[cur], mt[cur ^ 1], lane);
    cur ^= 1;
    const uint32_t* w32 = mt[cur];
    uint64_t v[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {  // every read of the block in flight at once
      const int w = r * 64 + lane;
      if (w < kVals) {
        if constexpr (WIDE) v[r] = (uint64_t)mt_temper(w32[2 * w]) << 32 | mt_temper(w32[2 * w + 1]);
        else v[r] = mt_temper(w32[w]);
        v[r] &= mask;
      } else {
        v[r] = ~0ull;  // past the block: never accepted (> rng)
      }
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const bool ok = v[r] <= rng;
      const uint64_t bal = __ballot(ok);
      const int64_t pos = count + __popcll(bal & below);
      if (ok && pos < n && v[r] != 0) atomicAdd(acc + pos, (unsigned long long)(neg ? p - v[r] : v[r]));
      count += __popcll(bal);
    }
  }
}

// total[e] = (first ? 0 : total[e]) + acc[e] mod p, reduced to [0, p); acc cleared for the next batch
__global__ void __launch_bounds__(kBlock)
k_mt_fold(unsigned long long* __restrict__ acc, int64_t* __restrict__ total, int64_t n, uint64_t p, int first) {
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += (int64_t)gridDim.x * kBlock) {
    const uint64_t a = acc[e] % p;
    uint64_t t = first ? a : (uint64_t)total[e] + a;
    if (t >= p) t -= p;
    total[e] = (int64_t)t;
    acc[e] = 0;
  }
}

// ---------------------------------------------------------------- jump-ahead expansion (r03)
// One wave per stream is latency-bound (38.7 ms for 32 streams x 11.7 M draws on a GPU that is
// mostly idle).  With jump-ahead every stream is cut into C chunks of J words that waves generate in
// parallel: chunk c starts from the state c*J words past the seed, W_c[j] = XOR_{i: g_i} x_{i+j}
// with g = x^(cJ) mod phi (mt_poly.h; the host computes and caches the polynomials), x the stream's
// word sequence from its seed.  Numpy's draws are accepted or rejected one by one, so a first pass
// counts the accepted draws of every chunk, a scan turns the counts into the chunks' first output
// positions, and a second pass regenerates each chunk and places its accepted draws there.  The last
// chunk runs on until the stream has its n draws, so an underestimated C costs time, never bits.
constexpr int kMtSeqWords = 624 * 34;  // x_0 .. x_21215 >= 19937 + 623 words: every x_{i+j} of a jump

// x_0 .. x_{kMtSeqWords-1} of every stream (one wave each), to global memory
__global__ void __launch_bounds__(64) k_mt_seq(const uint32_t* __restrict__ seeds, uint32_t* __restrict__ seq) {
  __shared__ uint32_t mt[2][kMtN];
  const int lane = threadIdx.x;
  uint32_t* out = seq + (size_t)blockIdx.x * kMtSeqWords;
  if (lane == 0) {
    uint32_t x = seeds[blockIdx.x];
    for (int i = 0; i < kMtN; ++i) {
      mt[0][i] = x;
      x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)(i + 1);
    }
  }
  __syncthreads();
  int cur = 0;
  for (int b = 0; b < kMtSeqWords / kMtN; ++b) {
    for (int i = lane; i < kMtN; i += 64) out[b * kMtN + i] = mt[cur][i];
    if (b + 1 == kMtSeqWords / kMtN) break;
    mt_next_block(mt[cur], mt[cur ^ 1], lane);
    cur ^= 1;
  }
}

// W_c for chunk c = blockIdx.x + 1 of stream blockIdx.y: the correlation of the stream's sequence
// with the set bits of x^(cJ) mod phi, given by the host as two lists of bit positions, even then
// odd, each stored as the index of the aligned word pair it reads, floor(i / 2) (row of `stride` int32
// per chunk: E, O, 0, 0, E even, O odd; E and O padded to multiples of 32 with the zero-window
// positions kMtPadEven / kMtPadOdd).  The sequence sits in LDS (85 KB, 8-byte aligned); the positions
// are read by scalar loads.  Word pairs: for an even position i thread u reads the aligned pair
// (x_{i+2u}, x_{i+2u+1}) -> words 2u, 2u+1; for an odd i the aligned pair (x_{i+2u-1}, x_{i+2u}) ->
// words 2u-1, 2u: one ds_read_b64 per thread and position (256 B/clk) instead of two 4-byte reads.
// 640 threads = two groups of 320 (313 needed: u = 0..312), each taking half of every list; the
// halves, then the neighbour's odd pair, are combined through LDS at the end.
constexpr int kMtJumpSeq = 19937 + 624;  // words of the sequence a jump reads (x_0 .. x_20560)
constexpr int kMtPadEven = 20562;        // pad positions: their windows (the next 626 words) are zero
constexpr int kMtPadOdd = 20563;
constexpr int kMtJumpLds = 20562 + 640;  // LDS words of the sequence + the zero region
constexpr int kMtJumpThreads = 640;
__global__ void __launch_bounds__(kMtJumpThreads) k_mt_jump(const uint32_t* __restrict__ seq,
                                                            const int32_t* __restrict__ pos, int stride, int chunks,
                                                            uint32_t* __restrict__ windows) {
  typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
  __shared__ __attribute__((aligned(16))) uint32_t xs[kMtJumpLds];
  __shared__ u32x2v cmb[2][320];
  const int tid = threadIdx.x;
  const int grp = __builtin_amdgcn_readfirstlane(tid / 320), u = tid % 320;  // 320 = 5 whole waves
  const int s = blockIdx.y, c = blockIdx.x + 1;
  {  // the sequence into LDS: 16-byte loads, all of a thread's in flight before its stores
    const u32x4* src4 = (const u32x4*)(seq + (size_t)s * kMtSeqWords);  // 84,864-byte rows: aligned
    u32x4* xs4 = (u32x4*)xs;
    constexpr int NV = kMtJumpLds / 4, R = (NV + kMtJumpThreads - 1) / kMtJumpThreads;
    constexpr int NS = (kMtJumpSeq + 3) / 4;  // vectors holding sequence words (the last one partly)
    u32x4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int q = tid + r * kMtJumpThreads;
      v[r] = q < NS ? src4[q] : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int q = tid + r * kMtJumpThreads;
      if (q == NS - 1) {  // words past x_20560 are zero
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (4 * q + j >= kMtJumpSeq) v[r][j] = 0u;
      }
      if (q < NV) xs4[q] = v[r];
    }
  }
  __syncthreads();  // the sequence is in LDS
  const int32_t* row = pos + (size_t)(c - 1) * stride;
  const int E = row[0], O = row[1];
  const int32_t* lists = row + 4;
  u32x2v ae = {0u, 0u}, ao = {0u, 0u};
  const u32x2v* xp = (const u32x2v*)xs;  // the sequence as aligned word pairs
  // the two lists, one after the other; group g takes the g-th half of each
  for (int pass = 0; pass < 2; ++pass) {
    const int len = pass ? O : E;
    const int32_t* lp = lists + (pass ? E : 0);
    // positions by scalar loads (uniform addresses, 16 per s_load_dwordx16): no LDS cycles for them
    // (r03u interleaved A/B: 2.60-2.62 ms with the positions staged in LDS and read as broadcasts,
    // 2.53-2.54 ms this way)
    const int half = len / 2;  // a multiple of 16
    const int32_t* gp = lp + grp * half;
    u32x2v acc = {0u, 0u};
    for (int k = 0; k < half; k += 16) {
      int ii[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) ii[q] = gp[k + q];
#pragma unroll
      for (int q = 0; q < 16; ++q) acc ^= xp[ii[q] + u];  // aligned pair: ds_read_b64
    }
    if (pass) ao ^= acc;
    else ae ^= acc;
  }
  // combine the groups' halves, then words 2u = E.x ^ O.y and 2u + 1 = E.y ^ O(u+1).x
  __syncthreads();
  if (grp == 1) {
    cmb[0][u] = ae;
    cmb[1][u] = ao;
  }
  __syncthreads();
  if (grp == 0) {
    ae ^= cmb[0][u];
    ao ^= cmb[1][u];
  }
  __syncthreads();
  if (grp == 0) cmb[1][u] = ao;  // every thread's odd pair, for its left neighbour
  __syncthreads();
  if (grp == 0 && u < kMtN / 2) {
    uint32_t* out = windows + ((size_t)s * chunks + c) * kMtN;
    out[2 * u] = ae.x ^ ao.y;
    out[2 * u + 1] = ae.y ^ cmb[1][u + 1].x;
  }
}

// Pass 1 (PLACE = false): accepted draws of chunks 0 .. chunks-2 of every stream -> counts[s][c].
// Pass 2 (PLACE = true): chunk c stores its accepted draws, signed (p - v for a negative stream, 0
// stays 0), into the stream's plane from output position offs[s][c] on (the last chunk until the
// stream has n): plain coalesced stores, every position of a plane written exactly once (the planes
// replace k_mt_randint's uint64 atomics, which cost 4.8x the generation in this pass).
// Chunk 0 starts from the seeded state (x_0..x_623 of seq), chunk c > 0 from W_c; a chunk is
// jwords words = jwords / 624 blocks.
template <bool WIDE, bool PLACE>
__global__ void __launch_bounds__(64)
k_mt_chunk(const uint32_t* __restrict__ seq, const uint32_t* __restrict__ windows, int chunks, int64_t jwords,
           uint64_t rng, uint64_t mask, uint64_t p, int64_t n, const int8_t* __restrict__ signs,
           int64_t* __restrict__ counts, const int64_t* __restrict__ offs, void* __restrict__ planes, int64_t pstride) {
  using PT = typename std::conditional<WIDE, uint64_t, uint32_t>::type;
  PT* plane = (PT*)planes + (size_t)blockIdx.y * pstride;
  __shared__ uint32_t mt[2][kMtN];
  const int lane = threadIdx.x;
  const int c = blockIdx.x, s = blockIdx.y;
  const bool last = c == chunks - 1;
  int64_t count = PLACE ? offs[(size_t)s * chunks + c] : 0;
  if (PLACE && count >= n) return;  // every output position is taken by earlier chunks
  const uint32_t* w0 = c == 0 ? seq + (size_t)s * kMtSeqWords : windows + ((size_t)s * chunks + c) * kMtN;
  for (int i = lane; i < kMtN; i += 64) mt[0][i] = w0[i];
  __syncthreads();
  const bool neg = signs[s] < 0;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  constexpr int kVals = WIDE ? kMtN / 2 : kMtN;
  constexpr int kRounds = (kVals + 63) / 64;
  int cur = 0;
  const int64_t blocks = jwords / kMtN;
  for (int64_t b = 0; (PLACE && last) ? count < n : b < blocks; ++b) {
    mt_next_block(mt[cur], mt[cur ^ 1], lane);
    cur ^= 1;
    const uint32_t* w32 = mt[cur];
    uint64_t v[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const int w = r * 64 + lane;
      if (w < kVals) {
        if constexpr (WIDE) v[r] = (uint64_t)mt_temper(w32[2 * w]) << 32 | mt_temper(w32[2 * w + 1]);
        else v[r] = mt_temper(w32[w]);
        v[r] &= mask;
      } else {
        v[r] = ~0ull;
      }
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const bool ok = v[r] <= rng;
      const uint64_t bal = __ballot(ok);
      if constexpr (PLACE) {
        const int64_t pos = count + __popcll(bal & below);
        if (ok && pos < n) plane[pos] = (PT)((neg && v[r] != 0) ? p - v[r] : v[r]);
      }
      count += __popcll(bal);
    }
    if (PLACE && count >= n) break;
  }
  if (!PLACE && lane == 0) counts[(size_t)s * chunks + c] = count;
}

// total[e] = (first ? 0 : total[e]) + sum over the g planes of element e, mod p (planes hold values
// in [0, p), pstride elements apart, a multiple of 4: 32-bit planes are read as 16-byte vectors of
// four elements and summed in uint64, reduced once; 64-bit planes add modulo p one by one)
template <bool WIDE>
__global__ void __launch_bounds__(kBlock)
k_mt_fold_planes(const void* __restrict__ planes, int g, int64_t n, int64_t pstride, uint64_t p,
                 int64_t* __restrict__ total, int first) {
  if constexpr (WIDE) {
    for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += (int64_t)gridDim.x * kBlock) {
      uint64_t t = first ? 0 : (uint64_t)total[e];
      const uint64_t* pl = (const uint64_t*)planes + e;
      for (int s = 0; s < g; ++s) {
        t += __builtin_nontemporal_load(pl + (size_t)s * pstride);
        if (t >= p) t -= p;
      }
      total[e] = (int64_t)t;
    }
  } else {
    const int64_t nv = (n + 3) / 4;
    for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kBlock) {
      const int64_t e = 4 * v;
      uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
      const u32x4* pl = (const u32x4*)((const uint32_t*)planes + e);
      for (int s = 0; s < g; ++s) {
        const u32x4 x = __builtin_nontemporal_load(pl + (size_t)s * (pstride / 4));
        t0 += x[0];
        t1 += x[1];
        t2 += x[2];
        t3 += x[3];
      }
      const uint64_t tt[4] = {t0, t1, t2, t3};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (e + j >= n) break;
        uint64_t t = tt[j] % p;
        if (!first) {
          t += (uint64_t)total[e + j];
          if (t >= p) t -= p;
        }
        total[e + j] = (int64_t)t;
      }
    }
  }
}

// offs[s][c] = sum of counts[s][0..c-1] (exclusive scan over a stream's chunks)
__global__ void k_mt_scan(const int64_t* __restrict__ counts, int64_t* __restrict__ offs, int streams, int chunks) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= streams) return;
  int64_t run = 0;
  for (int c = 0; c < chunks; ++c) {
    offs[(size_t)s * chunks + c] = run;
    if (c < chunks - 1) run += counts[(size_t)s * chunks + c];
  }
}

}  // namespace

// ============================================================================================ ABI
extern "C" {

namespace {
int finite_sum_impl(fa_ctx* ctx, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                    const void* const* d_in, const void* const* d_mask, int64_t prime, int flags,
                    void* const* d_out_finite, int32_t q_bits, double scale, void* const* d_out_real,
                    void* hip_stream, int64_t sstr) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (k <= 0 || num_segments <= 0 || !seg_numel || !d_in)
    return fail(FA_ERR_INVALID, "fa_finite_sum: invalid arguments");
  if (prime <= 0) return fail(FA_ERR_INVALID, "fa_finite_sum: prime must be > 0");
  if (flags & ~(FA_FINITE_MOD_FIRST | FA_FINITE_MOD_EACH | FA_FINITE_MOD_END | FA_FINITE_REAL_F64))
    return fail(FA_ERR_INVALID, "fa_finite_sum: unknown flags 0x%x", flags);
  if (d_out_real && (q_bits < 0 || q_bits > 62)) return fail(FA_ERR_INVALID, "fa_finite_sum: q_bits must be in [0, 62]");
  int nseg = 0;
  int64_t tiles = 0;
  for (int s = 0; s < num_segments; ++s) {
    if (seg_numel[s] < 0) return fail(FA_ERR_INVALID, "segment %d has negative numel", s);
    if (seg_numel[s] == 0) continue;
    const bool fo = d_out_finite && d_out_finite[s], ro = d_out_real && d_out_real[s];
    if (!fo && !ro) return fail(FA_ERR_INVALID, "segment %d: no output", s);
    for (int i = 0; i < k; ++i)
      if (!d_in[(int64_t)s * k + i]) return fail(FA_ERR_INVALID, "segment %d client %d: input NULL", s, i);
    ++nseg;
    tiles += (seg_numel[s] + kTile - 1) / kTile;
  }
  if (nseg == 0) return FA_OK;
  if (tiles > 0x7FFFFFFFll) return fail(FA_ERR_INVALID, "too many tiles");
  const size_t seg_bytes = align16(sizeof(FSeg) * nseg);
  const size_t ptr_bytes = sizeof(void*) * (size_t)nseg * k;
  const size_t bytes = seg_bytes + ptr_bytes;
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  fa_ctx::Slot* slot = nullptr;
  int rc = acquire_slot(ctx, bytes, &slot);
  if (rc) return rc;
  char* h = (char*)slot->host;
  FSeg* hs = (FSeg*)h;
  const void** hp = (const void**)(h + seg_bytes);
  int j = 0;
  int64_t t0 = 0;
  for (int s = 0; s < num_segments; ++s) {
    const int64_t n = seg_numel[s];
    if (n == 0) continue;
    FSeg sg;
    sg.numel = n;
    sg.tile_start = t0;
    sg.ptr_base = j * k;
    sg.mask = d_mask ? (const long long*)d_mask[s] : nullptr;
    sg.out_fin = d_out_finite ? (long long*)d_out_finite[s] : nullptr;
    sg.out_real = d_out_real ? d_out_real[s] : nullptr;
    const uintptr_t ra = (flags & FA_FINITE_REAL_F64) ? 15u : 7u;
    bool aligned = (!sg.out_fin || al16(sg.out_fin)) && (!sg.out_real || ((uintptr_t)sg.out_real & ra) == 0);
    for (int i = 0; i < k; ++i) {
      const void* p = d_in[(int64_t)s * k + i];
      hp[(int64_t)j * k + i] = p;
      aligned = aligned && al16(p);
    }
    sg.aligned = (aligned && (!sg.mask || al16(sg.mask))) ? 1 : 0;
    if (sstr && !sg.aligned) return fail(FA_ERR_INVALID, "tiled inputs, mask and outputs must be aligned");
    hs[j] = sg;
    t0 += (n + kTile - 1) / kTile;
    ++j;
  }
  rc = stage(slot, bytes, st);
  if (rc) return rc;
  const char* dv = (const char*)slot->dev;
  const ModP mp = make_modp(prime);
  Dequant dq;
  dq.half = (double)(prime - 1) / 2.0;
  dq.pd = (double)prime;
  dq.inv_pow2q = std::ldexp(1.0, -q_bits);
  dq.scale = (float)scale;
  const dim3 grid((unsigned)tiles), blk(kBlock);
  if (flags & FA_FINITE_MOD_EACH)
    hipLaunchKernelGGL((k_finite_sum<true>), grid, blk, 0, st, (const FSeg*)dv, nseg,
                       (const void* const*)(dv + seg_bytes), k, flags, mp, dq, sstr);
  else
    hipLaunchKernelGGL((k_finite_sum<false>), grid, blk, 0, st, (const FSeg*)dv, nseg,
                       (const void* const*)(dv + seg_bytes), k, flags, mp, dq, sstr);
  FA_HIP(hipGetLastError());
  return release(slot, st);
}
}  // namespace

int fa_finite_sum(fa_ctx* ctx, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                  const void* const* d_in, const void* const* d_mask, int64_t prime, int flags,
                  void* const* d_out_finite, int32_t q_bits, double scale, void* const* d_out_real,
                  void* hip_stream) {
  return finite_sum_impl(ctx, num_segments, seg_numel, k, d_in, d_mask, prime, flags, d_out_finite, q_bits, scale,
                         d_out_real, hip_stream, 0);
}

int fa_finite_sum_tiled(fa_ctx* ctx, int64_t n, int32_t k, const void* const* d_in, int64_t tile_stride,
                        const void* d_mask, int64_t prime, int flags, void* d_out_finite, int32_t q_bits,
                        double scale, void* d_out_real, void* hip_stream) {
  if (n < 0) return fail(FA_ERR_INVALID, "n must be >= 0");
  if (tile_stride <= 0 || tile_stride % FA_TILE_BYTES)
    return fail(FA_ERR_INVALID, "tile_stride must be a positive multiple of %d (got %lld)", FA_TILE_BYTES,
                (long long)tile_stride);
  const void* masks[1] = {d_mask};
  void* fin[1] = {d_out_finite};
  void* real[1] = {d_out_real};
  return finite_sum_impl(ctx, 1, &n, k, d_in, d_mask ? masks : nullptr, prime, flags,
                         d_out_finite ? fin : nullptr, q_bits, scale, d_out_real ? real : nullptr, hip_stream,
                         tile_stride);
}

int fa_finite_quantize(fa_ctx* ctx, int dtype, int32_t num_segments, const int64_t* seg_numel,
                       const void* const* d_x, const void* const* d_mask, int64_t prime, int32_t q_bits,
                       void* const* d_out, void* hip_stream) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (num_segments <= 0 || !seg_numel || !d_x || !d_out) return fail(FA_ERR_INVALID, "fa_finite_quantize: invalid arguments");
  if (dtype != FA_DTYPE_F32 && dtype != FA_DTYPE_F64 && dtype != FA_DTYPE_I64)
    return fail(FA_ERR_DTYPE, "fa_finite_quantize: dtype %d not supported (F32, F64, I64)", dtype);
  if (prime <= 0) return fail(FA_ERR_INVALID, "fa_finite_quantize: prime must be > 0");
  if (q_bits < 0 || q_bits > 62) return fail(FA_ERR_INVALID, "fa_finite_quantize: q_bits must be in [0, 62]");
  const int V = dtype == FA_DTYPE_F32 ? 4 : 2;
  const int64_t tile_elems = (int64_t)kBlock * V;
  const bool mask = d_mask != nullptr;
  int nseg = 0;
  int64_t tiles = 0;
  for (int s = 0; s < num_segments; ++s) {
    if (seg_numel[s] < 0) return fail(FA_ERR_INVALID, "segment %d has negative numel", s);
    if (seg_numel[s] == 0) continue;
    if (!d_x[s] || !d_out[s] || (mask && !d_mask[s])) return fail(FA_ERR_INVALID, "segment %d: NULL pointer", s);
    ++nseg;
    tiles += (seg_numel[s] + tile_elems - 1) / tile_elems;
  }
  if (nseg == 0) return FA_OK;
  if (tiles > 0x7FFFFFFFll) return fail(FA_ERR_INVALID, "too many tiles");
  const size_t bytes = sizeof(QSeg) * nseg;
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  fa_ctx::Slot* slot = nullptr;
  int rc = acquire_slot(ctx, bytes, &slot);
  if (rc) return rc;
  QSeg* hs = (QSeg*)slot->host;
  int j = 0;
  int64_t t0 = 0;
  for (int s = 0; s < num_segments; ++s) {
    const int64_t n = seg_numel[s];
    if (n == 0) continue;
    const bool al = al16(d_x[s]) && al16(d_out[s]) && (!mask || al16(d_mask[s]));
    hs[j] = QSeg{n, t0, d_x[s], mask ? (const long long*)d_mask[s] : nullptr, (long long*)d_out[s], al ? 1 : 0};
    t0 += (n + tile_elems - 1) / tile_elems;
    ++j;
  }
  rc = stage(slot, bytes, st);
  if (rc) return rc;
  QParams qp;
  qp.pow2q_f = std::ldexp(1.0f, q_bits);
  qp.pf = (float)prime;
  qp.pow2q_d = std::ldexp(1.0, q_bits);
  qp.pd = (double)prime;
  qp.q = q_bits;
  const ModP mp = make_modp(prime);
  const QSeg* ds = (const QSeg*)slot->dev;
  const dim3 grid((unsigned)tiles), blk(kBlock);
#define FA_Q(DT)                                                                              \
  if (mask) hipLaunchKernelGGL((k_finite_quant<DT, true>), grid, blk, 0, st, ds, nseg, qp, mp); \
  else hipLaunchKernelGGL((k_finite_quant<DT, false>), grid, blk, 0, st, ds, nseg, qp, mp);
  switch (dtype) {
    case FA_DTYPE_F32: FA_Q(FA_DTYPE_F32); break;
    case FA_DTYPE_F64: FA_Q(FA_DTYPE_F64); break;
    default: FA_Q(FA_DTYPE_I64); break;
  }
#undef FA_Q
  FA_HIP(hipGetLastError());
  return release(slot, st);
}

int fa_lcc_decode(fa_ctx* ctx, int32_t rows, int32_t k, int64_t m, const int64_t* coef, const void* d_f,
                  int64_t prime, int64_t n_out, void* d_out, void* hip_stream) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (rows <= 0 || k <= 0 || m <= 0 || !coef || !d_f || !d_out)
    return fail(FA_ERR_INVALID, "fa_lcc_decode: invalid arguments");
  if (prime <= 0) return fail(FA_ERR_INVALID, "fa_lcc_decode: prime must be > 0");
  if (n_out < 0 || n_out > (int64_t)rows * m) return fail(FA_ERR_INVALID, "fa_lcc_decode: n_out must be in [0, rows*m]");
  if (n_out == 0) return FA_OK;
  const int rows_needed = (int)((n_out + m - 1) / m);
  const int64_t blocks = (m + kBlock - 1) / kBlock;
  if (blocks > 0x7FFFFFFFll) return fail(FA_ERR_INVALID, "too many columns");
  // float64 path precondition: coefficients in [0, p) and (p-1)^2 * k < 2^53
  bool f64 = (unsigned __int128)(prime - 1) * (unsigned __int128)(prime - 1) * (unsigned __int128)k <
             ((unsigned __int128)1 << 53);
  for (int64_t t = 0; f64 && t < (int64_t)rows_needed * k; ++t) f64 = coef[t] >= 0 && coef[t] < prime;
  const int passes = (rows_needed + kRBF - 1) / kRBF;
  const size_t i64_bytes = align16(sizeof(int64_t) * (size_t)rows_needed * k);
  const size_t f64_bytes = f64 ? align16(sizeof(double) * (size_t)passes * k * kRBF) : 0;
  const size_t redo_bytes = f64 ? sizeof(int) * (size_t)blocks : 0;
  const size_t bytes = i64_bytes + f64_bytes + redo_bytes;
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  fa_ctx::Slot* slot = nullptr;
  int rc = acquire_slot(ctx, bytes, &slot);
  if (rc) return rc;
  char* h = (char*)slot->host;
  memcpy(h, coef, sizeof(int64_t) * (size_t)rows_needed * k);
  if (f64) {
    double* cT = (double*)(h + i64_bytes);
    for (int ps = 0; ps < passes; ++ps)
      for (int i = 0; i < k; ++i)
        for (int r = 0; r < kRBF; ++r) {
          const int j = ps * kRBF + r;
          cT[((int64_t)ps * k + i) * kRBF + r] = j < rows_needed ? (double)coef[(int64_t)j * k + i] : 0.0;
        }
  }
  rc = stage(slot, bytes, st);
  if (rc) return rc;
  char* dv = (char*)slot->dev;
  const ModP mp = make_modp(prime);
  if (f64 && ctx->variant != 1) {  // variant 1 forces the int64 path (A/B and test hook)
    int* redo = (int*)(dv + i64_bytes + f64_bytes);
    FA_HIP(hipMemsetAsync(redo, 0, redo_bytes, st));
    hipLaunchKernelGGL(k_lcc_decode_f64, dim3((unsigned)blocks), dim3(kBlock), 0, st, (const double*)(dv + i64_bytes),
                       rows_needed, k, m, (const long long*)d_f, n_out, (long long*)d_out, mp, redo);
    hipLaunchKernelGGL(k_lcc_decode, dim3((unsigned)blocks), dim3(kBlock), 0, st, (const long long*)dv,
                       rows_needed, k, m, (const long long*)d_f, n_out, (long long*)d_out, mp, (const int*)redo);
  } else {
    hipLaunchKernelGGL(k_lcc_decode, dim3((unsigned)blocks), dim3(kBlock), 0, st, (const long long*)dv,
                       rows_needed, k, m, (const long long*)d_f, n_out, (long long*)d_out, mp, (const int*)nullptr);
  }
  FA_HIP(hipGetLastError());
  return release(slot, st);
}


}  // extern "C"

namespace {
// FA_MT_JUMP=0: every stream sequential (k_mt_randint); FA_MT_JUMP_LOG2=k: chunks of 624 << k words
bool mt_jump_enabled() {
  const char* e = getenv("FA_MT_JUMP");
  return !(e && e[0] == '0');
}
// chunk size J = 624 << log2: about 2,048 chunk waves over all streams (8 per CU), in [624 << 2, 624 << 14]
int mt_jump_log2(double exp_words, int streams) {
  const char* e = getenv("FA_MT_JUMP_LOG2");
  if (e) {
    const int v = atoi(e);
    return v < 0 ? 0 : v > 20 ? 20 : v;
  }
  const double per = exp_words * std::max(1, streams) / (624.0 * 2048.0);
  int k = 2;
  while (k < 14 && (double)(1ll << (k + 1)) <= per) ++k;
  return k;
}

// The set-bit positions of x^(cJ) mod phi, c = 1..count, on the device (ctx->mt_poly_dev; one row
// of `stride` int32 per chunk: E, O, 0, 0, the E even positions, the O odd ones, each list padded to a
// multiple of 32 with kMtPadEven / kMtPadOdd; stride a multiple of 4: every list 16-byte aligned).  Host polynomials are cached per J (mt_poly.h); the device table is rebuilt
// only when J or the count grows.
int mt_jump_tables(fa_ctx* ctx, uint64_t J, int count, hipStream_t st) {
  if (ctx->mt_poly_dev && ctx->mt_poly_J == J && ctx->mt_poly_count >= count) return FA_OK;
  if (fa_mt::charpoly().empty()) return fail(FA_ERR_INVALID, "fa_mt_randint_sum: MT19937 characteristic polynomial not found");
  const std::vector<fa_mt::Poly> g = fa_mt::jump_polys(J, count);
  std::vector<std::vector<int32_t>> ev((size_t)count), od((size_t)count);
  int stride = 0;
  for (int c = 0; c < count; ++c) {
    for (int i = 0; i < fa_mt::kDeg; ++i)
      if (fa_mt::get_bit(g[(size_t)c], i)) (i & 1 ? od : ev)[(size_t)c].push_back(i >> 1);  // pair index
    while (ev[(size_t)c].size() % 32) ev[(size_t)c].push_back(kMtPadEven >> 1);
    while (od[(size_t)c].size() % 32) od[(size_t)c].push_back(kMtPadOdd >> 1);
    stride = std::max<int>(stride, 4 + (int)(ev[(size_t)c].size() + od[(size_t)c].size()));  // 4 + a multiple of 32
  }
  std::vector<int32_t> tab((size_t)count * stride, 0);
  for (int c = 0; c < count; ++c) {
    int32_t* r = &tab[(size_t)c * stride];
    r[0] = (int32_t)ev[(size_t)c].size();
    r[1] = (int32_t)od[(size_t)c].size();
    std::copy(ev[(size_t)c].begin(), ev[(size_t)c].end(), r + 4);
    std::copy(od[(size_t)c].begin(), od[(size_t)c].end(), r + 4 + ev[(size_t)c].size());
  }
  FA_HIP(hipStreamSynchronize(st));  // a previous table may still be read by queued kernels
  if (ctx->mt_live) FA_HIP(hipEventSynchronize(ctx->mt_ev));  // ... also on another stream
  if (ctx->mt_poly_dev) FA_HIP(hipFree(ctx->mt_poly_dev));
  ctx->mt_poly_dev = nullptr;
  ctx->mt_poly_count = 0;
  if (hipMalloc(&ctx->mt_poly_dev, tab.size() * sizeof(int32_t)) != hipSuccess)
    return fail(FA_ERR_NOMEM, "fa_mt_randint_sum: jump table allocation failed");
  FA_HIP(hipMemcpy(ctx->mt_poly_dev, tab.data(), tab.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  ctx->mt_poly_J = J;
  ctx->mt_poly_count = count;
  ctx->mt_poly_stride = stride;
  return FA_OK;
}

// device bytes for the per-stream planes of one group (FA_MT_PLANE_MB, default 2 GiB)
uint64_t mt_plane_budget() {
  const char* e = getenv("FA_MT_PLANE_MB");
  const long long mb = e ? atoll(e) : 2048;
  return (uint64_t)std::max<long long>(1, mb) << 20;
}

// >= bytes of device work space in ctx->mt_dev (grown, never shrunk)
int mt_work(fa_ctx* ctx, size_t bytes, hipStream_t st) {
  if (ctx->mt_cap >= bytes) return FA_OK;
  FA_HIP(hipStreamSynchronize(st));
  if (ctx->mt_live) FA_HIP(hipEventSynchronize(ctx->mt_ev));
  if (ctx->mt_dev) FA_HIP(hipFree(ctx->mt_dev));
  ctx->mt_dev = nullptr;
  ctx->mt_cap = 0;
  if (hipMalloc(&ctx->mt_dev, bytes) != hipSuccess) return fail(FA_ERR_NOMEM, "fa_mt_randint_sum: %zu bytes of work space", bytes);
  ctx->mt_cap = bytes;
  return FA_OK;
}
}  // namespace

extern "C" {

size_t fa_mt_randint_sum_scratch_bytes(int64_t n) { return n > 0 ? sizeof(uint64_t) * (size_t)n : 0; }

int fa_mt_randint_sum(fa_ctx* ctx, int32_t num_streams, const uint32_t* seeds, const int8_t* signs, int64_t prime,
                      int64_t n, void* d_out, void* d_scratch, size_t scratch_bytes, void* hip_stream) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (num_streams < 0 || n < 0 || prime <= 0 || (num_streams > 0 && (!seeds || !signs)) || (n > 0 && !d_out))
    return fail(FA_ERR_INVALID, "fa_mt_randint_sum: invalid arguments");
  if (n > 0 && (!d_scratch || scratch_bytes < fa_mt_randint_sum_scratch_bytes(n)))
    return fail(FA_ERR_INVALID, "fa_mt_randint_sum: scratch must hold %zu bytes", fa_mt_randint_sum_scratch_bytes(n));
  for (int s = 0; s < num_streams; ++s)
    if (signs[s] != 1 && signs[s] != -1)
      return fail(FA_ERR_INVALID, "fa_mt_randint_sum: sign %d of stream %d", signs[s], s);
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  if (n == 0) return FA_OK;
  const uint64_t p = (uint64_t)prime, rng = p - 1;
  uint64_t mask = rng;
  for (int sh = 1; sh < 64; sh <<= 1) mask |= mask >> sh;
  const bool wide = rng > 0xFFFFFFFFull;
  FA_HIP(hipMemsetAsync(d_out, 0, sizeof(int64_t) * (size_t)n, st));
  if (num_streams == 0 || rng == 0) return FA_OK;  // randint(0, 1) draws nothing and is all zeros
  // streams per batch: a batch's sum of values in [0, p) must not wrap 64 bits
  const uint64_t per = std::min<uint64_t>((uint64_t)num_streams, UINT64_MAX / rng);
  const size_t seed_b = align16(sizeof(uint32_t) * num_streams);
  const size_t tab = seed_b + align16((size_t)num_streams);
  const unsigned fold_blocks = (unsigned)std::min<int64_t>((n + kBlock - 1) / kBlock, 4096);
  // jump-ahead: C chunks of J words per stream when the stream is long enough for >= 2 of them
  const double exp_words = (double)n * (wide ? 2.0 : 1.0) * ((double)mask + 1.0) / ((double)rng + 1.0);
  // streams per group: their planes (n values each) within the plane budget; the chunk size is chosen
  // for the streams of one group (the groups run one after another)
  const size_t es = wide ? 8 : 4;
  const uint64_t G = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)num_streams, mt_plane_budget() / (((uint64_t)n + 3) / 4 * 4 * es)));
  const uint64_t J = 624ull << mt_jump_log2(exp_words, (int)G);
  const int C = mt_jump_enabled() ? (int)std::min<double>(std::floor(exp_words / (double)J), 4096.0) : 0;
  const size_t seq_b = align16(sizeof(uint32_t) * kMtSeqWords * G), win_b = align16(sizeof(uint32_t) * kMtN * C * G);
  const int64_t pstride = (n + 3) / 4 * 4;  // plane stride: every plane 16-byte aligned
  const size_t cnt_b = align16(sizeof(int64_t) * C * G), pl_b = (size_t)G * pstride * es;
  int rc;
  if (C >= 2) {  // everything that can fail before the staging slot is taken (a taken slot is always released)
    rc = mt_jump_tables(ctx, J, C - 1, st);
    if (rc) return rc;
    rc = mt_work(ctx, seq_b + win_b + 2 * cnt_b + pl_b, st);
    if (rc) return rc;
    if (!ctx->mt_ev && hipEventCreateWithFlags(&ctx->mt_ev, hipEventDisableTiming) != hipSuccess) {
      ctx->mt_ev = nullptr;
      return fail(FA_ERR_HIP, "fa_mt_randint_sum: hipEventCreate failed");
    }
  }
  fa_ctx::Slot* slot = nullptr;
  rc = acquire_slot(ctx, tab, &slot);
  if (rc) return rc;
  char* h = (char*)slot->host;
  memcpy(h, seeds, sizeof(uint32_t) * num_streams);
  memcpy(h + seed_b, signs, (size_t)num_streams);
  rc = stage(slot, tab, st);
  if (rc) return rc;
  const uint32_t* dseeds = (const uint32_t*)slot->dev;
  const int8_t* dsigns = (const int8_t*)((const char*)slot->dev + seed_b);
  if (C >= 2) {
    // the work space is shared by every call on this ctx: a previous call queued on another stream
    // must be done with it before these kernels overwrite it
    if (ctx->mt_live && hipStreamWaitEvent(st, ctx->mt_ev, 0) != hipSuccess) {
      (void)release(slot, st);
      return fail(FA_ERR_HIP, "fa_mt_randint_sum: hipStreamWaitEvent failed");
    }
    char* w = (char*)ctx->mt_dev;
    uint32_t* dseq = (uint32_t*)w;
    uint32_t* dwin = (uint32_t*)(w + seq_b);
    int64_t* dcnt = (int64_t*)(w + seq_b + win_b);
    int64_t* doff = (int64_t*)(w + seq_b + win_b + cnt_b);
    void* dpl = w + seq_b + win_b + 2 * cnt_b;
    const int32_t* dpos = (const int32_t*)ctx->mt_poly_dev;
    for (uint64_t s0 = 0; s0 < (uint64_t)num_streams; s0 += G) {
      const unsigned b = (unsigned)std::min<uint64_t>(G, (uint64_t)num_streams - s0);
      hipLaunchKernelGGL(k_mt_seq, dim3(b), dim3(64), 0, st, dseeds + s0, dseq);
      hipLaunchKernelGGL(k_mt_jump, dim3(C - 1, b), dim3(kMtJumpThreads), 0, st, dseq, dpos, ctx->mt_poly_stride, C, dwin);
      if (wide) {
        hipLaunchKernelGGL((k_mt_chunk<true, false>), dim3(C - 1, b), dim3(64), 0, st, dseq, dwin, C, (int64_t)J, rng,
                           mask, p, n, dsigns + s0, dcnt, (const int64_t*)nullptr, dpl, pstride);
        hipLaunchKernelGGL(k_mt_scan, dim3((b + 63) / 64), dim3(64), 0, st, dcnt, doff, (int)b, C);
        hipLaunchKernelGGL((k_mt_chunk<true, true>), dim3(C, b), dim3(64), 0, st, dseq, dwin, C, (int64_t)J, rng,
                           mask, p, n, dsigns + s0, dcnt, (const int64_t*)doff, dpl, pstride);
        hipLaunchKernelGGL((k_mt_fold_planes<true>), dim3(fold_blocks), dim3(kBlock), 0, st, (const void*)dpl, (int)b,
                           n, pstride, p, (int64_t*)d_out, s0 == 0 ? 1 : 0);
      } else {
        hipLaunchKernelGGL((k_mt_chunk<false, false>), dim3(C - 1, b), dim3(64), 0, st, dseq, dwin, C, (int64_t)J,
                           rng, mask, p, n, dsigns + s0, dcnt, (const int64_t*)nullptr, dpl, pstride);
        hipLaunchKernelGGL(k_mt_scan, dim3((b + 63) / 64), dim3(64), 0, st, dcnt, doff, (int)b, C);
        hipLaunchKernelGGL((k_mt_chunk<false, true>), dim3(C, b), dim3(64), 0, st, dseq, dwin, C, (int64_t)J,
                           rng, mask, p, n, dsigns + s0, dcnt, (const int64_t*)doff, dpl, pstride);
        hipLaunchKernelGGL((k_mt_fold_planes<false>), dim3(fold_blocks), dim3(kBlock), 0, st, (const void*)dpl,
                           (int)b, n, pstride, p, (int64_t*)d_out, s0 == 0 ? 1 : 0);
      }
    }
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipEventRecord(ctx->mt_ev, st);
    if (e != hipSuccess) {
      (void)release(slot, st);
      return fail(FA_ERR_HIP, "fa_mt_randint_sum: %s", hipGetErrorString(e));
    }
    ctx->mt_live = true;
    return release(slot, st);
  }
  if (hipMemsetAsync(d_scratch, 0, sizeof(uint64_t) * (size_t)n, st) != hipSuccess) {
    (void)release(slot, st);
    return fail(FA_ERR_HIP, "fa_mt_randint_sum: hipMemsetAsync of the scratch failed");
  }
  int first = 1;
  for (uint64_t s0 = 0; s0 < (uint64_t)num_streams; s0 += per) {
    const unsigned b = (unsigned)std::min<uint64_t>(per, (uint64_t)num_streams - s0);
    if (wide)
      hipLaunchKernelGGL(k_mt_randint<true>, dim3(b), dim3(64), 0, st, dseeds + s0, dsigns + s0, rng, mask, p, n,
                         (unsigned long long*)d_scratch);
    else
      hipLaunchKernelGGL(k_mt_randint<false>, dim3(b), dim3(64), 0, st, dseeds + s0, dsigns + s0, rng, mask, p, n,
                         (unsigned long long*)d_scratch);
    hipLaunchKernelGGL(k_mt_fold, dim3(fold_blocks), dim3(kBlock), 0, st, (unsigned long long*)d_scratch,
                       (int64_t*)d_out, n, p, first);
    first = 0;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    (void)release(slot, st);
    return fail(FA_ERR_HIP, "fa_mt_randint_sum: %s", hipGetErrorString(e));
  }
  return release(slot, st);
}

}  // extern "C"
