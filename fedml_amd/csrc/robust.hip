// robust.hip -- MI355X (gfx950) kernels + C ABI of the robust-aggregation family
// (include/fedagg_robust.h): coordinate-wise median over the clients and Krum's pairwise
// squared distances.
//
// Coordinate-wise median (k_median): torch.median over the client axis is a SELECTION, so the
// result is one of the inputs, bit for bit.  One lane owns one coordinate: it loads the K client
// values (all loads in flight at once), maps them to order-preserving uint32 keys (unsigned order
// == numeric order, -0.0 just below +0.0), pads to B = K rounded up to 8 with low/high sentinels
// that put the lower median at rank (B-1)/2, and selects that rank with a pruned odd-even merge
// network (median_nets.h: 283 min/max for B = 32, 1,233 for B = 72, 2,299 for B = 128, vs 480 /
// 3,584 / 3,584 for a full bitonic sort of the next power of two).  ATen's exact rules are kept: a NaN anywhere in the column returns the FIRST NaN;
// among equal values the client index decides, which only matters for +-0 -- both cases (a NaN
// seen, or a zero selected) take a short in-order rescan of the column.
// K <= 128 runs the network; larger K and float64 a rank-counting kernel (O(K^2) per coordinate).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "fa_internal.h"
#include "fedagg_robust.h"
#include "median_nets.h"

using namespace fa_detail;

namespace {


// Raw element loads in the global address space (global_load_*: vmcnt only).  Generic (flat)
// loads also count in lgkmcnt, so every s_waitcnt for the next scalar pointer load drained them and
// the per-client loads of a column ran one HBM round trip at a time.
template <typename T>
__device__ __forceinline__ T gld(const void* p, int64_t e) {
  return ((const __attribute__((address_space(1))) T*)p)[e];
}

// non-temporal: each client element is read once (K = 16 / 32 medians 6% / 3% faster)
template <typename T>
__device__ __forceinline__ T gld_nt(const void* p, int64_t e) {
  return __builtin_nontemporal_load((const __attribute__((address_space(1))) T*)p + e);
}

// uniform base + 32-bit byte offset (zero-extended): selects the saddr form of global_load
template <typename T>
__device__ __forceinline__ T gld_nt_off(const void* p, unsigned off) {
  return __builtin_nontemporal_load((const __attribute__((address_space(1))) T*)((const char*)p + off));
}

template <int DT> struct MedT;
template <> struct MedT<FA_DTYPE_F32> {
  using S = unsigned;
  static constexpr int kBytes = 4;
  __device__ static float load(const void* p, int64_t e) { return gld_nt<float>(p, e); }
  __device__ static float load_off(const void* p, unsigned off) { return gld_nt_off<float>(p, off); }
  __device__ static void store(void* p, int64_t e, float v) { ((float*)p)[e] = v; }
  __device__ static void store_bits(void* p, int64_t e, const void* src) { ((unsigned*)p)[e] = ((const unsigned*)src)[e]; }
  __device__ static void store_bits_off(void* p, int64_t e, const void* src, unsigned off) {
    ((unsigned*)p)[e] = gld_nt_off<unsigned>(src, off);
  }
};
template <> struct MedT<FA_DTYPE_BF16> {
  static constexpr int kBytes = 2;
  __device__ static float load(const void* p, int64_t e) {
    return __uint_as_float((unsigned)gld_nt<unsigned short>(p, e) << 16);
  }
  __device__ static float load_off(const void* p, unsigned off) {
    return __uint_as_float((unsigned)gld_nt_off<unsigned short>(p, off) << 16);
  }
  __device__ static void store(void* p, int64_t e, float v) {
    ((unsigned short*)p)[e] = (unsigned short)(__float_as_uint(v) >> 16);  // exact: v came from bf16
  }
  __device__ static void store_bits(void* p, int64_t e, const void* src) {
    ((unsigned short*)p)[e] = ((const unsigned short*)src)[e];
  }
  __device__ static void store_bits_off(void* p, int64_t e, const void* src, unsigned off) {
    ((unsigned short*)p)[e] = gld_nt_off<unsigned short>(src, off);
  }
};
template <> struct MedT<FA_DTYPE_F16> {
  static constexpr int kBytes = 2;
  __device__ static float load(const void* p, int64_t e) {
    return (float)__builtin_bit_cast(_Float16, gld_nt<unsigned short>(p, e));
  }
  __device__ static float load_off(const void* p, unsigned off) {
    return (float)__builtin_bit_cast(_Float16, gld_nt_off<unsigned short>(p, off));
  }
  __device__ static void store(void* p, int64_t e, float v) {
    ((unsigned short*)p)[e] = __builtin_bit_cast(unsigned short, (_Float16)v);  // exact: v came from f16
  }
  __device__ static void store_bits(void* p, int64_t e, const void* src) {
    ((unsigned short*)p)[e] = ((const unsigned short*)src)[e];
  }
  __device__ static void store_bits_off(void* p, int64_t e, const void* src, unsigned off) {
    ((unsigned short*)p)[e] = gld_nt_off<unsigned short>(src, off);
  }
};

// order-preserving key of a float (unsigned order == numeric order for non-NaN values; -0.0 sorts
// just below +0.0, which the zero rescan below accounts for)
__device__ __forceinline__ unsigned fkey(float x) {
  const unsigned u = __float_as_uint(x);
  return u ^ ((unsigned)((int)u >> 31) | 0x80000000u);
}
constexpr unsigned kPosZeroKey = 0x80000000u, kNegZeroKey = 0x7FFFFFFFu;
__device__ __forceinline__ float fkey_inv(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

struct MSeg {
  int64_t numel;
  int64_t tile_start;
  void* out;
  int64_t tstride;  // 0: flat client segments; > 0: tile-interleaved inputs, bytes between a client's tiles
  int32_t ptr_base;
  int32_t pad;
};
static_assert(sizeof(MSeg) == 40, "MSeg layout");

// Byte offset of a workgroup's first column e0 from a client's segment start: flat segments e0 * SZ;
// tiled inputs (tstride > 0, FA_TILE_BYTES tiles of E elements; fedml_amd/arena.py tiled=True)
// (e0 / E) * tstride + (e0 % E) * SZ.  A workgroup's columns never straddle a tile (its column count
// divides E), so a client's element is `uniform base (SGPRs: pointer + this offset) + the lane's
// 32-bit byte offset` in both layouts -- every load keeps global_load's saddr form, for any segment size.
template <int SZ>
__device__ __forceinline__ int64_t col_base(int64_t e0, int64_t tstride) {
  constexpr int64_t E = FA_TILE_BYTES / SZ;
  return tstride ? (e0 / E) * tstride + (e0 % E) * SZ : e0 * SZ;
}
__device__ __forceinline__ const void* at(const void* p, int64_t ub) { return (const char*)p + ub; }

// Rare cases, resolved by an in-order rescan of the column: a NaN anywhere -> ATen returns the
// FIRST NaN; a zero selected -> the selected rank r falls in the block of (equal) zeros, which ATen
// orders by client index -> the (r - #negatives)-th zero in client order.
// Client i's element of this lane: at(in[i], ub) + boff (col_base); the result goes to out[e].
template <int DT>
__device__ __forceinline__ void store_rare(const void* const* in, int64_t ub, unsigned boff, int k, int64_t e, int r,
                                           bool nan, void* out) {
  if (nan) {
    for (int i = 0; i < k; ++i) {
      const float x = MedT<DT>::load_off(at(in[i], ub), boff);
      if (x != x) { MedT<DT>::store_bits_off(out, e, at(in[i], ub), boff); return; }
    }
  }
  int negc = 0;
  for (int i = 0; i < k; ++i) negc += MedT<DT>::load_off(at(in[i], ub), boff) < 0.0f;
  int seen = 0;
  for (int i = 0; i < k; ++i) {
    const float x = MedT<DT>::load_off(at(in[i], ub), boff);
    if (x == 0.0f) {
      if (seen == r - negc) { MedT<DT>::store_bits_off(out, e, at(in[i], ub), boff); return; }
      ++seen;
    }
  }
}

// One lane per coordinate.  Loads: the column's K client pointers first (scalar loads), then all
// B element loads (clamped, unconditional) before any is consumed.  Keys: the K real keys, then
// L = (B-1)/2 - (K-1)/2 low sentinels (0, below every non-NaN key) and high sentinels
// (0xFFFFFFFF) for the rest, so the lower median of the reals is rank (B-1)/2 of all B keys --
// which the pruned network select_mid<B> (median_nets.h) computes.  B = K rounded up to 8.
// One coordinate: all B element loads (clamped to the column's last coordinate when !live, so every
// load is unconditional) before any is consumed, keys + sentinels, the network, the rare-case rescan
// (k_median_pk's odd last coordinate).
template <int DT, int B>
__device__ __forceinline__ void median_col(const void* const* in, int64_t ub, unsigned boff, int k, int64_t e,
                                           bool live, void* out) {
  const void* p[B];
#pragma unroll
  for (int i = 0; i < B; ++i) p[i] = at(in[min(i, k - 1)], ub);
  float x[B];
#pragma unroll
  for (int i = 0; i < B; ++i) x[i] = MedT<DT>::load_off(p[i], boff);  // clamped: every load unconditional
  const int lo_end = k + (B - 1) / 2 - ((k - 1) >> 1);          // sentinels [k, lo_end) are low
  unsigned key[B];
  bool nan = false;
#pragma unroll
  for (int i = 0; i < B; ++i) {
    nan = nan || (i < k && x[i] != x[i]);
    key[i] = i < k ? fkey(x[i]) : (i < lo_end ? 0u : 0xFFFFFFFFu);
  }
  const unsigned kr = select_mid<B>(key);
  if (!live) return;
  const int r = (k - 1) >> 1;
  if (nan || kr == kPosZeroKey || kr == kNegZeroKey) store_rare<DT>(in, ub, boff, k, e, r, nan, out);
  else MedT<DT>::store(out, e, fkey_inv(kr));
}

// Branch-free form (r02), used whenever every segment's byte size fits in 32 bits: the generic
// form below compiles `i < k ? key : sentinel` and `nan || ...` (k a runtime value) into an
// exec-mask branch with its own s_waitcnt per client -- ~3,000 scalar and branch instructions ahead
// of B = 128's 2,175 min/max -- and keeps a 64-bit VGPR address per client (B = 128: 158 VGPRs).
// Here the sentinels are uniform selects (no branch) and every load is `uniform base (SGPRs) + ONE
// shared 32-bit byte offset` (global_load ... saddr).  Measured (r02j): K = 128 1.58 -> 1.45 ms,
// K = 96 1.11 -> 0.88, K = 64 0.62 -> 0.59, K = 32 0.278 -> 0.272 ms; bit-exact (same network).
// EXACT (k == B, no sentinels): the selects are dropped at compile time (K = 128: 1.53 -> 1.45 ms).
// Float keys (r03): the network runs on the loaded floats with IEEE 754-2019 minimum / maximum
// (median_nets.h, v_minimum3_f32 / v_maximum3_f32): their order is the uint32 keys' order on every
// non-NaN value (-0 < +0 included), so the same bits are selected, and a NaN anywhere in the column
// makes the selected value NaN (every input reaches the selected output) -- no per-key conversion
// or NaN test (5-6 VALU a key in the uint32-key form, commit 9aaf2ea).  Sentinels are -inf / +inf (a
// tie with a real infinity selects the same bits).  Interleaved A/B (profiles/r03ac): K = 64 0.606 ->
// 0.535 ms, K = 32 unchanged.
template <int DT, int B, bool EXACT, int W = (B > 64 ? 2 : (B > 56 ? 3 : (B > 32 ? 4 : 5)))>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W)))
k_median_off(const MSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k) {
  if constexpr (EXACT) k = B;
  const int64_t tile = blockIdx.x;
  const MSeg sg = segs[nseg > 1 ? find_seg(segs, nseg, tile) : 0];
  const int64_t e0 = (tile - sg.tile_start) * kBlock, e = e0 + threadIdx.x;
  const bool live = e < sg.numel;
  const int64_t ec = live ? e : sg.numel - 1;
  const void* const* in = ptrs + sg.ptr_base;
  const int64_t ub = col_base<MedT<DT>::kBytes>(e0, sg.tstride);
  const unsigned boff = (unsigned)(ec - e0) * (unsigned)MedT<DT>::kBytes;
  const int lo_end = k + (B - 1) / 2 - ((k - 1) >> 1);  // sentinels [k, lo_end) low, [lo_end, B) high
  float x[B];
#pragma unroll
  for (int i = 0; i < B; ++i) x[i] = MedT<DT>::load_off(at(in[min(i, k - 1)], ub), boff);
  if constexpr (!EXACT) {
#pragma unroll
    for (int i = 0; i < B; ++i) x[i] = i < k ? x[i] : (i < lo_end ? -__builtin_inff() : __builtin_inff());
  }
  const float kr = select_mid<B>(x);
  if (!live) return;
  const int r = (k - 1) >> 1;
  const bool nan = kr != kr;
  if (nan || kr == 0.0f) store_rare<DT>(in, ub, boff, k, e, r, nan, sg.out);
  else MedT<DT>::store(sg.out, e, kr);
}

// Two lanes per column, K in (64, 128] (r02).  k_median_off at B = 128 holds 128 keys per lane:
// 256 VGPRs with spills, 2 waves per SIMD (1 wave without spills was slower still: K = 128 1.49 ->
// 1.99 ms), so HBM latency is exposed between the network's phases.  Here a column's B = 2N keys
// (B = K rounded up to 8, as k_median_off) are split between two lanes of different waves: waves 0-1
// of the workgroup hold clients 0..N-1 of 128 columns, waves 2-3 clients N..2N-1 of the same columns
// (the half index is wave-uniform, so every load keeps the SGPR-base + 32-bit-offset form).  Each lane
// sorts its N keys (SortNet<N>, median_nets.h: 1,086 min/max for N = 64, the same work as half of
// B = 128's pruned selection network), the upper lanes hand their sorted keys to the lower lanes
// through LDS, and the lower median -- rank N-1 of the 2N keys -- is max_j min(A[j], C[N-1-j]) (the N
// pairwise minima of a sorted A and a reversed sorted C are the N smallest keys).  Padding as
// k_median_off, all of it in the upper half, sentinels -inf / +inf.  Float keys as k_median_off (r03):
// a NaN in either half turns that half's sorted keys NaN and so the merged value (r02's uint32 keys
// found a NaN as a sorted key outside [key(-inf), key(+inf)]; K = 100 1.009 -> 0.955 ms, K = 128
// within 1 %, profiles/r03ac).  N keys + the merge fit 128 VGPRs
// (4 waves per SIMD).  Same keys and rare-case rules as k_median_off: bit-exact.
constexpr int k2lCols = kBlock / 2;  // columns per workgroup
#ifndef MEDIAN_2L_W
#define MEDIAN_2L_W (N <= 40 ? 8 : N <= 48 ? 6 : 5)
#endif
template <int DT, int N, bool EXACT>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(MEDIAN_2L_W)))
k_median_2l(const MSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k, int xcd) {
  constexpr int B = 2 * N;
  if constexpr (EXACT) k = B;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  __shared__ u32x4 xs[N / 4][k2lCols];  // the upper lanes' N sorted keys, [quad][column]
  const int h = __builtin_amdgcn_readfirstlane((int)threadIdx.x / k2lCols);  // half: wave-uniform
  const int c = (int)threadIdx.x % k2lCols;
  const int64_t tile = xcd ? xcd_tile_map(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  const MSeg sg = segs[nseg > 1 ? find_seg(segs, nseg, tile) : 0];
  const int64_t e0 = (tile - sg.tile_start) * k2lCols, e = e0 + c;
  const bool live = e < sg.numel;
  const int64_t ec = live ? e : sg.numel - 1;
  const void* const* in = ptrs + sg.ptr_base;
  const int64_t ub = col_base<MedT<DT>::kBytes>(e0, sg.tstride);
  const unsigned boff = (unsigned)(ec - e0) * (unsigned)MedT<DT>::kBytes;
  const int base = N * h;
  const int lo_end = k + (B - 1) / 2 - ((k - 1) >> 1);  // slots [k, lo_end) low sentinels, [lo_end, B) high
  float x[N];
#pragma unroll
  for (int t = 0; t < N; ++t) x[t] = MedT<DT>::load_off(at(in[min(base + t, k - 1)], ub), boff);
  if constexpr (!EXACT) {
#pragma unroll
    for (int t = N - 8; t < N; ++t)  // K > B - 8: only the upper half's last 8 slots can hold sentinels
      x[t] = base + t < k ? x[t] : (base + t < lo_end ? -__builtin_inff() : __builtin_inff());
  }
  SortNet<N>::run(x);  // a NaN input turns every sorted output NaN
  if (h == 1) {
#pragma unroll
    for (int q = 0; q < N / 4; ++q)
      xs[q][c] = u32x4{__float_as_uint(x[4 * q]), __float_as_uint(x[4 * q + 1]), __float_as_uint(x[4 * q + 2]),
                       __float_as_uint(x[4 * q + 3])};
  }
  __syncthreads();
  if (h == 1) return;
  float kr = -__builtin_inff();
#pragma unroll
  for (int q = 0; q < N / 4; ++q) {
    const u32x4 b = xs[q][c];
    kr = kmax(kr, kmin(x[N - 1 - 4 * q], __uint_as_float(b.x)));
    kr = kmax(kr, kmin(x[N - 2 - 4 * q], __uint_as_float(b.y)));
    kr = kmax(kr, kmin(x[N - 3 - 4 * q], __uint_as_float(b.z)));
    kr = kmax(kr, kmin(x[N - 4 - 4 * q], __uint_as_float(b.w)));
  }
  if (!live) return;
  const int r = (k - 1) >> 1;
  const bool nan = kr != kr;
  if (nan || kr == 0.0f) store_rare<DT>(in, ub, boff, k, e, r, nan, sg.out);
  else MedT<DT>::store(sg.out, e, kr);
}

// (B > 64: median_col's body written out -- called through median_col, B = 128 took 256 VGPRs,
// 1 wave/SIMD, 1.6 -> 2.2 ms; B <= 64 the other way round)
template <int DT, int B>
__global__ void __launch_bounds__(kBlock)
k_median(const MSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k) {
  const int64_t tile = blockIdx.x;
  const MSeg sg = segs[nseg > 1 ? find_seg(segs, nseg, tile) : 0];
  const int64_t e0 = (tile - sg.tile_start) * kBlock, e = e0 + threadIdx.x;
  const bool live = e < sg.numel;
  const int64_t ec = live ? e : sg.numel - 1;
  const void* const* in = ptrs + sg.ptr_base;
  const int64_t ub = col_base<MedT<DT>::kBytes>(e0, sg.tstride);
  const unsigned boff = (unsigned)(ec - e0) * (unsigned)MedT<DT>::kBytes;
  if constexpr (B <= 64) {  // measured faster through median_col up to 64 (K = 64: 0.74 -> 0.64 ms)
    median_col<DT, B>(in, ub, boff, k, e, live, sg.out);
    return;
  }
  const void* p[B];
#pragma unroll
  for (int i = 0; i < B; ++i) p[i] = at(in[min(i, k - 1)], ub);
  float x[B];
#pragma unroll
  for (int i = 0; i < B; ++i) x[i] = MedT<DT>::load_off(p[i], boff);  // clamped: every load unconditional
  const int lo_end = k + (B - 1) / 2 - ((k - 1) >> 1);          // sentinels [k, lo_end) are low
  unsigned key[B];
  bool nan = false;
#pragma unroll
  for (int i = 0; i < B; ++i) {
    nan = nan || (i < k && x[i] != x[i]);
    key[i] = i < k ? fkey(x[i]) : (i < lo_end ? 0u : 0xFFFFFFFFu);
  }
  const unsigned kr = select_mid<B>(key);
  if (!live) return;
  const int r = (k - 1) >> 1;
  if (nan || kr == kPosZeroKey || kr == kNegZeroKey) store_rare<DT>(in, ub, boff, k, e, r, nan, sg.out);
  else MedT<DT>::store(sg.out, e, fkey_inv(kr));
}

// 16-bit types, two coordinates per lane: one 4-byte load per client, the two 16-bit keys packed in
// one register and the same network on v_pk_min_u16 / v_pk_max_u16 (half the loads and min/max
// instructions of one coordinate per lane).  Needs 4-byte aligned client and output pointers (the
// host checks); a column pair cut by the segment end takes the one-coordinate path.
__device__ __forceinline__ unsigned k16(unsigned u) { return u ^ ((u & 0x8000u) ? 0xFFFFu : 0x8000u); }
__device__ __forceinline__ unsigned k16_inv(unsigned k) { return (k & 0x8000u) ? (k & 0x7FFFu) : (~k & 0xFFFFu); }
template <int DT> __device__ __forceinline__ bool nan16(unsigned u) {
  return (u & 0x7FFFu) > (DT == FA_DTYPE_BF16 ? 0x7F80u : 0x7C00u);
}

template <int DT, int B>
__global__ void __launch_bounds__(kBlock)
k_median_pk(const MSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k) {
  const int64_t tile = blockIdx.x;
  const MSeg sg = segs[nseg > 1 ? find_seg(segs, nseg, tile) : 0];
  const int64_t e0 = (tile - sg.tile_start) * kBlock * 2, e = e0 + threadIdx.x * 2;
  if (e >= sg.numel) return;
  const void* const* in = ptrs + sg.ptr_base;
  const int64_t ub = col_base<2>(e0, sg.tstride);
  const unsigned boff = (unsigned)(e - e0) * 2u;
  if (e + 1 == sg.numel) {  // odd segment length: the last coordinate alone
    median_col<DT, B>(in, ub, boff, k, e, true, sg.out);
    return;
  }
  const void* p[B];
#pragma unroll
  for (int i = 0; i < B; ++i) p[i] = at(in[min(i, k - 1)], ub);
  unsigned w[B];
#pragma unroll
  for (int i = 0; i < B; ++i) w[i] = gld_nt_off<unsigned>(p[i], boff);
  const int lo_end = k + (B - 1) / 2 - ((k - 1) >> 1);
  fa_u16x2 key[B];
  bool nan0 = false, nan1 = false;
#pragma unroll
  for (int i = 0; i < B; ++i) {
    const unsigned lo = w[i] & 0xFFFFu, hi = w[i] >> 16;
    nan0 = nan0 || (i < k && nan16<DT>(lo));
    nan1 = nan1 || (i < k && nan16<DT>(hi));
    const unsigned short sent = i < lo_end ? (unsigned short)0 : (unsigned short)0xFFFF;
    key[i] = i < k ? fa_u16x2{(unsigned short)k16(lo), (unsigned short)k16(hi)} : fa_u16x2{sent, sent};
  }
  const fa_u16x2 kr = select_mid<B>(key);
  const int r = (k - 1) >> 1;
  const unsigned k0 = kr.x, k1 = kr.y;
  const bool rare0 = nan0 || k0 == 0x8000u || k0 == 0x7FFFu;  // NaN seen / a zero selected
  const bool rare1 = nan1 || k1 == 0x8000u || k1 == 0x7FFFu;
  if (!rare0 && !rare1) {
    ((unsigned*)sg.out)[e >> 1] = k16_inv(k0) | (k16_inv(k1) << 16);
    return;
  }
  if (rare0) store_rare<DT>(in, ub, boff, k, e, r, nan0, sg.out);
  else ((unsigned short*)sg.out)[e] = (unsigned short)k16_inv(k0);
  if (rare1) store_rare<DT>(in, ub, boff + 2u, k, e + 1, r, nan1, sg.out);
  else ((unsigned short*)sg.out)[e + 1] = (unsigned short)k16_inv(k1);
}

// Any K (and float64): rank counting, ATen's order (value, client index), NaN first.
template <typename T> __device__ __forceinline__ T ldv(const void* p, int64_t e) { return ((const T*)p)[e]; }

// client element at(p, ub) + lane offset c (elements), as a double
template <int DT>
__device__ __forceinline__ double load_d(const void* p, int64_t c) {
  if constexpr (DT == FA_DTYPE_F64) return gld<double>(p, c);
  else return (double)MedT<DT>::load(p, c);
}
template <int DT>
__device__ __forceinline__ void copy_bits(void* out, int64_t e, const void* src, int64_t c) {
  if constexpr (DT == FA_DTYPE_F64) ((unsigned long long*)out)[e] = ((const unsigned long long*)src)[c];
  else MedT<DT>::store_bits_off(out, e, src, (unsigned)c * (unsigned)MedT<DT>::kBytes);
}
template <int DT> constexpr int elem_bytes() { if constexpr (DT == FA_DTYPE_F64) return 8; else return MedT<DT>::kBytes; }

template <int DT>
__global__ void __launch_bounds__(kBlock)
k_median_rank(const MSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k) {
  const int64_t tile = blockIdx.x;
  const MSeg sg = segs[nseg > 1 ? find_seg(segs, nseg, tile) : 0];
  const int64_t e0 = (tile - sg.tile_start) * kBlock, e = e0 + threadIdx.x;
  if (e >= sg.numel) return;
  const void* const* in = ptrs + sg.ptr_base;
  const int64_t ub = col_base<elem_bytes<DT>()>(e0, sg.tstride);
  const int64_t c = e - e0;
  for (int i = 0; i < k; ++i) {
    const double xi = load_d<DT>(at(in[i], ub), c);
    if (xi != xi) { copy_bits<DT>(sg.out, e, at(in[i], ub), c); return; }
  }
  const int r = (k - 1) >> 1;
  for (int i = 0; i < k; ++i) {
    const double xi = load_d<DT>(at(in[i], ub), c);
    int less = 0, eq_before = 0;
    for (int j = 0; j < k; ++j) {
      const double xj = load_d<DT>(at(in[j], ub), c);
      less += xj < xi;
      eq_before += (xj == xi) && (j < i);
    }
    if (less + eq_before == r) { copy_bits<DT>(sg.out, e, at(in[i], ub), c); return; }
  }
}

// FA_MEDIAN_FULL=0 forces the generic (branching, 64-bit address) form (A/B measurement)
bool full_enabled() {
  static const int on = [] {
    const char* e = getenv("FA_MEDIAN_FULL");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on != 0;
}

// Lanes per column for K in (64, 128]: 2 = k_median_2l, 1 = one lane (k_median_off).  FA_MEDIAN_LANES
// forces a form (read at every call: A/B measurement and tests); FA_MEDIAN_2L=0 keeps one lane.
// (r03: a four-lanes-per-column form measured 19-30 % slower than k_median_2l and was removed)
constexpr int kMedian2lMin = 64;   // every K in (64, 128] (r02y: K = 65 and 96 within 2 % either way, the rest faster;
                                   // r02ab: at B = 40..64 the split measured 0-11 % slower, not used)
int median_lanes(int dtype, int k, bool packed, bool off32) {
  static const int mode2 = [] {
    const char* e = getenv("FA_MEDIAN_2L");
    return e ? atoi(e) : -1;
  }();
  if (dtype == FA_DTYPE_F64 || packed || !off32 || !full_enabled() || mode2 == 0 || k <= 64 || k > 128) return 1;
  const char* e = getenv("FA_MEDIAN_LANES");
  const int m = e ? atoi(e) : -1;
  if (m == 1 || m == 2) return m;
  return k > kMedian2lMin ? 2 : 1;
}

template <int DT>
void launch_median(int k, bool packed, bool off32, int lanes, dim3 grid, hipStream_t st, const MSeg* ds,
                   int nseg, const void* const* dp) {
  if constexpr (DT != FA_DTYPE_F64) {
    if (lanes == 2) {
      // FA_MEDIAN_XCD=1: XCD-contiguous tile map (A/B measurement)
      static const int xm = [] {
        const char* e = getenv("FA_MEDIAN_XCD");
        return e && e[0] == '1' ? 1 : 0;
      }();
      switch ((k + 7) / 8) {  // B = K rounded up to 8, N = B / 2 keys per lane
#define FA_M2(Q)                                                                                                  \
  case Q:                                                                                                       \
    if (k == 8 * Q) hipLaunchKernelGGL((k_median_2l<DT, 4 * Q, true>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k, xm); \
    else hipLaunchKernelGGL((k_median_2l<DT, 4 * Q, false>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k, xm);          \
    return;
        FA_M2(9) FA_M2(10) FA_M2(11) FA_M2(12) FA_M2(13) FA_M2(14) FA_M2(15) FA_M2(16)
#undef FA_M2
        default: break;
      }
    }
  }
  if constexpr (DT == FA_DTYPE_F64) {
    hipLaunchKernelGGL((k_median_rank<DT>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k);
  } else {
    switch ((k + 7) / 8) {  // bucket B = K rounded up to 8 (median_nets.h)
#define FA_MB(Q)                                                                                       \
  case Q:                                                                                            \
    if constexpr (DT != FA_DTYPE_F32 && Q <= 8)  /* packed: K <= 64 (see fa_coord_median) */  \
      if (packed) {                                                                                  \
        hipLaunchKernelGGL((k_median_pk<DT, 8 * Q>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k);     \
        return;                                                                                      \
      }                                                                                              \
    if (off32 && full_enabled() && k == 8 * Q)                                                       \
      hipLaunchKernelGGL((k_median_off<DT, 8 * Q, true>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k); \
    else if (off32 && full_enabled())                                                                \
      hipLaunchKernelGGL((k_median_off<DT, 8 * Q, false>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k); \
    else                                                                                             \
      hipLaunchKernelGGL((k_median<DT, 8 * Q>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k);          \
    return;
      FA_MB(1) FA_MB(2) FA_MB(3) FA_MB(4) FA_MB(5) FA_MB(6) FA_MB(7) FA_MB(8)
      FA_MB(9) FA_MB(10) FA_MB(11) FA_MB(12) FA_MB(13) FA_MB(14) FA_MB(15) FA_MB(16)
#undef FA_MB
      default: break;
    }
    hipLaunchKernelGGL((k_median_rank<DT>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k);
  }
}

}  // namespace

// ============================================================================================ ABI
namespace {
int median_impl(fa_ctx* ctx, int dtype, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                const void* const* d_in, int64_t tstride, void* const* d_out, void* hip_stream) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (k <= 0 || num_segments <= 0 || !seg_numel || !d_in || !d_out)
    return fail(FA_ERR_INVALID, "fa_coord_median: invalid arguments");
  if (dtype != FA_DTYPE_F32 && dtype != FA_DTYPE_BF16 && dtype != FA_DTYPE_F16 && dtype != FA_DTYPE_F64)
    return fail(FA_ERR_DTYPE, "fa_coord_median: dtype %d not supported (F32, BF16, F16, F64)", dtype);
  if (tstride < 0 || tstride % FA_TILE_BYTES)
    return fail(FA_ERR_INVALID, "fa_coord_median_tiled: tile_stride must be a positive multiple of %d (got %lld)",
                FA_TILE_BYTES, (long long)tstride);
  // bf16 / f16 with 4-byte aligned pointers, K <= 64: two coordinates per lane (k_median_pk;
  // bf16 K = 16 / 32 / 64: 0.127 / 0.251 / 0.655 -> 0.106 / 0.205 / 0.572 ms.  K = 128 took 2.44 ms
  // packed vs 1.51 ms one per lane: 128 live keys + 128 pointers exceed the register file)
  bool packed = (dtype == FA_DTYPE_BF16 || dtype == FA_DTYPE_F16) && k <= 64;
  for (int s = 0; s < num_segments && packed; ++s) {
    if (seg_numel[s] <= 0) continue;
    packed = d_out[s] && (uintptr_t)d_out[s] % 4 == 0;
    for (int i = 0; i < k && packed; ++i) packed = (uintptr_t)d_in[(int64_t)s * k + i] % 4 == 0;
  }
  // every kernel addresses a client's element as a uniform 64-bit base (the workgroup's first column,
  // col_base) + a 32-bit lane offset, so any segment size takes the branch-free forms (r03: segments
  // over 4 GB took the generic k_median)
  const bool off32 = true;
  const int lanes = median_lanes(dtype, k, packed, off32);
  const int64_t tile_elems = packed ? 2 * kBlock : lanes == 2 ? k2lCols : kBlock;
  int nseg = 0;
  int64_t tiles = 0;
  for (int s = 0; s < num_segments; ++s) {
    if (seg_numel[s] < 0) return fail(FA_ERR_INVALID, "segment %d has negative numel", s);
    if (seg_numel[s] == 0) continue;
    if (!d_out[s]) return fail(FA_ERR_INVALID, "segment %d: output NULL", s);
    for (int i = 0; i < k; ++i)
      if (!d_in[(int64_t)s * k + i]) return fail(FA_ERR_INVALID, "segment %d client %d: input NULL", s, i);
    ++nseg;
    tiles += (seg_numel[s] + tile_elems - 1) / tile_elems;
  }
  if (nseg == 0) return FA_OK;
  if (tiles > 0x7FFFFFFFll) return fail(FA_ERR_INVALID, "too many tiles");
  const size_t seg_bytes = align16(sizeof(MSeg) * nseg);
  const size_t ptr_bytes = sizeof(void*) * (size_t)nseg * k;
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  fa_ctx::Slot* slot = nullptr;
  int rc = acquire_slot(ctx, seg_bytes + ptr_bytes, &slot);
  if (rc) return rc;
  char* h = (char*)slot->host;
  MSeg* hs = (MSeg*)h;
  const void** hp = (const void**)(h + seg_bytes);
  int j = 0;
  int64_t t0 = 0;
  for (int s = 0; s < num_segments; ++s) {
    const int64_t n = seg_numel[s];
    if (n == 0) continue;
    for (int i = 0; i < k; ++i) hp[(int64_t)j * k + i] = d_in[(int64_t)s * k + i];
    hs[j] = MSeg{n, t0, d_out[s], tstride, j * k, 0};
    t0 += (n + tile_elems - 1) / tile_elems;
    ++j;
  }
  rc = stage(slot, seg_bytes + ptr_bytes, st, true);
  if (rc) return rc;
  const char* dv = (const char*)slot->dev;
  const MSeg* ds = (const MSeg*)dv;
  const void* const* dp = (const void* const*)(dv + seg_bytes);
  const dim3 grid((unsigned)tiles);
  switch (dtype) {
    case FA_DTYPE_F32: launch_median<FA_DTYPE_F32>(k, packed, off32, lanes, grid, st, ds, nseg, dp); break;
    case FA_DTYPE_BF16: launch_median<FA_DTYPE_BF16>(k, packed, off32, lanes, grid, st, ds, nseg, dp); break;
    case FA_DTYPE_F16: launch_median<FA_DTYPE_F16>(k, packed, off32, lanes, grid, st, ds, nseg, dp); break;
    default: launch_median<FA_DTYPE_F64>(k, packed, off32, lanes, grid, st, ds, nseg, dp); break;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    (void)release(slot, st);
    return fail(FA_ERR_HIP, "fa_coord_median: %s", hipGetErrorString(e));
  }
  return release(slot, st);
}
}  // namespace

extern "C" {

int fa_coord_median(fa_ctx* ctx, int dtype, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                    const void* const* d_in, void* const* d_out, void* hip_stream) {
  return median_impl(ctx, dtype, num_segments, seg_numel, k, d_in, 0, d_out, hip_stream);
}

int fa_coord_median_tiled(fa_ctx* ctx, int dtype, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                          const void* const* d_in, int64_t tile_stride, void* const* d_out, void* hip_stream) {
  if (tile_stride <= 0) return fail(FA_ERR_INVALID, "fa_coord_median_tiled: tile_stride must be > 0");
  return median_impl(ctx, dtype, num_segments, seg_numel, k, d_in, tile_stride, d_out, hip_stream);
}

}  // extern "C"

// ============================================================================================
// Krum's pairwise squared distances (krum_defense.py:52-66): D[i][j] = sum_e (x_i[e] - x_j[e])^2
// over the clients' weight vectors, float32 inputs, every pair (i < j) in ONE pass over the data.
// A workgroup stages a chunk of coordinates of all K clients in LDS (transposed [e][client],
// so 4 clients of one coordinate are one 16-byte LDS read), and each thread owns one 4x4
// client-pair tile (upper triangle) -- 16 differences per 2 LDS reads, packed fp32 -- over a slice
// of `ce` coordinates of the chunk (pair_split).  Software pipeline: chunk i is computed from one LDS
// buffer while chunk i + 1 (already in registers) is written to the other and chunk i + 2 is loaded
// from HBM -- one barrier per chunk, HBM latency behind the pair loop.  Sums: float32 over runs of
// <= kPE coordinates, float64 across runs.
// Per-block float64 partials of the upper triangle go to a scratch buffer and a second kernel
// adds them in block order (deterministic).
namespace {

constexpr int kPE = 64;       // longest float32 run (coordinates); small-K esplit cap
constexpr int kMaxPairK = 128;
constexpr int kMaxPairThreads = 1024;
constexpr int kNPS = 16;      // k_pairdist: elements of one client staged per thread and chunk
constexpr int kNPL = 8;       // k_pairdist_lane: coordinates of one client staged per lane and chunk

// Work split of k_pairdist: ntiles 4x4 pair tiles (upper triangle), one per thread, times `esplit`
// coordinate slices: a workgroup is ntiles * esplit threads (<= 1024; K <= 128 -> ntiles <= 528).
// Staging: `rows` = nthreads / kp threads per client, np elements each; a chunk is pe = ce * esplit
// coordinates, every slice exactly ce (a uniform trip count: the pair loop runs on a scalar
// counter).  ntiles <= 128: esplit = 256 / ntiles (e.g. K = 32 keeps 252 of 256 threads busy);
// larger: see below (measured, K = 100: 3 x 325 threads, 72-coordinate chunks, 3.9 ms vs 5.1 ms
// with 325 threads and 24-coordinate chunks).  The LDS row stride is KPAD + 4 floats with KPAD the
// next of 16 / 32 / 64 / 96 / 128 >= kp, a compile-time constant (immediate LDS offsets).
// Staging: kp <= 32 -- k_pairdist_lane, a lane per client, 8 consecutive coordinates by two 16-byte
// loads; larger K -- k_pairdist, `rows` lanes per client reading consecutive floats, 16 elements per
// thread (r02: K = 64 / 100 / 128: 2.59 / 3.99 / 6.58 -> 2.0 / 3.7 / 6.38 ms; at K <= 32 the
// per-element form's extra instructions cost more than its coalescing gains).
struct PairSplit { int kp, kpad, nb, ntiles, esplit, nthreads, rows, ce, pe, nblocks, dgroups, npl; bool lane; };
// k_pairdist_lane: coordinates staged per lane and chunk, 16 (r03g interleaved A/B, 2 x 2 runs: K = 16 /
// 32 0.214-0.217 / 0.580-0.597 ms at 8 -> 0.195-0.196 / 0.533-0.561 at 16); FA_PAIR_NPL=8 restores kNPL
int pair_npl() {
  static const int v = [] {
    const char* e = getenv("FA_PAIR_NPL");
    return e && atoi(e) == kNPL ? kNPL : 16;
  }();
  return v;
}
// Tiles: 4x4 pair tiles of the STRICT upper triangle of 4-client blocks (bi < bj), one per thread and
// coordinate slice; the pairs inside a block (6 per block) are spread over all threads as a second,
// small phase per chunk (see k_pairdist), so no thread computes the 10 wasted slots of a diagonal tile
// and the workgroup is a whole number of waves (r03: K = 128 took 528 threads = 9 waves with diagonal
// tiles -> one workgroup per CU at 96 VGPRs; 496 tiles -> 512 threads, two workgroups per CU).
PairSplit pair_split(int k) {
  PairSplit q;
  q.kp = (k + 3) & ~3;
  q.kpad = q.kp <= 64 ? 64 : q.kp <= 96 ? 96 : 128;  // k_pairdist (kp > 32)
  q.nb = q.kp / 4;
  q.ntiles = q.nb * (q.nb - 1) / 2;
  auto waves = [](int th) { return (th + 63) / 64 * 64; };
  if (q.ntiles == 0) {
    q.esplit = 1;
  } else if (q.kp <= 32) {  // k_pairdist_lane: about 256 threads (r03e sweep, K = 32: 9 x 28 tiles best)
    q.esplit = std::max(1, std::min(kPE, kBlock / q.ntiles));
  } else {
    // k_pairdist: the most slices whose waves stay >= 90% full, up to 512 threads while the tiles are
    // few (<= 128) and 1024 otherwise -- r03e sweep: K = 64 / 100 / 128 fastest at 4 / 3 / 2 slices
    // (512 / 960 / 1024 threads: 1.56 / 3.69 / 5.18 ms vs 2.63 / 6.19 / 5.44 ms at one or two)
    const int cap = q.ntiles <= 128 ? 512 : kMaxPairThreads;
    q.esplit = 1;
    for (int e = 1; waves(e * q.ntiles) <= cap; ++e)
      if ((double)(e * q.ntiles) / waves(e * q.ntiles) >= 0.9) q.esplit = e;
  }
  // measurement override (tools/krum_split.sh sweeps): FA_PAIR_SPLIT="esplit"
  static const char* ov = getenv("FA_PAIR_SPLIT");
  const int oe = ov ? atoi(ov) : 0;
  if (oe >= 1 && q.ntiles > 0 && waves(oe * q.ntiles) <= kMaxPairThreads) q.esplit = oe;
  q.nthreads = std::max(64, waves(q.ntiles * q.esplit));
  if (q.nthreads < q.kp) q.nthreads = waves(q.kp);  // every client needs a staging thread
  q.rows = q.nthreads / q.kp;
  q.lane = q.kp <= 32;
  q.npl = kNPL;
  if (q.lane) {  // k_pairdist_lane: slices of pe / esplit coordinates, not necessarily equal
    q.npl = pair_npl();
    q.pe = q.rows * q.npl;
    q.ce = 0;
  } else {
    // a slice is one float32 run at most, and every element of a chunk has a staging thread
    q.ce = std::max(1, std::min(kPE, q.rows * kNPS / q.esplit));
    // two LDS buffers of pe rows: at most 80 KB, so two workgroups share a CU -- or, for a workgroup of
    // more than 512 threads (alone on its CU at <= 128 VGPRs), up to 150 KB (FA_PAIR_LDS_KB; r03f:
    // K = 100 / 128 3.67 / 5.10 -> 3.40 / 4.89 ms with 150 vs 80)
    static const char* lk = getenv("FA_PAIR_LDS_KB");
    const size_t cap_kb = q.nthreads <= 512 ? 80 : lk && atoi(lk) >= 16 && atoi(lk) <= 150 ? atoi(lk) : 150;
    while (q.ce > 1 && 2 * sizeof(float) * (size_t)q.ce * q.esplit * (q.kpad + 4) > cap_kb * 1024) --q.ce;
    q.pe = q.ce * q.esplit;
  }
  q.dgroups = q.nthreads / q.nb;  // threads per block in the within-block phase
  q.nblocks = 1024;  // workgroups (each writes all pair partials once)
  static const char* ob = getenv("FA_PAIR_BLOCKS");  // measurement override (A/B runs, r02v)
  if (ob && atoi(ob) >= 64 && atoi(ob) <= 16384) q.nblocks = atoi(ob);
  return q;
}

// LDS bytes a pair kernel launch needs: the two staging buffers, and in the epilogue the slice
// reduction of the tiles (esplit > 1) and the within-block reduction (6 doubles per thread).
size_t pair_lds_bytes(const PairSplit& q) {
  const int stride = q.lane ? q.kp + 4 : q.kpad + 4;
  size_t lds = 2 * sizeof(float) * (size_t)q.pe * stride;
  if (q.esplit > 1) lds = std::max(lds, sizeof(double) * 16 * (size_t)q.ntiles);
  return std::max(lds, sizeof(double) * 6 * (size_t)q.nthreads);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct PSeg {
  int64_t numel;
  int64_t tile_start;   // first chunk of this segment (find_seg keys on it)
  int32_t ptr_base;
  int32_t pad;
  int64_t pad2;
};
static_assert(sizeof(PSeg) == 32, "PSeg layout");

// The reference's difference `v_i - v_j` is computed in the vectorized model's dtype
// (krum_defense.py:52-60: torch.cat of the weights, then `(v1 - v2).norm()`): for bfloat16 / float16
// models every difference is the float32 difference rounded to that type (ATen's CPU sub: float
// arithmetic, one rounding to the storage type), then squared and summed in float.  RT: 0 = float32
// (no rounding), 1 = bfloat16, 2 = float16 (round to nearest even; overflow -> inf, NaN stays NaN).
template <int RT>
__device__ __forceinline__ f32x2 round_diff(f32x2 d) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
  if constexpr (RT == 1) return __builtin_convertvector(__builtin_convertvector(d, bf16x2), f32x2);
  else if constexpr (RT == 2) return __builtin_convertvector(__builtin_convertvector(d, f16x2), f32x2);
  else return d;
}


// tile -> (bi, bj), bi < bj: row-major over the strict upper triangle of nb blocks
__device__ __forceinline__ void tile_blocks(int tile, int nb, int& bi, int& bj) {
  int r = 0, rem = tile;
  while (rem >= nb - 1 - r) { rem -= nb - 1 - r; ++r; }
  bi = r;
  bj = r + 1 + rem;
}

__device__ __forceinline__ int64_t pair_index(int i, int j, int k) {  // i < j
  return (int64_t)i * k - (int64_t)i * (i + 1) / 2 + (j - i - 1);
}

// One coordinate of a 4x4 pair tile: clients 4bi..4bi+3 (a) against 4bj..4bj+3 (b), packed fp32
// (v_pk_add_f32 / v_pk_fma_f32): pair (x, y), (x, y+1) per instruction -- the same per-element IEEE
// sub and fused multiply-add as the scalar form, half the VALU issue slots.
template <int RT>
__device__ __forceinline__ void pair_tile(const float4 a, const float4 b, f32x2 (&acc)[8]) {
  // a's lanes broadcast by shuffles of its two halves (op_sel on the packed subtraction, no v_mov)
  const f32x2 a01 = {a.x, a.y}, a23 = {a.z, a.w};
  const f32x2 b01 = {b.x, b.y}, b23 = {b.z, b.w};
  const f32x2 ax[4] = {__builtin_shufflevector(a01, a01, 0, 0), __builtin_shufflevector(a01, a01, 1, 1),
                       __builtin_shufflevector(a23, a23, 0, 0), __builtin_shufflevector(a23, a23, 1, 1)};
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const f32x2 d0 = round_diff<RT>(ax[x] - b01), d1 = round_diff<RT>(ax[x] - b23);
    acc[2 * x] = __builtin_elementwise_fma(d0, d0, acc[2 * x]);
    acc[2 * x + 1] = __builtin_elementwise_fma(d1, d1, acc[2 * x + 1]);
  }
}

// The within-block phase: thread t sums the 6 pairs (4b + i, 4b + j), i < j < 4, of block b = t % nb
// over the chunk's coordinates e = t / nb, t / nb + dg, ... (dg = threads per block) -- one 16-byte
// LDS read and 3 packed differences per coordinate; float32 runs, float64 across runs, as the tiles.
template <int RT>
struct Within {
  f32x2 acc[3];
  double accd[6];
  int run;
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int u = 0; u < 3; ++u) acc[u] = f32x2{0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < 6; ++u) accd[u] = 0.0;
    run = 0;
  }
  __device__ __forceinline__ void flush() {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      accd[2 * u] += (double)acc[u].x;
      accd[2 * u + 1] += (double)acc[u].y;
      acc[u] = f32x2{0.0f, 0.0f};
    }
    run = 0;
  }
  __device__ __forceinline__ void add(const float* lb, int stride, int pe, int e0, int dg, int b) {
    for (int e = e0; e < pe; e += dg) {
      const float4 v = *(const float4*)&lb[e * stride + 4 * b];
      const f32x2 x = round_diff<RT>(f32x2{v.x, v.x} - f32x2{v.y, v.z});  // (0,1) (0,2)
      const f32x2 y = round_diff<RT>(f32x2{v.x, v.y} - f32x2{v.w, v.z});  // (0,3) (1,2)
      const f32x2 z = round_diff<RT>(f32x2{v.y, v.z} - f32x2{v.w, v.w});  // (1,3) (2,3)
      acc[0] = __builtin_elementwise_fma(x, x, acc[0]);
      acc[1] = __builtin_elementwise_fma(y, y, acc[1]);
      acc[2] = __builtin_elementwise_fma(z, z, acc[2]);
    }
  }
  // after each chunk: dmax = most coordinates one chunk adds (uniform)
  __device__ __forceinline__ void step(int dmax) {
    run += dmax;
    if (run + dmax > kPE) flush();
  }
};

// Epilogue of both pair kernels: the block's partials of every pair (i < j < k) into `out` -- the
// tiles (their esplit slices added in slice order through LDS), then the within-block pairs (the dg
// threads of a block added in thread order through LDS).  Every thread of the block calls it.
__device__ __forceinline__ void pair_epilogue(float* lds, const double (&accd)[16], bool pact, int es, int tile,
                                              int bi, int bj, int ntiles, int esplit, int nb, int k,
                                              const double (&waccd)[6], bool dact, int dg, double* out) {
  const int t = threadIdx.x;
  double* red = (double*)lds;
  if (esplit == 1) {
    if (pact) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int i = 4 * bi + u / 4, j = 4 * bj + u % 4;
        if (j < k) out[pair_index(i, j, k)] = accd[u];
      }
    }
  } else {
    __syncthreads();
    for (int s = 0; s < esplit; ++s) {
      if (pact && es == s) {
#pragma unroll
        for (int u = 0; u < 16; ++u) red[tile * 16 + u] = (s == 0 ? 0.0 : red[tile * 16 + u]) + accd[u];
      }
      __syncthreads();
    }
    for (int idx = t; idx < ntiles * 16; idx += (int)blockDim.x) {
      const int u = idx % 16;
      int r, c;
      tile_blocks(idx / 16, nb, r, c);
      const int i = 4 * r + u / 4, j = 4 * c + u % 4;
      if (j < k) out[pair_index(i, j, k)] = red[idx];
    }
  }
  __syncthreads();  // LDS reused for the within-block sums
  if (dact) {
#pragma unroll
    for (int p = 0; p < 6; ++p) red[t * 6 + p] = waccd[p];
  }
  __syncthreads();
  for (int idx = t; idx < nb * 6; idx += (int)blockDim.x) {
    const int b = idx / 6, p = idx % 6;
    double sum = 0.0;
    for (int g = 0; g < dg; ++g) sum += red[(g * nb + b) * 6 + p];
    const int i = 4 * b + (p < 3 ? 0 : p < 5 ? 1 : 2), j = 4 * b + (p < 3 ? p + 1 : p < 5 ? p - 1 : 3);
    if (j < k) out[pair_index(i, j, k)] = sum;
  }
}

// K <= 32 (kp <= 32): the r01 form -- a lane per client stages 8 consecutive coordinates (two 16-byte
// loads), slices of pe / esplit coordinates (pe = rows * 8); measured faster there than the
// strided form below (K = 16 / 32: 0.20 / 0.59 vs 0.27 / 0.65 ms)
template <bool VEC, int RT, bool PF, int NPL>
__global__ void __launch_bounds__(kMaxPairThreads) __attribute__((amdgpu_waves_per_eu(4)))
k_pairdist_lane(const PSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k, int kp,
           int64_t nchunks, int ntiles, int esplit, int pe, double* __restrict__ partial,
           const double* __restrict__ guard, double limit) {
  if (guard && *guard <= limit) return;  // the Gram form's result stands (fa_pairwise_sqdist_gram)
  extern __shared__ float lds[];              // [2][pe][kp + 4]
  const int stride = kp + 4;
  const int nb = kp / 4;
  const int t = threadIdx.x;                     // blockDim.x >= ntiles * esplit, whole waves
  const bool pact = t < ntiles * esplit;         // the rest only stage and take part in the within phase
  const int es = pact ? t / ntiles : 0;          // coordinate slice
  const int tile = pact ? t % ntiles : 0;
  int bi = 0, bj = 1;
  if (pact) tile_blocks(tile, nb, bi, bj);
  const int dg = (int)blockDim.x / nb;           // within-block phase: threads per block
  const bool dact = t < dg * nb;
  const int db = t % nb, de0 = t / nb;
  Within<RT> wb;
  wb.init();
  double accd[16];
  f32x2 acc[8];
  int run = 0;  // coordinates summed in acc since the last flush
#pragma unroll
  for (int u = 0; u < 16; ++u) accd[u] = 0.0;
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = f32x2{0.0f, 0.0f};
  auto flush = [&]() {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      accd[2 * u] += (double)acc[u].x;
      accd[2 * u + 1] += (double)acc[u].y;
      acc[u] = f32x2{0.0f, 0.0f};
    }
    run = 0;
  };
  const int e_lo = (int)((int64_t)es * pe / esplit), e_hi = (int)((int64_t)(es + 1) * pe / esplit);
  // staging role: client sc, NPL consecutive coordinates from se of every chunk (pe = (nthreads / kp)
  // * NPL, so the row (t / kp) < nthreads / kp of a staging thread is exactly se < pe).  Registers
  // hold the next chunk while the current one is computed (see the pipeline below); they go to LDS
  // transposed, [e][client].
  const int sc = t % kp, se = (t / kp) * NPL;
  const bool sact = se < pe && sc < k;
  const bool swr = se < pe;            // clients k..kp-1 are staged as zeros
  float v[NPL];
  int cseg = -1;
  const float* src = nullptr;
  int64_t snum = 0;
  auto load = [&](int64_t ch) {
    const int si = nseg > 1 ? find_seg(segs, nseg, ch) : 0;
    const PSeg sg = segs[si];
    if (si != cseg) {  // one pointer load per segment, not per chunk
      cseg = si;
      src = sact ? (const float*)ptrs[sg.ptr_base + sc] : nullptr;
      snum = sg.numel;
    }
    const int64_t b0 = (ch - sg.tile_start) * pe + se;
    if (!sact) {
#pragma unroll
      for (int u = 0; u < NPL; ++u) v[u] = 0.0f;
    } else if (b0 + NPL <= snum) {  // whole run: one base address, immediate offsets
      const __attribute__((address_space(1))) float* g = (const __attribute__((address_space(1))) float*)(src + b0);
      if constexpr (VEC) {
        typedef float f32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int u = 0; u < NPL / 4; ++u) {
          const f32x4 q = ((const __attribute__((address_space(1))) f32x4*)g)[u];
          v[4 * u] = q.x;
          v[4 * u + 1] = q.y;
          v[4 * u + 2] = q.z;
          v[4 * u + 3] = q.w;
        }
      } else {
#pragma unroll
        for (int u = 0; u < NPL; ++u) v[u] = g[u];
      }
    } else {  // the segment's last run: coordinates past the end add 0 to every sum
#pragma unroll
      for (int u = 0; u < NPL; ++u) v[u] = b0 + u < snum ? gld<float>(src, b0 + u) : 0.0f;
    }
  };
  // two LDS buffers: chunk i is computed from buffer i & 1 while chunk i + 1 is written to the other
  // (and chunk i + 2 loads into registers) -- one barrier per chunk
  const int bufsz = pe * stride;
  auto put = [&](int buf) {
    if (swr) {
#pragma unroll
      for (int u = 0; u < NPL; ++u) lds[buf * bufsz + (se + u) * stride + sc] = v[u];
    }
  };
  // each workgroup takes a contiguous run of chunks: a 128-byte line split between two chunks is then
  // fetched once, by one workgroup (grid-strided chunks put the halves on different CUs / XCDs: K = 32
  // read 1.43x its bytes)
  const int64_t c0 = nchunks * blockIdx.x / gridDim.x, c1 = nchunks * (blockIdx.x + 1) / gridDim.x;
  if (c0 < c1) {
    load(c0);
    put(0);
    if (c0 + 1 < c1) load(c0 + 1);
  }
  __syncthreads();
  int cur = 0;
  for (int64_t ch = c0; ch < c1; ++ch, cur ^= 1) {
    const float* lb = lds + cur * bufsz;
    // packed fp32 (v_pk_add_f32 / v_pk_fma_f32): pair (x, y), (x, y+1) per instruction -- the same
    // per-element IEEE sub and fused multiply-add as the scalar form, half the VALU issue slots
    if (pact && e_hi > e_lo) {
      // PF: the next coordinate's two 16-byte reads are issued before this one's arithmetic, so the
      // LDS latency hides behind it (r03c PMC: 39% of wave cycles waiting, lgkmcnt(0) after each read)
      const float* pa = lb + 4 * bi;
      const float* pb = lb + 4 * bj;
      float4 a = *(const float4*)&pa[e_lo * stride];
      float4 b = *(const float4*)&pb[e_lo * stride];
#pragma unroll 4
      for (int e = e_lo; e < e_hi; ++e) {
        float4 an = a, bn = b;
        if constexpr (PF) {
          const int e1 = e + 1 < e_hi ? e + 1 : e;
          an = *(const float4*)&pa[e1 * stride];
          bn = *(const float4*)&pb[e1 * stride];
        } else {
          a = *(const float4*)&pa[e * stride];
          b = *(const float4*)&pb[e * stride];
        }
        pair_tile<RT>(a, b, acc);
        if constexpr (PF) { a = an; b = bn; }
      }
    }
    run += e_hi - e_lo;
    if (run + (e_hi - e_lo) > kPE) flush();  // float runs of <= kPE coordinates, then float64
    if (dact) wb.add(lb, stride, pe, de0, dg, db);
    wb.step((pe + dg - 1) / dg);
    if (ch + 1 < c1) {
      put(cur ^ 1);  // buffer cur ^ 1 was last read before the previous barrier
      if (ch + 2 < c1) load(ch + 2);
    }
    __syncthreads();
  }
  flush();
  wb.flush();
  pair_epilogue(lds, accd, pact, es, tile, bi, bj, ntiles, esplit, nb, k, wb.accd, dact, dg,
                partial + (int64_t)blockIdx.x * ((int64_t)k * (k - 1) / 2));
}

// waves_per_eu(4): <= 128 VGPRs, the budget at which a CU holds 16 waves (MI355X_MICROARCH.md: waves
// per CU halve at 64 / 128 VGPRs) -- two 8-wave workgroups of 512 threads (K = 128)
template <int KPAD, int RT, bool PF>
__global__ void __launch_bounds__(kMaxPairThreads) __attribute__((amdgpu_waves_per_eu(4)))
k_pairdist(const PSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k, int kp,
           int64_t nchunks, int ntiles, int esplit, int ce, int rows, double* __restrict__ partial,
           const double* __restrict__ guard, double limit) {
  if (guard && *guard <= limit) return;  // the Gram form's result stands (fa_pairwise_sqdist_gram)
  constexpr int S = KPAD + 4;                    // LDS row stride (floats), 16-byte rows
  constexpr int NP = kNPS;
  extern __shared__ float lds[];                 // [2][pe][S]
  const int pe = ce * esplit;
  const int nb = kp / 4;
  const int t = threadIdx.x;                     // blockDim.x >= ntiles * esplit, whole waves
  const bool pact = t < ntiles * esplit;         // the rest only stage and take part in the within phase
  const int es = pact ? t / ntiles : 0;          // coordinate slice
  const int tile = pact ? t % ntiles : 0;
  int bi = 0, bj = 1;
  if (pact) tile_blocks(tile, nb, bi, bj);
  const int dg = (int)blockDim.x / nb;           // within-block phase: threads per block
  const bool dact = t < dg * nb;
  const int db = t % nb, de0 = t / nb;
  Within<RT> wb;
  wb.init();
  double accd[16];
  f32x2 acc[8];
  int run = 0;  // coordinates summed in acc since the last flush (uniform)
#pragma unroll
  for (int u = 0; u < 16; ++u) accd[u] = 0.0;
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = f32x2{0.0f, 0.0f};
  auto flush = [&]() {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      accd[2 * u] += (double)acc[u].x;
      accd[2 * u + 1] += (double)acc[u].y;
      acc[u] = f32x2{0.0f, 0.0f};
    }
    run = 0;
  };
  // staging role: client sc = t / rows, elements sr, sr + rows, ... of every chunk -- consecutive
  // lanes read consecutive floats of one client (rows * 4 contiguous bytes per client and load; a
  // lane per client had made every load touch 64 lines: K = 64 staging alone took 2.6 ms), and their
  // LDS stores [e][sc] fall on distinct banks (S = 4 mod 32: bank 4 * sr + sc).  Registers hold the
  // next chunk while the current one is computed (see the pipeline below).
  const int sc = t / rows, sr = t % rows;
  const int sstep = rows;              // element step of a staging thread
  const bool sact = sc < k;
  const bool swr = sc < kp;            // clients k..kp-1 are staged as zeros
  float v[NP];
  int cseg = -1;
  const float* src = nullptr;
  int64_t snum = 0;
  auto load = [&](int64_t ch) {
    const int si = nseg > 1 ? find_seg(segs, nseg, ch) : 0;
    const PSeg sg = segs[si];
    if (si != cseg) {  // one pointer load per segment, not per chunk
      cseg = si;
      src = sact ? (const float*)ptrs[sg.ptr_base + sc] : nullptr;
      snum = sg.numel;
    }
    const int64_t b0 = (ch - sg.tile_start) * pe;
    // elements of this chunk inside the segment: all of them but in the segment's last chunk, where
    // coordinates past the end add 0 to every sum
    const int lim = sact ? (int)std::min<int64_t>(pe, snum - b0) : 0;
    const __attribute__((address_space(1))) float* g =
        (const __attribute__((address_space(1))) float*)(sact ? src + b0 + sr : nullptr);
    const int n = lim > sr ? (lim - sr + sstep - 1) / sstep : 0;  // elements u < n are inside
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      v[u] = u < n ? *g : 0.0f;
      g += sstep;
    }
  };
  // two LDS buffers: chunk i is computed from buffer i & 1 while chunk i + 1 is written to the other
  // (and chunk i + 2 loads into registers) -- one barrier per chunk
  const int bufsz = pe * S;
  const int nput = swr && pe > sr ? std::min(NP, (pe - sr + sstep - 1) / sstep) : 0;
  const int rstep = sstep * S;
  auto put = [&](int buf) {
    float* l = lds + buf * bufsz + sr * S + sc;
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      if (u < nput) *l = v[u];
      l += rstep;
    }
  };
  // each workgroup takes a contiguous run of chunks: a 128-byte line split between two chunks is then
  // fetched once, by one workgroup (grid-strided chunks put the halves on different CUs / XCDs: K = 32
  // read 1.43x its bytes)
  const int64_t c0 = nchunks * blockIdx.x / gridDim.x, c1 = nchunks * (blockIdx.x + 1) / gridDim.x;
  if (c0 < c1) {
    load(c0);
    put(0);
    if (c0 + 1 < c1) load(c0 + 1);
  }
  __syncthreads();
  int cur = 0;
  const int off_a = es * ce * S + 4 * bi, off_b = es * ce * S + 4 * bj;
  for (int64_t ch = c0; ch < c1; ++ch, cur ^= 1) {
    const float* pa = lds + cur * bufsz + off_a;
    const float* pb = lds + cur * bufsz + off_b;
    // packed fp32 (v_pk_add_f32 / v_pk_fma_f32): pair (x, y), (x, y+1) per instruction -- the same
    // per-element IEEE sub and fused multiply-add as the scalar form, half the VALU issue slots
    if (pact) {
      float4 a = *(const float4*)pa;
      float4 b = *(const float4*)pb;
#pragma unroll 4
      for (int i = 0; i < ce; ++i) {
        float4 an = a, bn = b;
        if constexpr (PF) {  // next coordinate's reads in flight during this one's arithmetic
          const int i1 = i + 1 < ce ? i + 1 : i;
          an = *(const float4*)(pa + i1 * S);
          bn = *(const float4*)(pb + i1 * S);
        } else {
          a = *(const float4*)(pa + i * S);
          b = *(const float4*)(pb + i * S);
        }
        pair_tile<RT>(a, b, acc);
        if constexpr (PF) { a = an; b = bn; }
      }
    }
    run += ce;
    if (run + ce > kPE) flush();  // float runs of <= kPE coordinates, then float64
    if (dact) wb.add(lds + cur * bufsz, S, pe, de0, dg, db);
    wb.step((pe + dg - 1) / dg);
    if (ch + 1 < c1) {
      put(cur ^ 1);  // buffer cur ^ 1 was last read before the previous barrier
      if (ch + 2 < c1) load(ch + 2);
    }
    __syncthreads();
  }
  flush();
  wb.flush();
  pair_epilogue(lds, accd, pact, es, tile, bi, bj, ntiles, esplit, nb, k, wb.accd, dact, dg,
                partial + (int64_t)blockIdx.x * ((int64_t)k * (k - 1) / 2));
}

// float64 models (krum_defense.py:50-66 over vectorize_weight's float64 vector, common/utils.py:8-30):
// every difference and square in float64, as the reference computes them (no float32 step).  A rare
// path, written for clarity: a workgroup stages kC64 coordinates of all k clients in LDS ([e][client]
// doubles), each thread owns pairs p = t, t + 256, ... (<= 32 of them, k <= 128) and adds their
// squared differences over the chunk with float64 FMAs; per-block partials go through
// k_pairdist_reduce like the float32 kernels'.
constexpr int kC64 = 32;
__global__ void __launch_bounds__(kBlock)
k_pairdist_f64(const PSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k,
               int64_t nchunks, double* __restrict__ partial) {
  extern __shared__ double ldsd[];  // [kC64][k]
  const int t = threadIdx.x;
  const int npairs = k * (k - 1) / 2;
  constexpr int kPPT = (kMaxPairK * (kMaxPairK - 1) / 2 + kBlock - 1) / kBlock;  // 32
  double acc[kPPT];
  int pij[kPPT];  // i | j << 8 of pair t + q * kBlock
#pragma unroll
  for (int q = 0; q < kPPT; ++q) {
    acc[q] = 0.0;
    const int p = t + q * kBlock;
    int i = 0, rem = p;
    if (p < npairs)
      while (rem >= k - 1 - i) { rem -= k - 1 - i; ++i; }
    pij[q] = p < npairs ? (i | ((i + 1 + rem) << 8)) : 0;
  }
  const int64_t c0 = nchunks * blockIdx.x / gridDim.x, c1 = nchunks * (blockIdx.x + 1) / gridDim.x;
  for (int64_t ch = c0; ch < c1; ++ch) {
    const int si = nseg > 1 ? find_seg(segs, nseg, ch) : 0;
    const PSeg sg = segs[si];
    const int64_t b0 = (ch - sg.tile_start) * kC64;
    __syncthreads();  // the previous chunk's reads are done
    for (int idx = t; idx < kC64 * k; idx += kBlock) {  // consecutive threads: consecutive coordinates
      const int i = idx / kC64, e = idx % kC64;
      const double* src = (const double*)ptrs[sg.ptr_base + i];
      ldsd[e * k + i] = b0 + e < sg.numel ? src[b0 + e] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kPPT; ++q) {
      if (t + q * kBlock < npairs) {
        const int i = pij[q] & 0xff, j = pij[q] >> 8;
        double s = acc[q];
        for (int e = 0; e < kC64; ++e) {
          const double d = ldsd[e * k + i] - ldsd[e * k + j];
          s = __builtin_fma(d, d, s);
        }
        acc[q] = s;
      }
    }
  }
  double* out = partial + (int64_t)blockIdx.x * npairs;
#pragma unroll
  for (int q = 0; q < kPPT; ++q)
    if (t + q * kBlock < npairs) out[t + q * kBlock] = acc[q];
}

__global__ void __launch_bounds__(kBlock)
k_pairdist_reduce(const double* __restrict__ partial, int nblocks, int k, double* __restrict__ d,
                  const double* __restrict__ guard, double limit) {
  if (guard && *guard <= limit) return;
  // kRP pairs per workgroup, kBlock / kRP lanes per pair: lane l sums blocks l, l + L, ... (each
  // load row = kRP consecutive pairs), then the L lane sums are added in lane order -- a fixed
  // order, so the result is deterministic.  (A single thread per pair made this a serial chain of
  // nblocks loads: ~0.5 ms of latency at 1,024 blocks.)
  constexpr int kRP = 8, L = kBlock / kRP;
  __shared__ double red[L][kRP + 1];
  const int64_t npairs = (int64_t)k * (k - 1) / 2;
  const int pl = threadIdx.x % kRP, lane = threadIdx.x / kRP;
  const int64_t p = (int64_t)blockIdx.x * kRP + pl;
  double s = 0.0;
  if (p < npairs)
    for (int b = lane; b < nblocks; b += L) s += partial[(int64_t)b * npairs + p];
  red[lane][pl] = s;
  __syncthreads();
  if (lane == 0 && p < npairs) {
    double t = 0.0;
    for (int l = 0; l < L; ++l) t += red[l][pl];
    int i = 0;  // p -> (i, j)
    int64_t rem = p;
    while (rem >= k - 1 - i) { rem -= k - 1 - i; ++i; }
    const int j = i + 1 + (int)rem;
    d[(int64_t)i * k + j] = t;
    d[(int64_t)j * k + i] = t;
  }
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < k; i += kBlock) d[(int64_t)i * k + i] = 0.0;
}


// ---------------------------------------------------------------------------------------------
// Gram form of the pairwise distances on the matrix cores (r05, float32 models):
//   D_ij = A_i + A_j - 2 G_ij,  G = Y Y^T,  A_i = G_ii,  y_i[e] = x_i[e] - c[e]
// with c a robust per-coordinate centre (the median of clients 0..4: with at most two of them
// Byzantine it lies inside the honest clients' range, so the honest pairs' cancellation stays small).
// One multiply-add per pair-coordinate on v_mfma_f32_32x32x2_f32 (f32 in / f32 accumulate, the FP32
// vector rate), instead of the direct form's sub + fma on the VALU; operands read once per 32x32 tile.
// The form cancels: relative error ~ eps * kappa_ij, kappa_ij = (A_i + A_j) / D_ij -- the distance
// kernel reports max kappa (k_gram_reduce's tail) and the binding reruns the direct kernel when it is large
// or not finite (fedml_amd/engine.py pairwise_sqdist).
//
// Layout: a workgroup owns a contiguous run of chunks (kGE coordinates of one segment, all clients);
// a chunk is staged x -> LDS [client][kGS] (coalesced 16-byte loads of each client row, the next chunk
// in registers while this one is computed), the centre row is computed once per chunk, and every wave
// runs the MFMAs of its tile(s) (32x32 client blocks bi <= bj, upper triangle incl. the diagonal) over
// its share of the chunk's coordinate groups: lane l takes client 32*b + (l & 31) and coordinates
// 8g + 4*(l >> 5) + 0..3 (one ds_read_b128 feeds four MFMAs; A and B are the same fragment layout,
// so k runs over (8g + u, 8g + 4 + u)).  float32 runs of one chunk, float64 across chunks.
constexpr int kGE = 128;       // coordinates per chunk
constexpr int kGS = kGE + 4;   // LDS row stride (floats): 16-byte rows, b128 reads conflict-free
typedef float gf16 __attribute__((ext_vector_type(16)));
typedef float gf4 __attribute__((ext_vector_type(4)));

template <int KB, bool S16 = false> struct GramCfg {
  static constexpr int T = KB * (KB + 1) / 2;             // 32x32 tiles, upper triangle
  static constexpr int R = S16 ? (KB == 4 ? 1 : 4) : KB == 1 ? 4 : KB == 2 ? 4 : KB == 3 ? 2 : 1;  // coordinate splits
  static constexpr int W = S16 ? (KB == 4 ? 12 : 16) : T * R;  // waves per workgroup, one (tile, split) each:
                                                          // 4 / 12 / 12 / 10 -- a multiple of the CU's 4
                                                          // SIMDs except K > 96 (3, 3, 2, 2 tiles per SIMD),
                                                          // whose S16 form runs 12 waves of three 16x16 tiles;
                                                          // K in (32, 64] S16: 16 waves, 4 tile sets x 4 splits
  static constexpr int NT = W * 64;
  static constexpr int KP = 32 * KB;
  static constexpr int NLD = (KP * (kGE / 4) + NT - 1) / NT;  // staged 16-byte vectors per thread
  static constexpr int LDS_FLOATS = 2 * KP * kGS + W * kGE;   // two chunk buffers + a centre row per wave
};

// (r05k: a register ring of 2-4 staged chunks measured slower at K = 32 -- the compiler waits vmcnt(0)
// at every put whatever the depth; r05m: chunks dealt round-robin over the workgroups, within noise.
// Both knobs were removed)

// K in (96, 128], S16 form: 12 waves, each three 16x16 tiles of the 8 client blocks of 16 that share at
// most 3 blocks -- waves 0-3 the diagonal pairs {2a, 2a + 1} (tiles (2a,2a), (2a,2a+1), (2a+1,2a+1)),
// waves 4-11 the triangles of a decomposition of the remaining 24 block pairs (K_{2,2,2,2} into 8
// triangles, found by search): every one of the 36 upper 16x16 tiles once, 3 per wave, 3 waves per SIMD
__constant__ const int8_t kG16Blocks[12][3] = {{0, 1, 1}, {2, 3, 3}, {4, 5, 5}, {6, 7, 7}, {0, 2, 4}, {0, 3, 6},
                                               {0, 5, 7}, {1, 2, 7}, {1, 3, 5}, {1, 4, 6}, {2, 5, 6}, {3, 4, 7}};
// K in (32, 64], S16 form: 4 tile sets of the 4 client blocks -- the diagonal pairs {0, 1} and {2, 3}
// (3 tiles each) and the cross pairs (0, {2, 3}) and (1, {2, 3}) (2 tiles each) -- each over 4
// coordinate splits; wave w runs set (w % 4 + w / 4) % 4, split w / 4, so every SIMD (w % 4) holds
// two 3-tile and two 2-tile waves.  Row: {type (0 diagonal pair, 2 cross pair), block 0, 1, 2}.
__constant__ const int8_t kG16Sets2[4][4] = {{0, 0, 1, 1}, {0, 2, 3, 3}, {2, 0, 2, 3}, {2, 1, 2, 3}};
// K in (64, 96] (bf16x3 form, r06): the 6 client blocks of 16 as 7 sets of 3 tiles -- the diagonal pairs
// {0, 1}, {2, 3}, {4, 5} and the 4 triangles of K_{2,2,2} (one block of each pair) that cover the 12
// cross pairs once; wave w runs set w over the whole chunk.  Row: {type, block 0, 1, 2}.
__constant__ const int8_t kG16Sets3[7][4] = {{0, 0, 1, 1}, {0, 2, 3, 3}, {0, 4, 5, 5}, {1, 0, 2, 4},
                                             {1, 0, 3, 5}, {1, 1, 2, 5}, {1, 1, 3, 4}};

template <int KB>
__host__ __device__ constexpr int gram_T_c() { return KB * (KB + 1) / 2; }

template <int KB>
__device__ __forceinline__ void gram_tile_kb(int t, int& bi, int& bj) {
  int i = 0, rem = t;
  while (rem >= KB - i) { rem -= KB - i; ++i; }
  bi = i;
  bj = i + rem;
}

template <int KB, bool VEC, bool S16>
__global__ void __launch_bounds__((GramCfg<KB, S16>::NT)) __attribute__((amdgpu_waves_per_eu(S16 && KB == 4 ? 3 : 4)))
k_pair_gram(const PSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k,
            int64_t nchunks, double* __restrict__ partial, unsigned* __restrict__ ctr) {
  static_assert(!S16 || KB == 4 || KB == 2, "16x16 wave tables for 8 (K > 96) or 4 (K in (32, 64]) client blocks");
  using C = GramCfg<KB, S16>;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ctr = 0u;  // k_gram_reduce's arrival counter
  extern __shared__ __attribute__((aligned(16))) float gl[];
  float* const lds0 = gl;                       // [2][KP][kGS]
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  float* const cen = gl + 2 * C::KP * kGS + w * kGE;  // this wave's centre row (wave-private: no barrier)
  // 32x32 form: this wave's tile (bi, bj) and coordinate-group split r
  const int ti = w / C::R, r = w % C::R;
  int bi = 0, bj = 0;
  if constexpr (!S16) gram_tile_kb<KB>(ti, bi, bj);
  const bool diag = bi == bj;
  const int half = lane >> 5, lrow = lane & 31;
  const int ra = 32 * bi + lrow, rb = 32 * bj + lrow;
  // 16x16 form: lane (li, kk); this wave's tile set -- type 0: a diagonal pair (b0,b0), (b0,b1),
  // (b1,b1); 1: a triangle (b0,b1), (b0,b2), (b1,b2); 2: a cross pair (b0,b1), (b0,b2) -- and split
  const int li = lane & 15, kk = lane >> 4;
  const int r16 = KB == 4 ? 0 : w / 4, set16 = KB == 4 ? w : (w % 4 + w / 4) % 4;
  const int typ = KB == 4 ? (w < 4 ? 0 : 1) : kG16Sets2[set16][0];
  const bool dg = typ == 0;
  int blk[3] = {0, 0, 0};
  int ro[3] = {0, 0, 0};  // row offsets of client 16 b + li of the wave's blocks
  if constexpr (S16) {
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      blk[x] = KB == 4 ? kG16Blocks[w][x] : kG16Sets2[set16][1 + x];
      ro[x] = (16 * blk[x] + li) * kGS;
    }
  }
  constexpr int NACC = S16 ? 12 : 16;
  gf16 acc;
  gf4 a16[3];
  double accd[NACC];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
#pragma unroll
  for (int x = 0; x < 3; ++x) a16[x] = gf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < NACC; ++q) accd[q] = 0.0;
  // staging: 16-byte vector q of client (idx / (kGE/4)) = coordinates 4 q .. 4 q + 3 of the chunk
  constexpr int QV = kGE / 4;
  gf4 v[C::NLD];
  // this thread's client pointers for the current segment (one pointer load per segment, not per
  // chunk: a per-chunk pointer load put a full memory round trip before every data load)
  const float* src[C::NLD];
  int cseg = -1;
  auto load = [&](int64_t ch) {
    const int si = nseg > 1 ? find_seg(segs, nseg, ch) : 0;
    const PSeg sg = segs[si];
    if (si != cseg) {
      cseg = si;
#pragma unroll
      for (int u = 0; u < C::NLD; ++u) {
        const int idx = t + u * C::NT;
        const int cl = idx / QV;
        src[u] = (C::NLD * C::NT == C::KP * QV || idx < C::KP * QV) && cl < k
                     ? (const float*)ptrs[sg.ptr_base + cl] + 4 * (idx % QV) : nullptr;
      }
    }
    const int64_t b0 = (ch - sg.tile_start) * kGE;
    const bool full = VEC && b0 + kGE <= sg.numel;  // uniform: the segment's last chunk takes the slow path
    if (full) {  // every load issued before any is consumed
#pragma unroll
      for (int u = 0; u < C::NLD; ++u) {
        const gf4 z = {0.f, 0.f, 0.f, 0.f};
        v[u] = src[u] ? *(const __attribute__((address_space(1))) gf4*)(src[u] + b0) : z;
      }
    } else {
#pragma unroll
      for (int u = 0; u < C::NLD; ++u) {
        const int idx = t + u * C::NT;
        gf4 x = {0.f, 0.f, 0.f, 0.f};
        if (src[u]) {
          const int64_t left = sg.numel - (b0 + 4 * (idx % QV));
#pragma unroll
          for (int z = 0; z < 4; ++z) if (z < left) x[z] = gld<float>(src[u] + b0, z);
        }
        v[u] = x;
      }
    }
  };
  auto put = [&](int buf) {
    float* L = lds0 + buf * C::KP * kGS;
#pragma unroll
    for (int u = 0; u < C::NLD; ++u) {
      const int idx = t + u * C::NT;
      if (C::NLD * C::NT == C::KP * QV || idx < C::KP * QV) *(gf4*)&L[(idx / QV) * kGS + 4 * (idx % QV)] = v[u];
    }
  };
  const int64_t c0 = nchunks * blockIdx.x / gridDim.x, c1 = nchunks * (blockIdx.x + 1) / gridDim.x;
  if (c0 < c1) {
    load(c0);
    put(0);
    if (c0 + 1 < c1) load(c0 + 1);
  }
  __syncthreads();
  int cur = 0;
  for (int64_t ch = c0; ch < c1; ++ch, cur ^= 1) {
    const float* L = lds0 + cur * C::KP * kGS;
    // the centre of the chunk's coordinates, by every wave for itself: the median of clients 0..4
    // (fewer clients: of 0..2, or client 0); padding coordinates are 0 everywhere, so y = 0 there
#pragma unroll
    for (int e = lane; e < kGE; e += 64) {
      float c;
      if (k >= 5) {
        const float a = L[e], b = L[kGS + e], cc = L[2 * kGS + e], d = L[3 * kGS + e], f = L[4 * kGS + e];
        c = __builtin_amdgcn_fmed3f(f, fmaxf(fminf(a, b), fminf(cc, d)), fminf(fmaxf(a, b), fmaxf(cc, d)));
      } else if (k >= 3) {
        c = __builtin_amdgcn_fmed3f(L[e], L[kGS + e], L[2 * kGS + e]);
      } else {
        c = L[e];
      }
      cen[e] = c;
    }
    __builtin_amdgcn_wave_barrier();  // the wave's own LDS writes are seen by its later reads (in order)
    // no padding mask: rows >= k are staged as zeros and their G entries are never read
    if constexpr (S16) {
      // lane (li, kk) reads unit 4 G + kk (coordinates 16 G + 4 kk .. + 3) of its blocks' rows: the k
      // index of MFMA m is coordinate 16 G + 4 kk + m (any assignment works when A and B agree);
      // rows 528 bytes apart, so the 16 rows of one b128 read hit distinct banks
#pragma unroll
      for (int gi = 0; gi < kGE / 16 / C::R; ++gi) {
        const int G = r16 + gi * C::R;
        const int u4 = 4 * (4 * G + kk);
        const gf4 cc = *(const gf4*)&cen[u4];
        const gf4 y0 = *(const gf4*)&L[ro[0] + u4] - cc;
        const gf4 y1 = *(const gf4*)&L[ro[1] + u4] - cc;
        if (dg) {  // (a,a), (a,b), (b,b)
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            a16[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(y0[m], y0[m], a16[0], 0, 0, 0);
            a16[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(y0[m], y1[m], a16[1], 0, 0, 0);
            a16[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(y1[m], y1[m], a16[2], 0, 0, 0);
          }
        } else if (typ == 1) {  // (p,q), (p,r), (q,r)
          const gf4 y2 = *(const gf4*)&L[ro[2] + u4] - cc;
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            a16[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(y0[m], y1[m], a16[0], 0, 0, 0);
            a16[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(y0[m], y2[m], a16[1], 0, 0, 0);
            a16[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(y1[m], y2[m], a16[2], 0, 0, 0);
          }
        } else {  // (a,p), (a,q)
          const gf4 y2 = *(const gf4*)&L[ro[2] + u4] - cc;
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            a16[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(y0[m], y1[m], a16[0], 0, 0, 0);
            a16[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(y0[m], y2[m], a16[1], 0, 0, 0);
          }
        }
      }
    } else {
      const float* La = L + ra * kGS + 4 * half;
      const float* Lb = L + rb * kGS + 4 * half;
      const float* cr = cen + 4 * half;
#pragma unroll
      for (int g = r; g < kGE / 8; g += C::R) {
        const gf4 cc = *(const gf4*)&cr[8 * g];
        const gf4 ya = *(const gf4*)&La[8 * g] - cc;
        const gf4 yb = diag ? ya : *(const gf4*)&Lb[8 * g] - cc;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ya.x, yb.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ya.y, yb.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ya.z, yb.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ya.w, yb.w, acc, 0, 0, 0);
      }
    }
    // float32 runs of FL chunks (FL kGE / R coordinates of this split: 128 / 256) -> float64
    constexpr int FL = KB == 1 ? 4 : 2;
    if ((ch - c0) % FL == FL - 1 || ch + 1 == c1) {
      if constexpr (S16) {
#pragma unroll
        for (int x = 0; x < 3; ++x)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            accd[4 * x + q] += (double)a16[x][q];
            a16[x][q] = 0.0f;
          }
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          accd[q] += (double)acc[q];
          acc[q] = 0.0f;
        }
      }
    }
    if (ch + 1 < c1) {
      put(cur ^ 1);  // chunk ch + 1 (in registers); buffer cur ^ 1 was last read before the last barrier
      if (ch + 2 < c1) load(ch + 2);
    }
    __syncthreads();  // one barrier per chunk
  }
  if constexpr (S16) {
    // 16x16 C/D layout: register q of lane l is row 4 (l >> 4) + q, column l & 15 of its tile; tile
    // (A, B) of the 16-blocks lands in 32x32 tile (A / 2, B / 2), quadrant (A % 2, B % 2), of this
    // block's partial (the k_gram_reduce layout); a diagonal 32x32 tile's lower-left quadrant, never
    // read, is written as zeros by its diagonal-pair wave.  K in (32, 64]: the 4 splits of a set are
    // summed in split order through LDS first (the chunk buffers are free now)
    if constexpr (C::R > 1) {
      double* red = (double*)gl;  // [W][12][64]
#pragma unroll
      for (int q = 0; q < 12; ++q) red[(int64_t)w * 768 + q * 64 + lane] = accd[q];
      __syncthreads();
      if (r16 != 0) return;
#pragma unroll
      for (int q = 0; q < 12; ++q)
        for (int rr = 1; rr < C::R; ++rr) accd[q] += red[(int64_t)(4 * rr + ((set16 - rr + 4) % 4)) * 768 + q * 64 + lane];
    }
    double* o = partial + (int64_t)blockIdx.x * C::T * 1024;
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      if (typ == 2 && x == 2) break;  // a cross pair has two tiles
      const int pa = x == 2 ? 1 : 0, pb = dg ? (x == 0 ? 0 : 1) : (x == 0 ? 1 : 2);
      const int A = blk[pa], Bk = blk[pb];
      const int I = A >> 1, J = Bk >> 1;
      const int t32 = I * KB - I * (I - 1) / 2 + (J - I);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        o[(int64_t)t32 * 1024 + (16 * (A & 1) + 4 * kk + q) * 32 + 16 * (Bk & 1) + li] = accd[4 * x + q];
    }
    if (dg) {
      const int I = blk[0] >> 1, t32 = I * KB - I * (I - 1) / 2;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[(int64_t)t32 * 1024 + (16 + 4 * kk + q) * 32 + li] = 0.0;
    }
    return;
  } else {
    // the R splits of a tile summed in split order through LDS (the chunk buffers are free now), then
    // partial[(block * T + tile) * 1024 + row * 32 + col]; C/D layout of the 32x32 f32 MFMA: register q
    // of lane l holds row (q & 3) + 8 (q >> 2) + 4 (l >> 5), column l & 31
    double* red = (double*)gl;  // [W][1024]
    if (C::R > 1) {
#pragma unroll
      for (int q = 0; q < 16; ++q) red[(int64_t)w * 1024 + q * 64 + lane] = accd[q];
      __syncthreads();
    }
    if (r == 0) {
      double* o = partial + ((int64_t)blockIdx.x * C::T + ti) * 1024;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        double sm = accd[q];
        for (int rr = 1; rr < C::R; ++rr) sm += red[(int64_t)(w + rr) * 1024 + q * 64 + lane];
        const int row = (q & 3) + 8 * (q >> 2) + 4 * half;
        o[row * 32 + lrow] = sm;
      }
    }
  }
}

// K in (96, 128], bf16x3 split form (r06).  The f32-input MFMA issues at the FP32 vector rate (32
// cycles per v_mfma_f32_16x16x4_f32 on a SIMD); the bf16 MFMA is 16x faster per product
// (v_mfma_f32_16x16x32_bf16: 32 products per lane pair in 16 cycles).  So y = x - c (float32, as the
// forms above) is split EXACTLY into three bf16 values, y = h + m + l (8 + 8 + 8 significant bits of
// y's 24; each remainder is exact in float32), once per element and chunk into three LDS planes, and
//   G_ab = H_a H_b^T + H_a M_b^T + M_a H_b^T + H_a L_b^T + L_a H_b^T + M_a M_b^T
// on the bf16 matrix cores, accumulated in float32 (the dropped M L^T + L M^T + L L^T are <= 2^-25 of
// a product: below the float32 rounding of the sum).  Per chunk and tile that is 4 groups x 6 MFMAs
// x 16 cycles = 384 instead of 32 x 32 = 1,024 MFMA cycles; the split costs ~5 VALU per element,
// once per workgroup instead of once per wave and operand read.
// Per chunk (128 coordinates, the same 12-wave tile map as the S16 form, kG16Blocks): A) the staged
// rows 0..4 go to LDS; barrier; B) every thread computes the chunk's centre (median of clients 0..4)
// at its one coordinate quad (r06: no centre rows); C) every thread splits its staged elements into the planes, then issues the
// next chunk's loads (in flight during the MFMAs); barrier; D) MFMAs.  The planes are single-buffered:
// the barrier of the next chunk's step A separates its step C from this chunk's reads.
constexpr int kG3S = kGE + 8;  // bf16 per plane row: 272-byte rows, 16-lane b128 reads conflict-free
typedef __bf16 gbf8 __attribute__((ext_vector_type(8)));
typedef __bf16 gbf4 __attribute__((ext_vector_type(4)));
// L = 1 (K in (32, 64] only, the default there): 8 waves in 2 splits, two workgroups per CU -- two
// chunks of loads in flight per CU instead of one: K = 64 1.01-1.03 -> 0.84-0.86 ms (profiles/r06s)
template <int KB, int L = 0>
struct Gram3Cfg {
  static_assert(KB >= 2 && KB <= 4, "16x16 wave tables for 4, 6 or 8 client blocks of 16");
  static_assert(L == 0 || KB <= 3, "the two-workgroup layouts are for 4 or 6 client blocks of 16");
  static constexpr int KP = 32 * KB, QV = kGE / 4;
  static constexpr int W = KB == 4 ? 12 : KB == 3 ? 7 : L ? 8 : 16, NT = W * 64;
  static constexpr int R = KB == 2 ? (L ? 2 : 4) : 1;          // coordinate splits (groups of 32 per chunk / R)
  static constexpr int FL = KB == 2 && !L ? 2 : 1;              // chunks per float32 run (64 products at K <= 64)
  static constexpr int NLD = (KP * QV + NT - 1) / NT;           // staged 16-byte vectors per thread (6 / 7 / 2)
  static constexpr bool PRE = KB != 2 && !L;                    // next group's fragments read ahead (VGPRs)
  static constexpr int PLANE = KP * kG3S;                       // bf16 per plane
  static constexpr size_t PLANE_BYTES = (size_t)3 * PLANE * 2;  // h, m, l
  // L = 1 at K in (64, 96] (the default there): the client pointers in LDS instead of 7 pointer
  // pairs per thread and two planes live at a time in the MFMA phase -- the registers a second
  // workgroup per CU needs (124 of 128 per lane; 2 x 81.7 KB of LDS): K = 96 1.45-1.47 -> 1.37-1.39 ms
  // (profiles/r06y)
  static constexpr bool PT = L && KB == 3;
  static constexpr size_t STAGE = PLANE_BYTES + sizeof(float) * 5 * kGE + (PT ? sizeof(void*) * KP : 0);
  static_assert(NT % QV == 0, "a thread's staged vectors share one coordinate quad (its centre)");
  static constexpr size_t RED = R > 1 ? sizeof(double) * W * 768 : 0;               // the splits' sums
  static constexpr size_t LDS = STAGE > RED ? STAGE : RED;
};

__device__ __forceinline__ float bf_f(__bf16 b) { return (float)b; }

template <int KB, bool VEC, int L = 0>
__global__ void __launch_bounds__((Gram3Cfg<KB, L>::NT)) __attribute__((amdgpu_waves_per_eu(KB >= 3 && !L ? 3 : 4)))
k_pair_gram3(const PSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k,
             int64_t nchunks, double* __restrict__ partial, unsigned* __restrict__ ctr) {
  using C = Gram3Cfg<KB, L>;
  constexpr int QV = C::QV;
  if (blockIdx.x == 0 && threadIdx.x == 0) *ctr = 0u;  // k_gram_reduce's arrival counter
  extern __shared__ __attribute__((aligned(16))) char g3[];
  __bf16* const planes = (__bf16*)g3;
  float* const c5 = (float*)(g3 + C::PLANE_BYTES);  // [5][kGE] raw rows 0..4
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 15, kk = lane >> 4;
  // the wave's tile set (the S16 forms' tables): type 0 a diagonal pair (b0,b0), (b0,b1), (b1,b1);
  // 1 a triangle (b0,b1), (b0,b2), (b1,b2); 2 a cross pair (b0,b1), (b0,b2) -- and its coordinate split
  const int set16 = KB >= 3 ? w : (w % 4 + w / 4) % 4;
  const int r16 = KB >= 3 ? 0 : w / 4;
  const int typ = KB == 4 ? (w < 4 ? 0 : 1) : KB == 3 ? kG16Sets3[set16][0] : kG16Sets2[set16][0];
  const bool dg = typ == 0;
  const int ntile = typ == 2 ? 2 : 3;
  int blk[3], ro[3];
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    blk[x] = KB == 4 ? kG16Blocks[w][x] : KB == 3 ? kG16Sets3[set16][1 + x] : kG16Sets2[set16][1 + x];
    ro[x] = (16 * blk[x] + li) * kG3S + 8 * kk;
  }
  gf4 a16[3];
  double accd[12];
#pragma unroll
  for (int x = 0; x < 3; ++x) a16[x] = gf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 12; ++q) accd[q] = 0.0;
  gf4 v[C::NLD];
  const float* src[C::PT ? 1 : C::NLD];
  const float** const ptab = (const float**)(g3 + C::PLANE_BYTES + sizeof(float) * 5 * kGE);  // [KP] if PT
  int cseg = -1;
  auto load = [&](int64_t ch) {  // as k_pair_gram: client rows, coalesced 16-byte loads
    const int si = nseg > 1 ? find_seg(segs, nseg, ch) : 0;
    const PSeg sg = segs[si];
    if (si != cseg) {
      cseg = si;
      if constexpr (C::PT) {  // (a uniform branch: every thread reaches both barriers)
        __syncthreads();      // every thread's loads from the previous segment's table are issued
        if (t < C::KP) ptab[t] = t < k ? (const float*)ptrs[sg.ptr_base + t] : nullptr;
        __syncthreads();
      } else {
#pragma unroll
        for (int u = 0; u < C::NLD; ++u) {
          const int idx = t + u * C::NT;
          const int cl = idx / QV;
          src[u] = idx < C::KP * QV && cl < k ? (const float*)ptrs[sg.ptr_base + cl] + 4 * (idx % QV) : nullptr;
        }
      }
    }
    auto srcp = [&](int u) -> const float* {
      if constexpr (C::PT) {
        const int idx = t + u * C::NT;
        const float* b = idx < C::KP * QV ? ptab[idx / QV] : nullptr;
        return b ? b + 4 * (idx % QV) : nullptr;
      } else {
        return src[u];
      }
    };
    const int64_t b0 = (ch - sg.tile_start) * kGE;
    if (VEC && b0 + kGE <= sg.numel) {
#pragma unroll
      for (int u = 0; u < C::NLD; ++u) {
        const gf4 z = {0.f, 0.f, 0.f, 0.f};
        const float* sp = srcp(u);
        v[u] = sp ? *(const __attribute__((address_space(1))) gf4*)(sp + b0) : z;
      }
    } else {
#pragma unroll
      for (int u = 0; u < C::NLD; ++u) {
        const int idx = t + u * C::NT;
        gf4 x = {0.f, 0.f, 0.f, 0.f};
        const float* sp = srcp(u);
        if (sp) {
          const int64_t left = sg.numel - (b0 + 4 * (idx % QV));
#pragma unroll
          for (int z = 0; z < 4; ++z) if (z < left) x[z] = gld<float>(sp + b0, z);
        }
        v[u] = x;
      }
    }
  };
  const int64_t c0 = nchunks * blockIdx.x / gridDim.x, c1 = nchunks * (blockIdx.x + 1) / gridDim.x;
  if (c0 < c1) load(c0);
  for (int64_t ch = c0; ch < c1; ++ch) {
    // A) rows 0..4 (staged by threads 0..159 in their first vector) to LDS
    if (t < 5 * QV) *(gf4*)&c5[(t / QV) * kGE + 4 * (t % QV)] = v[0];
    __syncthreads();  // also: every wave is done reading the planes of chunk ch - 1
    // B) the chunk's centre at this thread's coordinate quad (every staged vector of the thread is at
    // quad t % QV): the median of clients 0..4 (k > 32 here)
    const int q = t % QV;
    gf4 cq;
    {
      const gf4 a = *(const gf4*)&c5[4 * q], b = *(const gf4*)&c5[kGE + 4 * q],
                 c = *(const gf4*)&c5[2 * kGE + 4 * q], d = *(const gf4*)&c5[3 * kGE + 4 * q],
                 f = *(const gf4*)&c5[4 * kGE + 4 * q];
#pragma unroll
      for (int z = 0; z < 4; ++z)
        cq[z] = __builtin_amdgcn_fmed3f(f[z], fmaxf(fminf(a[z], b[z]), fminf(c[z], d[z])),
                                        fminf(fmaxf(a[z], b[z]), fmaxf(c[z], d[z])));
    }
    // C) y = x - c split into h + m + l, written to the three planes
#pragma unroll
    for (int u = 0; u < C::NLD; ++u) {
      const int idx = t + u * C::NT;
      if (C::NLD * C::NT == C::KP * QV || idx < C::KP * QV) {
        const int cl = idx / QV;
        const gf4 y = v[u] - cq;
        gbf4 h, m, l;
#pragma unroll
        for (int z = 0; z < 4; ++z) {
          h[z] = (__bf16)y[z];
          const float r = y[z] - bf_f(h[z]);
          m[z] = (__bf16)r;
          l[z] = (__bf16)(r - bf_f(m[z]));
        }
        __bf16* const row = planes + cl * kG3S + 4 * q;
        *(gbf4*)row = h;
        *(gbf4*)(row + C::PLANE) = m;
        *(gbf4*)(row + 2 * C::PLANE) = l;
      }
    }
    if (ch + 1 < c1) load(ch + 1);  // in flight during the MFMAs
    __syncthreads();
    // D) the wave's 16x16 tiles over its groups of 32 coordinates of the chunk, one code path per
    // tile-set type (the operand registers of every MFMA fixed at compile time: no fragment copies)
    // with the next group's fragments read before this group's MFMAs
    auto tiles = [&](auto typc) {
      constexpr int TYP = decltype(typc)::value;
      constexpr int NB = TYP == 0 ? 2 : 3, NT3 = TYP == 2 ? 2 : 3;
      constexpr int NG = kGE / 32 / C::R;
      if constexpr (C::PT) {
        // (the two-workgroup layout at K in (64, 96]: 128 registers per lane) two planes live at a
        // time -- H and M for M M, H M, M H, then L in M's registers for H L, L H and H H
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
          const int G = r16 + gi * C::R;
          gbf8 fh[NB], fx[NB];
#pragma unroll
          for (int x = 0; x < NB; ++x) {
            fh[x] = *(const gbf8*)&planes[ro[x] + 32 * G];
            fx[x] = *(const gbf8*)&planes[C::PLANE + ro[x] + 32 * G];
          }
#pragma unroll
          for (int x = 0; x < NT3; ++x) {
            const int pa = x == 2 ? 1 : 0, pb = TYP == 0 ? (x == 0 ? 0 : 1) : (x == 0 ? 1 : 2);
            gf4 acc = a16[x];
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[pa], fx[pb], acc, 0, 0, 0);  // M M
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[pa], fx[pb], acc, 0, 0, 0);  // H M
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[pa], fh[pb], acc, 0, 0, 0);  // M H
            a16[x] = acc;
          }
#pragma unroll
          for (int x = 0; x < NB; ++x) fx[x] = *(const gbf8*)&planes[2 * C::PLANE + ro[x] + 32 * G];
#pragma unroll
          for (int x = 0; x < NT3; ++x) {
            const int pa = x == 2 ? 1 : 0, pb = TYP == 0 ? (x == 0 ? 0 : 1) : (x == 0 ? 1 : 2);
            gf4 acc = a16[x];
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[pa], fx[pb], acc, 0, 0, 0);  // H L
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[pa], fh[pb], acc, 0, 0, 0);  // L H
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh[pa], fh[pb], acc, 0, 0, 0);  // H H
            a16[x] = acc;
          }
        }
        return;
      }
      gbf8 f[NB][3], fn[NB][3];
      auto rd = [&](gbf8 (&d)[NB][3], int G) {
#pragma unroll
        for (int x = 0; x < NB; ++x)
#pragma unroll
          for (int p = 0; p < 3; ++p) d[x][p] = *(const gbf8*)&planes[p * C::PLANE + ro[x] + 32 * G];
      };
      rd(f, r16);
#pragma unroll
      for (int gi = 0; gi < NG; ++gi) {
        if (C::PRE && gi + 1 < NG) rd(fn, r16 + (gi + 1) * C::R);
#pragma unroll
        for (int x = 0; x < NT3; ++x) {
          // type 0: (0,0), (0,1), (1,1); type 1: (0,1), (0,2), (1,2); type 2: (0,1), (0,2)
          const int pa = x == 2 ? 1 : 0, pb = TYP == 0 ? (x == 0 ? 0 : 1) : (x == 0 ? 1 : 2);
          gf4 acc = a16[x];
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[pa][1], f[pb][1], acc, 0, 0, 0);  // M M
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[pa][0], f[pb][2], acc, 0, 0, 0);  // H L
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[pa][2], f[pb][0], acc, 0, 0, 0);  // L H
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[pa][0], f[pb][1], acc, 0, 0, 0);  // H M
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[pa][1], f[pb][0], acc, 0, 0, 0);  // M H
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[pa][0], f[pb][0], acc, 0, 0, 0);  // H H
          a16[x] = acc;
        }
        if (gi + 1 < NG) {
          if constexpr (C::PRE) {
#pragma unroll
            for (int x = 0; x < NB; ++x)
#pragma unroll
              for (int p = 0; p < 3; ++p) f[x][p] = fn[x][p];
          } else {
            rd(f, r16 + (gi + 1) * C::R);
          }
        }
      }
    };
    if (typ == 0) tiles(std::integral_constant<int, 0>{});
    else if (KB == 4 || typ == 1) tiles(std::integral_constant<int, 1>{});
    else tiles(std::integral_constant<int, 2>{});
    // float32 runs -> float64: every chunk for K > 96 (128 coordinates, 24 MFMAs per tile: the bf16
    // MFMA's accumulation carries a small bias that grows with the run, profiles/r06b), every second
    // chunk for K <= 64 (64 coordinates of the split, 12 MFMAs)
    if (C::FL == 1 || (ch - c0) % C::FL == C::FL - 1 || ch + 1 == c1) {
#pragma unroll
      for (int x = 0; x < 3; ++x)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          accd[4 * x + q] += (double)a16[x][q];
          a16[x][q] = 0.0f;
        }
    }
  }
  // epilogue: as k_pair_gram<KB, *, true> -- the splits summed in split order through LDS (the planes
  // are free now), then 16x16 tile (A, B) into 32x32 tile (A / 2, B / 2), quadrant (A % 2, B % 2); a
  // diagonal 32x32 tile's lower-left quadrant written as zeros
  __syncthreads();
  if constexpr (C::R > 1) {
    double* red = (double*)g3;  // [W][12][64]
#pragma unroll
    for (int q = 0; q < 12; ++q) red[(int64_t)w * 768 + q * 64 + lane] = accd[q];
    __syncthreads();
    if (r16 != 0) return;
#pragma unroll
    for (int q = 0; q < 12; ++q)
      for (int rr = 1; rr < C::R; ++rr) accd[q] += red[(int64_t)(4 * rr + ((set16 - rr + 4) % 4)) * 768 + q * 64 + lane];
  }
  double* o = partial + (int64_t)blockIdx.x * gram_T_c<KB>() * 1024;
#pragma unroll
  for (int x = 0; x < 3; ++x) {
    if (x == 2 && typ == 2) break;
    const int pa = x == 2 ? 1 : 0, pb = dg ? (x == 0 ? 0 : 1) : (x == 0 ? 1 : 2);
    const int A = blk[pa], Bk = blk[pb];
    const int I = A >> 1, J = Bk >> 1;
    const int t32 = I * KB - I * (I - 1) / 2 + (J - I);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      o[(int64_t)t32 * 1024 + (16 * (A & 1) + 4 * kk + q) * 32 + 16 * (Bk & 1) + li] = accd[4 * x + q];
  }
  if (dg) {
    const int I = blk[0] >> 1, t32 = I * KB - I * (I - 1) / 2;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[(int64_t)t32 * 1024 + (16 + 4 * kk + q) * 32 + li] = 0.0;
  }
  (void)ntile;
}

// K <= 32 with an LDS-DMA ring (r05).  The register-staged kernel above waits vmcnt(0) for its one
// chunk in flight at every put (the compiler cannot count a ring of register loads across the loop:
// r05k, depths 2-4 all slower), and its time splits (r05o, measurement knobs on a first 4-wave ring
// kernel): the read alone 251 us, + MFMA 104, + the centre 42 (every wave computed all 128), + the
// float64 flush 29 -- the compute was not hidden under the read.  So: ONE workgroup of 16 waves per
// CU (4 per SIMD), a ring of NB 32-KB chunk buffers filled by global_load_lds_dwordx4 (no staging
// registers, no ds_write pass), NB - 1 chunks in flight across the one raw s_barrier per chunk with a
// counted vmcnt (2 DMA instructions per thread and chunk: vmcnt(2 (NB - 2)) retires exactly chunk
// i); each wave computes the centre of only ITS 16 coordinates, and flushes float32 into float64
// every second chunk (64 products per run).  One wave-instruction of DMA writes one client row
// (64 lanes x 16 bytes = 256 coordinates), lane-linear, so the bank swizzle goes on the SOURCE
// address: physical unit p of row r holds coordinates 4 (p ^ (r & 15)) .. + 3 (16 rows read at one
// unit offset hit 16 distinct units: conflict-free ds_read_b128).  Rows k..31 load client 0's
// coordinates and are zeroed by the mask, as the register kernel's zero rows are (a non-finite input
// makes D non-finite either way, and the kappa guard hands the call to the direct kernels).  Only
// full 256-coordinate chunks go through the ring (tile_start = the segment's first full chunk, pad =
// 1 when a partial chunk follows); partial chunks are taken after the ring has drained, segment s by
// workgroup s % gridDim.x, through bounds-checked register loads.
// CW coordinates per chunk, WV waves per workgroup (each wave: CW / (8 WV) = 2 groups of every chunk)
template <int NB, int CW, int WV>
__global__ void __launch_bounds__(64 * WV) __attribute__((amdgpu_waves_per_eu(4)))
k_pair_gram_ring(const PSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k,
                 int64_t nfull, double* __restrict__ partial, unsigned* __restrict__ ctr) {
  constexpr int RS = CW, BUF = 32 * RS;        // floats per client row / per ring buffer
  constexpr int U = CW / 4, RPI = 64 / U;      // 16-byte units per row, rows per DMA wave-instruction
  constexpr int IPW = 32 / RPI / WV;           // DMA instructions per wave and chunk
  constexpr int NT = 64 * WV;
  static_assert(CW == 16 * WV && IPW >= 1 && U >= 16, "16 coordinates per wave and chunk");
  static_assert(NB * BUF * 4 >= WV * 768 * 8, "the epilogue's float64 wave sums reuse the ring");
  extern __shared__ __attribute__((aligned(16))) float gl[];  // [NB][32][CW] swizzled, then [WV][16] centres
  if (blockIdx.x == 0 && threadIdx.x == 0) *ctr = 0u;  // k_gram_reduce's arrival counter
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);  // coordinates 16 w .. 16 w + 15 of every chunk
  float* const cen = gl + NB * BUF + w * 16;
  // 16x16x4 MFMA lanes: i = lane & 15 (client i of block 0, 16 + i of block 1), kk = lane >> 4
  const int li = lane & 15, kk = lane >> 4;
  gf4 t00 = {0.f, 0.f, 0.f, 0.f}, t01 = t00, t11 = t00;  // tiles (0,0), (0,1), (1,1) of the 32x32 G
  double a00[4] = {0, 0, 0, 0}, a01[4] = {0, 0, 0, 0}, a11[4] = {0, 0, 0, 0};
  const float* cp[IPW];  // DMA j of this wave: client rows RPI (IPW w + j) + lane / U
  int cseg = -1;
  int64_t cbase = 0;
  auto seg_ptrs = [&](int si) {
    const PSeg sg = segs[si];
    cseg = si;
    cbase = sg.tile_start;
#pragma unroll
    for (int j = 0; j < IPW; ++j) {
      const int r0 = RPI * (IPW * w + j);  // wave-uniform: the row pointers are scalar loads
      const void* p0 = ptrs[sg.ptr_base + (r0 < k ? r0 : 0)];
      const void* p1 = RPI > 1 ? ptrs[sg.ptr_base + (r0 + 1 < k ? r0 + 1 : 0)] : p0;
      const int row = r0 + lane / U;
      cp[j] = (const float*)(lane / U ? p1 : p0) + 4 * ((lane % U) ^ (row & 15));
    }
  };
  auto issue = [&](int64_t ch, int buf) {  // full chunk ch -> ring buffer buf
    const int si = nseg > 1 ? find_seg(segs, nseg, ch) : 0;
    if (si != cseg) seg_ptrs(si);
    const int64_t off = (ch - cbase) * CW;
#pragma unroll
    for (int j = 0; j < IPW; ++j)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(cp[j] + off),
                                       (__attribute__((address_space(3))) void*)(gl + buf * BUF + RPI * (IPW * w + j) * RS),
                                       16, 0, 0);
  };
  // G on v_mfma_f32_16x16x4_f32 over the three tiles of the upper triangle (the 32x32 form's (1,0)
  // quadrant is the (0,1) tile transposed: 3 x 32 instead of 2 x 64 MFMA cycles per 4 coordinates;
  // K <= 16 needs tile (0,0) alone).  This wave takes coordinates 16 w .. 16 w + 15 of the chunk: lane
  // (li, kk) reads 16-byte unit 4 w + kk of client rows li and 16 + li (one ds_read_b128 each; the k
  // index of MFMA m is coordinate 4 kk + m -- any assignment works when A and B agree).  Rows >= k hold
  // client 0's coordinates (DMA) or zeros (partial chunks): their G entries are never read.
  auto compute = [&](const float* L, bool flush) {
    if (lane < 16) {  // the centre of this wave's 16 coordinates (median of clients 0..4)
      const int u = 4 * w + (lane >> 2), z = lane & 3;
      float c;
      if (k >= 5) {
        const float a0 = L[4 * u + z], b0 = L[RS + 4 * (u ^ 1) + z], c0 = L[2 * RS + 4 * (u ^ 2) + z],
                    d0 = L[3 * RS + 4 * (u ^ 3) + z], f0 = L[4 * RS + 4 * (u ^ 4) + z];
        c = __builtin_amdgcn_fmed3f(f0, fmaxf(fminf(a0, b0), fminf(c0, d0)), fminf(fmaxf(a0, b0), fmaxf(c0, d0)));
      } else if (k >= 3) {
        c = __builtin_amdgcn_fmed3f(L[4 * u + z], L[RS + 4 * (u ^ 1) + z], L[2 * RS + 4 * (u ^ 2) + z]);
      } else {
        c = L[4 * u + z];
      }
      cen[lane] = c;
    }
    __builtin_amdgcn_wave_barrier();
    const int pu = 4 * ((4 * w + kk) ^ li);  // physical unit of logical unit 4 w + kk in rows li and 16 + li
    const gf4 cc = *(const gf4*)&cen[4 * kk];
    const gf4 y0 = *(const gf4*)&L[li * RS + pu] - cc;
    if (k > 16) {
      const gf4 y1 = *(const gf4*)&L[(16 + li) * RS + pu] - cc;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        t00 = __builtin_amdgcn_mfma_f32_16x16x4f32(y0[m], y0[m], t00, 0, 0, 0);
        t01 = __builtin_amdgcn_mfma_f32_16x16x4f32(y0[m], y1[m], t01, 0, 0, 0);
        t11 = __builtin_amdgcn_mfma_f32_16x16x4f32(y1[m], y1[m], t11, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int m = 0; m < 4; ++m) t00 = __builtin_amdgcn_mfma_f32_16x16x4f32(y0[m], y0[m], t00, 0, 0, 0);
    }
    if (flush) {  // float32 runs of 4 chunks (64 products per entry) -> float64
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a00[q] += (double)t00[q];
        a01[q] += (double)t01[q];
        a11[q] += (double)t11[q];
        t00[q] = t01[q] = t11[q] = 0.0f;
      }
    }
  };
  // this workgroup's run of full chunks; ring fill past its end re-loads chunk 0 (L2-resident after
  // the first) into a buffer nobody reads, so every iteration has NB - 1 chunks in flight
  const int64_t G = gridDim.x, B = blockIdx.x;
  const int64_t c0 = nfull * B / G, n = nfull * (B + 1) / G - c0;
  if (n > 0) {
#pragma unroll
    for (int s = 0; s < NB - 1; ++s) issue(s < n ? c0 + s : 0, s);
    for (int64_t i = 0; i < n; ++i) {
      // s_waitcnt vmcnt(IPW (NB - 2)) lgkmcnt(0) (gfx9 encoding: vmcnt [3:0] + [15:14], expcnt [6:4] = 7: no wait)
      __builtin_amdgcn_s_waitcnt(0x0070 | ((IPW * (NB - 2)) & 0xF) | (((IPW * (NB - 2)) >> 4) << 14));
      __builtin_amdgcn_s_barrier();  // chunk i landed for every wave; every wave is done with buffer (i - 1) % NB
      const int64_t nx = i + NB - 1;
      issue(nx < n ? c0 + nx : 0, (int)(nx % NB));
      compute(gl + (int)(i % NB) * BUF, (i & 3) == 3 || i + 1 == n);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0): the fill loads landed
  __syncthreads();
  // the partial chunks: segment s's last (numel % CW coordinates) by workgroup s % G, register loads
  // with bounds into buffer 0 (the same swizzle), then the same compute
  for (int64_t si = B; si < nseg; si += G) {
    const PSeg sg = segs[si];
    if (!sg.pad) continue;
    const int64_t b0 = (sg.numel / CW) * CW, left = sg.numel - b0;
    for (int idx = t; idx < 32 * U; idx += NT) {
      const int row = idx / U, u = idx % U;
      gf4 x = {0.f, 0.f, 0.f, 0.f};
      if (row < k) {
        const float* p = (const float*)ptrs[sg.ptr_base + row] + b0;
#pragma unroll
        for (int z = 0; z < 4; ++z) if (4 * u + z < left) x[z] = gld<float>(p, 4 * u + z);
      }
      *(gf4*)&gl[row * RS + 4 * (u ^ (row & 15))] = x;
    }
    __syncthreads();
    compute(gl, true);
    __syncthreads();
  }
  // the WV waves' sums added in wave order through LDS, then partial[block * 1024 + row * 32 + col]
  // (16x16 C/D layout: register q of lane l is row 4 (l >> 4) + q, column l & 15 of its tile; the
  // lower-left quadrant, never read, is written as zeros)
  double* red = (double*)gl;  // [WV][12][64]
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    red[(int64_t)w * 768 + q * 64 + lane] = a00[q];
    red[(int64_t)w * 768 + (4 + q) * 64 + lane] = a01[q];
    red[(int64_t)w * 768 + (8 + q) * 64 + lane] = a11[q];
  }
  __syncthreads();
  if (w == 0) {
    double* o = partial + (int64_t)blockIdx.x * 1024;
#pragma unroll
    for (int q = 0; q < 12; ++q) {
      double sum = red[q * 64 + lane];
      for (int v = 1; v < WV; ++v) sum += red[(int64_t)v * 768 + q * 64 + lane];
      const int tile = q >> 2, row = 4 * kk + (q & 3), col = li;
      const int R = tile == 2 ? 16 + row : row, C = tile == 0 ? col : 16 + col;
      o[R * 32 + C] = sum;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) o[(16 + 4 * kk + q) * 32 + li] = 0.0;
  }
}

// G entries of the T tiles summed over the per-block partials in a fixed order: a workgroup of 16
// waves takes 16 consecutive entries (entry = tile * 1024 + row * 32 + col) and splits the partial
// rows 64 ways (128-byte row reads), then the 64 split sums are added in split order through LDS;
// written to g (KP x KP, upper tiles only).
// The LAST workgroup to finish (an arrival counter the Gram kernel zeroed; release / acquire at agent
// scope around it) then forms D_ij = A_i + A_j - 2 G_ij for every pair into the k x k matrix and the
// largest kappa_ij = (A_i + A_j) / D_ij (+inf for D_ij <= 0 or a NaN) into *kmax -- the former
// k_gram_dist / k_gram_kmax launches, in this kernel's tail.
constexpr int kGRW = 16;  // waves per k_gram_reduce workgroup
template <int KB>
__global__ void __launch_bounds__(64 * kGRW)
k_gram_reduce(const double* __restrict__ partial, int nparts, double* __restrict__ g, int k, double* __restrict__ d,
              double* __restrict__ kmax, unsigned* __restrict__ ctr) {
  using C = GramCfg<KB>;
  __shared__ double red[kGRW * 64];
  __shared__ int last;
  // lane = (row lane rl, entry el): a workgroup takes kGRE consecutive entries and splits the rows
  // 64 ways (16 waves x 4 row lanes), so every lane has at most nparts / 64 rows to add (r05: one
  // entry per lane and 16 row splits left 32 dependent-latency rows per lane at K <= 32's 512
  // partials); each row read is kGRE x 8 = 128 contiguous bytes
  constexpr int kGRE = 16, RS = kGRW * 64 / kGRE;
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  const int el = lane % kGRE, rl = lane / kGRE;
  const int rs = v * (64 / kGRE) + rl;  // this lane's row split, 0 .. RS - 1
  const int64_t nent = (int64_t)C::T * 1024;
  const int64_t e = (int64_t)blockIdx.x * kGRE + el;
  double s = 0.0;
  int b = rs;
  for (; b + 7 * RS < nparts; b += 8 * RS) {  // 8 loads in flight, added in row order
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = partial[(int64_t)(b + u * RS) * nent + e];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += x[u];
  }
  for (; b < nparts; b += RS) s += partial[(int64_t)b * nent + e];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < kGRE) {  // the RS split sums in split order
    double tsum = 0.0;
    for (int u = 0; u < RS; ++u) tsum += red[(u / (64 / kGRE)) * 64 + (u % (64 / kGRE)) * kGRE + threadIdx.x];
    int bi, bj;
    gram_tile_kb<KB>((int)(e / 1024), bi, bj);
    const int row = (int)(e % 1024) / 32, col = (int)(e % 32);
    g[(int64_t)(32 * bi + row) * C::KP + 32 * bj + col] = tsum;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == gridDim.x - 1;
    if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (!last) return;
  double m = 0.0;
  for (int idx = threadIdx.x; idx < k * k; idx += 64 * kGRW) {
    const int i = idx / k, j = idx % k;
    if (j > i) {
      const double ai = g[(int64_t)i * C::KP + i], aj = g[(int64_t)j * C::KP + j], gij = g[(int64_t)i * C::KP + j];
      const double dd = ai + aj - 2.0 * gij;
      d[(int64_t)i * k + j] = dd;
      d[(int64_t)j * k + i] = dd;
      const double kap = (ai + aj) / dd;
      m = fmax(m, dd > 0.0 && kap >= 0.0 ? kap : __builtin_inf());  // NaN, negative or D <= 0: +inf
    } else if (j == i) {
      d[(int64_t)i * k + i] = 0.0;
    }
  }
  red[threadIdx.x] = m;
  __syncthreads();
  for (int w2 = 32 * kGRW; w2 > 0; w2 >>= 1) {
    if ((int)threadIdx.x < w2) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w2]);
    __syncthreads();
  }
  if (threadIdx.x == 0) *kmax = red[0];
}

bool gram_s16() {  // K in (32, 64] and (96, 128]: the 16x16 forms (FA_GRAM16=0: the 32x32 forms, A/B)
  static const bool on = [] {
    const char* e = getenv("FA_GRAM16");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool gram3() {  // K in (32, 128]: the bf16x3 split form (FA_GRAM3=0: the f32-input forms, A/B)
  static const bool on = [] {
    const char* e = getenv("FA_GRAM3");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool gram3_l2() {  // K in (32, 64]: the two-workgroup bf16x3 layout (Gram3Cfg<2, 1>; FA_GRAM3_L2=0: one, A/B)
  static const bool on = [] {
    const char* e = getenv("FA_GRAM3_L2");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool gram3_l3() {  // K in (64, 96]: the two-workgroup bf16x3 layout (Gram3Cfg<3, 1>; FA_GRAM3_L3=0: one, A/B)
  static const bool on = [] {
    const char* e = getenv("FA_GRAM3_L3");
    return !(e && e[0] == '0');
  }();
  return on;
}

int gram_glds() {  // K <= 32: the LDS-DMA ring kernel (FA_GRAM_GLDS=0: the register-staged k_pair_gram<1>, A/B)
  static const int d = [] {
    const char* e = getenv("FA_GRAM_GLDS");
    return e && e[0] == '0' ? 0 : 8;
  }();
  return d;
}

// workgroups: one per CU for K > 32 (12 / 12 / 10 waves, <= 128 VGPRs: 16 waves per CU); K <= 32 below
int gram_nblocks(int64_t nchunks, int kb) {
  static const int ov = [] {  // FA_GRAM_BLOCKS: measurement override (A/B)
    const char* e = getenv("FA_GRAM_BLOCKS");
    return e ? atoi(e) : 0;
  }();
  const bool two = (kb == 2 && gram3() && gram3_l2()) || (kb == 3 && gram3() && gram3_l3());  // 2 WGs / CU
  const int64_t cap = ov >= 64 && ov <= 8192 ? ov : two ? 512 : kb >= 2 ? 256 : 1024;
  return (int)std::max<int64_t>(1, std::min<int64_t>(nchunks, cap));
}

int gram_T(int kb) { return kb * (kb + 1) / 2; }
int gram_chunk(int) { return kGE; }

size_t gram_scratch(int32_t num_segments, const int64_t* seg_numel, int32_t k) {
  const int kb = (k + 31) / 32;
  int64_t nchunks = 0;
  for (int s = 0; s < num_segments; ++s)
    if (seg_numel[s] > 0) nchunks += (seg_numel[s] + gram_chunk(kb) - 1) / gram_chunk(kb);
  const size_t parts = (size_t)gram_nblocks(nchunks, kb);
  return align16(sizeof(double) * (parts * gram_T(kb) * 1024 + (size_t)(32 * kb) * (32 * kb) + 128));
}

size_t gram_lds(int kb) {
  const int T = gram_T(kb), R = kb == 1 ? 4 : kb == 2 ? 4 : kb == 3 ? 2 : 1;
  const bool s16 = (kb == 4 || kb == 2) && gram_s16();
  const int W = s16 ? (kb == 4 ? 12 : 16) : T * R;
  const size_t stage = sizeof(float) * (2 * (size_t)(32 * kb) * kGS + (size_t)W * kGE);
  return std::max(stage, sizeof(double) * (s16 ? 768 : 1024) * (size_t)W);  // the epilogue's split reduction
}

int pairdist_direct(fa_ctx* ctx, int diff_dtype, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                    const void* const* d_in, void* d_dist, void* d_scratch, size_t scratch_bytes, void* hip_stream,
                    const double* guard, double limit);

// The Gram form's error model and the guard it sets (Krum; calibrated on the box by
// tools/krum_kappa_sweep.py and tests/test_gpu_krum_band.py, profiles/r06b).  A G entry is accumulated
// in float32 runs of n products and the runs are added in float64.  With one random rounding per
// product (the MFMA's accumulator; the measured errors fit this, not one rounding per instruction)
// the run sums' error is ~0.25 u n sqrt(P) t for P coordinates of mean term t, i.e. sigma(A) / A ~
// 0.25 u n / sqrt(P) (u = 2^-24); D = A_i + A_j - 2 G_ij collects three such errors, so
// sigma(D) / D ~ 0.30 kappa u n / sqrt(P).  Measured (r06b, forced Gram form, max over every pair):
// K = 128, P = 1 M, kappa 15.8: 2.7e-7 = 3.8 sigma; K = 128, P = 11.7 M, kappa 1.29: 7e-9 = 4 sigma.
// The guard keeps the Gram result only while MARGIN sigma(D) / D <= 1e-6 (MARGIN = 6):
//   kappa <= 1e-6 / (6 x 0.30 x 2^-24 x n / sqrt(P)) = 9.3 sqrt(P) / n.
// Large models are unaffected (P = 11.7 M, K = 128: 124 > 16); small ones with long runs hand over to
// the direct kernel at lower kappa (P = 7,850, K = 128: 3.2).
// The bf16x3 split forms (k_pair_gram3) add a size-independent part: their measured error per unit
// kappa levels off with P (max over every pair, P >= 1 M: K in (96, 128] 5.4e-8 with 2-chunk runs
// (profiles/r06b), 2.1e-8 with 1-chunk runs (r06d); K in (32, 64] 7.4e-9) -- a bias of the bf16 MFMA's
// float32 accumulation that grows with the run -- so their bound is kappa (6 sigma(P) + b) <= 1e-6
// with b = 4e-8 / 1.2e-8, 1.9x / 1.6x the measured level.
struct GramRun {
  int n;     // float32 products per run of one G entry
  double b;  // size-independent relative error per unit kappa (0 for the f32-input forms)
};
GramRun gram_run(int kb, bool glds) {
  if (glds) return {64, 0.0};  // k_pair_gram_ring: 16 products per chunk, flushed every 4 chunks
  const bool g3 = kb >= 2 && gram3();
  switch (kb) {
    case 1: return {128, 0.0};                        // R = 4, FL = 4
    case 2: return {64, g3 ? 1.2e-8 : 0.0};           // f32: R = 4, FL = 2; bf16x3: R = 2, FL = 1 -- 64 either way
    case 3: return {128, g3 ? 4e-8 : 0.0};            // f32: R = 2, FL = 2; bf16x3: R = 1, FL = 1 (as K > 96)
    default: return g3 ? GramRun{128, 4e-8} : GramRun{256, 0.0};  // bf16x3: FL = 1; f32: R = 1, FL = 2
  }
}
constexpr double kGramSigma = 0.30 * 5.9604644775390625e-8;  // sigma(D) / D per unit kappa x sqrt(P) / n
double gram_kappa_bound(int64_t p_total, GramRun r) {
  return 1e-6 / (6.0 * kGramSigma * r.n / std::sqrt((double)std::max<int64_t>(p_total, 1)) + r.b);
}
bool gram_vec(int32_t num_segments, const int64_t* seg_numel, int32_t k, const void* const* d_in) {
  bool vec = true;
  for (int s = 0; s < num_segments; ++s)
    if (seg_numel[s] > 0)
      for (int i = 0; i < k; ++i) vec = vec && d_in[(int64_t)s * k + i] && ((uintptr_t)d_in[(int64_t)s * k + i] % 16 == 0);
  return vec;
}

}  // namespace

extern "C" {

int fa_pairwise_sqdist(fa_ctx* ctx, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                       const void* const* d_in, void* d_dist, void* d_scratch, size_t scratch_bytes,
                       void* hip_stream) {
  return fa_pairwise_sqdist_rt(ctx, FA_DTYPE_F32, num_segments, seg_numel, k, d_in, d_dist, d_scratch,
                               scratch_bytes, hip_stream);
}

int fa_pairwise_sqdist_rt(fa_ctx* ctx, int diff_dtype, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                          const void* const* d_in, void* d_dist, void* d_scratch, size_t scratch_bytes,
                          void* hip_stream) {
  return pairdist_direct(ctx, diff_dtype, num_segments, seg_numel, k, d_in, d_dist, d_scratch, scratch_bytes,
                         hip_stream, nullptr, 0.0);
}

}  // extern "C"

namespace {
// The direct (difference) kernels.  guard != nullptr: every launch returns at once unless *guard >
// limit -- the Gram form's fallback, decided on the device (no host round trip).
int pairdist_direct(fa_ctx* ctx, int diff_dtype, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                    const void* const* d_in, void* d_dist, void* d_scratch, size_t scratch_bytes, void* hip_stream,
                    const double* guard, double limit) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (diff_dtype != FA_DTYPE_F32 && diff_dtype != FA_DTYPE_BF16 && diff_dtype != FA_DTYPE_F16 &&
      diff_dtype != FA_DTYPE_F64)
    return fail(FA_ERR_INVALID, "fa_pairwise_sqdist_rt: diff_dtype must be F32, BF16, F16 or F64 (got %d)",
                diff_dtype);
  const bool f64 = diff_dtype == FA_DTYPE_F64;
  const int rt = diff_dtype == FA_DTYPE_BF16 ? 1 : diff_dtype == FA_DTYPE_F16 ? 2 : 0;
  if (k < 2 || k > kMaxPairK || num_segments <= 0 || !seg_numel || !d_in || !d_dist)
    return fail(FA_ERR_INVALID, "fa_pairwise_sqdist: invalid arguments (2 <= k <= %d)", kMaxPairK);
  const PairSplit q = pair_split(k);
  const int kp = q.kp, ntiles = q.ntiles, esplit = q.esplit, pe = q.pe;
  if (q.nthreads > kMaxPairThreads) return fail(FA_ERR_INVALID, "fa_pairwise_sqdist: k too large");
  int nseg = 0;
  int64_t nchunks = 0, nchunks64 = 0;
  for (int s = 0; s < num_segments; ++s) {
    if (seg_numel[s] < 0) return fail(FA_ERR_INVALID, "segment %d has negative numel", s);
    if (seg_numel[s] == 0) continue;
    for (int i = 0; i < k; ++i)
      if (!d_in[(int64_t)s * k + i]) return fail(FA_ERR_INVALID, "segment %d client %d: input NULL", s, i);
    ++nseg;
    nchunks += (seg_numel[s] + pe - 1) / pe;
    nchunks64 += (seg_numel[s] + kC64 - 1) / kC64;
  }
  const int64_t npairs = (int64_t)k * (k - 1) / 2;
  // workgroups: the same count for every diff dtype (fa_pairwise_sqdist_scratch_bytes sizes the
  // partials by it), float64 chunks spread over them
  const int nblocks = (int)std::max<int64_t>(1, std::min<int64_t>(nchunks, q.nblocks));
  if (scratch_bytes < sizeof(double) * (size_t)npairs * nblocks || !d_scratch)
    return fail(FA_ERR_INVALID, "fa_pairwise_sqdist: scratch must hold %zu bytes",
                sizeof(double) * (size_t)npairs * nblocks);
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  if (nseg == 0) {
    FA_HIP(hipMemsetAsync(d_dist, 0, sizeof(double) * (size_t)k * k, st));
    return FA_OK;
  }
  const size_t seg_bytes = align16(sizeof(PSeg) * nseg);
  const size_t ptr_bytes = sizeof(void*) * (size_t)nseg * k;
  fa_ctx::Slot* slot = nullptr;
  int rc = acquire_slot(ctx, seg_bytes + ptr_bytes, &slot);
  if (rc) return rc;
  char* h = (char*)slot->host;
  PSeg* hs = (PSeg*)h;
  const void** hp = (const void**)(h + seg_bytes);
  int j = 0;
  int64_t c0 = 0;
  const int64_t cpe = f64 ? kC64 : pe;  // coordinates per chunk
  for (int s = 0; s < num_segments; ++s) {
    const int64_t n = seg_numel[s];
    if (n == 0) continue;
    for (int i = 0; i < k; ++i) hp[(int64_t)j * k + i] = d_in[(int64_t)s * k + i];
    hs[j] = PSeg{n, c0, j * k, 0, 0};
    c0 += (n + cpe - 1) / cpe;
    ++j;
  }
  rc = stage(slot, seg_bytes + ptr_bytes, st, true);
  if (rc) return rc;
  const char* dv = (const char*)slot->dev;
  // FA_PAIR_PF=1: the next coordinate's LDS reads issued before this one's arithmetic.  Off by default:
  // r03g interleaved A/B, 2 x 2 runs, slower at every K (K = 32 / 64 / 128: 0.580-0.597 / 1.591-1.592 /
  // 4.97-5.00 ms without vs 0.598-0.616 / 1.627-1.634 / 5.12-5.14 with) -- at 16 waves per CU the LDS
  // latency is hidden by the other waves, and the extra 8 VGPRs of operands cost more
  static const int pf = [] {
    const char* e = getenv("FA_PAIR_PF");
    return e && e[0] == '1' ? 1 : 0;
  }();
  if (f64) {
    hipLaunchKernelGGL(k_pairdist_f64, dim3((unsigned)nblocks), dim3(kBlock), sizeof(double) * kC64 * k, st,
                       (const PSeg*)dv, nseg, (const void* const*)(dv + seg_bytes), k, nchunks64, (double*)d_scratch);
  } else if (q.lane) {
    const size_t lds = pair_lds_bytes(q);
    bool vec = true;  // 16-byte loads: every client segment 16-byte aligned (chunk starts are multiples of 8)
    for (int i = 0; i < j * k; ++i) vec = vec && ((uintptr_t)hp[i] % 16 == 0);
#define FA_PDL(V, R) if (pf) FA_PDL1(V, R, true); else FA_PDL1(V, R, false)
#define FA_PDL1(V, R, P) if (q.npl == 16) FA_PDL2(V, R, P, 16); else FA_PDL2(V, R, P, kNPL)
#define FA_PDL2(V, R, P, NP) hipLaunchKernelGGL((k_pairdist_lane<V, R, P, NP>), dim3((unsigned)nblocks), dim3((unsigned)q.nthreads), \
      lds, st, (const PSeg*)dv, nseg, (const void* const*)(dv + seg_bytes), k, kp, nchunks, ntiles, esplit, pe,      \
      (double*)d_scratch, guard, limit)
    if (vec) {
      if (rt == 1) FA_PDL(true, 1); else if (rt == 2) FA_PDL(true, 2); else FA_PDL(true, 0);
    } else {
      if (rt == 1) FA_PDL(false, 1); else if (rt == 2) FA_PDL(false, 2); else FA_PDL(false, 0);
    }
#undef FA_PDL
#undef FA_PDL1
#undef FA_PDL2
  } else {
    const size_t lds = pair_lds_bytes(q);
#define FA_PD(KPAD, R) if (pf) FA_PD2(KPAD, R, true); else FA_PD2(KPAD, R, false)
#define FA_PD2(KPAD, R, P) hipLaunchKernelGGL((k_pairdist<KPAD, R, P>), dim3((unsigned)nblocks), dim3((unsigned)q.nthreads), \
      lds, st, (const PSeg*)dv, nseg, (const void* const*)(dv + seg_bytes), k, kp, nchunks, ntiles, esplit, q.ce,   \
      q.rows, (double*)d_scratch, guard, limit)
#define FA_PDR(KPAD) if (rt == 1) FA_PD(KPAD, 1); else if (rt == 2) FA_PD(KPAD, 2); else FA_PD(KPAD, 0)
    switch (q.kpad) {
      case 64: FA_PDR(64); break;
      case 96: FA_PDR(96); break;
      default: FA_PDR(128); break;
    }
#undef FA_PDR
#undef FA_PD
#undef FA_PD2
  }
  const dim3 blk(kBlock);
  hipLaunchKernelGGL(k_pairdist_reduce, dim3((unsigned)((npairs + 7) / 8)), blk, 0,
                     st, (const double*)d_scratch, nblocks, k, (double*)d_dist, guard, limit);
  FA_HIP(hipGetLastError());
  return release(slot, st);
}
}  // namespace

extern "C" {

size_t fa_pairwise_sqdist_scratch_bytes(int32_t num_segments, const int64_t* seg_numel, int32_t k) {
  if (k < 2 || num_segments <= 0 || !seg_numel) return 0;
  const PairSplit q = pair_split(k);
  int64_t nchunks = 0;
  for (int s = 0; s < num_segments; ++s)
    if (seg_numel[s] > 0) nchunks += (seg_numel[s] + q.pe - 1) / q.pe;
  const int64_t nblocks = std::max<int64_t>(1, std::min<int64_t>(nchunks, q.nblocks));
  return sizeof(double) * (size_t)((int64_t)k * (k - 1) / 2) * (size_t)nblocks;
}


size_t fa_pairwise_sqdist_gram_scratch_bytes(int32_t num_segments, const int64_t* seg_numel, int32_t k) {
  if (k < 2 || k > kMaxPairK || num_segments <= 0 || !seg_numel) return 0;
  // the Gram form's partials + G + row maxima, then the guarded direct kernels' partials
  return gram_scratch(num_segments, seg_numel, k) + fa_pairwise_sqdist_scratch_bytes(num_segments, seg_numel, k);
}

int fa_pairwise_sqdist_gram(fa_ctx* ctx, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                            const void* const* d_in, void* d_dist, void* d_kappa_max, double kappa_limit,
                            void* d_scratch, size_t scratch_bytes, void* hip_stream) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (k < 2 || k > kMaxPairK || num_segments <= 0 || !seg_numel || !d_in || !d_dist || !d_kappa_max)
    return fail(FA_ERR_INVALID, "fa_pairwise_sqdist_gram: invalid arguments (2 <= k <= %d)", kMaxPairK);
  const int kbc = (k + 31) / 32;
  const bool vec = gram_vec(num_segments, seg_numel, k, d_in);
  // K <= 32 on 16-byte aligned clients: the LDS-DMA ring kernel (256-coordinate chunks), whose chunk
  // index runs over FULL chunks only (tile_start = the segment's first full chunk, pad = 1: a partial
  // chunk follows)
  const int glds = kbc == 1 && vec ? gram_glds() : 0;
  const int cs = glds ? 128 : gram_chunk(kbc);
  int nseg = 0;
  int64_t nchunks = 0;
  for (int s = 0; s < num_segments; ++s) {
    if (seg_numel[s] < 0) return fail(FA_ERR_INVALID, "segment %d has negative numel", s);
    if (seg_numel[s] == 0) continue;
    for (int i = 0; i < k; ++i)
      if (!d_in[(int64_t)s * k + i]) return fail(FA_ERR_INVALID, "segment %d client %d: input NULL", s, i);
    ++nseg;
    nchunks += (seg_numel[s] + cs - 1) / cs;
  }
  const size_t need = fa_pairwise_sqdist_gram_scratch_bytes(num_segments, seg_numel, k);
  if (scratch_bytes < need || !d_scratch)
    return fail(FA_ERR_INVALID, "fa_pairwise_sqdist_gram: scratch must hold %zu bytes", need);
  const size_t gram_bytes = gram_scratch(num_segments, seg_numel, k);
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  if (nseg == 0) {
    FA_HIP(hipMemsetAsync(d_dist, 0, sizeof(double) * (size_t)k * k, st));
    FA_HIP(hipMemsetAsync(d_kappa_max, 0, sizeof(double), st));
    return FA_OK;
  }
  const size_t seg_bytes = align16(sizeof(PSeg) * nseg);
  const size_t ptr_bytes = sizeof(void*) * (size_t)nseg * k;
  fa_ctx::Slot* slot = nullptr;
  int rc = acquire_slot(ctx, seg_bytes + ptr_bytes, &slot);
  if (rc) return rc;
  PSeg* hs = (PSeg*)slot->host;
  const void** hp = (const void**)((char*)slot->host + seg_bytes);
  int j = 0;
  int64_t c0 = 0;
  for (int s = 0; s < num_segments; ++s) {
    const int64_t n = seg_numel[s];
    if (n == 0) continue;
    for (int i = 0; i < k; ++i) hp[(int64_t)j * k + i] = d_in[(int64_t)s * k + i];
    hs[j] = PSeg{n, c0, j * k, glds && n % cs ? 1 : 0, 0};
    c0 += glds ? n / cs : (n + cs - 1) / cs;
    ++j;
  }
  rc = stage(slot, seg_bytes + ptr_bytes, st, true);
  if (rc) return rc;
  const char* dv = (const char*)slot->dev;
  const int kb = kbc;
  const int nblocks = gram_nblocks(nchunks, kb);
  double* part = (double*)d_scratch;
  double* gm = part + (size_t)nblocks * gram_T(kb) * 1024;
  unsigned* ctr = (unsigned*)(gm + (size_t)(32 * kb) * (32 * kb));  // k_gram_reduce's arrival counter
  const PSeg* sg = (const PSeg*)dv;
  const void* const* pp = (const void* const*)(dv + seg_bytes);
  const int ntr = gram_T(kb) * 1024 / 16;  // k_gram_reduce workgroups (16 entries each)
  const size_t lds = gram_lds(kb);
#define FA_GR(KB, S)                                                                                           \
  do {                                                                                                         \
    if (vec)                                                                                                   \
      hipLaunchKernelGGL((k_pair_gram<KB, true, S>), dim3((unsigned)nblocks), dim3(GramCfg<KB, S>::NT), lds,    \
                         st, sg, nseg, pp, k, nchunks, part, ctr);                                             \
    else                                                                                                       \
      hipLaunchKernelGGL((k_pair_gram<KB, false, S>), dim3((unsigned)nblocks), dim3(GramCfg<KB, S>::NT), lds,   \
                         st, sg, nseg, pp, k, nchunks, part, ctr);                                             \
    hipLaunchKernelGGL((k_gram_reduce<KB>), dim3((unsigned)ntr), dim3(64 * kGRW), 0, st, (const double*)part,    \
                       nblocks, gm, k, (double*)d_dist, (double*)d_kappa_max, ctr);                           \
  } while (0)
#define FA_GR3(KB, L)                                                                                          \
  do {                                                                                                         \
    if (vec)                                                                                                   \
      hipLaunchKernelGGL((k_pair_gram3<KB, true, L>), dim3((unsigned)nblocks), dim3(Gram3Cfg<KB, L>::NT),       \
                         (Gram3Cfg<KB, L>::LDS), st, sg, nseg, pp, k, nchunks, part, ctr);                      \
    else                                                                                                       \
      hipLaunchKernelGGL((k_pair_gram3<KB, false, L>), dim3((unsigned)nblocks), dim3(Gram3Cfg<KB, L>::NT),      \
                         (Gram3Cfg<KB, L>::LDS), st, sg, nseg, pp, k, nchunks, part, ctr);                      \
    hipLaunchKernelGGL((k_gram_reduce<KB>), dim3((unsigned)ntr), dim3(64 * kGRW), 0, st, (const double*)part,    \
                       nblocks, gm, k, (double*)d_dist, (double*)d_kappa_max, ctr);                           \
  } while (0)
  if (glds) {  // c0 = the full-chunk count; two 8-wave workgroups per CU
    // the workgroup count the scratch was sized for (gram_scratch -> gram_nblocks), at most 512
    const int nbg = std::min(gram_nblocks(nchunks, 1), 512);
    const size_t lg = (size_t)4 * 32 * cs * sizeof(float) + (size_t)glds * 16 * sizeof(float);
    hipLaunchKernelGGL((k_pair_gram_ring<4, 128, 8>), dim3((unsigned)nbg), dim3(512), lg, st, sg, nseg, pp, k, c0,
                       part, ctr);
    hipLaunchKernelGGL((k_gram_reduce<1>), dim3((unsigned)ntr), dim3(64 * kGRW), 0, st, (const double*)part, nbg, gm,
                       k, (double*)d_dist, (double*)d_kappa_max, ctr);
  } else switch (kb) {
    case 1: FA_GR(1, false); break;
    case 2:
      if (gram3() && gram3_l2()) FA_GR3(2, 1);  // the bf16x3 split form (K in (32, 64])
      else if (gram3()) FA_GR3(2, 0);
      else if (gram_s16()) FA_GR(2, true);
      else FA_GR(2, false);
      break;
    case 3:
      if (gram3() && gram3_l3()) FA_GR3(3, 1);  // the bf16x3 split form (K in (64, 96])
      else if (gram3()) FA_GR3(3, 0);
      else FA_GR(3, false);
      break;
    default:
      if (gram3()) {  // the bf16x3 split form (K in (96, 128])
        FA_GR3(4, 0);
      } else if (gram_s16()) {
        FA_GR(4, true);
      } else {
        FA_GR(4, false);
      }
      break;
  }
#undef FA_GR
#undef FA_GR3
  FA_HIP(hipGetLastError());
  rc = release(slot, st);
  if (rc || kappa_limit <= 0.0) return rc;
  // the guarded direct kernels: they run (and overwrite d_dist) only if kappa_max exceeds the limit
  // the error model allows at this size (fa_pairwise_sqdist_gram_limit)
  int64_t ptot = 0;
  for (int s = 0; s < num_segments; ++s) ptot += std::max<int64_t>(seg_numel[s], 0);
  const double lim = std::min(kappa_limit, gram_kappa_bound(ptot, gram_run(kb, glds != 0)));
  return pairdist_direct(ctx, FA_DTYPE_F32, num_segments, seg_numel, k, d_in, d_dist, (char*)d_scratch + gram_bytes,
                         scratch_bytes - gram_bytes, hip_stream, (const double*)d_kappa_max, lim);
}

double fa_pairwise_sqdist_gram_limit(int32_t num_segments, const int64_t* seg_numel, int32_t k,
                                     const void* const* d_in, double kappa_limit) {
  if (k < 2 || k > kMaxPairK || num_segments <= 0 || !seg_numel || !d_in || kappa_limit <= 0.0) return 0.0;
  const int kb = (k + 31) / 32;
  const bool glds = kb == 1 && gram_vec(num_segments, seg_numel, k, d_in) && gram_glds();
  int64_t ptot = 0;
  for (int s = 0; s < num_segments; ++s) ptot += std::max<int64_t>(seg_numel[s], 0);
  return std::min(kappa_limit, gram_kappa_bound(ptot, gram_run(kb, glds)));
}

}  // extern "C"
