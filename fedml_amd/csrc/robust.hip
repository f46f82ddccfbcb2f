// robust.hip -- MI355X (gfx950) kernels + C ABI of the robust-aggregation family
// (include/fedagg_robust.h): coordinate-wise median over the clients and Krum's pairwise
// squared distances.
//
// Coordinate-wise median (k_median): torch.median over the client axis is a SELECTION, so the
// result is one of the inputs, bit for bit.  One lane owns one coordinate: it streams the K client
// values into registers as order-preserving uint32 keys (floats mapped so that unsigned order ==
// numeric order, -0.0 folded onto +0.0), sorts them with a bitonic network padded to P2 = next
// power of two with max-key sentinels (P2 (P2 log2 P2 ...)/4 compare-exchanges, each a v_min_u32 +
// v_max_u32 on compile-time register indices), and takes key[(K-1)/2] (uniform index -> one select
// chain).  ATen's exact rules are kept: a NaN anywhere in the column returns the FIRST NaN; among
// equal values the client index decides, which only matters for +-0 -- both cases (a NaN seen, or
// a zero selected) take a short in-order rescan of the column.
// Compute per coordinate ~P2 log2^2 P2 ops vs K*s bytes of HBM: memory-bound to K ~ 64, roughly
// balanced at K = 128.  Larger K: a rank-counting kernel (O(K^2) per coordinate, L2-resident).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstring>

#include "fa_internal.h"
#include "fedagg_robust.h"

using namespace fa_detail;

namespace {

constexpr int kMaxP2 = 64;  // largest column one lane sorts (a 128-key network takes the compiler minutes)

template <int DT> struct MedT;
template <> struct MedT<FA_DTYPE_F32> {
  using S = unsigned;
  __device__ static float load(const void* p, int64_t e) { return ((const float*)p)[e]; }
  __device__ static void store(void* p, int64_t e, float v) { ((float*)p)[e] = v; }
  __device__ static void store_bits(void* p, int64_t e, const void* src) { ((unsigned*)p)[e] = ((const unsigned*)src)[e]; }
};
template <> struct MedT<FA_DTYPE_BF16> {
  __device__ static float load(const void* p, int64_t e) {
    return __uint_as_float((unsigned)((const unsigned short*)p)[e] << 16);
  }
  __device__ static void store(void* p, int64_t e, float v) {
    ((unsigned short*)p)[e] = (unsigned short)(__float_as_uint(v) >> 16);  // exact: v came from bf16
  }
  __device__ static void store_bits(void* p, int64_t e, const void* src) {
    ((unsigned short*)p)[e] = ((const unsigned short*)src)[e];
  }
};
template <> struct MedT<FA_DTYPE_F16> {
  __device__ static float load(const void* p, int64_t e) {
    return (float)__builtin_bit_cast(_Float16, ((const unsigned short*)p)[e]);
  }
  __device__ static void store(void* p, int64_t e, float v) {
    ((unsigned short*)p)[e] = __builtin_bit_cast(unsigned short, (_Float16)v);  // exact: v came from f16
  }
  __device__ static void store_bits(void* p, int64_t e, const void* src) {
    ((unsigned short*)p)[e] = ((const unsigned short*)src)[e];
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
  int32_t ptr_base;
  int32_t pad;
};
static_assert(sizeof(MSeg) == 32, "MSeg layout");

template <int P2>
__device__ __forceinline__ void bitonic_sort(unsigned (&key)[P2]) {
#pragma unroll
  for (int size = 2; size <= P2; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
#pragma unroll
      for (int i = 0; i < P2; ++i) {
        const int j = i ^ stride;
        if (j > i) {
          const unsigned lo = min(key[i], key[j]), hi = max(key[i], key[j]);
          if ((i & size) == 0) { key[i] = lo; key[j] = hi; }
          else { key[i] = hi; key[j] = lo; }
        }
      }
    }
  }
}

// Rare cases, resolved by an in-order rescan of the column: a NaN anywhere -> ATen returns the
// FIRST NaN; a zero selected -> the selected rank r falls in the block of (equal) zeros, which ATen
// orders by client index -> the (r - #negatives)-th zero in client order.
template <int DT>
__device__ __forceinline__ void store_rare(const void* const* in, int k, int64_t e, int r, bool nan, void* out) {
  if (nan) {
    for (int i = 0; i < k; ++i) {
      const float x = MedT<DT>::load(in[i], e);
      if (x != x) { MedT<DT>::store_bits(out, e, in[i]); return; }
    }
  }
  int negc = 0;
  for (int i = 0; i < k; ++i) negc += MedT<DT>::load(in[i], e) < 0.0f;
  int seen = 0;
  for (int i = 0; i < k; ++i) {
    const float x = MedT<DT>::load(in[i], e);
    if (x == 0.0f) {
      if (seen == r - negc) { MedT<DT>::store_bits(out, e, in[i]); return; }
      ++seen;
    }
  }
}

template <int DT, int P2>
__global__ void __launch_bounds__(kBlock)
k_median(const MSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k) {
  const int64_t tile = blockIdx.x;
  const MSeg sg = segs[nseg > 1 ? find_seg(segs, nseg, tile) : 0];
  const int64_t e = (tile - sg.tile_start) * kBlock + threadIdx.x;
  const bool live = e < sg.numel;
  const int64_t ec = live ? e : sg.numel - 1;
  const void* const* in = ptrs + sg.ptr_base;
  unsigned key[P2];
  bool nan = false;
#pragma unroll
  for (int i = 0; i < P2; ++i) {
    const float x = MedT<DT>::load(in[min(i, k - 1)], ec);  // clamped: every load unconditional
    nan = nan || (i < k && x != x);                          // P2 - k < P2 / 2 sentinels
    key[i] = i < k ? fkey(x) : 0xFFFFFFFFu;
  }
  bitonic_sort<P2>(key);
  const int r = (k - 1) >> 1;
  unsigned kr = key[0];
#pragma unroll
  for (int i = 1; i < P2; ++i) kr = (i == r) ? key[i] : kr;  // uniform r: folds to one select chain
  if (!live) return;
  if (nan || kr == kPosZeroKey || kr == kNegZeroKey) store_rare<DT>(in, k, e, r, nan, sg.out);
  else MedT<DT>::store(sg.out, e, fkey_inv(kr));
}

// 64 < K <= 128: two lanes per coordinate, each sorting the keys of 64 clients (lane 2p: clients
// 0..63, lane 2p+1: clients 64..127, max-key sentinels past K).  One cross-lane bitonic step
// (lane 2p keeps min(A[i], B[63-i]), a bitonic sequence holding the 64 smallest keys) and a 64-key
// bitonic merge leave the 64 smallest keys sorted in lane 2p -- and rank (K-1)/2 <= 63 is among
// them.  Segment tiles are kBlock/2 coordinates (MSeg.tile_start counts those tiles).
template <int DT>
__global__ void __launch_bounds__(kBlock)
k_median2(const MSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k) {
  constexpr int H = kMaxP2;
  const int64_t tile = blockIdx.x;
  const MSeg sg = segs[nseg > 1 ? find_seg(segs, nseg, tile) : 0];
  const int half = threadIdx.x & 1;
  const int64_t e = (tile - sg.tile_start) * (kBlock / 2) + (threadIdx.x >> 1);
  const bool live = e < sg.numel;
  const int64_t ec = live ? e : sg.numel - 1;
  const void* const* in = ptrs + sg.ptr_base;
  unsigned key[H];
  bool nan = false;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const int c = half * H + i;
    const float x = MedT<DT>::load(in[min(c, k - 1)], ec);  // clamped: the load is unconditional
    nan = nan || (c < k && x != x);
    key[i] = c < k ? fkey(x) : 0xFFFFFFFFu;
  }
  bitonic_sort<H>(key);
  // cross-lane step of the 128-key bitonic merge (partner = lane ^ 1)
#pragma unroll
  for (int i = 0; i < H / 2; ++i) {  // pairs (i, H-1-i): both partner values read before either is written
    const unsigned o_hi = __shfl_xor(key[H - 1 - i], 1), o_lo = __shfl_xor(key[i], 1);
    key[i] = half == 0 ? min(key[i], o_hi) : max(key[i], o_hi);
    key[H - 1 - i] = half == 0 ? min(key[H - 1 - i], o_lo) : max(key[H - 1 - i], o_lo);
  }
  // bitonic merge of the (bitonic) lower half into ascending order
#pragma unroll
  for (int stride = H >> 1; stride > 0; stride >>= 1) {
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const int j = i ^ stride;
      if (j > i) {
        const unsigned lo = min(key[i], key[j]), hi = max(key[i], key[j]);
        key[i] = lo;
        key[j] = hi;
      }
    }
  }
  const int partner_nan = __shfl_xor((int)nan, 1);  // every lane shuffles (no short-circuit)
  nan = nan || partner_nan != 0;
  if (half != 0 || !live) return;
  const int r = (k - 1) >> 1;
  unsigned kr = key[0];
#pragma unroll
  for (int i = 1; i < H; ++i) kr = (i == r) ? key[i] : kr;
  if (nan || kr == kPosZeroKey || kr == kNegZeroKey) store_rare<DT>(in, k, e, r, nan, sg.out);
  else MedT<DT>::store(sg.out, e, fkey_inv(kr));
}

// Any K (and float64): rank counting, ATen's order (value, client index), NaN first.
template <typename T> __device__ __forceinline__ T ldv(const void* p, int64_t e) { return ((const T*)p)[e]; }

template <int DT>
__device__ __forceinline__ double load_d(const void* p, int64_t e) {
  if constexpr (DT == FA_DTYPE_F64) return ((const double*)p)[e];
  else return (double)MedT<DT>::load(p, e);
}
template <int DT>
__device__ __forceinline__ void copy_bits(void* out, int64_t e, const void* src) {
  if constexpr (DT == FA_DTYPE_F64) ((unsigned long long*)out)[e] = ((const unsigned long long*)src)[e];
  else MedT<DT>::store_bits(out, e, src);
}

template <int DT>
__global__ void __launch_bounds__(kBlock)
k_median_rank(const MSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k) {
  const int64_t tile = blockIdx.x;
  const MSeg sg = segs[nseg > 1 ? find_seg(segs, nseg, tile) : 0];
  const int64_t e = (tile - sg.tile_start) * kBlock + threadIdx.x;
  if (e >= sg.numel) return;
  const void* const* in = ptrs + sg.ptr_base;
  for (int i = 0; i < k; ++i) {
    if (load_d<DT>(in[i], e) != load_d<DT>(in[i], e)) { copy_bits<DT>(sg.out, e, in[i]); return; }
  }
  const int r = (k - 1) >> 1;
  for (int i = 0; i < k; ++i) {
    const double xi = load_d<DT>(in[i], e);
    int less = 0, eq_before = 0;
    for (int j = 0; j < k; ++j) {
      const double xj = load_d<DT>(in[j], e);
      less += xj < xi;
      eq_before += (xj == xi) && (j < i);
    }
    if (less + eq_before == r) { copy_bits<DT>(sg.out, e, in[i]); return; }
  }
}

template <int DT>
void launch_median(int k, dim3 grid, dim3 grid2, hipStream_t st, const MSeg* ds, int nseg, const void* const* dp) {
  if constexpr (DT == FA_DTYPE_F64) {
    hipLaunchKernelGGL((k_median_rank<DT>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k);
  } else {
    if (k <= 4) { hipLaunchKernelGGL((k_median<DT, 4>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k); return; }
    if (k <= 8) { hipLaunchKernelGGL((k_median<DT, 8>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k); return; }
    if (k <= 16) { hipLaunchKernelGGL((k_median<DT, 16>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k); return; }
    if (k <= 32) { hipLaunchKernelGGL((k_median<DT, 32>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k); return; }
    if (k <= 64) { hipLaunchKernelGGL((k_median<DT, 64>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k); return; }
    if (k <= 2 * kMaxP2) {  // two lanes per coordinate: half the grid's coordinates per block
      hipLaunchKernelGGL((k_median2<DT>), grid2, dim3(kBlock), 0, st, ds, nseg, dp, k);
      return;
    }
    hipLaunchKernelGGL((k_median_rank<DT>), grid, dim3(kBlock), 0, st, ds, nseg, dp, k);
  }
}

}  // namespace

// ============================================================================================ ABI
extern "C" {

int fa_coord_median(fa_ctx* ctx, int dtype, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                    const void* const* d_in, void* const* d_out, void* hip_stream) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (k <= 0 || num_segments <= 0 || !seg_numel || !d_in || !d_out)
    return fail(FA_ERR_INVALID, "fa_coord_median: invalid arguments");
  if (dtype != FA_DTYPE_F32 && dtype != FA_DTYPE_BF16 && dtype != FA_DTYPE_F16 && dtype != FA_DTYPE_F64)
    return fail(FA_ERR_DTYPE, "fa_coord_median: dtype %d not supported (F32, BF16, F16, F64)", dtype);
  // coordinates per tile: kBlock, or kBlock/2 when two lanes share a coordinate (64 < k <= 128)
  const bool two_lane = dtype != FA_DTYPE_F64 && k > kMaxP2 && k <= 2 * kMaxP2;
  const int64_t tile_elems = two_lane ? kBlock / 2 : kBlock;
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
    hs[j] = MSeg{n, t0, d_out[s], j * k, 0};
    t0 += (n + tile_elems - 1) / tile_elems;
    ++j;
  }
  rc = stage(slot, seg_bytes + ptr_bytes, st);
  if (rc) return rc;
  const char* dv = (const char*)slot->dev;
  const MSeg* ds = (const MSeg*)dv;
  const void* const* dp = (const void* const*)(dv + seg_bytes);
  const dim3 grid((unsigned)tiles);
  switch (dtype) {
    case FA_DTYPE_F32: launch_median<FA_DTYPE_F32>(k, grid, grid, st, ds, nseg, dp); break;
    case FA_DTYPE_BF16: launch_median<FA_DTYPE_BF16>(k, grid, grid, st, ds, nseg, dp); break;
    case FA_DTYPE_F16: launch_median<FA_DTYPE_F16>(k, grid, grid, st, ds, nseg, dp); break;
    default: launch_median<FA_DTYPE_F64>(k, grid, grid, st, ds, nseg, dp); break;
  }
  FA_HIP(hipGetLastError());
  return release(slot, st);
}

}  // extern "C"

// ============================================================================================
// Krum's pairwise squared distances (krum_defense.py:52-66): D[i][j] = sum_e (x_i[e] - x_j[e])^2
// over the clients' weight vectors, float32 inputs, every pair (i < j) in ONE pass over the data.
// A workgroup stages a chunk of kPE coordinates of all K clients in LDS (transposed [e][client],
// so 4 clients of one coordinate are one 16-byte LDS read), and each thread owns up to TPT 4x4
// client-pair tiles (upper triangle) -- 16 differences per 2 LDS reads -- over a slice of the
// chunk's coordinates.  Sums: float32 within a chunk slice (<= kPE terms), float64 across chunks.
// Per-block float64 partials of the upper triangle go to a scratch buffer and a second kernel
// adds them in block order (deterministic).  VALU-bound for large K (K^2/2 pair updates per
// coordinate against 4K bytes).
namespace {

constexpr int kPE = 64;       // coordinates per LDS chunk
constexpr int kMaxPairK = 128;

struct PSeg {
  int64_t numel;
  int64_t tile_start;   // first chunk of this segment (find_seg keys on it)
  int32_t ptr_base;
  int32_t pad;
  int64_t pad2;
};
static_assert(sizeof(PSeg) == 32, "PSeg layout");

template <int TPT>
__global__ void __launch_bounds__(kBlock)
k_pairdist(const PSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k, int kp,
           int64_t nchunks, int ntiles, int esplit, double* __restrict__ partial) {
  extern __shared__ float lds[];              // [kPE][kp + 4]
  const int stride = kp + 4;
  const int nb = kp / 4;
  const int t = threadIdx.x;
  // work split: TPT == 1 -> tile t % ntiles, coordinate slice t / ntiles (esplit slices);
  //             TPT  > 1 -> tiles t, t + kBlock, ... (esplit == 1)
  const int es = TPT == 1 ? t / ntiles : 0;
  const bool active = es < esplit;
  const int tile0 = TPT == 1 ? t % ntiles : t;
  int bi[TPT], bj[TPT];
  bool tv[TPT];
#pragma unroll
  for (int q = 0; q < TPT; ++q) {
    const int tile = tile0 + q * kBlock;
    tv[q] = active && tile < ntiles;
    int r = 0, rem = tv[q] ? tile : 0;  // tile -> (bi, bj), bi <= bj, row-major upper triangle
    while (rem >= nb - r) { rem -= nb - r; ++r; }
    bi[q] = r;
    bj[q] = r + rem;
  }
  double accd[TPT][16];
#pragma unroll
  for (int q = 0; q < TPT; ++q)
#pragma unroll
    for (int u = 0; u < 16; ++u) accd[q][u] = 0.0;
  const int per = kPE / esplit;  // coordinates of a chunk per slice
  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const PSeg sg = segs[nseg > 1 ? find_seg(segs, nseg, ch) : 0];
    const int64_t e0 = (ch - sg.tile_start) * kPE;
    const void* const* in = ptrs + sg.ptr_base;
    __syncthreads();  // the previous chunk is consumed
    // stage: client c, coordinate e -> lds[e * stride + c]; clients >= k and coordinates past the
    // segment end are zero (they add 0 to every sum).  Loads are unconditional (clamped) so the
    // unrolled loop keeps 8 in flight per lane.
    {
      const int e = t & (kPE - 1);
      const bool ev = e0 + e < sg.numel;
      const int64_t ge = ev ? e0 + e : sg.numel - 1;
#pragma unroll 8
      for (int c = t / kPE; c < kp; c += kBlock / kPE) {
        const float v = ((const float*)in[min(c, k - 1)])[ge];
        lds[e * stride + c] = (ev && c < k) ? v : 0.0f;
      }
    }
    __syncthreads();
    if (active) {
      float acc[TPT][16];
#pragma unroll
      for (int q = 0; q < TPT; ++q)
#pragma unroll
        for (int u = 0; u < 16; ++u) acc[q][u] = 0.0f;
      for (int e = es * per; e < (es + 1) * per; ++e) {
#pragma unroll
        for (int q = 0; q < TPT; ++q) {
          if (!tv[q]) continue;
          const float4 a = *(const float4*)&lds[e * stride + 4 * bi[q]];
          const float4 b = *(const float4*)&lds[e * stride + 4 * bj[q]];
          const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) {
              const float d = __fsub_rn(av[x], bv[y]);
              acc[q][x * 4 + y] = __fmaf_rn(d, d, acc[q][x * 4 + y]);
            }
        }
      }
#pragma unroll
      for (int q = 0; q < TPT; ++q)
#pragma unroll
        for (int u = 0; u < 16; ++u) accd[q][u] += (double)acc[q][u];
    }
  }
  // reduce the esplit slices of each tile through LDS (reused as double scratch), then write the
  // block's upper-triangle partials: pair (i, j), i < j -> index i*k - i*(i+1)/2 + (j - i - 1)
  __syncthreads();
  double* red = (double*)lds;  // [ntiles * 16] doubles, fits: kPE*(kp+4)*4 >= 16*8*ntiles? see host
  const int64_t npairs = (int64_t)k * (k - 1) / 2;
  double* out = partial + (int64_t)blockIdx.x * npairs;
  if (TPT == 1) {
    for (int s = 0; s < esplit; ++s) {
      if (active && es == s) {
#pragma unroll
        for (int u = 0; u < 16; ++u) red[tile0 * 16 + u] = (s == 0 ? 0.0 : red[tile0 * 16 + u]) + accd[0][u];
      }
      __syncthreads();
    }
    for (int idx = t; idx < ntiles * 16; idx += kBlock) {
      const int tile = idx / 16, u = idx % 16;
      int r = 0, rem = tile;
      while (rem >= nb - r) { rem -= nb - r; ++r; }
      const int i = 4 * r + u / 4, j = 4 * (r + rem) + u % 4;
      if (i < j && j < k) out[(int64_t)i * k - (int64_t)i * (i + 1) / 2 + (j - i - 1)] = red[idx];
    }
  } else {
#pragma unroll
    for (int q = 0; q < TPT; ++q) {
      if (!tv[q]) continue;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int i = 4 * bi[q] + u / 4, j = 4 * bj[q] + u % 4;
        if (i < j && j < k) out[(int64_t)i * k - (int64_t)i * (i + 1) / 2 + (j - i - 1)] = accd[q][u];
      }
    }
  }
}

__global__ void __launch_bounds__(kBlock)
k_pairdist_reduce(const double* __restrict__ partial, int nblocks, int k, double* __restrict__ d) {
  const int64_t npairs = (int64_t)k * (k - 1) / 2;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < npairs; p += (int64_t)gridDim.x * kBlock) {
    double s = 0.0;
    for (int b = 0; b < nblocks; ++b) s += partial[(int64_t)b * npairs + p];
    // p -> (i, j)
    int i = 0;
    int64_t rem = p;
    while (rem >= k - 1 - i) { rem -= k - 1 - i; ++i; }
    const int j = i + 1 + (int)rem;
    d[(int64_t)i * k + j] = s;
    d[(int64_t)j * k + i] = s;
  }
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < k; i += kBlock) d[(int64_t)i * k + i] = 0.0;
}

}  // namespace

extern "C" {

int fa_pairwise_sqdist(fa_ctx* ctx, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                       const void* const* d_in, void* d_dist, void* d_scratch, size_t scratch_bytes,
                       void* hip_stream) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (k < 2 || k > kMaxPairK || num_segments <= 0 || !seg_numel || !d_in || !d_dist)
    return fail(FA_ERR_INVALID, "fa_pairwise_sqdist: invalid arguments (2 <= k <= %d)", kMaxPairK);
  const int kp = (k + 3) & ~3;
  const int nb = kp / 4;
  const int ntiles = nb * (nb + 1) / 2;
  int tpt = (ntiles + kBlock - 1) / kBlock;
  int esplit = 1;
  if (tpt == 1) {
    esplit = kBlock / ntiles;
    int p2 = 1;
    while (p2 * 2 <= esplit && p2 * 2 <= kPE) p2 *= 2;
    esplit = p2;
  }
  if (tpt > 3) return fail(FA_ERR_INVALID, "fa_pairwise_sqdist: k too large");
  int nseg = 0;
  int64_t nchunks = 0;
  for (int s = 0; s < num_segments; ++s) {
    if (seg_numel[s] < 0) return fail(FA_ERR_INVALID, "segment %d has negative numel", s);
    if (seg_numel[s] == 0) continue;
    for (int i = 0; i < k; ++i)
      if (!d_in[(int64_t)s * k + i]) return fail(FA_ERR_INVALID, "segment %d client %d: input NULL", s, i);
    ++nseg;
    nchunks += (seg_numel[s] + kPE - 1) / kPE;
  }
  const int64_t npairs = (int64_t)k * (k - 1) / 2;
  const int nblocks = (int)std::max<int64_t>(1, std::min<int64_t>(nchunks, 1024));
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
  for (int s = 0; s < num_segments; ++s) {
    const int64_t n = seg_numel[s];
    if (n == 0) continue;
    for (int i = 0; i < k; ++i) hp[(int64_t)j * k + i] = d_in[(int64_t)s * k + i];
    hs[j] = PSeg{n, c0, j * k, 0, 0};
    c0 += (n + kPE - 1) / kPE;
    ++j;
  }
  rc = stage(slot, seg_bytes + ptr_bytes, st);
  if (rc) return rc;
  const char* dv = (const char*)slot->dev;
  size_t lds = sizeof(float) * (size_t)kPE * (kp + 4);
  lds = std::max(lds, sizeof(double) * 16 * (size_t)ntiles);
  const dim3 grid((unsigned)nblocks), blk(kBlock);
#define FA_PD(T)                                                                                     \
  hipLaunchKernelGGL((k_pairdist<T>), grid, blk, lds, st, (const PSeg*)dv, nseg,                       \
                     (const void* const*)(dv + seg_bytes), k, kp, nchunks, ntiles, esplit, (double*)d_scratch)
  if (tpt == 1) FA_PD(1);
  else if (tpt == 2) FA_PD(2);
  else FA_PD(3);
#undef FA_PD
  hipLaunchKernelGGL(k_pairdist_reduce, dim3((unsigned)std::min<int64_t>((npairs + kBlock - 1) / kBlock, 64)), blk, 0,
                     st, (const double*)d_scratch, nblocks, k, (double*)d_dist);
  FA_HIP(hipGetLastError());
  return release(slot, st);
}

size_t fa_pairwise_sqdist_scratch_bytes(int32_t num_segments, const int64_t* seg_numel, int32_t k) {
  if (k < 2 || num_segments <= 0 || !seg_numel) return 0;
  int64_t nchunks = 0;
  for (int s = 0; s < num_segments; ++s)
    if (seg_numel[s] > 0) nchunks += (seg_numel[s] + kPE - 1) / kPE;
  const int64_t nblocks = std::max<int64_t>(1, std::min<int64_t>(nchunks, 1024));
  return sizeof(double) * (size_t)((int64_t)k * (k - 1) / 2) * (size_t)nblocks;
}

}  // extern "C"
