// fedagg.hip -- MI355X (gfx950 / CDNA4) kernels and C ABI of the FedAvg-family aggregation engine.
//
// Public contract: include/fedagg.h (which reference loop each entry replaces, exact arithmetic).
//
// Design (DESIGN.md has the numbers):
//  * The path is an HBM-bound ordered reduction over K client streams: per output element it reads
//    K inputs and writes one.  No MFMA (0.5 flop/B) and no LDS staging (no data reuse): every lane
//    owns V consecutive elements (one 16-byte vector) of one tile and walks the K clients IN ORDER,
//    which is what makes the result bit-identical to the reference's client-ordered CPU loop.
//  * Bandwidth comes from memory-level parallelism: the client loop is unrolled by U with all U
//    16-byte loads issued before any is consumed (U KiB in flight per wave), so a CU with ~8-20
//    resident waves keeps >= 64 KiB of HBM reads in flight.  Out-of-range clients in the last group
//    are loaded from a clamped (valid) index and skipped on the uniform accumulate branch, so no
//    load sits behind a branch (hipcc would otherwise wait vmcnt(0) per load).
//  * Inputs are read exactly once -> non-temporal loads; the output is written once -> non-temporal
//    stores.  (Mixing re-reads neighbours, so fa_mix keeps the default cache policy.)
//  * A whole state_dict (many tensors of one dtype) is one launch: a device-resident segment table
//    maps each 256-thread tile to (segment, offset) by a wave-uniform binary search (scalar loads).
//  * Arithmetic: op(.) = IEEE op in float/double, rounded once to the storage type, never fused
//    (compiled with -ffp-contract=off, __f*_rn intrinsics).  The accumulator starts at -0.0, which
//    is the exact identity of IEEE addition (-0 + t == t bitwise for every t, incl. +-0, NaN, Inf),
//    so "acc = t_0" needs no select.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>

#include <mutex>

#include <algorithm>
#include <climits>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <type_traits>
#include <vector>

#include "fa_internal.h"

using namespace fa_detail;

namespace {


// --------------------------------------------------------------------------------------------
// Device-resident descriptors (staged per call from pinned host memory).

struct MixRow {             // one output row of a mixing matrix
  int32_t begin, end;     // CSR entry range
  void* out;
  void* out2;             // PushSum z output (or null)
  double scale;           // PushSum post-scale (1/omega)
};
static_assert(sizeof(MixRow) == 32, "MixRow layout");

// --------------------------------------------------------------------------------------------
// Exact per-op arithmetic.
__device__ __forceinline__ float op_mul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float op_add(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float op_div(float a, float b) { return __fdiv_rn(a, b); }
__device__ __forceinline__ double op_mul(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double op_add(double a, double b) { return __dadd_rn(a, b); }
__device__ __forceinline__ double op_div(double a, double b) { return __ddiv_rn(a, b); }

__device__ __forceinline__ float bf16_round(float x) { return (float)(__bf16)x; }
__device__ __forceinline__ unsigned bf16_bits(float x) {
  return (unsigned)__builtin_bit_cast(unsigned short, (__bf16)x);
}
// The f32 -> f16 rounding must see a MATERIALISED f32 value: otherwise the gfx950 backend folds
// fptrunc(fmul(fpext(h), c)) into v_fma_mixlo_f16, which rounds the exact product to f16 ONCE,
// while the reference (PyTorch CPU) rounds it to f32 first and then to f16 (double rounding).
// The empty asm pins the f32 intermediate in a VGPR (no instruction is emitted).
__device__ __forceinline__ float pin_f32(float x) {
  asm("" : "+v"(x));
  return x;
}
__device__ __forceinline__ float f16_round(float x) { return (float)(_Float16)pin_f32(x); }
__device__ __forceinline__ unsigned f16_bits(float x) {
  return (unsigned)__builtin_bit_cast(unsigned short, (_Float16)pin_f32(x));
}
__device__ __forceinline__ float f16_from_bits(unsigned b) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)b);
}

// --------------------------------------------------------------------------------------------
// Element traits per (input dtype, mode):
//   R     raw element value after unpacking (exact widening: float for f32/bf16/f16)
//   A     accumulator / op type;  C coefficient type;  D divisor type
//   V     elements per 16-byte input vector;  IN_BYTES / OUT_BYTES element sizes
//   term  t_i of the contract;  acc   op(acc + t);  zero  the exact additive identity
template <int DT, int MODE> struct Tr;

template <int MODE> struct TrFloatBase {
  using A = float; using C = float; using D = float; using R = float;
  __device__ static C coef(double c) { return (float)c; }
  __device__ static D div(double d) { return (float)d; }
  __device__ static A zero() { return -0.0f; }
};

template <int MODE> struct Tr<FA_DTYPE_F32, MODE> : TrFloatBase<MODE> {
  static constexpr int V = 4, IN_BYTES = 4, OUT_BYTES = 4;
  __device__ static float rnd(float x) { return x; }
  __device__ static void unpack(u32x4 r, float (&x)[V]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = __uint_as_float(r[j]);
  }
  __device__ static float ld1(const void* p, int64_t e) { return ((const float*)p)[e]; }
  __device__ static void st1(void* p, int64_t e, float v) { ((float*)p)[e] = v; }
  __device__ static void stv(void* p, const float (&a)[V]) {
    u32x4 w = {__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]), __float_as_uint(a[3])};
    __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x4*)p);
  }
};

template <int MODE> struct Tr<FA_DTYPE_BF16, MODE> : TrFloatBase<MODE> {
  static constexpr int V = 8, IN_BYTES = 2, OUT_BYTES = 2;
  __device__ static float rnd(float x) { return bf16_round(x); }
  __device__ static void unpack(u32x4 r, float (&x)[V]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[2 * j] = __uint_as_float(r[j] << 16);
      x[2 * j + 1] = __uint_as_float(r[j] & 0xFFFF0000u);
    }
  }
  __device__ static float ld1(const void* p, int64_t e) {
    return __uint_as_float((unsigned)((const unsigned short*)p)[e] << 16);
  }
  __device__ static void st1(void* p, int64_t e, float v) { ((unsigned short*)p)[e] = (unsigned short)bf16_bits(v); }
  __device__ static void stv(void* p, const float (&a)[V]) {
    u32x4 w;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = bf16_bits(a[2 * j]) | (bf16_bits(a[2 * j + 1]) << 16);
    __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x4*)p);
  }
};

template <int MODE> struct Tr<FA_DTYPE_F16, MODE> : TrFloatBase<MODE> {
  static constexpr int V = 8, IN_BYTES = 2, OUT_BYTES = 2;
  __device__ static float rnd(float x) { return f16_round(x); }
  __device__ static void unpack(u32x4 r, float (&x)[V]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[2 * j] = f16_from_bits(r[j] & 0xFFFFu);
      x[2 * j + 1] = f16_from_bits(r[j] >> 16);
    }
  }
  __device__ static float ld1(const void* p, int64_t e) { return f16_from_bits(((const unsigned short*)p)[e]); }
  __device__ static void st1(void* p, int64_t e, float v) { ((unsigned short*)p)[e] = (unsigned short)f16_bits(v); }
  __device__ static void stv(void* p, const float (&a)[V]) {
    u32x4 w;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = f16_bits(a[2 * j]) | (f16_bits(a[2 * j + 1]) << 16);
    __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x4*)p);
  }
};

template <int MODE> struct Tr<FA_DTYPE_F64, MODE> {
  using A = double; using C = double; using D = double; using R = double;
  static constexpr int V = 2, IN_BYTES = 8, OUT_BYTES = 8;
  __device__ static C coef(double c) { return c; }
  __device__ static D div(double d) { return d; }
  __device__ static A zero() { return -0.0; }
  __device__ static double rnd(double x) { return x; }
  __device__ static void unpack(u32x4 r, double (&x)[V]) {
    x[0] = __builtin_bit_cast(double, u32x2{r[0], r[1]});
    x[1] = __builtin_bit_cast(double, u32x2{r[2], r[3]});
  }
  __device__ static double ld1(const void* p, int64_t e) { return ((const double*)p)[e]; }
  __device__ static void st1(void* p, int64_t e, double v) { ((double*)p)[e] = v; }
  __device__ static void stv(void* p, const double (&a)[V]) {
    u32x2 lo = __builtin_bit_cast(u32x2, a[0]), hi = __builtin_bit_cast(u32x2, a[1]);
    u32x4 w = {lo[0], lo[1], hi[0], hi[1]};
    __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x4*)p);
  }
};

// int64 inputs, weighted modes: float32 output (PyTorch type promotion int64 (*) float -> float32)
template <int MODE> struct Tr<FA_DTYPE_I64, MODE> {
  using A = float; using R = long long; using D = float;
  using C = typename std::conditional<MODE == FA_MODE_MUL_N_DIV_N, long long, float>::type;
  static constexpr int V = 2, IN_BYTES = 8, OUT_BYTES = 4;
  __device__ static C coef(double c) { return (C)c; }
  __device__ static D div(double d) { return (float)d; }
  __device__ static A zero() { return -0.0f; }
  __device__ static float rnd(float x) { return x; }
  __device__ static void unpack(u32x4 r, long long (&x)[V]) {
    x[0] = __builtin_bit_cast(long long, u32x2{r[0], r[1]});
    x[1] = __builtin_bit_cast(long long, u32x2{r[2], r[3]});
  }
  __device__ static long long ld1(const void* p, int64_t e) { return ((const long long*)p)[e]; }
  __device__ static void st1(void* p, int64_t e, float v) { ((float*)p)[e] = v; }
  __device__ static void stv(void* p, const float (&a)[V]) {
    u32x2 w = {__float_as_uint(a[0]), __float_as_uint(a[1])};
    __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x2*)p);
  }
};

// int64 inputs, plain sum: int64 output, two's-complement wrap
template <> struct Tr<FA_DTYPE_I64, FA_MODE_SUM> {
  using A = unsigned long long; using R = long long; using C = float; using D = float;
  static constexpr int V = 2, IN_BYTES = 8, OUT_BYTES = 8;
  __device__ static C coef(double) { return 0.f; }
  __device__ static D div(double) { return 0.f; }
  __device__ static A zero() { return 0ull; }
  __device__ static A rnd(A x) { return x; }
  __device__ static void unpack(u32x4 r, long long (&x)[V]) {
    x[0] = __builtin_bit_cast(long long, u32x2{r[0], r[1]});
    x[1] = __builtin_bit_cast(long long, u32x2{r[2], r[3]});
  }
  __device__ static long long ld1(const void* p, int64_t e) { return ((const long long*)p)[e]; }
  __device__ static void st1(void* p, int64_t e, A v) { ((unsigned long long*)p)[e] = v; }
  __device__ static void stv(void* p, const A (&a)[V]) {
    u32x2 lo = __builtin_bit_cast(u32x2, a[0]), hi = __builtin_bit_cast(u32x2, a[1]);
    u32x4 w = {lo[0], lo[1], hi[0], hi[1]};
    __builtin_nontemporal_store(w, (__attribute__((address_space(1))) u32x4*)p);
  }
};

// t_i of the contract
template <int DT, int MODE>
__device__ __forceinline__ typename Tr<DT, MODE>::A term(typename Tr<DT, MODE>::R x,
                                                         typename Tr<DT, MODE>::C c,
                                                         typename Tr<DT, MODE>::D d) {
  using T = Tr<DT, MODE>;
  if constexpr (DT == FA_DTYPE_I64) {
    if constexpr (MODE == FA_MODE_SUM) {
      return (unsigned long long)x;
    } else if constexpr (MODE == FA_MODE_MUL_W) {
      return op_mul((float)x, c);
    } else {  // int64 * int64 (wrapping), then true_divide in float32
      return op_div((float)(long long)((unsigned long long)x * (unsigned long long)c), d);
    }
  } else {
    if constexpr (MODE == FA_MODE_SUM) {
      return x;
    } else if constexpr (MODE == FA_MODE_MUL_W) {
      return T::rnd(op_mul(x, c));
    } else {
      return T::rnd(op_div(T::rnd(op_mul(x, c)), d));
    }
  }
}

template <int DT, int MODE>
__device__ __forceinline__ typename Tr<DT, MODE>::A accum(typename Tr<DT, MODE>::A acc,
                                                          typename Tr<DT, MODE>::A t) {
  if constexpr (DT == FA_DTYPE_I64 && MODE == FA_MODE_SUM) {
    return acc + t;
  } else {
    return Tr<DT, MODE>::rnd(op_add(acc, t));
  }
}

// Client tensors are plain device allocations: load through the GLOBAL address space so hipcc
// emits global_load_dwordx4 (in-order vmcnt accounting) instead of flat_load_dwordx4.
typedef const __attribute__((address_space(1))) u32x4* gp_u32x4;

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const void* p) {
  gp_u32x4 g = (gp_u32x4)p;
  if constexpr (NT) return __builtin_nontemporal_load(g);
  else return *g;
}


// --------------------------------------------------------------------------------------------
// The ordered weighted-sum kernel.  One workgroup = one tile of kBlock*V*S elements of one segment:
// lane l owns the S vectors at e0 + s*kBlock*V (each slot coalesced across the wave).  Clients are
// consumed in groups of U; with PF (prefetch) the next group's U*S loads are issued before the
// current group is consumed, so a wave keeps up to 2*U*S KiB in flight.
template <int DT, int MODE, int U, int S, bool NT>
struct WsumBody {
  using T = Tr<DT, MODE>;
  using A = typename T::A;
  using R = typename T::R;
  static constexpr int V = T::V;
  static constexpr int64_t SLOT_BYTES = (int64_t)kBlock * V * T::IN_BYTES;

  // sst: bytes between the input slots of one lane (SLOT_BYTES for flat inputs; the arena's tile
  // stride for tile-interleaved inputs, fa_weighted_sum_tiled)
  __device__ static void load(u32x4 (&r)[U][S], const void* const* __restrict__ in, int i0, int k,
                              int64_t boff, int64_t sst = SLOT_BYTES) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u, k - 1);  // clamped: every load unconditional
      const char* p = (const char*)in[i] + boff;
#pragma unroll
      for (int s = 0; s < S; ++s) r[u][s] = ld16<NT>(p + s * sst);
    }
  }
  // element index of flat element e in an input whose 4-KiB slots are `sst` bytes apart
  __device__ static int64_t phys(int64_t e, int64_t sst) {
    constexpr int64_t TV = (int64_t)kBlock * V;
    return (e / TV) * (sst / T::IN_BYTES) + e % TV;
  }
  template <bool GUARD>
  __device__ static void consume(A (&acc)[S][V], const u32x4 (&r)[U][S], const double* __restrict__ coef,
                                 int i0, int k, typename T::D d) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!GUARD || i0 + u < k) {  // wave-uniform
        const typename T::C c = T::coef(coef[i0 + u]);
#pragma unroll
        for (int s = 0; s < S; ++s) {
          R x[V];
          T::unpack(r[u][s], x);
#pragma unroll
          for (int v = 0; v < V; ++v) acc[s][v] = accum<DT, MODE>(acc[s][v], term<DT, MODE>(x[v], c, d));
        }
      }
    }
  }
};

// One workgroup's tile of an ordered weighted reduction (the body of k_wsum and k_wsum_pair).
template <int DT, int MODE, int U, int S, bool NT, bool PF>
__device__ __forceinline__ void wsum_tile(const Seg* __restrict__ segs, int nseg, const double* __restrict__ coef,
                                          const void* const* __restrict__ ptrs, int k, double divisor,
                                          int64_t sstr, int64_t tile) {
  using B = WsumBody<DT, MODE, U, S, NT>;
  using T = typename B::T;
  using A = typename B::A;
  constexpr int V = T::V;
  constexpr int64_t TILE = (int64_t)kBlock * V * S;

  const Seg sg = segs[nseg > 1 ? find_seg(segs, nseg, tile) : 0];
  const int64_t tl = tile - sg.tile_start;
  const int64_t base = tl * TILE;
  const void* const* in = ptrs + sg.ptr_base;
  const typename T::D d = T::div(divisor);
  const int64_t sst = sstr ? sstr : B::SLOT_BYTES;  // flat: slot s of tile tl is tile tl*S+s

  if (sg.aligned && base + TILE <= sg.numel) {
    const int64_t e0 = base + (int64_t)threadIdx.x * V;
    const int64_t boff = tl * S * sst + (int64_t)threadIdx.x * V * T::IN_BYTES;
    A acc[S][V];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[s][v] = T::zero();
    if constexpr (PF) {
      u32x4 ra[U][S], rb[U][S];
      B::load(ra, in, 0, k, boff, sst);
      int i0 = 0;
      // two groups per trip so the ping-pong buffers keep fixed registers
      for (; i0 + 2 * U < k; i0 += 2 * U) {
        B::load(rb, in, i0 + U, k, boff, sst);
        B::template consume<false>(acc, ra, coef, i0, k, d);
        B::load(ra, in, i0 + 2 * U, k, boff, sst);
        B::template consume<false>(acc, rb, coef, i0 + U, k, d);
      }
      if (i0 + U < k) {
        B::load(rb, in, i0 + U, k, boff, sst);
        B::template consume<false>(acc, ra, coef, i0, k, d);
        B::template consume<true>(acc, rb, coef, i0 + U, k, d);
      } else {
        B::template consume<true>(acc, ra, coef, i0, k, d);
      }
    } else {
      // whole groups unguarded: a guarded consume (a wave-uniform branch per client) let hipcc sink
      // the group's second load into its branch, issued only after the first client's arithmetic and
      // waited for with vmcnt(0) -- one serialized memory round trip per group of U clients (r06)
      int i0 = 0;
      for (; i0 + U <= k; i0 += U) {
        u32x4 r[U][S];
        B::load(r, in, i0, k, boff, sst);
        B::template consume<false>(acc, r, coef, i0, k, d);
      }
      if (i0 < k) {
        u32x4 r[U][S];
        B::load(r, in, i0, k, boff, sst);
        B::template consume<true>(acc, r, coef, i0, k, d);
      }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) T::stv((char*)sg.out + (e0 + (int64_t)s * kBlock * V) * T::OUT_BYTES, acc[s]);
  } else {
    // tail tile or unaligned segment: coalesced scalar loads, same arithmetic
    const int64_t end = min(base + TILE, sg.numel);
    for (int64_t e = base + threadIdx.x; e < end; e += kBlock) {
      A acc = T::zero();
      const int64_t pe = B::phys(e, sst);
      // unrolled: the loads of 8 clients issue before their chain of accumulations (a long client list
      // issued one load per round trip: r04x / r04aa, the 512-client hier tail tile ran ~0.25 ms alone)
#pragma unroll 8
      for (int i = 0; i < k; ++i)
        acc = accum<DT, MODE>(acc, term<DT, MODE>(T::ld1(in[i], pe), T::coef(coef[i]), d));
      T::st1(sg.out, e, acc);
    }
  }
}

// xcd = 1: workgroup -> tile mapping by XCD (the dispatcher deals workgroups to the 8 XCDs
// round-robin; XCD x then walks a contiguous eighth of the tiles, so one XCD's L2 and address
// translation caches see a few segments' allocations instead of all of them)
__device__ __forceinline__ int64_t xcd_tile(int64_t bid, int64_t tiles) { return xcd_tile_map(bid, tiles); }

constexpr int kXcdMinClients = 32;  // single flat segments with at least this many client vectors: XCD map

bool xcd_map_single() {  // FA_XCD_MAP=2: XCD-contiguous tiles for single-segment staged launches too (A/B)
  static const int on = [] {
    const char* e = getenv("FA_XCD_MAP");
    return e && e[0] == '2' ? 1 : 0;
  }();
  return on != 0;
}

bool xcd_map_enabled() {  // FA_XCD_MAP=0: round-robin workgroup -> tile order everywhere (A/B)
  static const int on = [] {
    const char* e = getenv("FA_XCD_MAP");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on != 0;
}

// XCD-contiguous tiles (xcd_tile) with workgroup 0 and the workgroup the map gives the last tile
// swapped: the ragged last tile still starts first (a bijection of [0, tiles))
__device__ __forceinline__ int64_t xcd_tail_first(int64_t bid, int64_t tiles) {
  const int64_t m = xcd_tile(bid, tiles);
  if (bid == 0) return tiles - 1;
  return m == tiles - 1 ? xcd_tile(0, tiles) : m;
}

// one segment: workgroup 0 takes the last tile (ragged: the scalar path, one pass over every client
// per element) so that it overlaps the stream instead of running alone after it (r04aa / r04ab)
__device__ __forceinline__ int64_t tail_first(int nseg) {
  return nseg == 1 ? (blockIdx.x == 0 ? (int64_t)gridDim.x - 1 : (int64_t)blockIdx.x - 1) : (int64_t)blockIdx.x;
}

template <int DT, int MODE, int U, int S, bool NT, bool PF>
__global__ void __launch_bounds__(kBlock)
k_wsum(const Seg* __restrict__ segs, int nseg, const double* __restrict__ coef,
       const void* const* __restrict__ ptrs, int k, double divisor, int64_t sstr, int xcd) {
  const int64_t t = xcd ? (nseg == 1 ? xcd_tail_first(blockIdx.x, gridDim.x) : xcd_tile(blockIdx.x, gridDim.x))
                        : tail_first(nseg);
  wsum_tile<DT, MODE, U, S, NT, PF>(segs, nseg, coef, ptrs, k, divisor, sstr, t);
}

// Descriptor tables (segments | coefficients | pointers) small enough to travel as the kernel's
// argument: the launch then needs no staged host->device copy (one ~2.5 us blit plus its dependency
// gap on the stream per launch -- a visible share of a 0.26 ms cfg2 round or of a multi-GPU step's
// eight chunk launches).  The tables are read with scalar loads from the kernarg segment, exactly
// as from the staged buffer.
constexpr int kInlineBytes = 3072;
struct InlineDesc {
  alignas(16) char raw[kInlineBytes];
};

template <int DT, int MODE, int U, int S, bool NT, bool PF>
__global__ void __launch_bounds__(kBlock)
k_wsum_inl(const InlineDesc dsc, int nseg, int coef_off, int ptr_off, int k, double divisor, int64_t sstr, int xcd) {
  const char* b = dsc.raw;
  const int64_t t = xcd ? xcd_tail_first((int64_t)blockIdx.x, (int64_t)gridDim.x) : tail_first(nseg);
  wsum_tile<DT, MODE, U, S, NT, PF>((const Seg*)b, nseg, (const double*)(b + coef_off),
                                    (const void* const*)(b + ptr_off), k, divisor, sstr, t);
}

// A float dtype group and the state_dict's int64 group (BatchNorm num_batches_tracked counters,
// promoted to fp32 by the reference's `x * w`) in ONE launch: the int64 tiles take the first
// workgroups, so their latency-bound ordered loop (~10 us as a launch of its own for ResNet-18-GN's
// 20 counters) overlaps the float group's stream instead of following it with a second launch and
// a second descriptor copy.  Same per-element arithmetic as two k_wsum launches.
template <int DT, int MODE, int U, int S, bool PF>
__global__ void __launch_bounds__(kBlock)
k_wsum_pair(const Seg* __restrict__ segs0, int nseg0, const void* const* __restrict__ ptrs0, int64_t sstr0,
            const Seg* __restrict__ segs1, int nseg1, const void* const* __restrict__ ptrs1, int64_t sstr1,
            int64_t tiles1, const double* __restrict__ coef, int k, double divisor, int xcd) {
  const int64_t t = xcd ? xcd_tile(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;  // see k_wsum
  if (t < tiles1)
    wsum_tile<FA_DTYPE_I64, MODE, 8, 1, true, false>(segs1, nseg1, coef, ptrs1, k, divisor, sstr1, t);
  else
    wsum_tile<DT, MODE, U, S, true, PF>(segs0, nseg0, coef, ptrs0, k, divisor, sstr0, t - tiles1);
}

// k_wsum_pair with its tables as the kernel argument (layout of PairTables)
template <int DT, int MODE, int U, int S, bool PF>
__global__ void __launch_bounds__(kBlock)
k_wsum_pair_inl(const InlineDesc dsc, int nseg0, int nseg1, int seg1_off, int coef_off, int ptr0_off, int ptr1_off,
                int64_t sstr0, int64_t sstr1, int64_t tiles1, int k, double divisor) {
  const char* b = dsc.raw;
  const double* coef = (const double*)(b + coef_off);
  const int64_t t = blockIdx.x;
  if (t < tiles1)
    wsum_tile<FA_DTYPE_I64, MODE, 8, 1, true, false>((const Seg*)(b + seg1_off), nseg1, coef,
                                                     (const void* const*)(b + ptr1_off), k, divisor, sstr1, t);
  else
    wsum_tile<DT, MODE, U, S, true, PF>((const Seg*)b, nseg0, coef, (const void* const*)(b + ptr0_off), k, divisor,
                                        sstr0, t - tiles1);
}

// --------------------------------------------------------------------------------------------
// Two-level (grouped) ordered reduction in ONE pass over the clients: for every group g (a
// contiguous client range), the group partial G_g = ordered reduction of its clients (MODE), then
// the group epilogue t_g (none / op(G_g * c_g) / op(op(G_g * c_g) / d_g)), then out = ordered sum
// of t_g.  This is the reference's two-level arithmetic -- hierarchical FL (group FedAvg, then the
// cloud's (G*n)/N or the SP trainer's G*(N_g/N)), fedavg_seq (worker partials, then a plain sum) --
// with every intermediate kept in registers: bit-identical to running the levels as separate
// launches, minus the intermediate HBM round trips.
struct GroupDesc {
  int32_t begin, end;  // client range
  double mul;          // epilogue coefficient c_g
  double div;          // epilogue divisor d_g
  int64_t pad;
};
static_assert(sizeof(GroupDesc) == 32, "GroupDesc layout");

template <int DT, int MODE, int U, bool NT>
__global__ void __launch_bounds__(kBlock)
k_wsum_grouped(const Seg* __restrict__ segs, const double* __restrict__ coef,
               const void* const* __restrict__ ptrs, double divisor,
               const GroupDesc* __restrict__ groups, int ngroups, int gmode, int64_t sstr) {
  using B = WsumBody<DT, MODE, U, 1, NT>;
  using T = typename B::T;
  using A = typename B::A;
  constexpr int V = T::V;
  constexpr int64_t TILE = (int64_t)kBlock * V;
  // workgroup 0 takes the LAST tile (ragged: the scalar path, one pass over every client per element)
  // so that it overlaps the stream instead of running alone at the end -- r04aa: cfg4 (512 clients,
  // 11.70 M coordinates) 3.80 -> 3.55 ms; the size had run as slow as 12.58 M (profiles/r04x)
  const int64_t tile = blockIdx.x == 0 ? (int64_t)gridDim.x - 1 : (int64_t)blockIdx.x - 1;
  const Seg sg = segs[0];
  const int64_t base = tile * TILE;
  const void* const* in = ptrs;
  const typename T::D d = T::div(divisor);
  const int64_t sst = sstr ? sstr : B::SLOT_BYTES;

  auto epilogue = [&](A g, const GroupDesc& gd) -> A {
    if (gmode == FA_MODE_MUL_W) return T::rnd(op_mul(g, (A)gd.mul));
    if (gmode == FA_MODE_MUL_N_DIV_N) return T::rnd(op_div(T::rnd(op_mul(g, (A)gd.mul)), (A)gd.div));
    return g;
  };

  if (sg.aligned && base + TILE <= sg.numel) {
    const int64_t e0 = base + (int64_t)threadIdx.x * V;
    const int64_t boff = tile * sst + (int64_t)threadIdx.x * V * T::IN_BYTES;
    A out[V];
#pragma unroll
    for (int v = 0; v < V; ++v) out[v] = T::zero();
    for (int g = 0; g < ngroups; ++g) {
      const GroupDesc gd = groups[g];
      A acc[1][V];
#pragma unroll
      for (int v = 0; v < V; ++v) acc[0][v] = T::zero();
      int i0 = gd.begin;
      for (; i0 + U <= gd.end; i0 += U) {  // whole groups unguarded (see wsum_tile)
        u32x4 r[U][1];
        B::load(r, in, i0, gd.end, boff, sst);
        B::template consume<false>(acc, r, coef, i0, gd.end, d);
      }
      if (i0 < gd.end) {
        u32x4 r[U][1];
        B::load(r, in, i0, gd.end, boff, sst);
        B::template consume<true>(acc, r, coef, i0, gd.end, d);
      }
#pragma unroll
      for (int v = 0; v < V; ++v) out[v] = accum<DT, MODE>(out[v], epilogue(acc[0][v], gd));
    }
    T::stv((char*)sg.out + e0 * T::OUT_BYTES, out);
  } else {
    const int64_t end = min(base + TILE, sg.numel);
    for (int64_t e = base + threadIdx.x; e < end; e += kBlock) {
      A out = T::zero();
      const int64_t pe = B::phys(e, sst);
      for (int g = 0; g < ngroups; ++g) {
        const GroupDesc gd = groups[g];
        A acc = T::zero();
#pragma unroll 8
        for (int i = gd.begin; i < gd.end; ++i)
          acc = accum<DT, MODE>(acc, term<DT, MODE>(T::ld1(in[i], pe), T::coef(coef[i]), d));
        out = accum<DT, MODE>(out, epilogue(acc, gd));
      }
      T::st1(sg.out, e, out);
    }
  }
}

// --------------------------------------------------------------------------------------------
// FedOpt server step fused into the aggregation (simulation/mpi/fedopt/FedOptAggregator.py:
// 104-131): per element the FedAvg average (ordered, in registers), the pseudo-gradient
// g = param - avg, and torch.optim.SGD's update of the global parameter and its momentum buffer,
// in place.  The reference runs FedAvg, a state_dict round trip and a CPU optimizer step; PyTorch's
// CPU add(alpha) is a fused multiply-add, so every `x + a*y` here is one __fmaf_rn (pinned by the
// g10 fixtures).  fp32 parameters; segments = parameter tensors (Seg.out = the parameter).
enum { SGD_MOMENTUM = 1, SGD_NESTEROV = 2, SGD_WD = 4, SGD_FIRST = 8 };

__device__ __forceinline__ float sgd_update(float p, float avg, float& buf, float neg_lr, float mom,
                                            float damp1, float wd, int flags) {
  float g = __fsub_rn(p, avg);
  if (flags & SGD_WD) g = __fmaf_rn(p, wd, g);
  if (flags & SGD_MOMENTUM) {
    buf = (flags & SGD_FIRST) ? g : __fmaf_rn(g, damp1, __fmul_rn(buf, mom));
    g = (flags & SGD_NESTEROV) ? __fmaf_rn(buf, mom, g) : buf;
  }
  return __fmaf_rn(g, neg_lr, p);
}

// torch.optim.RMSprop (centered=False) on CPU tensors, reachable from the reference's FedOpt as
// server_optimizer="rmsprop" (OptRepo passes lr and momentum).  ATen's CPU op sequence:
// square_avg.mul_(alpha).addcmul_(g, g, value=1-alpha) -> fma((1-alpha)*g, g, sq*alpha);
// avg = sqrt(square_avg) + eps; momentum: buf = buf*m + g/avg (addcdiv), p += -lr*buf (FMA);
// else p = p + (-lr*g)/avg.  ATen's sqrt there is MKL-VML (not correctly rounded): parity is
// within 1e-6 relative, not bit-exact.  State starts at zero (torch initialises it so).
struct RmsArgs { float alpha, one_m_alpha, eps; };

__device__ __forceinline__ float rmsprop_update(float p, float avg, float& sq, float& buf, float neg_lr, float mom,
                                                float wd, const RmsArgs& ra, int flags) {
  float g = __fsub_rn(p, avg);
  if (flags & SGD_WD) g = __fmaf_rn(p, wd, g);
  sq = __fmaf_rn(__fmul_rn(ra.one_m_alpha, g), g, __fmul_rn(sq, ra.alpha));
  // correctly rounded float sqrt: the float32 __fsqrt_rn lowers to v_sqrt_f32 (~1 ulp) on gfx950;
  // the float64 sqrt is correctly rounded and float64 -> float32 rounding of a sqrt is innocuous
  const float den = __fadd_rn(__double2float_rn(__dsqrt_rn((double)sq)), ra.eps);
  if (flags & SGD_MOMENTUM) {
    buf = __fadd_rn(__fmul_rn(buf, mom), __fdiv_rn(g, den));
    return __fmaf_rn(buf, neg_lr, p);
  }
  return __fadd_rn(p, __fdiv_rn(__fmul_rn(neg_lr, g), den));
}

// OPT 0: SGD (bufs = momentum); OPT 1: RMSprop (bufs = momentum, bufs2 = square_avg)
template <int U, bool NT, int OPT>
__device__ __forceinline__ void fedavg_sgd_tile(const Seg* __restrict__ segs, int nseg, const double* __restrict__ coef,
                                                const void* const* __restrict__ ptrs, int k,
                                                void* const* __restrict__ bufs, float neg_lr, float mom, float damp1,
                                                float wd, int flags, int64_t sstr, void* const* __restrict__ bufs2,
                                                RmsArgs ra, int64_t tile) {
  using B = WsumBody<FA_DTYPE_F32, FA_MODE_MUL_W, U, 1, NT>;
  using T = typename B::T;
  constexpr int V = T::V;
  constexpr int64_t TILE = (int64_t)kBlock * V;
  const int s = nseg > 1 ? find_seg(segs, nseg, tile) : 0;
  const Seg sg = segs[s];
  float* param = (float*)sg.out;
  float* mbuf = (float*)bufs[s];
  float* sqb = OPT == 1 ? (float*)bufs2[s] : nullptr;
  const int64_t tl = tile - sg.tile_start;
  const int64_t base = tl * TILE;
  const void* const* in = ptrs + sg.ptr_base;
  const float d = 0.f;
  const int64_t sst = sstr ? sstr : B::SLOT_BYTES;
  const bool read_buf = (flags & SGD_MOMENTUM) && !(flags & SGD_FIRST);

  if (sg.aligned && base + TILE <= sg.numel) {
    const int64_t e0 = base + (int64_t)threadIdx.x * V;
    const int64_t boff = tl * sst + (int64_t)threadIdx.x * V * 4;
    // the parameter and momentum loads are issued first: their latency hides under the client stream
    u32x4 p4 = ld16<true>(param + e0);
    u32x4 b4 = {0, 0, 0, 0}, q4 = {0, 0, 0, 0};
    if (read_buf) b4 = ld16<true>(mbuf + e0);
    if (OPT == 1 && !(flags & SGD_FIRST)) q4 = ld16<true>(sqb + e0);
    float acc[1][V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[0][v] = -0.0f;
    int i0 = 0;
    for (; i0 + U <= k; i0 += U) {  // whole groups unguarded (see wsum_tile)
      u32x4 r[U][1];
      B::load(r, in, i0, k, boff, sst);
      B::template consume<false>(acc, r, coef, i0, k, d);
    }
    if (i0 < k) {
      u32x4 r[U][1];
      B::load(r, in, i0, k, boff, sst);
      B::template consume<true>(acc, r, coef, i0, k, d);
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float b = __uint_as_float(b4[v]);
      if constexpr (OPT == 1) {
        float q = __uint_as_float(q4[v]);
        p4[v] = __float_as_uint(rmsprop_update(__uint_as_float(p4[v]), acc[0][v], q, b, neg_lr, mom, wd, ra, flags));
        q4[v] = __float_as_uint(q);
      } else {
        p4[v] = __float_as_uint(sgd_update(__uint_as_float(p4[v]), acc[0][v], b, neg_lr, mom, damp1, wd, flags));
      }
      b4[v] = __float_as_uint(b);
    }
    __builtin_nontemporal_store(p4, (__attribute__((address_space(1))) u32x4*)(param + e0));
    if (flags & SGD_MOMENTUM) __builtin_nontemporal_store(b4, (__attribute__((address_space(1))) u32x4*)(mbuf + e0));
    if constexpr (OPT == 1) __builtin_nontemporal_store(q4, (__attribute__((address_space(1))) u32x4*)(sqb + e0));
  } else {
    const int64_t end = min(base + TILE, sg.numel);
    for (int64_t e = base + threadIdx.x; e < end; e += kBlock) {
      const int64_t pe = B::phys(e, sst);
      float acc = -0.0f;
#pragma unroll 8
      for (int i = 0; i < k; ++i)
        acc = accum<FA_DTYPE_F32, FA_MODE_MUL_W>(
            acc, term<FA_DTYPE_F32, FA_MODE_MUL_W>(T::ld1(in[i], pe), T::coef(coef[i]), d));
      float b = read_buf ? mbuf[e] : 0.f;
      if constexpr (OPT == 1) {
        float q = (flags & SGD_FIRST) ? 0.f : sqb[e];
        param[e] = rmsprop_update(param[e], acc, q, b, neg_lr, mom, wd, ra, flags);
        sqb[e] = q;
      } else {
        param[e] = sgd_update(param[e], acc, b, neg_lr, mom, damp1, wd, flags);
      }
      if (flags & SGD_MOMENTUM) mbuf[e] = b;
    }
  }
}

template <int U, bool NT, int OPT = 0>
__global__ void __launch_bounds__(kBlock)
k_fedavg_sgd(const Seg* __restrict__ segs, int nseg, const double* __restrict__ coef,
             const void* const* __restrict__ ptrs, int k, void* const* __restrict__ bufs, float neg_lr,
             float mom, float damp1, float wd, int flags, int64_t sstr, void* const* __restrict__ bufs2,
             RmsArgs ra) {
  fedavg_sgd_tile<U, NT, OPT>(segs, nseg, coef, ptrs, k, bufs, neg_lr, mom, damp1, wd, flags, sstr, bufs2, ra,
                              tail_first(nseg));
}

// the same with its tables (Seg[nseg] | coef[k] | bufs[nseg] | bufs2[nseg] | ptrs[nseg * k]) as the
// kernel argument (see InlineDesc)
template <int U, bool NT, int OPT = 0>
__global__ void __launch_bounds__(kBlock)
k_fedavg_sgd_inl(const InlineDesc dsc, int nseg, int coef_off, int buf_off, int buf2_off, int ptr_off, int k,
                 float neg_lr, float mom, float damp1, float wd, int flags, int64_t sstr, RmsArgs ra) {
  const char* b = dsc.raw;
  fedavg_sgd_tile<U, NT, OPT>((const Seg*)b, nseg, (const double*)(b + coef_off), (const void* const*)(b + ptr_off),
                              k, (void* const*)(b + buf_off), neg_lr, mom, damp1, wd, flags, sstr,
                              (void* const*)(b + buf2_off), ra, tail_first(nseg));
}

// --------------------------------------------------------------------------------------------
// Mixing / gossip kernel: one workgroup = one element tile, looping over every output row so that
// an input shared by neighbouring rows is re-read from L2 / Infinity Cache, not HBM.  Rows go in
// groups of RG: the loads of all RG rows (up to MAXD entries each, clamped like k_wsum) are issued
// before any is consumed, so a wave keeps RG*MAXD KiB in flight -- RG-1 of every RG rows' new
// neighbour is an L2 hit for a ring, so without the grouping a wave would hold only ~1 HBM miss.
// Rows with more than MAXD entries take ceil(deg / MAXD) passes (dense rows, e.g. 8x8 mixing).
template <int DT, int RG, int MAXD, bool POST>
__global__ void __launch_bounds__(kBlock)
k_mix(const MixRow* __restrict__ rows, int nrows, const int32_t* __restrict__ cols,
      const double* __restrict__ vals, const void* const* __restrict__ in, int64_t n, int aligned,
      int64_t isst, int64_t osst) {
  using T = Tr<DT, FA_MODE_MUL_W>;
  constexpr int V = T::V;
  constexpr int64_t TILE = (int64_t)kBlock * V;
  const int64_t bt = tail_first(1);  // the ragged last tile (scalar path over every row) first
  const int64_t base = bt * TILE;
  const float dz = 0.f;
  // 4-KiB slot strides of the inputs / outputs: TILE * bytes (flat) or an arena's tile stride
  const int64_t ist = isst ? isst : TILE * T::IN_BYTES, ost = osst ? osst : TILE * T::OUT_BYTES;

  if (aligned && base + TILE <= n) {
    const int64_t boff = bt * ist + (int64_t)threadIdx.x * V * T::IN_BYTES;
    const int64_t ooff = bt * ost + (int64_t)threadIdx.x * V * T::OUT_BYTES;
    for (int r0 = 0; r0 < nrows; r0 += RG) {
      int beg[RG], end[RG];
      int maxd = 0;
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        const int r = min(r0 + g, nrows - 1);
        beg[g] = rows[r].begin;
        end[g] = rows[r].end;
        maxd = max(maxd, end[g] - beg[g]);
      }
      float acc[RG][V];
#pragma unroll
      for (int g = 0; g < RG; ++g)
#pragma unroll
        for (int v = 0; v < V; ++v) acc[g][v] = -0.0f;
      for (int p = 0; p < maxd; p += MAXD) {
        u32x4 x4[RG][MAXD];
#pragma unroll
        for (int g = 0; g < RG; ++g)
#pragma unroll
          for (int u = 0; u < MAXD; ++u) {
            const int j = min(beg[g] + p + u, end[g] - 1);
            x4[g][u] = ld16<false>((const char*)in[cols[j]] + boff);
          }
#pragma unroll
        for (int g = 0; g < RG; ++g)
#pragma unroll
          for (int u = 0; u < MAXD; ++u) {
            if (beg[g] + p + u < end[g]) {  // wave-uniform
              const float c = (float)vals[beg[g] + p + u];
              float x[V];
              T::unpack(x4[g][u], x);
#pragma unroll
              for (int v = 0; v < V; ++v)
                acc[g][v] = accum<DT, FA_MODE_MUL_W>(acc[g][v], term<DT, FA_MODE_MUL_W>(x[v], c, dz));
            }
          }
      }
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        if (r0 + g < nrows) {
          const MixRow& row = rows[r0 + g];
          T::stv((char*)row.out + ooff, acc[g]);
          if constexpr (POST) {
            const float s = (float)row.scale;
            float z[V];
#pragma unroll
            for (int v = 0; v < V; ++v) z[v] = T::rnd(op_mul(acc[g][v], s));
            T::stv((char*)row.out2 + ooff, z);
          }
        }
      }
    }
  } else {
    const int64_t end = min(base + TILE, n);
    for (int r = 0; r < nrows; ++r) {
      const MixRow row = rows[r];
      for (int64_t e = base + threadIdx.x; e < end; e += kBlock) {
        const int64_t pi = (e / TILE) * (ist / T::IN_BYTES) + e % TILE;
        const int64_t po = (e / TILE) * (ost / T::OUT_BYTES) + e % TILE;
        float acc = -0.0f;
        for (int j = row.begin; j < row.end; ++j)
          acc = accum<DT, FA_MODE_MUL_W>(
              acc, term<DT, FA_MODE_MUL_W>(T::ld1(in[cols[j]], pi), (float)vals[j], dz));
        T::st1(row.out, po, acc);
        if constexpr (POST) T::st1(row.out2, po, T::rnd(op_mul(acc, (float)row.scale)));
      }
    }
  }
}

// --------------------------------------------------------------------------------------------
// Banded mixing (ring-like gossip): every entry of row r reads input (r + off + d) mod num_in with
// d in {-1, 0, +1} (host-checked); NT: non-temporal input loads (the default launch).  Rows are walked in order with a register sliding window over
// the inputs, so each input tile is loaded ONCE per workgroup (k_mix re-reads neighbours through
// L2/MALL: +8 % HBM traffic at 256 nodes).  Per group of RG rows the RG new window slots are loaded
// together; each CSR entry picks its slot by a wave-uniform switch (scalar branches, no VALU select),
// so the accumulation order is still the CSR order, bit for bit.
template <int DT, int RG, bool POST, bool NT = false>
__global__ void __launch_bounds__(kBlock)
k_mix_band(const MixRow* __restrict__ rows, int nrows, const int32_t* __restrict__ cols,
           const double* __restrict__ vals, const void* const* __restrict__ in, int num_in, int off,
           int64_t n, int64_t isst, int64_t osst, int xcd) {
  using T = Tr<DT, FA_MODE_MUL_W>;
  constexpr int V = T::V;
  constexpr int64_t TILE = (int64_t)kBlock * V;
  const int64_t bt0 = xcd ? xcd_tile(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;  // see k_wsum
  // workgroup 0 (tile 0 under either map) takes the last, ragged tile: its scalar path walks every row
  const int64_t bt = bt0 == 0 ? (int64_t)gridDim.x - 1 : bt0 - 1;
  const int64_t base = bt * TILE;
  const float dz = 0.f;
  const int64_t ist = isst ? isst : TILE * T::IN_BYTES, ost = osst ? osst : TILE * T::OUT_BYTES;
  auto wrap = [num_in](int c) { c %= num_in; return c < 0 ? c + num_in : c; };

  if (base + TILE <= n) {
    const int64_t boff = bt * ist + (int64_t)threadIdx.x * V * T::IN_BYTES;
    const int64_t ooff = bt * ost + (int64_t)threadIdx.x * V * T::OUT_BYTES;
    u32x4 win[RG + 2];  // win[s] = input (r0 + off - 1 + s) mod num_in
    win[0] = ld16<NT>((const char*)in[wrap(off - 1)] + boff);
    win[1] = ld16<NT>((const char*)in[wrap(off)] + boff);
    for (int r0 = 0; r0 < nrows; r0 += RG) {
#pragma unroll
      for (int g = 0; g < RG; ++g) win[2 + g] = ld16<NT>((const char*)in[wrap(r0 + off + 1 + g)] + boff);
#pragma unroll
      for (int g = 0; g < RG; ++g) {
        if (r0 + g < nrows) {  // wave-uniform
          const MixRow row = rows[r0 + g];
          float acc[V];
#pragma unroll
          for (int v = 0; v < V; ++v) acc[v] = -0.0f;
          for (int j = row.begin; j < row.end; ++j) {
            const int rel = wrap(cols[j] - (r0 + g + off) + 1);  // 0, 1 or 2 (host-checked)
            const float c = (float)vals[j];
            float x[V];
            if (rel == 0) T::unpack(win[g], x);
            else if (rel == 1) T::unpack(win[g + 1], x);
            else T::unpack(win[g + 2], x);
#pragma unroll
            for (int v = 0; v < V; ++v)
              acc[v] = accum<DT, FA_MODE_MUL_W>(acc[v], term<DT, FA_MODE_MUL_W>(x[v], c, dz));
          }
          T::stv((char*)row.out + ooff, acc);
          if constexpr (POST) {
            const float sc = (float)row.scale;
#pragma unroll
            for (int v = 0; v < V; ++v) acc[v] = T::rnd(op_mul(acc[v], sc));
            T::stv((char*)row.out2 + ooff, acc);
          }
        }
      }
      win[0] = win[RG];
      win[1] = win[RG + 1];
    }
  } else {
    const int64_t end = min(base + TILE, n);
    for (int r = 0; r < nrows; ++r) {
      const MixRow row = rows[r];
      for (int64_t e = base + threadIdx.x; e < end; e += kBlock) {
        const int64_t pi = (e / TILE) * (ist / T::IN_BYTES) + e % TILE;
        const int64_t po = (e / TILE) * (ost / T::OUT_BYTES) + e % TILE;
        float acc = -0.0f;
        for (int j = row.begin; j < row.end; ++j)
          acc = accum<DT, FA_MODE_MUL_W>(
              acc, term<DT, FA_MODE_MUL_W>(T::ld1(in[cols[j]], pi), (float)vals[j], dz));
        T::st1(row.out, po, acc);
        if constexpr (POST) T::st1(row.out2, po, T::rnd(op_mul(acc, (float)row.scale)));
      }
    }
  }
}

// PushSum's weight on the device (client_pushsum.py:127-156): omega'_r = the row's ordered sum
// omega_r * W_rr + sum_j omega_j * W_jr in float32 -- the same CSR order and per-op rounding as the
// models' mixing rows (the reference's omega is a numpy float32: `omega *= W[i][i]`, then `+=` of
// each sender's `omega_j * W`, in receive order) -- and the row's post-scale 1/omega' (float32
// division, `1.0 / self.omega`), written into the staged row table the mixing kernel reads next.
__global__ void __launch_bounds__(kBlock)
k_pushsum_omega(MixRow* __restrict__ rows, int nrows, const int32_t* __restrict__ cols,
                const double* __restrict__ vals, const float* __restrict__ omega_in, float* __restrict__ omega_out) {
  const int r = blockIdx.x * kBlock + threadIdx.x;
  if (r >= nrows) return;
  const MixRow row = rows[r];
  float acc = -0.0f;
  for (int j = row.begin; j < row.end; ++j)
    acc = accum<FA_DTYPE_F32, FA_MODE_MUL_W>(acc, term<FA_DTYPE_F32, FA_MODE_MUL_W>(omega_in[cols[j]], (float)vals[j], 0.f));
  omega_out[r] = acc;
  rows[r].scale = (double)op_div(1.0f, acc);
}

// The band offset `off` for which every entry of row r is input (r + off + {-1,0,1}) mod num_in,
// or INT_MIN if the CSR is not banded that way.
int band_offset(int32_t rows, const int32_t* row_ptr, const int32_t* cols, int32_t num_in) {
  if (rows <= 0 || num_in < 3) return INT32_MIN;
  auto md = [num_in](int x) { x %= num_in; return x < 0 ? x + num_in : x; };
  int cand[3];
  int nc = 0;
  if (row_ptr[1] <= row_ptr[0]) return INT32_MIN;
  const int c0 = cols[row_ptr[0]];
  for (int d = -1; d <= 1; ++d) cand[nc++] = md(c0 - d);  // row 0: off in {c0+1, c0, c0-1}
  for (int ci = 0; ci < nc; ++ci) {
    const int off = cand[ci];
    bool ok = true;
    for (int r = 0; r < rows && ok; ++r)
      for (int j = row_ptr[r]; j < row_ptr[r + 1] && ok; ++j) {
        const int rel = md(cols[j] - (r + off) + 1);
        ok = rel <= 2;
      }
    if (ok) return off;
  }
  return INT32_MIN;
}

}  // namespace

// --------------------------------------------------------------------------------------------
// Host side (error reporting and the staging slots live in fa_detail, see fa_internal.h).
namespace {

// Kernel variants (performance only; every variant computes the identical result).
struct Variant { int U, S; bool NT, PF; };
constexpr Variant kVariants[] = {
    {8, 1, true, false},   // 0: default
    {4, 1, true, false},   // 1
    {16, 1, true, false},  // 2
    {8, 1, false, false},  // 3: default-policy loads
    {4, 2, true, false},   // 4
    {8, 2, true, false},   // 5
    {4, 4, true, false},   // 6
    {8, 1, true, true},    // 7: double-buffered prefetch
    {4, 2, true, true},    // 8
};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

template <int DT, int MODE, int U, int S, bool NT, bool PF>
void launch_wsum(int64_t tiles, hipStream_t st, const Seg* segs, int nseg, const double* coef,
                 const void* const* ptrs, int k, double divisor, int64_t sstr) {
  // multi-segment tables (separate tensors): XCD-contiguous tiles, FA_XCD_MAP=0 turns it off.  r02ao
  // interleaved A/B: fragmented metric (26,112 tensors) 10.76-10.83 -> 10.64 ms.  One flat segment
  // keeps the hardware's round-robin (tools/layout_probe.py: an XCD-contiguous split read 6.38-6.45
  // vs 6.62-6.72 TB/s there).
  const int xcd = xcd_map_enabled() && (nseg > 1 || xcd_map_single() || (sstr == 0 && k >= kXcdMinClients)) ? 1 : 0;
  hipLaunchKernelGGL((k_wsum<DT, MODE, U, S, NT, PF>), dim3((unsigned)tiles), dim3(kBlock), 0, st, segs,
                     nseg, coef, ptrs, k, divisor, sstr, xcd);
}

// tables as the kernel argument: only the automatic shapes (variant 0: U = 8, S = 1; 5: U = 8, S = 2)
template <int DT, int MODE>
void launch_wsum_inl(int variant, int64_t tiles, hipStream_t st, const InlineDesc& dsc, int nseg, int coef_off,
                     int ptr_off, int k, double divisor, int64_t sstr) {
  // one flat segment over many separately placed client vectors (not a tiled arena): XCD-contiguous
  // tiles, so the workgroups sharing a CU / XCD read neighbouring tiles and reuse their address
  // translations (r05e, 128 separate fp32[125 M] buffers, 2 interleaved reps: 10.43-10.58 ->
  // 10.26-10.30 ms; UTCL1 misses -27 %, profiles/r05b/translation_summary.json)
  const int xcd = nseg == 1 && sstr == 0 && k >= kXcdMinClients && xcd_map_enabled() ? 1 : 0;
  if (variant == 5)
    hipLaunchKernelGGL((k_wsum_inl<DT, MODE, 8, 2, true, false>), dim3((unsigned)tiles), dim3(kBlock), 0, st, dsc,
                       nseg, coef_off, ptr_off, k, divisor, sstr, xcd);
  else
    hipLaunchKernelGGL((k_wsum_inl<DT, MODE, 8, 1, true, false>), dim3((unsigned)tiles), dim3(kBlock), 0, st, dsc,
                       nseg, coef_off, ptr_off, k, divisor, sstr, xcd);
}

template <int DT>
void dispatch_inl(int mode, int variant, int64_t tiles, hipStream_t st, const InlineDesc& dsc, int nseg,
                  int coef_off, int ptr_off, int k, double divisor, int64_t sstr) {
  switch (mode) {
    case FA_MODE_MUL_W: launch_wsum_inl<DT, FA_MODE_MUL_W>(variant, tiles, st, dsc, nseg, coef_off, ptr_off, k, divisor, sstr); break;
    case FA_MODE_MUL_N_DIV_N: launch_wsum_inl<DT, FA_MODE_MUL_N_DIV_N>(variant, tiles, st, dsc, nseg, coef_off, ptr_off, k, divisor, sstr); break;
    default: launch_wsum_inl<DT, FA_MODE_SUM>(variant, tiles, st, dsc, nseg, coef_off, ptr_off, k, divisor, sstr); break;
  }
}

template <int DT, int MODE>
void dispatch_variant(int variant, int64_t tiles, hipStream_t st, const Seg* segs, int nseg,
                      const double* coef, const void* const* ptrs, int k, double divisor, int64_t sstr) {
#define FA_V(ID, U, S, NT, PF) \
  case ID: launch_wsum<DT, MODE, U, S, NT, PF>(tiles, st, segs, nseg, coef, ptrs, k, divisor, sstr); break;
  switch (variant) {
    FA_V(1, 4, 1, true, false)
    FA_V(2, 16, 1, true, false)
    FA_V(3, 8, 1, false, false)
    FA_V(4, 4, 2, true, false)
    FA_V(5, 8, 2, true, false)
    FA_V(6, 4, 4, true, false)
    FA_V(7, 8, 1, true, true)
    FA_V(8, 4, 2, true, true)
    default: launch_wsum<DT, MODE, 8, 1, true, false>(tiles, st, segs, nseg, coef, ptrs, k, divisor, sstr);
  }
#undef FA_V
}

template <int DT>
int dispatch_mode(int mode, int variant, int64_t tiles, hipStream_t st, const Seg* segs, int nseg,
                  const double* coef, const void* const* ptrs, int k, double divisor, int64_t sstr) {
  switch (mode) {
    case FA_MODE_MUL_W: dispatch_variant<DT, FA_MODE_MUL_W>(variant, tiles, st, segs, nseg, coef, ptrs, k, divisor, sstr); break;
    case FA_MODE_MUL_N_DIV_N: dispatch_variant<DT, FA_MODE_MUL_N_DIV_N>(variant, tiles, st, segs, nseg, coef, ptrs, k, divisor, sstr); break;
    case FA_MODE_SUM: dispatch_variant<DT, FA_MODE_SUM>(variant, tiles, st, segs, nseg, coef, ptrs, k, divisor, sstr); break;
    default: return fail(FA_ERR_DTYPE, "unknown mode %d", mode);
  }
  return FA_OK;
}

int elems_per_vec(int dtype) {
  switch (dtype) {
    case FA_DTYPE_F32: return 4;
    case FA_DTYPE_BF16: case FA_DTYPE_F16: return 8;
    case FA_DTYPE_F64: case FA_DTYPE_I64: return 2;
    default: return 0;
  }
}

}  // namespace


// ============================================================================================
// fa_detail: host helpers shared with the other translation units (fa_internal.h).
namespace fa_detail {

namespace {
thread_local char g_last_error[512] = "";
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
  return code;
}

const char* last_error() { return g_last_error; }

// r05: a per-call event record at release() put a marker between a call's kernels and the next
// launch on the device (profiles/r05j: 5.6 us between k_gram_dist and the guarded direct kernels,
// 14 us between calls).  Only a table COPY needs ordering after the slot's previous readers: a use
// that found its table already staged (the steady state of repeated rounds) records no event -- the
// slot's next use is predicted to hit too, and if it copies instead, it records the event then, at
// the end of the readers' stream -- while a use that copied records one at release(), so the next
// copy can overlap the calls in between.  The host waits only for a copy still reading the host
// buffer before rewriting it.  FA_SLOT_EVENT=1: an event per call and a host wait (A/B).
bool slot_event_mode() {
  static const int on = [] {
    const char* e = getenv("FA_SLOT_EVENT");
    return e && e[0] == '1' ? 1 : 0;
  }();
  return on != 0;
}

int acquire_slot(fa_ctx* ctx, size_t bytes, fa_ctx::Slot** out) {
  fa_ctx::Slot& s = ctx->slots[ctx->next];
  ctx->next = (ctx->next + 1) % kSlots;
  // a use that never reached release() (its caller failed after stage(), possibly after queueing
  // kernels that read `dev` on a stream the slot never recorded) leaves the device buffer's contents
  // and readers unknown: copy again next time, and only after every queued reader is done (a device
  // sync -- an error path, never taken by a call that succeeds)
  if (s.acquired) {
    s.shadow_ok = false;
    FA_HIP(hipDeviceSynchronize());
  }
  s.acquired = true;
  if (s.pending) {
    FA_HIP(hipEventSynchronize(s.ev));
    s.pending = false;
  }
  if (s.copy_live) {  // the host buffer is rewritten next: the last copy from it must have read it
    FA_HIP(hipEventSynchronize(s.staged));
    s.copy_live = false;
  }
  if (s.cap < bytes) {
    // the buffers are freed: every earlier reader of `dev` (any stream) must be done
    if (s.used) FA_HIP(hipDeviceSynchronize());
    size_t cap = align16(std::max(bytes, std::max<size_t>(2 * s.cap, 16384)));
    if (s.host) FA_HIP(hipHostFree(s.host));
    if (s.dev) FA_HIP(hipFree(s.dev));
    s.host = s.dev = nullptr;
    s.cap = 0;
    s.shadow_ok = false;
    s.used = false;
    // mapped: the staging copy is a kernel reading it over PCIe (stage())
    if (hipHostMalloc(&s.host, cap, hipHostMallocMapped) != hipSuccess)
      return fail(FA_ERR_NOMEM, "hipHostMalloc(%zu) failed", cap);
    if (hipHostGetDevicePointer(&s.hmap, s.host, 0) != hipSuccess) s.hmap = nullptr;
    if (hipMalloc(&s.dev, cap) != hipSuccess) return fail(FA_ERR_NOMEM, "hipMalloc(%zu) failed", cap);
    s.cap = cap;
  }
  *out = &s;
  return FA_OK;
}

namespace {
// descriptor tables host -> device: 16-byte units read from the mapped pinned slot
__global__ void __launch_bounds__(kBlock) k_stage_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int n16) {
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < n16; i += gridDim.x * kBlock) dst[i] = src[i];
}

bool stage_kernel_enabled() {
  static const int on = [] {
    const char* e = getenv("FA_STAGE_COPY");  // "0": hipMemcpyAsync (measurement A/B)
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on != 0;
}
}  // namespace

// A table of up to 256 KB goes by a copy kernel: hipMemcpyAsync from pinned memory ran as a separate
// copy whose completion the aggregation kernel then waited for (~30 us of GPU time per call at 3,904
// pointers, cfg2 through agg() on separate tensors).  The copy kernel runs on a per-device side
// stream and the caller's stream waits for it (an event), so back-to-back calls copy call n+1's table
// while call n's kernel is still running; the slot's device buffer is free (acquire_slot waited for
// its previous reader).  FA_STAGE_SIDE=0: the copy on the caller's stream (A/B).
namespace {
bool stage_side_enabled() {
  static const int on = [] {
    const char* e = getenv("FA_STAGE_SIDE");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on != 0;
}
hipStream_t side_stream() {
  static std::mutex m;
  static hipStream_t ss[64] = {};
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return nullptr;
  std::lock_guard<std::mutex> g(m);
  if (!ss[d] && hipStreamCreateWithFlags(&ss[d], hipStreamNonBlocking) != hipSuccess) ss[d] = nullptr;
  return ss[d];
}
}  // namespace

// r04: a state_dict round over the SAME client tensors as the slot's last use (the bench's steps, and
// rounds whose updates the caching allocator places at the same addresses) stages a byte-identical
// table; its copy and the cross-queue wait behind it cost ~14 us of GPU idle per call at cfg2's 3,904
// pointers (profiles/r04b: 19.8 us between k_wsum_pair kernels vs ~6 us without a staged table).
// FA_STAGE_REUSE=0: always copy (A/B).
namespace {
bool stage_reuse_enabled() {
  const char* e = getenv("FA_STAGE_REUSE");
  return !(e && e[0] == '0');
}
}  // namespace

int stage(fa_ctx::Slot* s, size_t bytes, hipStream_t st, bool reuse) {
  reuse = reuse && stage_reuse_enabled();
  if (!s->staged && hipEventCreateWithFlags(&s->staged, hipEventDisableTiming) != hipSuccess)
    return fail(FA_ERR_HIP, "hipEventCreate failed");
  if (reuse && s->shadow_ok && s->shadow.size() == bytes && memcmp(s->host, s->shadow.data(), bytes) == 0) {
    // the device buffer holds these bytes; while the copy that put them there may still be in
    // flight, the caller's stream waits for it (any stream: no bookkeeping of which streams did)
    const hipError_t q = hipEventQuery(s->staged);
    if (q == hipErrorNotReady) FA_HIP(hipStreamWaitEvent(st, s->staged, 0));
    else if (q != hipSuccess) FA_HIP(q);
    // readers on another stream: this stream's use is ordered after the slot's previous one, so the
    // readers of `dev` form one chain and a later copy, ordered after the last of them, is after all
    if (!slot_event_mode() && s->used && s->last != st) {
      if (!s->ev_live) FA_HIP(hipEventRecord(s->ev, s->last));
      FA_HIP(hipStreamWaitEvent(st, s->ev, 0));
    }
    s->hit = true;
    return FA_OK;
  }
  s->hit = false;
  // `dev` is about to be rewritten: the shadow is valid again only once the copy (and the caller
  // stream's wait for it) has been enqueued -- every failure below returns with it invalid
  s->shadow_ok = false;
  const bool evmode = slot_event_mode();
  if (s->hmap && bytes <= (256u << 10) && stage_kernel_enabled()) {
    const int n16 = (int)((bytes + 15) / 16);  // slots are >= 16 KB and 16-byte multiples
    const int blocks = std::max(1, std::min(64, (n16 + kBlock - 1) / kBlock));
    hipStream_t cs = st;
    if (stage_side_enabled()) {
      hipStream_t ss = side_stream();
      if (ss) cs = ss;
    }
    // the copy overwrites `dev`: after the slot's previous readers (stream order when they ran on
    // the copy's own stream; otherwise an event at their stream's current end)
    if (!evmode && s->used && s->last != cs) {
      if (!s->ev_live) FA_HIP(hipEventRecord(s->ev, s->last));
      FA_HIP(hipStreamWaitEvent(cs, s->ev, 0));
    }
    hipLaunchKernelGGL(k_stage_copy, dim3(blocks), dim3(kBlock), 0, cs, (const u32x4*)s->hmap, (u32x4*)s->dev, n16);
    FA_HIP(hipGetLastError());
    FA_HIP(hipEventRecord(s->staged, cs));
    if (cs != st) FA_HIP(hipStreamWaitEvent(st, s->staged, 0));
  } else {
    if (!evmode && s->used && s->last != st) {
      if (!s->ev_live) FA_HIP(hipEventRecord(s->ev, s->last));
      FA_HIP(hipStreamWaitEvent(st, s->ev, 0));
    }
    FA_HIP(hipMemcpyAsync(s->dev, s->host, bytes, hipMemcpyHostToDevice, st));
    FA_HIP(hipEventRecord(s->staged, st));
  }
  s->copy_live = true;
  if (reuse) {
    s->shadow.assign((const char*)s->host, (const char*)s->host + bytes);
    s->shadow_ok = true;
  }
  return FA_OK;
}

int release(fa_ctx::Slot* s, hipStream_t st) {
  const bool evmode = slot_event_mode();
  s->ev_live = false;
  if (evmode || !s->hit) {
    FA_HIP(hipEventRecord(s->ev, st));
    s->pending = evmode;
    s->ev_live = !evmode;
  }
  s->hit = false;
  s->last = st;
  s->used = true;
  s->acquired = false;
  return FA_OK;
}

}  // namespace fa_detail

// ============================================================================================ ABI
extern "C" {

int fa_abi_version(void) { return FA_ABI_VERSION; }

const char* fa_strerror(int code) {
  switch (code) {
    case FA_OK: return "FA_OK";
    case FA_ERR_INVALID: return "FA_ERR_INVALID";
    case FA_ERR_DTYPE: return "FA_ERR_DTYPE";
    case FA_ERR_HIP: return "FA_ERR_HIP";
    case FA_ERR_NOMEM: return "FA_ERR_NOMEM";
    case FA_ERR_COMM: return "FA_ERR_COMM";
    default: return "FA_ERR_UNKNOWN";
  }
}

const char* fa_last_error(void) { return fa_detail::last_error(); }

int fa_ctx_create(int hip_device, fa_ctx** out) {
  if (!out) return fail(FA_ERR_INVALID, "fa_ctx_create: out is NULL");
  *out = nullptr;
  int ndev = 0;
  FA_HIP(hipGetDeviceCount(&ndev));
  if (hip_device < 0 || hip_device >= ndev)
    return fail(FA_ERR_INVALID, "fa_ctx_create: device %d out of range [0,%d)", hip_device, ndev);
  DeviceGuard g(hip_device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", hip_device);
  fa_ctx* c = new (std::nothrow) fa_ctx();
  if (!c) return fail(FA_ERR_NOMEM, "fa_ctx_create: out of host memory");
  c->device = hip_device;
  for (auto& s : c->slots) {
    if (hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) {
      fa_ctx_destroy(c);
      return fail(FA_ERR_HIP, "hipEventCreate failed");
    }
  }
  *out = c;
  return FA_OK;
}

int fa_ctx_destroy(fa_ctx* c) {
  if (!c) return FA_OK;
  DeviceGuard g(c->device);
  bool used = false;
  for (auto& s : c->slots) used = used || s.used || s.copy_live;
  if (used) (void)hipDeviceSynchronize();  // the slots' last readers and copies, on any stream
  for (auto& s : c->slots) {
    if (s.pending && s.ev) (void)hipEventSynchronize(s.ev);
    if (s.ev) (void)hipEventDestroy(s.ev);
    if (s.staged) (void)hipEventDestroy(s.staged);
    if (s.host) (void)hipHostFree(s.host);
    if (s.dev) (void)hipFree(s.dev);
  }
  if (c->zc_ev) (void)hipEventDestroy(c->zc_ev);
  if (c->zc_host) (void)hipHostFree(c->zc_host);
  if (c->mt_live) (void)hipEventSynchronize(c->mt_ev);
  if (c->mt_ev) (void)hipEventDestroy(c->mt_ev);
  if (c->mt_dev) (void)hipFree(c->mt_dev);
  if (c->zc_counter) (void)hipFree(c->zc_counter);
  if (c->mt_poly_dev) (void)hipFree(c->mt_poly_dev);
  delete c;
  return FA_OK;
}

// Tuning knob (not part of the arithmetic contract): kernel variant for the weighted sum.
int fa_ctx_set_variant(fa_ctx* c, int variant) {
  if (!c || variant < 0 || variant >= kNumVariants)
    return fail(FA_ERR_INVALID, "fa_ctx_set_variant: variant must be in [0, %d)", kNumVariants);
  c->variant = variant;
  return FA_OK;
}

// Tuning knob (not part of the arithmetic contract): 0 disables the banded mixing kernel.
int fa_ctx_set_mix_band(fa_ctx* c, int enable) {
  if (!c) return fail(FA_ERR_INVALID, "fa_ctx_set_mix_band: ctx is NULL");
  c->mix_band = enable != 0;
  return FA_OK;
}

// A stream whose kernels run on `cu_count` of the device's CUs, spread evenly over the CU mask (so
// every XCD keeps a share).  The aggregation stream needs about half the CUs for the full HBM rate
// (tools/cumask_probe.py: 128-224 of 256 CUs stream 6.64-6.67 TB/s); on multi-GPU rounds the rest
// stay free for RCCL's kernels, so the collective of chunk c runs beside the partial of chunk c+1.
int fa_stream_create_cu_masked(int hip_device, int cu_count, void** out_stream) {
  if (!out_stream) return fail(FA_ERR_INVALID, "fa_stream_create_cu_masked: out_stream is NULL");
  *out_stream = nullptr;
  DeviceGuard g(hip_device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", hip_device);
  hipDeviceProp_t prop;
  FA_HIP(hipGetDeviceProperties(&prop, hip_device));
  const int total = prop.multiProcessorCount;
  if (cu_count <= 0 || cu_count > total)
    return fail(FA_ERR_INVALID, "cu_count must be in [1, %d] (got %d)", total, cu_count);
  const int words = (total + 31) / 32;
  uint32_t mask[64] = {0};
  if (words > 64) return fail(FA_ERR_INVALID, "device has too many CUs (%d)", total);
  for (int i = 0; i < total; ++i)
    if ((int64_t)i * cu_count / total != (int64_t)(i + 1) * cu_count / total) mask[i / 32] |= 1u << (i % 32);
  hipStream_t s = nullptr;
  FA_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask));
  *out_stream = (void*)s;
  return FA_OK;
}

int fa_stream_destroy(void* stream) {
  if (!stream) return FA_OK;
  FA_HIP(hipStreamDestroy((hipStream_t)stream));
  return FA_OK;
}

namespace {
// fa_weighted_sum_multi / fa_weighted_sum_tiled.  sstr = 0: flat inputs; otherwise (one segment)
// tile-interleaved inputs whose FA_TILE_BYTES slots are sstr bytes apart.
// FA_INLINE_DESC=0 forces the staged-table launches (A/B measurement)
bool inline_enabled() {
  static const int on = [] {
    const char* e = getenv("FA_INLINE_DESC");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on != 0;
}

int wsum_impl(fa_ctx* ctx, int dtype, int mode, int32_t num_segments, const int64_t* seg_numel, int32_t k,
              const void* const* d_in, const double* coef, double divisor, void* const* d_out,
              void* hip_stream, int64_t sstr) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (k <= 0) return fail(FA_ERR_INVALID, "k must be > 0 (got %d)", k);
  if (num_segments <= 0 || !seg_numel || !d_in || !d_out)
    return fail(FA_ERR_INVALID, "num_segments/seg_numel/d_in/d_out invalid");
  if (mode < FA_MODE_MUL_W || mode > FA_MODE_SUM) return fail(FA_ERR_DTYPE, "unknown mode %d", mode);
  const int V = elems_per_vec(dtype);
  if (V == 0) return fail(FA_ERR_DTYPE, "unknown dtype %d", dtype);
  if (mode != FA_MODE_SUM && !coef) return fail(FA_ERR_INVALID, "coef is NULL for a weighted mode");

  // count non-empty segments and tiles
  // variant 0 = automatic: few clients per launch (K <= 16, e.g. one GPU's share at N = 8) leave a
  // lane only 2 load groups, so two 16-byte vectors per lane (U = 8, S = 2, variant 5) keep more
  // bytes in flight: measured K = 16 x 125 M tiled 1.46 -> 1.37 ms; K >= 32 keeps (8, 1)
  const int variant = ctx->variant ? ctx->variant : (k <= 16 ? 5 : 0);
  const int64_t tile_elems = (int64_t)kBlock * V * kVariants[variant].S;
  int nseg = 0;
  int64_t tiles = 0;
  for (int s = 0; s < num_segments; ++s) {
    if (seg_numel[s] < 0) return fail(FA_ERR_INVALID, "segment %d has negative numel", s);
    if (seg_numel[s] == 0) continue;
    if (!d_out[s]) return fail(FA_ERR_INVALID, "segment %d: output is NULL", s);
    for (int i = 0; i < k; ++i)
      if (!d_in[(int64_t)s * k + i]) return fail(FA_ERR_INVALID, "segment %d client %d: input NULL", s, i);
    ++nseg;
    tiles += (seg_numel[s] + tile_elems - 1) / tile_elems;
  }
  if (nseg == 0) return FA_OK;
  if (tiles > 0x7FFFFFFFll) return fail(FA_ERR_INVALID, "too many tiles (%lld)", (long long)tiles);

  const size_t seg_bytes = align16(sizeof(Seg) * nseg);
  const size_t coef_bytes = align16(sizeof(double) * k);
  const size_t ptr_bytes = sizeof(void*) * (size_t)nseg * k;
  const size_t bytes = seg_bytes + coef_bytes + ptr_bytes;

  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  const bool inl = bytes <= (size_t)kInlineBytes && (variant == 0 || variant == 5) && inline_enabled();
  InlineDesc dsc;
  fa_ctx::Slot* slot = nullptr;
  int rc = FA_OK;
  if (!inl) {
    rc = acquire_slot(ctx, bytes, &slot);
    if (rc) return rc;
  }

  char* h = inl ? dsc.raw : (char*)slot->host;
  Seg* hs = (Seg*)h;
  double* hc = (double*)(h + seg_bytes);
  const void** hp = (const void**)(h + seg_bytes + coef_bytes);
  for (int i = 0; i < k; ++i) hc[i] = coef ? coef[i] : 0.0;
  int j = 0;
  int64_t t0 = 0;
  for (int s = 0; s < num_segments; ++s) {
    const int64_t n = seg_numel[s];
    if (n == 0) continue;
    bool aligned = al16(d_out[s]);
    for (int i = 0; i < k; ++i) {
      const void* p = d_in[(int64_t)s * k + i];
      hp[(int64_t)j * k + i] = p;
      aligned = aligned && al16(p);
    }
    if (sstr && !aligned) return fail(FA_ERR_INVALID, "tiled inputs and the output must be 16-byte aligned");
    hs[j] = Seg{n, t0, d_out[s], j * k, aligned ? 1 : 0};
    t0 += (n + tile_elems - 1) / tile_elems;
    ++j;
  }
  if (inl) {
    const int co = (int)seg_bytes, po = (int)(seg_bytes + coef_bytes);
    switch (dtype) {
      case FA_DTYPE_F32: dispatch_inl<FA_DTYPE_F32>(mode, variant, tiles, st, dsc, nseg, co, po, k, divisor, sstr); break;
      case FA_DTYPE_BF16: dispatch_inl<FA_DTYPE_BF16>(mode, variant, tiles, st, dsc, nseg, co, po, k, divisor, sstr); break;
      case FA_DTYPE_F16: dispatch_inl<FA_DTYPE_F16>(mode, variant, tiles, st, dsc, nseg, co, po, k, divisor, sstr); break;
      case FA_DTYPE_F64: dispatch_inl<FA_DTYPE_F64>(mode, variant, tiles, st, dsc, nseg, co, po, k, divisor, sstr); break;
      case FA_DTYPE_I64: dispatch_inl<FA_DTYPE_I64>(mode, variant, tiles, st, dsc, nseg, co, po, k, divisor, sstr); break;
    }
    FA_HIP(hipGetLastError());
    return FA_OK;
  }
  rc = stage(slot, bytes, st, true);
  if (rc) return rc;
  char* d = (char*)slot->dev;
  const Seg* ds = (const Seg*)d;
  const double* dc = (const double*)(d + seg_bytes);
  const void* const* dp = (const void* const*)(d + seg_bytes + coef_bytes);

  switch (dtype) {
    case FA_DTYPE_F32: rc = dispatch_mode<FA_DTYPE_F32>(mode, variant, tiles, st, ds, nseg, dc, dp, k, divisor, sstr); break;
    case FA_DTYPE_BF16: rc = dispatch_mode<FA_DTYPE_BF16>(mode, variant, tiles, st, ds, nseg, dc, dp, k, divisor, sstr); break;
    case FA_DTYPE_F16: rc = dispatch_mode<FA_DTYPE_F16>(mode, variant, tiles, st, ds, nseg, dc, dp, k, divisor, sstr); break;
    case FA_DTYPE_F64: rc = dispatch_mode<FA_DTYPE_F64>(mode, variant, tiles, st, ds, nseg, dc, dp, k, divisor, sstr); break;
    case FA_DTYPE_I64: rc = dispatch_mode<FA_DTYPE_I64>(mode, variant, tiles, st, ds, nseg, dc, dp, k, divisor, sstr); break;
  }
  if (rc) return rc;
  FA_HIP(hipGetLastError());
  return release(slot, st);
}
}  // namespace

extern "C++" {
namespace {
// A whole small round whose buffers sit in mapped host memory, on G <= kHost1MaxGroups workgroups
// (the flattened 16-byte vectors of every segment, Seg.tile_start = the segment's first vector; S
// vectors per thread and U clients per group with all their loads in flight before any is consumed:
// each group costs one PCIe round trip, and more CUs keep more reads in flight -- cfg1's round takes
// 25.7 / 17.9 / 14.6 / 13.7 / 15.0 us on 1 / 2 / 4 / 8 / 16 workgroups of 256 threads,
// profiles/r03n/doorbell_probe.json).  The ordered term/accum of wsum_tile; every thread's stores are
// made visible to the host, and the last workgroup to finish (a device-memory counter) stores `seq`
// into the completion word and resets the counter.
constexpr int kHost1Threads = 256, kHost1MaxGroups = 64;
template <int DT, int MODE>
__global__ void __launch_bounds__(kHost1Threads)
k_wsum_host1(const InlineDesc dsc, int nseg, int coef_off, int ptr_off, int k, double divisor, int64_t total_vec,
             unsigned long long* done, unsigned long long seq, unsigned* counter) {
  using T = Tr<DT, MODE>;
  using A = typename T::A;
  using R = typename T::R;
  constexpr int V = T::V, S = 2, U = 4;
  // the tables into LDS with one load per thread (lookups then cost no kernarg round trips)
  __shared__ u32x4 tab[kInlineBytes / 16];
  static_assert(kInlineBytes / 16 <= kHost1Threads, "one 16-byte load per thread");
  if (threadIdx.x < kInlineBytes / 16) tab[threadIdx.x] = ((const u32x4*)dsc.raw)[threadIdx.x];
  __syncthreads();
  const char* b = (const char*)tab;
  const Seg* segs = (const Seg*)b;
  const double* coef = (const double*)(b + coef_off);
  const void* const* ptrs = (const void* const*)(b + ptr_off);
  const typename T::D d = T::div(divisor);
  const int64_t nthr = (int64_t)gridDim.x * kHost1Threads, gt = (int64_t)blockIdx.x * kHost1Threads + threadIdx.x;
  for (int64_t base = 0; base < total_vec; base += nthr * S) {
    int64_t g[S];
    int si[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      g[s] = base + s * nthr + gt;
      si[s] = g[s] < total_vec ? find_seg(segs, nseg, g[s]) : -1;
    }
    A acc[S][V];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int v = 0; v < V; ++v) acc[s][v] = T::zero();
    for (int i0 = 0; i0 < k; i0 += U) {
      u32x4 r[S][U];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (si[s] < 0) continue;
        const Seg& sg = segs[si[s]];
        const int64_t boff = (g[s] - sg.tile_start) * 16;  // each client's slice is padded to 16 bytes
#pragma unroll
        for (int u = 0; u < U; ++u) r[s][u] = ld16<false>((const char*)ptrs[sg.ptr_base + min(i0 + u, k - 1)] + boff);
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (si[s] < 0) continue;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (i0 + u < k) {
            const typename T::C c = T::coef(coef[i0 + u]);
            R x[V];
            T::unpack(r[s][u], x);
#pragma unroll
            for (int v = 0; v < V; ++v) acc[s][v] = accum<DT, MODE>(acc[s][v], term<DT, MODE>(x[v], c, d));
          }
        }
      }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (si[s] < 0) continue;
      const Seg& sg = segs[si[s]];
      const int64_t e0 = (g[s] - sg.tile_start) * V;
      if (e0 + V <= sg.numel) {
        T::stv((char*)sg.out + e0 * T::OUT_BYTES, acc[s]);
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v)
          if (e0 + v < sg.numel) T::st1(sg.out, e0 + v, acc[s][v]);
      }
    }
  }
  __threadfence_system();  // this thread's result stores are visible to the host
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {  // the last workgroup: every other one's stores are visible
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <int DT>
void launch_host1(int mode, hipStream_t st, const InlineDesc& dsc, int nseg, int co, int po, int k, double divisor,
                  int64_t total_vec, unsigned long long* done, unsigned long long seq, unsigned* counter) {
  // one vector per thread up to kHost1MaxGroups workgroups
  const dim3 g((unsigned)std::min<int64_t>(kHost1MaxGroups, std::max<int64_t>(1, (total_vec + kHost1Threads - 1) / kHost1Threads)));
  const dim3 b(kHost1Threads);
  switch (mode) {
    case FA_MODE_MUL_W: hipLaunchKernelGGL((k_wsum_host1<DT, FA_MODE_MUL_W>), g, b, 0, st, dsc, nseg, co, po, k, divisor, total_vec, done, seq, counter); break;
    case FA_MODE_MUL_N_DIV_N: hipLaunchKernelGGL((k_wsum_host1<DT, FA_MODE_MUL_N_DIV_N>), g, b, 0, st, dsc, nseg, co, po, k, divisor, total_vec, done, seq, counter); break;
    default: hipLaunchKernelGGL((k_wsum_host1<DT, FA_MODE_SUM>), g, b, 0, st, dsc, nseg, co, po, k, divisor, total_vec, done, seq, counter); break;
  }
}

bool host1_enabled() {  // FA_HOST1=0: every host round through the device path's kernel + event (A/B)
  static const int on = [] {
    const char* e = getenv("FA_HOST1");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on != 0;
}
constexpr size_t kHost1MaxBytes = 1 << 20;  // input bytes up to which one workgroup serves the round
constexpr size_t kZcHeader = 256;           // completion word at the start of the mapped buffer
}  // namespace
}  // extern "C++"

int fa_weighted_sum_multi(fa_ctx* ctx, int dtype, int mode, int32_t num_segments,
                          const int64_t* seg_numel, int32_t k, const void* const* d_in,
                          const double* coef, double divisor, void* const* d_out, void* hip_stream) {
  return wsum_impl(ctx, dtype, mode, num_segments, seg_numel, k, d_in, coef, divisor, d_out, hip_stream, 0);
}

// Small host-resident rounds (the reference's quick_start: LR-MNIST, K = 2, 63 KB per client): the
// launch/copy latencies dominate, so the inputs are packed into ONE mapped pinned buffer and the
// kernel reads them -- and writes the result -- in place over PCIe (no H2D / D2H copies, one launch).
// Rounds whose tables fit the kernel argument and whose inputs are <= kHost1MaxBytes run in ONE
// workgroup (k_wsum_host1) that ends by storing a sequence number into the mapped buffer; the host
// spins on that word instead of an event wait (tools/doorbell_probe.hip on MI355X: launch + event
// 27.2 us, launch + completion word 22.2 us, a resident polling workgroup 18.6 us for cfg1's round).
// Larger rounds: the device path's kernel + one event wait.  Same per-element arithmetic either way.
int fa_weighted_sum_host(fa_ctx* ctx, int dtype, int mode, int32_t num_segments, const int64_t* seg_numel,
                         int32_t k, const void* const* h_in, const double* coef, double divisor, void* const* h_out,
                         void* hip_stream) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (k <= 0 || num_segments <= 0 || !seg_numel || !h_in || !h_out)
    return fail(FA_ERR_INVALID, "fa_weighted_sum_host: invalid arguments");
  const int V = elems_per_vec(dtype);
  if (V == 0) return fail(FA_ERR_DTYPE, "unknown dtype %d", dtype);
  if (num_segments > 4096 || k > 4096) return fail(FA_ERR_INVALID, "fa_weighted_sum_host: too many segments/clients");
  const size_t in_es = dtype == FA_DTYPE_F32 ? 4 : (dtype == FA_DTYPE_BF16 || dtype == FA_DTYPE_F16) ? 2 : 8;
  const size_t out_es = (dtype == FA_DTYPE_I64 && mode != FA_MODE_SUM) ? 4 : in_es;
  size_t total = 0;
  for (int s = 0; s < num_segments; ++s) {
    if (seg_numel[s] < 0) return fail(FA_ERR_INVALID, "segment %d has negative numel", s);
    total += (size_t)k * align16((size_t)seg_numel[s] * in_es) + align16((size_t)seg_numel[s] * out_es);
  }
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  if (!ctx->zc_ev) FA_HIP(hipEventCreateWithFlags(&ctx->zc_ev, hipEventDisableTiming));
  if (ctx->zc_cap < total + kZcHeader) {
    if (ctx->zc_host) FA_HIP(hipHostFree(ctx->zc_host));
    ctx->zc_host = ctx->zc_dev = nullptr;
    ctx->zc_cap = 0;
    const size_t cap = std::max<size_t>(total + kZcHeader, 1 << 20);
    // coherent: the device's reads and its completion word go straight over PCIe, no GPU caching
    if (hipHostMalloc(&ctx->zc_host, cap, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return fail(FA_ERR_NOMEM, "hipHostMalloc(%zu, mapped) failed", cap);
    FA_HIP(hipHostGetDevicePointer(&ctx->zc_dev, ctx->zc_host, 0));
    ctx->zc_cap = cap;
    memset(ctx->zc_host, 0, kZcHeader);
    ctx->zc_seq = 0;
  }
  if (!ctx->zc_counter) {  // the host1 kernel's workgroup counter (device memory, reset by its last user)
    if (hipMalloc((void**)&ctx->zc_counter, 256) != hipSuccess) return fail(FA_ERR_NOMEM, "hipMalloc(256) failed");
    FA_HIP(hipMemset(ctx->zc_counter, 0, 256));
  }
  std::vector<const void*> din((size_t)num_segments * k);
  std::vector<void*> dout(num_segments);
  size_t off = kZcHeader;
  char* hb = (char*)ctx->zc_host;
  char* db = (char*)ctx->zc_dev;
  for (int s = 0; s < num_segments; ++s) {
    const size_t nb = (size_t)seg_numel[s] * in_es;
    for (int i = 0; i < k; ++i) {
      const void* src = h_in[(size_t)s * k + i];
      if (!src && nb) return fail(FA_ERR_INVALID, "segment %d client %d: input NULL", s, i);
      if (nb) memcpy(hb + off, src, nb);
      din[(size_t)s * k + i] = db + off;
      off += align16(nb);
    }
    dout[s] = db + off;
    off += align16((size_t)seg_numel[s] * out_es);
  }
  // one workgroup + completion word when the tables fit the kernel argument and the round is small
  int nseg = 0;
  int64_t total_vec = 0;
  for (int s = 0; s < num_segments; ++s)
    if (seg_numel[s] > 0) ++nseg, total_vec += (seg_numel[s] + V - 1) / V;
  const size_t seg_b = align16(sizeof(Seg) * nseg), coef_b = align16(sizeof(double) * k);
  const size_t desc_b = seg_b + coef_b + sizeof(void*) * (size_t)nseg * k;
  if (host1_enabled() && nseg > 0 && desc_b <= (size_t)kInlineBytes && total <= kHost1MaxBytes) {
    InlineDesc dsc;
    Seg* hs = (Seg*)dsc.raw;
    double* hc = (double*)(dsc.raw + seg_b);
    const void** hp = (const void**)(dsc.raw + seg_b + coef_b);
    for (int i = 0; i < k; ++i) hc[i] = coef ? coef[i] : 0.0;
    int j = 0;
    int64_t v0 = 0;
    for (int s = 0; s < num_segments; ++s) {
      if (seg_numel[s] <= 0) continue;
      for (int i = 0; i < k; ++i) hp[(size_t)j * k + i] = din[(size_t)s * k + i];
      hs[j] = Seg{seg_numel[s], v0, dout[s], j * k, 1};
      v0 += (seg_numel[s] + V - 1) / V;
      ++j;
    }
    const unsigned long long seq = ++ctx->zc_seq;
    unsigned long long* done_d = (unsigned long long*)ctx->zc_dev;
    volatile unsigned long long* done_h = (volatile unsigned long long*)ctx->zc_host;
    hipStream_t st = (hipStream_t)hip_stream;
    const int co = (int)seg_b, po = (int)(seg_b + coef_b);
    switch (dtype) {
      case FA_DTYPE_F32: launch_host1<FA_DTYPE_F32>(mode, st, dsc, nseg, co, po, k, divisor, total_vec, done_d, seq, ctx->zc_counter); break;
      case FA_DTYPE_BF16: launch_host1<FA_DTYPE_BF16>(mode, st, dsc, nseg, co, po, k, divisor, total_vec, done_d, seq, ctx->zc_counter); break;
      case FA_DTYPE_F16: launch_host1<FA_DTYPE_F16>(mode, st, dsc, nseg, co, po, k, divisor, total_vec, done_d, seq, ctx->zc_counter); break;
      case FA_DTYPE_F64: launch_host1<FA_DTYPE_F64>(mode, st, dsc, nseg, co, po, k, divisor, total_vec, done_d, seq, ctx->zc_counter); break;
      default: launch_host1<FA_DTYPE_I64>(mode, st, dsc, nseg, co, po, k, divisor, total_vec, done_d, seq, ctx->zc_counter); break;
    }
    FA_HIP(hipGetLastError());
    // spin on the completion word; after 1 s fall back to a stream sync, which reports a fault
    const auto t0 = std::chrono::steady_clock::now();
    unsigned spins = 0;
    while (*done_h != seq) {
      if ((++spins & 1023u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
        FA_HIP(hipStreamSynchronize(st));
        if (*done_h != seq) {  // reset the workgroup counter so that the next round starts clean
          (void)hipMemset(ctx->zc_counter, 0, 256);
          return fail(FA_ERR_HIP, "fa_weighted_sum_host: the round finished without its completion word");
        }
        break;
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  } else {
    int rc = wsum_impl(ctx, dtype, mode, num_segments, seg_numel, k, din.data(), coef, divisor, dout.data(),
                       hip_stream, 0);
    if (rc) return rc;
    FA_HIP(hipEventRecord(ctx->zc_ev, (hipStream_t)hip_stream));
    FA_HIP(hipEventSynchronize(ctx->zc_ev));
  }
  for (int s = 0; s < num_segments; ++s) {
    const size_t nb = (size_t)seg_numel[s] * out_es;
    if (nb) {
      if (!h_out[s]) return fail(FA_ERR_INVALID, "segment %d: output NULL", s);
      memcpy(h_out[s], hb + ((char*)dout[s] - db), nb);
    }
  }
  return FA_OK;
}

int fa_weighted_sum(fa_ctx* ctx, int dtype, int mode, int64_t n, int32_t k, const void* const* d_in,
                    const double* coef, double divisor, void* d_out, void* hip_stream) {
  if (n < 0) return fail(FA_ERR_INVALID, "n must be >= 0");
  void* outs[1] = {d_out};
  return wsum_impl(ctx, dtype, mode, 1, &n, k, d_in, coef, divisor, outs, hip_stream, 0);
}

int fa_weighted_sum_tiled(fa_ctx* ctx, int dtype, int mode, int64_t n, int32_t k, const void* const* d_in,
                          int64_t tile_stride, const double* coef, double divisor, void* d_out,
                          void* hip_stream) {
  if (n < 0) return fail(FA_ERR_INVALID, "n must be >= 0");
  if (tile_stride <= 0 || tile_stride % FA_TILE_BYTES)
    return fail(FA_ERR_INVALID, "tile_stride must be a positive multiple of %d (got %lld)", FA_TILE_BYTES,
                (long long)tile_stride);
  void* outs[1] = {d_out};
  return wsum_impl(ctx, dtype, mode, 1, &n, k, d_in, coef, divisor, outs, hip_stream, tile_stride);
}

extern "C++" {
namespace {
// Tables of a pair launch: Seg0[nseg0] | Seg1[nseg1] | coef[k] | ptrs0[nseg0*k] | ptrs1[nseg1*k]
struct PairTables { int seg1, coef, ptr0, ptr1; size_t bytes; };

struct PairArgs {
  int nseg0, nseg1;
  int64_t sstr0, sstr1, tiles1;
  int k;
  double divisor;
};

template <int DT, int MODE, int S>
void launch_pair(int64_t tiles, hipStream_t st, const char* dev, const InlineDesc* dsc, const PairTables& L,
                 const PairArgs& a) {
  if (dsc)
    hipLaunchKernelGGL((k_wsum_pair_inl<DT, MODE, 8, S, false>), dim3((unsigned)tiles), dim3(kBlock), 0, st, *dsc,
                       a.nseg0, a.nseg1, L.seg1, L.coef, L.ptr0, L.ptr1, a.sstr0, a.sstr1, a.tiles1, a.k, a.divisor);
  else
    hipLaunchKernelGGL((k_wsum_pair<DT, MODE, 8, S, false>), dim3((unsigned)tiles), dim3(kBlock), 0, st,
                       (const Seg*)dev, a.nseg0, (const void* const*)(dev + L.ptr0), a.sstr0,
                       (const Seg*)(dev + L.seg1), a.nseg1, (const void* const*)(dev + L.ptr1), a.sstr1, a.tiles1,
                       (const double*)(dev + L.coef), a.k, a.divisor, xcd_map_enabled() && a.nseg0 > 1 ? 1 : 0);
}

template <int DT>
void pair_modes(int mode, bool k16, bool s4, int64_t tiles, hipStream_t st, const char* dev, const InlineDesc* dsc,
                const PairTables& L, const PairArgs& a) {
#define FA_PM(MODE) (s4 ? launch_pair<DT, MODE, 4>(tiles, st, dev, dsc, L, a) : k16 ? launch_pair<DT, MODE, 2>(tiles, st, dev, dsc, L, a) \
                         : launch_pair<DT, MODE, 1>(tiles, st, dev, dsc, L, a))
  switch (mode) {
    case FA_MODE_MUL_W: FA_PM(FA_MODE_MUL_W); break;
    case FA_MODE_MUL_N_DIV_N: FA_PM(FA_MODE_MUL_N_DIV_N); break;
    default: FA_PM(FA_MODE_SUM); break;
  }
#undef FA_PM
}

// A float dtype group (nseg0 segments) and the int64 group (nseg1 segments) of the same k clients in
// one launch; the int64 tiles first.  sstr = 0: one flat vector per segment and client, else the
// tiled-arena stride.
int pair_impl(fa_ctx* ctx, int dtype, int mode, int32_t nseg0, const int64_t* numel0, int32_t nseg1,
              const int64_t* numel1, int32_t k, const void* const* d_in0, const void* const* d_in1, int64_t sstr0,
              int64_t sstr1, const double* coef, double divisor, void* const* d_out0, void* const* d_out1,
              void* hip_stream) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (k <= 0) return fail(FA_ERR_INVALID, "k must be > 0 (got %d)", k);
  if (nseg0 < 0 || nseg1 < 0 || (nseg0 && (!numel0 || !d_in0 || !d_out0)) || (nseg1 && (!numel1 || !d_in1 || !d_out1)))
    return fail(FA_ERR_INVALID, "fa_weighted_sum_pair: NULL table");
  if (dtype != FA_DTYPE_F32 && dtype != FA_DTYPE_BF16 && dtype != FA_DTYPE_F16 && dtype != FA_DTYPE_F64)
    return fail(FA_ERR_DTYPE, "fa_weighted_sum_pair: dtype %d not supported (F32, BF16, F16, F64)", dtype);
  if (mode < FA_MODE_MUL_W || mode > FA_MODE_SUM) return fail(FA_ERR_DTYPE, "unknown mode %d", mode);
  if (mode != FA_MODE_SUM && !coef) return fail(FA_ERR_INVALID, "coef is NULL for a weighted mode");
  const int64_t strides[2] = {sstr0, sstr1};
  for (int g = 0; g < 2; ++g)
    if (strides[g] < 0 || strides[g] % FA_TILE_BYTES)
      return fail(FA_ERR_INVALID, "tile_stride must be 0 (row-major) or a positive multiple of %d (got %lld)",
                  FA_TILE_BYTES, (long long)strides[g]);
  // two 4-KiB slots per client and workgroup up to K = 16 (FA_PAIR_S=2 forces them for any K: A/B)
  static const bool s2 = [] {
    const char* e = getenv("FA_PAIR_S");
    return e && e[0] == '2';
  }();
  // FA_PAIR_S=4: four slots per client and workgroup (A/B: fewer address-translation misses per byte
  // on separately allocated tensors, profiles/r05c)
  // Default: four slots when the float group is flat (separate tensors / client-major rows, sstr0 = 0)
  // and K >= 32 -- r05f, cfg2 on 3,904 separate tensors, 3 interleaved pairs: 0.2776-0.2813 ->
  // 0.2727-0.2777 ms/step; the tiled arena keeps one slot (FA_PAIR_S=1 forces one slot everywhere)
  static const int s_env = [] {
    const char* e = getenv("FA_PAIR_S");
    return e ? atoi(e) : 0;
  }();
  const bool s4 = s_env == 4 || (s_env == 0 && sstr0 == 0 && k >= 32);
  const bool k16 = !s4 && s_env != 1 && (k <= 16 || s2);  // FA_PAIR_S=1: one slot for every K
  const int nsg[2] = {nseg0, nseg1};
  const int64_t* numel[2] = {numel0, numel1};
  const void* const* din[2] = {d_in0, d_in1};
  void* const* dout[2] = {d_out0, d_out1};
  const int64_t te[2] = {(int64_t)kBlock * elems_per_vec(dtype) * (s4 ? 4 : k16 ? 2 : 1),
                         (int64_t)kBlock * elems_per_vec(FA_DTYPE_I64)};
  int live[2] = {0, 0};
  int64_t tiles[2] = {0, 0};
  for (int g = 0; g < 2; ++g)
    for (int s = 0; s < nsg[g]; ++s) {
      if (numel[g][s] < 0) return fail(FA_ERR_INVALID, "group %d segment %d has negative numel", g, s);
      if (numel[g][s] == 0) continue;
      if (!dout[g][s]) return fail(FA_ERR_INVALID, "group %d segment %d: output is NULL", g, s);
      for (int i = 0; i < k; ++i)
        if (!din[g][(int64_t)s * k + i]) return fail(FA_ERR_INVALID, "group %d segment %d client %d: input NULL", g, s, i);
      ++live[g];
      tiles[g] += (numel[g][s] + te[g] - 1) / te[g];
    }
  if (live[0] == 0 || live[1] == 0) {  // one group: the ordinary launch
    if (live[0]) return wsum_impl(ctx, dtype, mode, nseg0, numel0, k, d_in0, coef, divisor, d_out0, hip_stream, sstr0);
    if (live[1]) return wsum_impl(ctx, FA_DTYPE_I64, mode, nseg1, numel1, k, d_in1, coef, divisor, d_out1, hip_stream, sstr1);
    return FA_OK;
  }
  if (tiles[0] + tiles[1] > 0x7FFFFFFFll) return fail(FA_ERR_INVALID, "too many tiles");
  PairTables L;
  L.seg1 = (int)(sizeof(Seg) * live[0]);
  L.coef = (int)align16(sizeof(Seg) * (live[0] + live[1]));
  L.ptr0 = L.coef + (int)align16(sizeof(double) * k);
  L.ptr1 = L.ptr0 + (int)(sizeof(void*) * live[0] * k);
  L.bytes = (size_t)L.ptr1 + sizeof(void*) * live[1] * (size_t)k;
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  const bool inl = L.bytes <= (size_t)kInlineBytes && inline_enabled();
  InlineDesc dsc;
  fa_ctx::Slot* slot = nullptr;
  int rc = FA_OK;
  if (!inl) {
    rc = acquire_slot(ctx, L.bytes, &slot);
    if (rc) return rc;
  }
  char* h = inl ? dsc.raw : (char*)slot->host;
  double* hc = (double*)(h + L.coef);
  for (int i = 0; i < k; ++i) hc[i] = coef ? coef[i] : 0.0;
  for (int g = 0; g < 2; ++g) {
    Seg* hs = (Seg*)(h + (g ? L.seg1 : 0));
    const void** hp = (const void**)(h + (g ? L.ptr1 : L.ptr0));
    int j = 0;
    int64_t t0 = 0;
    for (int s = 0; s < nsg[g]; ++s) {
      const int64_t n = numel[g][s];
      if (n == 0) continue;
      bool aligned = al16(dout[g][s]);
      for (int i = 0; i < k; ++i) {
        const void* q = din[g][(int64_t)s * k + i];
        hp[(int64_t)j * k + i] = q;
        aligned = aligned && al16(q);
      }
      if (strides[g] && !aligned) return fail(FA_ERR_INVALID, "tiled inputs and the output must be 16-byte aligned");
      hs[j] = Seg{n, t0, dout[g][s], j * k, aligned ? 1 : 0};
      t0 += (n + te[g] - 1) / te[g];
      ++j;
    }
  }
  const char* dev = nullptr;
  if (!inl) {
    rc = stage(slot, L.bytes, st, true);
    if (rc) return rc;
    dev = (const char*)slot->dev;
  }
  const PairArgs a{live[0], live[1], sstr0, sstr1, tiles[1], k, divisor};
  const int64_t total = tiles[0] + tiles[1];
  const InlineDesc* dp = inl ? &dsc : nullptr;
  switch (dtype) {
    case FA_DTYPE_F32: pair_modes<FA_DTYPE_F32>(mode, k16, s4, total, st, dev, dp, L, a); break;
    case FA_DTYPE_BF16: pair_modes<FA_DTYPE_BF16>(mode, k16, s4, total, st, dev, dp, L, a); break;
    case FA_DTYPE_F16: pair_modes<FA_DTYPE_F16>(mode, k16, s4, total, st, dev, dp, L, a); break;
    case FA_DTYPE_F64: pair_modes<FA_DTYPE_F64>(mode, k16, s4, total, st, dev, dp, L, a); break;
  }
  FA_HIP(hipGetLastError());
  return inl ? FA_OK : release(slot, st);
}
}  // namespace
}  // extern "C++"

int fa_weighted_sum_pair(fa_ctx* ctx, int dtype, int mode, int64_t n, int64_t n_i64, int32_t k,
                         const void* const* d_in, const void* const* d_in_i64, int64_t tile_stride,
                         int64_t tile_stride_i64, const double* coef, double divisor, void* d_out,
                         void* d_out_i64, void* hip_stream) {
  if (n < 0 || n_i64 < 0) return fail(FA_ERR_INVALID, "n must be >= 0");
  void* o0[1] = {d_out};
  void* o1[1] = {d_out_i64};
  return pair_impl(ctx, dtype, mode, 1, &n, 1, &n_i64, k, d_in, d_in_i64, tile_stride, tile_stride_i64, coef,
                   divisor, d_out ? o0 : nullptr, d_out_i64 ? o1 : nullptr, hip_stream);
}

int fa_weighted_sum_pair_multi(fa_ctx* ctx, int dtype, int mode, int32_t num_segments, const int64_t* seg_numel,
                               int32_t num_segments_i64, const int64_t* seg_numel_i64, int32_t k,
                               const void* const* d_in, const void* const* d_in_i64, const double* coef,
                               double divisor, void* const* d_out, void* const* d_out_i64, void* hip_stream) {
  return pair_impl(ctx, dtype, mode, num_segments, seg_numel, num_segments_i64, seg_numel_i64, k, d_in, d_in_i64, 0,
                   0, coef, divisor, d_out, d_out_i64, hip_stream);
}

namespace {
int grouped_impl(fa_ctx* ctx, int dtype, int mode, int64_t n, int32_t k, const void* const* d_in,
                 const double* coef, double divisor, int32_t num_groups, const int32_t* group_ptr,
                 int group_mode, const double* group_coef, const double* group_divisor,
                 void* d_out, void* hip_stream, int64_t sstr) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (k <= 0 || n < 0 || !d_in || !d_out || num_groups <= 0 || !group_ptr)
    return fail(FA_ERR_INVALID, "fa_weighted_sum_grouped: invalid arguments");
  if (dtype != FA_DTYPE_F32 && dtype != FA_DTYPE_BF16 && dtype != FA_DTYPE_F16 && dtype != FA_DTYPE_F64)
    return fail(FA_ERR_DTYPE, "fa_weighted_sum_grouped: dtype %d not supported (F32, BF16, F16, F64)", dtype);
  if (mode < FA_MODE_MUL_W || mode > FA_MODE_SUM || group_mode < FA_MODE_MUL_W || group_mode > FA_MODE_SUM)
    return fail(FA_ERR_DTYPE, "fa_weighted_sum_grouped: unknown mode");
  if (mode != FA_MODE_SUM && !coef) return fail(FA_ERR_INVALID, "coef is NULL for a weighted mode");
  if (group_mode != FA_MODE_SUM && !group_coef) return fail(FA_ERR_INVALID, "group_coef is NULL");
  if (group_mode == FA_MODE_MUL_N_DIV_N && !group_divisor) return fail(FA_ERR_INVALID, "group_divisor is NULL");
  if (group_ptr[0] != 0 || group_ptr[num_groups] != k)
    return fail(FA_ERR_INVALID, "group_ptr must start at 0 and end at k");
  for (int g = 0; g < num_groups; ++g)
    if (group_ptr[g + 1] <= group_ptr[g]) return fail(FA_ERR_INVALID, "group %d is empty", g);
  bool aligned = al16(d_out);
  for (int i = 0; i < k; ++i) {
    if (!d_in[i]) return fail(FA_ERR_INVALID, "client %d: input NULL", i);
    aligned = aligned && al16(d_in[i]);
  }
  if (n == 0) return FA_OK;
  if (sstr && !aligned) return fail(FA_ERR_INVALID, "tiled inputs and the output must be 16-byte aligned");
  const int64_t tile_elems = (int64_t)kBlock * elems_per_vec(dtype);
  const int64_t tiles = (n + tile_elems - 1) / tile_elems;
  if (tiles > 0x7FFFFFFFll) return fail(FA_ERR_INVALID, "too many tiles");
  const size_t seg_bytes = align16(sizeof(Seg));
  const size_t coef_bytes = align16(sizeof(double) * k);
  const size_t grp_bytes = sizeof(GroupDesc) * num_groups;
  const size_t ptr_bytes = sizeof(void*) * k;
  const size_t bytes = seg_bytes + coef_bytes + grp_bytes + ptr_bytes;
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  fa_ctx::Slot* slot = nullptr;
  int rc = acquire_slot(ctx, bytes, &slot);
  if (rc) return rc;
  char* h = (char*)slot->host;
  *(Seg*)h = Seg{n, 0, d_out, 0, aligned ? 1 : 0};
  double* hc = (double*)(h + seg_bytes);
  for (int i = 0; i < k; ++i) hc[i] = coef ? coef[i] : 0.0;
  GroupDesc* hg = (GroupDesc*)(h + seg_bytes + coef_bytes);
  for (int gi = 0; gi < num_groups; ++gi)
    hg[gi] = GroupDesc{group_ptr[gi], group_ptr[gi + 1], group_coef ? group_coef[gi] : 1.0,
                       group_divisor ? group_divisor[gi] : 1.0, 0};
  memcpy(h + seg_bytes + coef_bytes + grp_bytes, d_in, ptr_bytes);
  rc = stage(slot, bytes, st);
  if (rc) return rc;
  char* dv = (char*)slot->dev;
  const Seg* ds = (const Seg*)dv;
  const double* dc = (const double*)(dv + seg_bytes);
  const GroupDesc* dg = (const GroupDesc*)(dv + seg_bytes + coef_bytes);
  const void* const* dp = (const void* const*)(dv + seg_bytes + coef_bytes + grp_bytes);
  const dim3 grid((unsigned)tiles), blk(kBlock);
#define FA_G(DT, MODE) \
  hipLaunchKernelGGL((k_wsum_grouped<DT, MODE, 8, true>), grid, blk, 0, st, ds, dc, dp, divisor, dg, num_groups, group_mode, sstr)
#define FA_G_MODES(DT)                                   \
  switch (mode) {                                        \
    case FA_MODE_MUL_W: FA_G(DT, FA_MODE_MUL_W); break;  \
    case FA_MODE_MUL_N_DIV_N: FA_G(DT, FA_MODE_MUL_N_DIV_N); break; \
    default: FA_G(DT, FA_MODE_SUM); break;               \
  }
  switch (dtype) {
    case FA_DTYPE_F32: FA_G_MODES(FA_DTYPE_F32); break;
    case FA_DTYPE_BF16: FA_G_MODES(FA_DTYPE_BF16); break;
    case FA_DTYPE_F16: FA_G_MODES(FA_DTYPE_F16); break;
    case FA_DTYPE_F64: FA_G_MODES(FA_DTYPE_F64); break;
  }
#undef FA_G_MODES
#undef FA_G
  FA_HIP(hipGetLastError());
  return release(slot, st);
}
}  // namespace

int fa_weighted_sum_tiled_multi(fa_ctx* ctx, int dtype, int mode, int32_t num_segments, const int64_t* seg_numel,
                                int32_t k, const void* const* d_in, int64_t tile_stride, const double* coef,
                                double divisor, void* const* d_out, void* hip_stream) {
  if (tile_stride <= 0 || tile_stride % FA_TILE_BYTES)
    return fail(FA_ERR_INVALID, "tile_stride must be a positive multiple of %d (got %lld)", FA_TILE_BYTES,
                (long long)tile_stride);
  return wsum_impl(ctx, dtype, mode, num_segments, seg_numel, k, d_in, coef, divisor, d_out, hip_stream, tile_stride);
}

int fa_weighted_sum_grouped(fa_ctx* ctx, int dtype, int mode, int64_t n, int32_t k, const void* const* d_in,
                            const double* coef, double divisor, int32_t num_groups, const int32_t* group_ptr,
                            int group_mode, const double* group_coef, const double* group_divisor,
                            void* d_out, void* hip_stream) {
  return grouped_impl(ctx, dtype, mode, n, k, d_in, coef, divisor, num_groups, group_ptr, group_mode, group_coef,
                      group_divisor, d_out, hip_stream, 0);
}

int fa_weighted_sum_grouped_tiled(fa_ctx* ctx, int dtype, int mode, int64_t n, int32_t k, const void* const* d_in,
                                  int64_t tile_stride, const double* coef, double divisor, int32_t num_groups,
                                  const int32_t* group_ptr, int group_mode, const double* group_coef,
                                  const double* group_divisor, void* d_out, void* hip_stream) {
  if (tile_stride <= 0 || tile_stride % FA_TILE_BYTES)
    return fail(FA_ERR_INVALID, "tile_stride must be a positive multiple of %d (got %lld)", FA_TILE_BYTES,
                (long long)tile_stride);
  return grouped_impl(ctx, dtype, mode, n, k, d_in, coef, divisor, num_groups, group_ptr, group_mode, group_coef,
                      group_divisor, d_out, hip_stream, tile_stride);
}

namespace {
int fedavg_sgd_impl(fa_ctx* ctx, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                    const void* const* d_in, const double* coef, void* const* d_param, void* const* d_momentum,
                    double lr, double momentum, double dampening, double weight_decay, int nesterov,
                    int first_step, void* hip_stream, int64_t sstr, int opt = 0,
                    void* const* d_square_avg = nullptr, double alpha = 0.0, double eps = 0.0) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (opt == 1 && !d_square_avg) return fail(FA_ERR_INVALID, "fa_fedavg_rmsprop: square_avg buffers are NULL");
  if (k <= 0 || num_segments <= 0 || !seg_numel || !d_in || !coef || !d_param)
    return fail(FA_ERR_INVALID, "fa_fedavg_sgd: invalid arguments");
  if (momentum != 0.0 && !d_momentum) return fail(FA_ERR_INVALID, "fa_fedavg_sgd: momentum buffers are NULL");
  if (nesterov && (momentum <= 0.0 || dampening != 0.0))
    return fail(FA_ERR_INVALID, "fa_fedavg_sgd: nesterov needs momentum > 0 and dampening 0 (torch.optim.SGD)");
  const int64_t tile_elems = (int64_t)kBlock * 4;
  int nseg = 0;
  int64_t tiles = 0;
  for (int s = 0; s < num_segments; ++s) {
    if (seg_numel[s] < 0) return fail(FA_ERR_INVALID, "segment %d has negative numel", s);
    if (seg_numel[s] == 0) continue;
    if (!d_param[s] || (momentum != 0.0 && !d_momentum[s])) return fail(FA_ERR_INVALID, "segment %d: NULL", s);
    for (int i = 0; i < k; ++i)
      if (!d_in[(int64_t)s * k + i]) return fail(FA_ERR_INVALID, "segment %d client %d: input NULL", s, i);
    ++nseg;
    tiles += (seg_numel[s] + tile_elems - 1) / tile_elems;
  }
  if (nseg == 0) return FA_OK;
  if (tiles > 0x7FFFFFFFll) return fail(FA_ERR_INVALID, "too many tiles");
  const size_t seg_bytes = align16(sizeof(Seg) * nseg);
  const size_t coef_bytes = align16(sizeof(double) * k);
  const size_t buf_bytes = align16(sizeof(void*) * nseg);
  const size_t ptr_bytes = sizeof(void*) * (size_t)nseg * k;
  const size_t bytes = seg_bytes + coef_bytes + 2 * buf_bytes + ptr_bytes;
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  const bool inl = bytes <= (size_t)kInlineBytes && inline_enabled();
  InlineDesc dsc;
  fa_ctx::Slot* slot = nullptr;
  int rc = FA_OK;
  if (!inl) {
    rc = acquire_slot(ctx, bytes, &slot);
    if (rc) return rc;
  }
  char* h = inl ? dsc.raw : (char*)slot->host;
  Seg* hs = (Seg*)h;
  double* hc = (double*)(h + seg_bytes);
  void** hb = (void**)(h + seg_bytes + coef_bytes);
  void** hq = (void**)(h + seg_bytes + coef_bytes + buf_bytes);
  const void** hp = (const void**)(h + seg_bytes + coef_bytes + 2 * buf_bytes);
  for (int i = 0; i < k; ++i) hc[i] = coef[i];
  int j = 0;
  int64_t t0 = 0;
  for (int s = 0; s < num_segments; ++s) {
    const int64_t n = seg_numel[s];
    if (n == 0) continue;
    if (opt == 1 && !d_square_avg[s]) return fail(FA_ERR_INVALID, "segment %d: square_avg NULL", s);
    bool aligned = al16(d_param[s]) && (momentum == 0.0 || al16(d_momentum[s])) &&
                   (opt != 1 || al16(d_square_avg[s]));
    for (int i = 0; i < k; ++i) {
      const void* p = d_in[(int64_t)s * k + i];
      hp[(int64_t)j * k + i] = p;
      aligned = aligned && al16(p);
    }
    if (sstr && !aligned) return fail(FA_ERR_INVALID, "tiled inputs, parameter and momentum must be 16-byte aligned");
    hs[j] = Seg{n, t0, d_param[s], j * k, aligned ? 1 : 0};
    hb[j] = momentum != 0.0 ? d_momentum[s] : d_param[s];  // never dereferenced without momentum
    hq[j] = opt == 1 ? d_square_avg[s] : d_param[s];       // never dereferenced for SGD
    t0 += (n + tile_elems - 1) / tile_elems;
    ++j;
  }
  const int flags = (momentum != 0.0 ? SGD_MOMENTUM : 0) | (nesterov ? SGD_NESTEROV : 0) |
                    (weight_decay != 0.0 ? SGD_WD : 0) | (first_step ? SGD_FIRST : 0);
  const RmsArgs ra{(float)alpha, (float)(1.0 - alpha), (float)eps};
  if (inl) {
    const int co = (int)seg_bytes, bo = (int)(seg_bytes + coef_bytes), qo = (int)(seg_bytes + coef_bytes + buf_bytes),
              po = (int)(seg_bytes + coef_bytes + 2 * buf_bytes);
    if (opt == 1)
      hipLaunchKernelGGL((k_fedavg_sgd_inl<8, true, 1>), dim3((unsigned)tiles), dim3(kBlock), 0, st, dsc, nseg, co, bo,
                         qo, po, k, (float)(-lr), (float)momentum, 1.0f, (float)weight_decay, flags, sstr, ra);
    else
      hipLaunchKernelGGL((k_fedavg_sgd_inl<8, true, 0>), dim3((unsigned)tiles), dim3(kBlock), 0, st, dsc, nseg, co, bo,
                         qo, po, k, (float)(-lr), (float)momentum, (float)(1.0 - dampening), (float)weight_decay,
                         flags, sstr, ra);
    FA_HIP(hipGetLastError());
    return FA_OK;
  }
  rc = stage(slot, bytes, st);
  if (rc) return rc;
  char* dv = (char*)slot->dev;
  const Seg* ds = (const Seg*)dv;
  const double* dc = (const double*)(dv + seg_bytes);
  void* const* db = (void* const*)(dv + seg_bytes + coef_bytes);
  void* const* dq = (void* const*)(dv + seg_bytes + coef_bytes + buf_bytes);
  const void* const* dp = (const void* const*)(dv + seg_bytes + coef_bytes + 2 * buf_bytes);
  if (opt == 1)
    hipLaunchKernelGGL((k_fedavg_sgd<8, true, 1>), dim3((unsigned)tiles), dim3(kBlock), 0, st, ds, nseg, dc, dp, k,
                       db, (float)(-lr), (float)momentum, 1.0f, (float)weight_decay, flags, sstr, dq, ra);
  else
    hipLaunchKernelGGL((k_fedavg_sgd<8, true, 0>), dim3((unsigned)tiles), dim3(kBlock), 0, st, ds, nseg, dc, dp, k,
                       db, (float)(-lr), (float)momentum, (float)(1.0 - dampening), (float)weight_decay, flags, sstr,
                       dq, ra);
  FA_HIP(hipGetLastError());
  return release(slot, st);
}
}  // namespace

int fa_fedavg_sgd(fa_ctx* ctx, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                  const void* const* d_in, const double* coef, void* const* d_param, void* const* d_momentum,
                  double lr, double momentum, double dampening, double weight_decay, int nesterov,
                  int first_step, void* hip_stream) {
  return fedavg_sgd_impl(ctx, num_segments, seg_numel, k, d_in, coef, d_param, d_momentum, lr, momentum,
                         dampening, weight_decay, nesterov, first_step, hip_stream, 0);
}

int fa_fedavg_rmsprop(fa_ctx* ctx, int32_t num_segments, const int64_t* seg_numel, int32_t k,
                      const void* const* d_in, const double* coef, void* const* d_param,
                      void* const* d_square_avg, void* const* d_momentum, double lr, double alpha, double eps,
                      double weight_decay, double momentum, int first_step, void* hip_stream) {
  return fedavg_sgd_impl(ctx, num_segments, seg_numel, k, d_in, coef, d_param, d_momentum, lr, momentum, 0.0,
                         weight_decay, 0, first_step, hip_stream, 0, 1, d_square_avg, alpha, eps);
}

int fa_fedavg_sgd_tiled(fa_ctx* ctx, int64_t n, int32_t k, const void* const* d_in, int64_t tile_stride,
                        const double* coef, void* d_param, void* d_momentum, double lr, double momentum,
                        double dampening, double weight_decay, int nesterov, int first_step, void* hip_stream) {
  if (n < 0) return fail(FA_ERR_INVALID, "n must be >= 0");
  if (tile_stride <= 0 || tile_stride % FA_TILE_BYTES)
    return fail(FA_ERR_INVALID, "tile_stride must be a positive multiple of %d (got %lld)", FA_TILE_BYTES,
                (long long)tile_stride);
  void* params[1] = {d_param};
  void* moms[1] = {d_momentum};
  return fedavg_sgd_impl(ctx, 1, &n, k, d_in, coef, params, d_momentum ? moms : nullptr, lr, momentum, dampening,
                         weight_decay, nesterov, first_step, hip_stream, tile_stride);
}

namespace {
int mix_impl(fa_ctx* ctx, int dtype, int64_t n, int32_t rows, const int32_t* row_ptr,
             const int32_t* cols, const double* vals, int32_t num_in, const void* const* d_in,
             void* const* d_out, const double* post_scale, void* const* d_out2, void* hip_stream,
             int64_t isst, int64_t osst, const float* d_omega_in = nullptr, float* d_omega_out = nullptr) {
  static const double kOnes[1] = {1.0};
  const bool dev_omega = d_omega_in != nullptr;
  if (dev_omega && (!d_omega_out || !d_out2)) return fail(FA_ERR_INVALID, "fa_pushsum: omega_out / d_out2 NULL");
  if (dev_omega) post_scale = kOnes;  // the scales come from k_pushsum_omega, on the device
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (rows <= 0 || n < 0 || !row_ptr || !cols || !vals || !d_in || !d_out || num_in <= 0)
    return fail(FA_ERR_INVALID, "fa_mix: invalid arguments");
  if (dtype != FA_DTYPE_F32 && dtype != FA_DTYPE_BF16 && dtype != FA_DTYPE_F16)
    return fail(FA_ERR_DTYPE, "fa_mix: dtype %d not supported (F32, BF16, F16)", dtype);
  if (post_scale && !d_out2) return fail(FA_ERR_INVALID, "fa_mix: post_scale without d_out2");
  if (row_ptr[0] != 0) return fail(FA_ERR_INVALID, "fa_mix: row_ptr[0] must be 0");
  bool aligned = true;
  for (int r = 0; r < rows; ++r) {
    if (row_ptr[r + 1] <= row_ptr[r]) return fail(FA_ERR_INVALID, "fa_mix: row %d is empty", r);
    if (!d_out[r] || (post_scale && !d_out2[r])) return fail(FA_ERR_INVALID, "fa_mix: row %d output NULL", r);
    aligned = aligned && al16(d_out[r]) && (!post_scale || al16(d_out2[r]));
  }
  const int32_t nnz = row_ptr[rows];
  for (int j = 0; j < nnz; ++j)
    if (cols[j] < 0 || cols[j] >= num_in) return fail(FA_ERR_INVALID, "fa_mix: col %d out of range", cols[j]);
  for (int i = 0; i < num_in; ++i) {
    if (!d_in[i]) return fail(FA_ERR_INVALID, "fa_mix: input %d NULL", i);
    aligned = aligned && al16(d_in[i]);
  }
  if (n == 0 && !dev_omega) return FA_OK;
  if ((isst || osst) && !aligned) return fail(FA_ERR_INVALID, "fa_mix_tiled: inputs and outputs must be 16-byte aligned");
  const int V = elems_per_vec(dtype);
  const int64_t tiles = (n + (int64_t)kBlock * V - 1) / ((int64_t)kBlock * V);
  if (tiles > 0x7FFFFFFFll) return fail(FA_ERR_INVALID, "too many tiles");

  const size_t row_bytes = align16(sizeof(MixRow) * rows);
  const size_t col_bytes = align16(sizeof(int32_t) * nnz);
  const size_t val_bytes = align16(sizeof(double) * nnz);
  const size_t ptr_bytes = sizeof(void*) * num_in;
  const size_t bytes = row_bytes + col_bytes + val_bytes + ptr_bytes;

  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipStream_t st = (hipStream_t)hip_stream;
  fa_ctx::Slot* slot = nullptr;
  int rc = acquire_slot(ctx, bytes, &slot);
  if (rc) return rc;
  char* h = (char*)slot->host;
  MixRow* hr = (MixRow*)h;
  for (int r = 0; r < rows; ++r)
    hr[r] = MixRow{row_ptr[r], row_ptr[r + 1], d_out[r], post_scale ? d_out2[r] : nullptr,
                   post_scale && !dev_omega ? post_scale[r] : 1.0};
  memcpy(h + row_bytes, cols, sizeof(int32_t) * nnz);
  memcpy(h + row_bytes + col_bytes, vals, sizeof(double) * nnz);
  memcpy(h + row_bytes + col_bytes + val_bytes, d_in, ptr_bytes);
  rc = stage(slot, bytes, st);
  if (rc) return rc;
  char* d = (char*)slot->dev;
  const MixRow* drw = (const MixRow*)d;
  const int32_t* dcol = (const int32_t*)(d + row_bytes);
  const double* dval = (const double*)(d + row_bytes + col_bytes);
  const void* const* dptr = (const void* const*)(d + row_bytes + col_bytes + val_bytes);
  const dim3 grid((unsigned)tiles), blk(kBlock);
  const int al = aligned ? 1 : 0;
  if (dev_omega)
    hipLaunchKernelGGL(k_pushsum_omega, dim3((unsigned)((rows + kBlock - 1) / kBlock)), blk, 0, st, (MixRow*)drw, rows,
                       dcol, dval, d_omega_in, d_omega_out);
  if (n == 0) {
    FA_HIP(hipGetLastError());
    return release(slot, st);
  }
  int maxdeg = 0;
  for (int r = 0; r < rows; ++r) maxdeg = std::max(maxdeg, row_ptr[r + 1] - row_ptr[r]);
  const int band = (aligned && ctx->mix_band) ? band_offset(rows, row_ptr, cols, num_in) : INT32_MIN;
  if (band != INT32_MIN) {
    // non-temporal input loads by default (r03r interleaved A/B, cfg5 256-node ring: 5.23-5.32 ->
    // 4.41-4.42 ms; every model is read once per workgroup).  FA_BAND_VAR (A/B measurement): 0 cached
    // loads, 2 XCD-contiguous tiles, 3 both NT + XCD, 4 NT + XCD + 16-row groups (within 1 % of 1)
    static const int bv = [] {
      const char* e = getenv("FA_BAND_VAR");
      return e ? atoi(e) : 1;
    }();
    const int xm = (bv == 2 || bv >= 3) ? 1 : 0;
#define FA_BAND_K(DT, RG, POST, NT) \
    hipLaunchKernelGGL((k_mix_band<DT, RG, POST, NT>), grid, blk, 0, st, drw, rows, dcol, dval, dptr, num_in, band, n, isst, osst, xm)
#define FA_BAND(DT)                                                                                   \
  if (post_scale) {                                                                                   \
    if (bv == 1 || bv == 3) FA_BAND_K(DT, 8, true, true); else if (bv == 4) FA_BAND_K(DT, 16, true, true); \
    else FA_BAND_K(DT, 8, true, false);                                                               \
  } else {                                                                                            \
    if (bv == 1 || bv == 3) FA_BAND_K(DT, 8, false, true); else if (bv == 4) FA_BAND_K(DT, 16, false, true); \
    else FA_BAND_K(DT, 8, false, false);                                                              \
  }
    switch (dtype) {
      case FA_DTYPE_F32: FA_BAND(FA_DTYPE_F32); break;
      case FA_DTYPE_BF16: FA_BAND(FA_DTYPE_BF16); break;
      case FA_DTYPE_F16: FA_BAND(FA_DTYPE_F16); break;
    }
#undef FA_BAND
#undef FA_BAND_K
    FA_HIP(hipGetLastError());
    return release(slot, st);
  }
  // shape by row degree: ring-like (<= 3 entries), up to 4, or dense rows in passes of 8
#define FA_MIX_SHAPE(DT, RG, MAXD)                                                                     \
  if (post_scale)                                                                                      \
    hipLaunchKernelGGL((k_mix<DT, RG, MAXD, true>), grid, blk, 0, st, drw, rows, dcol, dval, dptr, n, al, isst, osst); \
  else                                                                                                 \
    hipLaunchKernelGGL((k_mix<DT, RG, MAXD, false>), grid, blk, 0, st, drw, rows, dcol, dval, dptr, n, al, isst, osst);
#define FA_MIX_LAUNCH(DT)                        \
  if (maxdeg <= 3) { FA_MIX_SHAPE(DT, 4, 3) }    \
  else if (maxdeg <= 4) { FA_MIX_SHAPE(DT, 4, 4) } \
  else { FA_MIX_SHAPE(DT, 2, 8) }
  switch (dtype) {
    case FA_DTYPE_F32: FA_MIX_LAUNCH(FA_DTYPE_F32); break;
    case FA_DTYPE_BF16: FA_MIX_LAUNCH(FA_DTYPE_BF16); break;
    case FA_DTYPE_F16: FA_MIX_LAUNCH(FA_DTYPE_F16); break;
  }
#undef FA_MIX_LAUNCH
#undef FA_MIX_SHAPE
  FA_HIP(hipGetLastError());
  return release(slot, st);
}
}  // namespace

int fa_mix(fa_ctx* ctx, int dtype, int64_t n, int32_t rows, const int32_t* row_ptr,
           const int32_t* cols, const double* vals, int32_t num_in, const void* const* d_in,
           void* const* d_out, const double* post_scale, void* const* d_out2, void* hip_stream) {
  return mix_impl(ctx, dtype, n, rows, row_ptr, cols, vals, num_in, d_in, d_out, post_scale, d_out2, hip_stream, 0, 0);
}

int fa_pushsum(fa_ctx* ctx, int dtype, int64_t n, int32_t rows, const int32_t* row_ptr, const int32_t* cols,
               const double* vals, int32_t num_in, const void* const* d_in, const float* d_omega_in,
               void* const* d_out, void* const* d_out2, float* d_omega_out, void* hip_stream) {
  if (!d_omega_in || !d_omega_out || !d_out2) return fail(FA_ERR_INVALID, "fa_pushsum: omega / z outputs NULL");
  return mix_impl(ctx, dtype, n, rows, row_ptr, cols, vals, num_in, d_in, d_out, nullptr, d_out2, hip_stream, 0, 0,
                  d_omega_in, d_omega_out);
}

int fa_mix_tiled(fa_ctx* ctx, int dtype, int64_t n, int32_t rows, const int32_t* row_ptr,
                 const int32_t* cols, const double* vals, int32_t num_in, const void* const* d_in,
                 int64_t in_tile_stride, void* const* d_out, int64_t out_tile_stride, const double* post_scale,
                 void* const* d_out2, void* hip_stream) {
  if (in_tile_stride <= 0 || in_tile_stride % FA_TILE_BYTES || out_tile_stride <= 0 ||
      out_tile_stride % FA_TILE_BYTES)
    return fail(FA_ERR_INVALID, "fa_mix_tiled: tile strides must be positive multiples of %d", FA_TILE_BYTES);
  return mix_impl(ctx, dtype, n, rows, row_ptr, cols, vals, num_in, d_in, d_out, post_scale, d_out2, hip_stream,
                  in_tile_stride, out_tile_stride);
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Read-stream probe (measurement only; no arithmetic contract): the weighted-sum kernel's access
// pattern with the arithmetic and the output stream removed.  The buffer is a run of FA_TILE_BYTES
// rows; workgroup b reads rows [b R, (b + 1) R) -- lane l the 16 bytes at l * 16 of every row, U = 8
// rows per load group (non-temporal, as k_wsum) -- and XORs them together.  With R = K on a tiled
// arena group this is exactly the address sequence k_wsum_inl issues on it, so its rate is the
// box's ceiling for that kernel on those very pages (bench.py: measured_read_ceiling).  The XOR is
// stored only if it equals a constant (never, in practice): the loads stay live without a write.
namespace {
template <int U>
__global__ void __launch_bounds__(kBlock)
k_read_probe(const char* __restrict__ buf, int64_t nrows, int rows_per_wg, unsigned* __restrict__ word) {
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t r1 = r0 + rows_per_wg < nrows ? r0 + rows_per_wg : nrows;
  const char* p = buf + (int64_t)threadIdx.x * 16;
  u32x4 acc = {0u, 0u, 0u, 0u};
  int64_t r = r0;
  for (; r + U <= r1; r += U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld16<true>(p + (r + u) * FA_TILE_BYTES);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  for (; r < r1; ++r) acc ^= ld16<true>(p + r * FA_TILE_BYTES);
  const unsigned x = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (x == 0x9E3779B9u) word[0] = x;
}
}  // namespace

extern "C" int fa_device_alloc_contiguous(fa_ctx* ctx, int64_t bytes, void** d_out) {
  if (!ctx || !d_out || bytes <= 0) return fail(FA_ERR_INVALID, "fa_device_alloc_contiguous: ctx, d_out, bytes > 0");
  *d_out = nullptr;
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  void* p = nullptr;
  const hipError_t e = hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocContiguous);
  if (e != hipSuccess || !p) {
    (void)hipGetLastError();  // not sticky: the caller falls back to an ordinary allocation
    return fail(FA_ERR_HIP, "hipExtMallocWithFlags(%lld bytes, contiguous): %s", (long long)bytes,
                hipGetErrorString(e));
  }
  *d_out = p;
  return FA_OK;
}

extern "C" int fa_device_free(fa_ctx* ctx, void* d_ptr) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (!d_ptr) return FA_OK;
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  FA_HIP(hipFree(d_ptr));
  return FA_OK;
}

extern "C" int fa_read_probe(fa_ctx* ctx, const void* d_buf, int64_t bytes, int32_t rows_per_workgroup,
                             void* d_word, void* hip_stream) {
  if (!ctx) return fail(FA_ERR_INVALID, "ctx is NULL");
  if (!d_buf || !d_word || !al16(d_buf) || bytes < FA_TILE_BYTES || rows_per_workgroup < 1 ||
      rows_per_workgroup > 65536)
    return fail(FA_ERR_INVALID, "fa_read_probe: 16-byte aligned buffer of >= %d bytes, 1 <= rows_per_workgroup "
                "<= 65536, and a device word are required", FA_TILE_BYTES);
  const int64_t nrows = bytes / FA_TILE_BYTES;
  const int64_t grid = (nrows + rows_per_workgroup - 1) / rows_per_workgroup;
  if (grid > 0x7FFFFFFF) return fail(FA_ERR_INVALID, "fa_read_probe: too many workgroups (%lld)", (long long)grid);
  DeviceGuard g(ctx->device);
  if (!g.ok) return fail(FA_ERR_HIP, "hipSetDevice(%d) failed", ctx->device);
  hipLaunchKernelGGL(k_read_probe<8>, dim3((unsigned)grid), dim3(kBlock), 0, (hipStream_t)hip_stream,
                     (const char*)d_buf, nrows, (int)rows_per_workgroup, (unsigned*)d_word);
  FA_HIP(hipGetLastError());
  return FA_OK;
}
