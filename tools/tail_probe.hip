// tail_probe.hip -- is cfg2's 1.5 GB round (K = 32 x 11.7 M fp32) losing time to the launch's tail?
// The aggregation's access pattern (K row streams of one allocation, 16-B non-temporal loads, one
// 16-B output vector per lane) with the arithmetic reduced to a xor, in four launch shapes:
//   block B threads, one tile of B x 16 B per client per workgroup (B = 256 is the product kernel),
//   or a persistent grid: G workgroups, each walking a contiguous run of tiles.
// Tool only (tools/tail_probe.py); not part of the product library.
#include <hip/hip_runtime.h>
#include <cstdint>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* gp;

template <int B, int U>
__device__ __forceinline__ void tile(const u32x4* const* __restrict__ ptrs, int k, int64_t t, u32x4* out) {
  const int64_t e = t * B + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (int i0 = 0; i0 < k; i0 += U) {
    u32x4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = __builtin_nontemporal_load((gp)(ptrs[min(i0 + u, k - 1)] + e));
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= r[u];
  }
  __builtin_nontemporal_store(acc, (__attribute__((address_space(1))) u32x4*)(out + e));
}

template <int B>
__global__ void __launch_bounds__(B) probe_tiles(const u32x4* const* __restrict__ ptrs, int k, u32x4* out) {
  tile<B, 8>(ptrs, k, blockIdx.x, out);
}

template <int B>
__global__ void __launch_bounds__(B) probe_persist(const u32x4* const* __restrict__ ptrs, int k, int64_t tiles,
                                                   u32x4* out) {
  const int64_t t0 = tiles * blockIdx.x / gridDim.x, t1 = tiles * (blockIdx.x + 1) / gridDim.x;
  for (int64_t t = t0; t < t1; ++t) tile<B, 8>(ptrs, k, t, out);
}

// mode 0: tiles (one per workgroup), 1: persistent with `grid` workgroups
extern "C" int tail_probe(const void* dptrs, int k, int64_t bytes_per_stream, void* out, int block, int mode,
                          int grid, void* stream) {
  const int64_t tiles = bytes_per_stream / (16 * (int64_t)block);
  hipStream_t st = (hipStream_t)stream;
  const u32x4* const* p = (const u32x4* const*)dptrs;
#define TP(BB)                                                                                                \
  if (block == BB) {                                                                                          \
    if (mode == 0) hipLaunchKernelGGL(probe_tiles<BB>, dim3((unsigned)tiles), dim3(BB), 0, st, p, k, (u32x4*)out); \
    else hipLaunchKernelGGL(probe_persist<BB>, dim3((unsigned)grid), dim3(BB), 0, st, p, k, tiles, (u32x4*)out); \
  }
  TP(64) TP(128) TP(256) TP(512)
#undef TP
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
