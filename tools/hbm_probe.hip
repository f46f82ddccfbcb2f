// hbm_probe.hip -- measures the practical HBM ceilings the aggregation kernel is compared with:
//   probe_read : read-only stream (16-B non-temporal loads, U in flight per lane), one word out/thread
//   probe_copy : 16-B load + 16-B store stream
// Tool only (tools/hbm_probe.py); not part of the product library.
#include <hip/hip_runtime.h>
#include <cstdint>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* gp;

template <int U>
__global__ void __launch_bounds__(256) probe_read(const u32x4* __restrict__ src, int64_t n16, unsigned* out) {
  unsigned acc = 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride * U) {
    u32x4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t j = i + u * stride;
      r[u] = j < n16 ? __builtin_nontemporal_load((gp)(src + j)) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= r[u][0] ^ r[u][1] ^ r[u][2] ^ r[u][3];
  }
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ void __launch_bounds__(256) probe_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load((gp)(src + i)), (__attribute__((address_space(1))) u32x4*)(dst + i));
}

// K separate streams, one 4-KiB tile of each per workgroup (the aggregation kernel's access
// pattern with the arithmetic removed): isolates the cost of reading 128 streams at once.
template <int U, bool WIDE_OUT>
__global__ void __launch_bounds__(256) probe_multi(const u32x4* const* __restrict__ ptrs, int k, unsigned* out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (int i0 = 0; i0 < k; i0 += U) {
    u32x4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = __builtin_nontemporal_load((gp)(ptrs[min(i0 + u, k - 1)] + e));
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= r[u];
  }
  if constexpr (WIDE_OUT)  // one 16-B output vector per lane, like the aggregation kernel
    __builtin_nontemporal_store(acc, (__attribute__((address_space(1))) u32x4*)((u32x4*)out + e));
  else
    out[e] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
}

extern "C" int hbm_probe_multi(const void* dptrs, int k, int64_t bytes_per_stream, void* out, int unroll, void* stream) {
  const int64_t tiles = bytes_per_stream / (16 * 256);
  if (unroll == 16) hipLaunchKernelGGL((probe_multi<16, false>), dim3(tiles), dim3(256), 0, (hipStream_t)stream, (const u32x4* const*)dptrs, k, (unsigned*)out);
  else if (unroll == -8) hipLaunchKernelGGL((probe_multi<8, true>), dim3(tiles), dim3(256), 0, (hipStream_t)stream, (const u32x4* const*)dptrs, k, (unsigned*)out);
  else hipLaunchKernelGGL((probe_multi<8, false>), dim3(tiles), dim3(256), 0, (hipStream_t)stream, (const u32x4* const*)dptrs, k, (unsigned*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int hbm_probe_read(const void* src, int64_t bytes, void* out, int blocks, int unroll, void* stream) {
  const int64_t n16 = bytes / 16;
  if (unroll == 4) hipLaunchKernelGGL(probe_read<4>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src, n16, (unsigned*)out);
  else if (unroll == 16) hipLaunchKernelGGL(probe_read<16>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src, n16, (unsigned*)out);
  else hipLaunchKernelGGL(probe_read<8>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src, n16, (unsigned*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int hbm_probe_copy(const void* src, void* dst, int64_t bytes, int blocks, void* stream) {
  hipLaunchKernelGGL(probe_copy, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src, (u32x4*)dst, bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
