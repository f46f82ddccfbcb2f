// layout_probe.hip -- tool only: is the client-major arena ([K][P], 128 streams) or a tile-interleaved
// arena ([P/T][K][T], each workgroup's reads one contiguous K*T run) closer to the read ceiling?
// Same 16-B non-temporal loads, U = 8 in flight, one 16-B store per lane, no arithmetic.
#include <hip/hip_runtime.h>
#include <cstdint>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4* gp;
typedef __attribute__((address_space(1))) u32x4* gpw;

// rows: client i at base + i*row16 (16-B units); workgroup b = 4-KiB column tile b
__global__ void __launch_bounds__(256) lp_rows(const u32x4* __restrict__ base, int64_t row16, int k, u32x4* out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (int i0 = 0; i0 < k; i0 += 8) {
    u32x4 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) r[u] = __builtin_nontemporal_load((gp)(base + (int64_t)min(i0 + u, k - 1) * row16 + e));
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= r[u];
  }
  __builtin_nontemporal_store(acc, (gpw)(out + e));
}

// tiled: tile t holds T16 16-B units of each client, client-major inside the tile
// (tile t, client i) at base + (t*k + i)*T16; workgroup b covers 256 units of one tile.
__global__ void __launch_bounds__(256) lp_tiled(const u32x4* __restrict__ base, int64_t T16, int k, u32x4* out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;   // output unit
  const int64_t t = e / T16, o = e - t * T16;
  const u32x4* tb = base + t * k * T16 + o;
  u32x4 acc = {0, 0, 0, 0};
  for (int i0 = 0; i0 < k; i0 += 8) {
    u32x4 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) r[u] = __builtin_nontemporal_load((gp)(tb + (int64_t)min(i0 + u, k - 1) * T16));
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= r[u];
  }
  __builtin_nontemporal_store(acc, (gpw)(out + e));
}

// tiled, XCD-aware: workgroup b runs on XCD b % 8; give each XCD a contiguous eighth of the tiles
__global__ void __launch_bounds__(256) lp_tiled_xcd(const u32x4* __restrict__ base, int k, u32x4* out) {
  const int64_t nb = gridDim.x, q = nb / 8, b = blockIdx.x;
  const int64_t tile = b < 8 * q ? (b % 8) * q + b / 8 : b;
  const int64_t e = tile * 256 + threadIdx.x;
  const u32x4* tb = base + tile * k * 256 + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (int i0 = 0; i0 < k; i0 += 8) {
    u32x4 r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) r[u] = __builtin_nontemporal_load((gp)(tb + (int64_t)min(i0 + u, k - 1) * 256));
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= r[u];
  }
  __builtin_nontemporal_store(acc, (gpw)(out + e));
}

extern "C" int lp_run(int mode, const void* base, int64_t p16, int k, int64_t t16, void* out, void* stream) {
  const int64_t blocks = p16 / 256;
  if (mode == 0) hipLaunchKernelGGL(lp_rows, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const u32x4*)base, p16, k, (u32x4*)out);
  else if (mode == 2) hipLaunchKernelGGL(lp_tiled_xcd, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const u32x4*)base, k, (u32x4*)out);
  else hipLaunchKernelGGL(lp_tiled, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const u32x4*)base, t16, k, (u32x4*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// CU-masked stream (hipExtStreamCreateWithCUMask): how many CUs does the tiled stream need for full
// HBM rate?  (Leaving CUs free for RCCL's kernels on multi-GPU runs.)
extern "C" int lp_masked_stream(int ncu_enabled, void** out_stream) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return -1;
  const int total = prop.multiProcessorCount;
  uint32_t mask[16] = {0};
  int words = (total + 31) / 32;
  // spread the disabled CUs evenly over the index space (XCDs/SEs interleave in the mask)
  for (int i = 0; i < total; ++i) {
    const bool on = (int64_t)i * ncu_enabled / total != (int64_t)(i + 1) * ncu_enabled / total;
    if (on) mask[i / 32] |= 1u << (i % 32);
  }
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, words, mask) != hipSuccess) return -2;
  *out_stream = (void*)s;
  return total;
}
