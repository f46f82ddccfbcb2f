// Read-pattern probe for the coordinate-wise median (tools/gpu_r03ae.sh): how fast can K client rows
// be streamed when every lane reads ONE 4-byte coordinate of each client (the median kernels' pattern,
// all K loads issued before any is used) versus 16 bytes (4 coordinates) of each client?  No network:
// the loaded values are reduced by a min (data-dependent, so nothing is dropped) and one value per
// coordinate is stored.  Output: one JSON line per form with the average kernel time over reps.
// r04: the same 4-byte-per-lane pattern on the tiled ClientArena layout (run_tiled).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

// global (not flat) loads, as the median kernels' gld_nt_off
template <typename T> __device__ __forceinline__ T ldnt(const T* p) {
  return __builtin_nontemporal_load((const __attribute__((address_space(1))) T*)p);
}

// one coordinate per lane: K 4-byte loads (uniform row base + 32-bit offset), then a min tree
template <int K>
__global__ void __launch_bounds__(256) k_w4(const float* const* __restrict__ rows, int64_t n, float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  float x[K];
#pragma unroll
  for (int i = 0; i < K; ++i) x[i] = ldnt(rows[i] + e);
  float m = x[0];
#pragma unroll
  for (int i = 1; i < K; ++i) m = __builtin_elementwise_minimum(m, x[i]);
  out[e] = m;
}

// four coordinates per lane: K 16-byte loads (running min: K x 16 B would not fit the registers)
template <int K>
__global__ void __launch_bounds__(256) k_w16(const float* const* __restrict__ rows, int64_t n, float* __restrict__ out) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (e >= n) return;
  f4 m = ldnt((const f4*)(rows[0] + e));
#pragma unroll
  for (int i = 1; i < K; ++i) m = __builtin_elementwise_minimum(m, ldnt((const f4*)(rows[i] + e)));  // loads hoisted by the compiler
  *(f4*)(out + e) = m;
}

// the tiled ClientArena layout [tiles][K][E] (E = 1024 floats): column e of client i at
// (e / E) * K * E + i * E + e % E -- a workgroup's 256 columns lie in one tile, its K rows 4 KiB apart
template <int K>
__global__ void __launch_bounds__(256) k_w4t(const float* __restrict__ arena, int64_t n, float* __restrict__ out) {
  constexpr int64_t E = 1024;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const float* base = arena + (e / E) * K * E + e % E;
  float x[K];
#pragma unroll
  for (int i = 0; i < K; ++i) x[i] = ldnt(base + i * E);
  float m = x[0];
#pragma unroll
  for (int i = 1; i < K; ++i) m = __builtin_elementwise_minimum(m, x[i]);
  out[e] = m;
}

template <int K>
void run_tiled(int64_t n, int reps) {
  constexpr int64_t E = 1024;
  const int64_t tiles = (n + E - 1) / E;
  float* arena;
  CK(hipMalloc(&arena, tiles * K * E * sizeof(float)));
  CK(hipMemset(arena, 0x3f, tiles * K * E * sizeof(float)));
  float* out;
  CK(hipMalloc(&out, n * sizeof(float)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned grid = (unsigned)((n + 255) / 256);
  auto launch = [&] { hipLaunchKernelGGL(k_w4t<K>, dim3(grid), dim3(256), 0, 0, (const float*)arena, n, out); };
  for (int w = 0; w < 3; ++w) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  const double bytes = (double)n * 4.0 * (K + 1);
  printf("{\"K\": %d, \"form\": \"4B/lane tiled\", \"ms\": %.4f, \"GBps\": %.1f}\n", K, ms, bytes / (ms * 1e-3) / 1e9);
  fflush(stdout);
  CK(hipFree(arena));
  CK(hipFree(out));
}

template <int K>
void run(int64_t n, int reps) {
  std::vector<float*> h(K);
  for (int i = 0; i < K; ++i) {
    CK(hipMalloc(&h[i], n * sizeof(float)));
    CK(hipMemset(h[i], 0x3f, n * sizeof(float)));
  }
  float** rows;
  CK(hipMalloc(&rows, K * sizeof(float*)));
  CK(hipMemcpy(rows, h.data(), K * sizeof(float*), hipMemcpyHostToDevice));
  float* out;
  CK(hipMalloc(&out, n * sizeof(float)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int form = 0; form < 2; ++form) {
    const unsigned grid = (unsigned)(form == 0 ? (n + 255) / 256 : (n / 4 + 255) / 256);
    auto launch = [&] {
      if (form == 0) hipLaunchKernelGGL(k_w4<K>, dim3(grid), dim3(256), 0, 0, (const float* const*)rows, n, out);
      else hipLaunchKernelGGL(k_w16<K>, dim3(grid), dim3(256), 0, 0, (const float* const*)rows, n, out);
    };
    for (int w = 0; w < 3; ++w) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double bytes = (double)n * 4.0 * (K + 1);
    printf("{\"K\": %d, \"form\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", K, form == 0 ? "4B/lane" : "16B/lane", ms,
           bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  }
  for (int i = 0; i < K; ++i) CK(hipFree(h[i]));
  CK(hipFree(rows));
  CK(hipFree(out));
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 11689512;  // ResNet-18's coordinates (the median bench)
  const int reps = 20;
  if (n % 4) return 1;
  run<32>(n, reps);
  run<64>(n, reps);
  run<128>(n, reps);
  run_tiled<32>(n, reps);
  run_tiled<128>(n, reps);
  return 0;
}
