// dpp_rate_probe.hip -- VALU issue rate of the pair-distance inner step on gfx950:
//   plain : t = b_i - a ; acc_i = fma(t, t, acc_i)                  (v_sub_f32 + v_fmac_f32)
//   dpp   : t = row_ror_d(b) - a ; acc_d = fma(t, t, acc_d)          (v_sub_f32_dpp + v_fmac_f32)
//   dpp2  : as dpp, two differences formed before their two fmas    (fewer s_nop hazards)
//   pk    : packed v_pk_add_f32 + v_pk_fma_f32 on float2
// 16 accumulators per lane, ITER x 16 steps; waves per SIMD set by the grid.  Prints ns and the
// achieved pair-steps per cycle per CU against the 128 lane-ops / clk / CU of non-packed FP32 VALU.
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o /tmp/dpp_rate_probe tools/dpp_rate_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <utility>

constexpr int ITER = 4096;

template <int D>
__device__ __forceinline__ float rot16(float v) {
  if constexpr (D == 0) return v;
  else return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x120 + (16 - D), 0xf, 0xf, true));
}

template <int MODE, int... D>
__device__ __forceinline__ void step(float a, float b, float (&acc)[16], std::integer_sequence<int, D...>) {
  if constexpr (MODE == 1) {
    ((acc[D] = __builtin_fmaf(rot16<D>(b) - a, rot16<D>(b) - a, acc[D])), ...);
  }
}

template <int D0, int D1>
__device__ __forceinline__ void sq2(float a, float b, float& x0, float& x1) {
  const float t0 = rot16<D0>(b) - a, t1 = rot16<D1>(b) - a;
  x0 = __builtin_fmaf(t0, t0, x0);
  x1 = __builtin_fmaf(t1, t1, x1);
}
template <int... D>
__device__ __forceinline__ void step2(float a, float b, float (&acc)[16], std::integer_sequence<int, D...>) {
  (sq2<2 * D, 2 * D + 1>(a, b, acc[2 * D], acc[2 * D + 1]), ...);
}

// software-pipelined: the next difference before this one's fma (sub_dpp, fma alternate; the
// temporary a sub_dpp writes is not the one the previous sub_dpp wrote)
template <int D, int N>
__device__ __forceinline__ void pipe(float a, float b, float t, float (&acc)[16]) {
  if constexpr (D + 1 < N) {
    const float tn = rot16<D + 1>(b) - a;
    acc[D] = __builtin_fmaf(t, t, acc[D]);
    pipe<D + 1, N>(a, b, tn, acc);
  } else {
    acc[D] = __builtin_fmaf(t, t, acc[D]);
  }
}

template <int MODE>
__global__ void __launch_bounds__(256) k(const float* in, float* out) {
  float acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  float a = in[threadIdx.x], b = in[threadIdx.x + 256];
  float bb[16];
  for (int i = 0; i < 16; ++i) bb[i] = in[threadIdx.x + 16 * i];
  for (int it = 0; it < ITER; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float t = bb[i] - a;
        acc[i] = __builtin_fmaf(t, t, acc[i]);
      }
    } else if constexpr (MODE == 2) step2(a, b, acc, std::make_integer_sequence<int, 8>{});
    else if constexpr (MODE == 4) pipe<0, 16>(a, b, b - a, acc);
    else step<MODE>(a, b, acc, std::make_integer_sequence<int, 16>{});
    a += 1.0f;
    b -= 1.0f;
  }
  float s = 0.0f;
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) kpk(const float* in, float* out) {
  f32x2 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x2{0.0f, 0.0f};
  f32x2 a = {in[threadIdx.x], in[threadIdx.x + 1]}, b = {in[threadIdx.x + 256], in[threadIdx.x + 257]};
  f32x2 bb[8];
  for (int i = 0; i < 8; ++i) bb[i] = f32x2{in[threadIdx.x + 16 * i], in[threadIdx.x + 16 * i + 8]};
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x2 t = bb[i] - a;
      acc[i] = __builtin_elementwise_fma(t, t, acc[i]);
    }
    a += 1.0f;
    b -= 1.0f;
  }
  float s = 0.0f;
  for (int i = 0; i < 8; ++i) s += acc[i].x + acc[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  float *in, *out;
  hipMalloc(&in, 4096 * 4);
  hipMemset(in, 0, 4096 * 4);
  const int cus = 256;
  hipMalloc(&out, (size_t)cus * 32 * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"plain", "dpp", "dpp2", "pk", "dpipe"};
  for (int wps : {2, 4, 8}) {        // waves per SIMD: blocks of 4 waves, wps blocks per CU
    const int blocks = cus * wps;
    for (int m = 0; m < 5; ++m) {
      auto launch = [&]() {
        if (m == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, in, out);
        if (m == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, in, out);
        if (m == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, in, out);
        if (m == 3) hipLaunchKernelGGL(kpk, dim3(blocks), dim3(256), 0, 0, in, out);
        if (m == 4) hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, in, out);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= 5;
      // pair-steps (one sub + one fma per lane) per launch
      const double steps = (double)blocks * 256 * ITER * 16;
      const double clk = 2.4e9 * ms * 1e-3;
      printf("waves/SIMD %d %-6s %.3f ms  lane-steps/clk/CU %.1f (VALU floor 64)\n", wps, names[m], ms,
             steps / clk / cus);
    }
  }
  return 0;
}
