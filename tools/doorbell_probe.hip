// Round-trip latency of a small host-resident FedAvg round (cfg1: K = 2 LR-MNIST updates, 7,850
// fp32 each) on one MI355X, three ways, each including the pack into mapped pinned memory and the
// copy of the result out of it:
//   launch+event : one launch per round + hipEventSynchronize (what fa_weighted_sum_host does);
//   launch+flag  : one launch per round, the host spins on a completion word the kernel writes;
//   doorbell     : a resident workgroup polls a doorbell word in mapped host memory, the host
//                  writes the round's sequence number and spins on the completion word.
// The resident kernel leaves after an idle period (wall clock, s_memrealtime) or on the stop word.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/doorbell_probe tools/doorbell_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

constexpr int P = 7850, K = 2, kThreads = 1024;

struct Ctl {
  unsigned long long doorbell;  // host -> device: round sequence number
  unsigned long long pad0[7];
  unsigned long long done;  // device -> host
  unsigned long long pad1[7];
  unsigned long long stop;  // host -> device
  unsigned long long pad2[7];
};

__device__ __forceinline__ unsigned long long ld_sys(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// out[e] = x0[e] * w0 + x1[e] * w1, rounded per op (the reference's avg = x0*w0; avg += x1*w1)
__device__ __forceinline__ void round_body(const float* in, float* out, float w0, float w1) {
  constexpr int V = P / 2;  // float2 per client (P even)
  const float2* a = (const float2*)in;
  const float2* b = (const float2*)(in + P);
  float2* o = (float2*)out;
  constexpr int R = (V + kThreads - 1) / kThreads;
  float2 xa[R], xb[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = r * kThreads + (int)threadIdx.x;
    if (i < V) {
      xa[r] = a[i];
      xb[r] = b[i];
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = r * kThreads + (int)threadIdx.x;
    if (i < V) {
      float2 v;
      v.x = __fadd_rn(__fmul_rn(xa[r].x, w0), __fmul_rn(xb[r].x, w1));
      v.y = __fadd_rn(__fmul_rn(xa[r].y, w0), __fmul_rn(xb[r].y, w1));
      o[i] = v;
    }
  }
  __threadfence_system();  // every wave's result stores performed before the completion word
}

__global__ void __launch_bounds__(kThreads) k_once(const float* in, float* out, float w0, float w1, Ctl* ctl,
                                                   unsigned long long seq) {
  round_body(in, out, w0, w1);
  __syncthreads();
  if (threadIdx.x == 0) st_sys(&ctl->done, seq);
}

// G workgroups, 16-byte loads, each workgroup a contiguous slice; the last one to finish (device
// counter) stores the completion word
__global__ void __launch_bounds__(256) k_multi(const float* in, float* out, float w0, float w1, Ctl* ctl,
                                               unsigned long long seq, unsigned* counter) {
  constexpr int V4 = P / 4;  // P = 7850 is not a multiple of 4: the last 2 floats separately
  const float4* a = (const float4*)in;
  const float4* b = (const float4*)(in + P + 2);  // client 1 starts 16-byte aligned (P + 2 floats pad)
  float4* o = (float4*)out;
  const int per = (V4 + gridDim.x - 1) / gridDim.x;
  const int lo = blockIdx.x * per, hi = min(V4, lo + per);
  constexpr int R = 8;
  float4 xa[R], xb[R];
  for (int base = lo; base < hi; base += 256 * R) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = base + r * 256 + (int)threadIdx.x;
      if (i < hi) { xa[r] = a[i]; xb[r] = b[i]; }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = base + r * 256 + (int)threadIdx.x;
      if (i < hi) {
        float4 v;
        v.x = __fadd_rn(__fmul_rn(xa[r].x, w0), __fmul_rn(xb[r].x, w1));
        v.y = __fadd_rn(__fmul_rn(xa[r].y, w0), __fmul_rn(xb[r].y, w1));
        v.z = __fadd_rn(__fmul_rn(xa[r].z, w0), __fmul_rn(xb[r].z, w1));
        v.w = __fadd_rn(__fmul_rn(xa[r].w, w0), __fmul_rn(xb[r].w, w1));
        o[i] = v;
      }
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x < P - 4 * V4) {
    const int e = 4 * V4 + threadIdx.x;
    out[e] = __fadd_rn(__fmul_rn(in[e], w0), __fmul_rn(in[P + 2 + e], w1));
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      st_sys(&ctl->done, seq);
    }
  }
}

__global__ void __launch_bounds__(kThreads) k_resident(const float* in, float* out, float w0, float w1, Ctl* ctl,
                                                       unsigned long long last, unsigned long long idle_ticks) {
  __shared__ unsigned long long job;
  unsigned long long t_last = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (threadIdx.x == 0) {
      unsigned long long d = ld_sys(&ctl->doorbell);
      while (d == last) {
        if (ld_sys(&ctl->stop)) { d = 0; break; }
        if (__builtin_amdgcn_s_memrealtime() - t_last > idle_ticks) { d = 0; break; }
        __builtin_amdgcn_s_sleep(1);
        d = ld_sys(&ctl->doorbell);
      }
      job = d;
    }
    __syncthreads();
    const unsigned long long j = job;
    if (j == 0) return;  // every thread leaves together
    round_body(in, out, w0, w1);
    __syncthreads();
    if (threadIdx.x == 0) st_sys(&ctl->done, j);
    last = j;
    t_last = __builtin_amdgcn_s_memrealtime();
    __syncthreads();  // job is rewritten only after every thread read it
  }
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 3000;
  std::vector<float> x0(P), x1(P), ref(P), res(P);
  srand(7);
  for (int i = 0; i < P; ++i) {
    x0[i] = (float)rand() / (float)RAND_MAX - 0.5f;
    x1[i] = (float)rand() / (float)RAND_MAX - 0.5f;
  }
  const float w0 = 300.f / 800.f, w1 = 500.f / 800.f;
  for (int i = 0; i < P; ++i) {
    volatile float a = x0[i] * w0, b = x1[i] * w1;
    ref[i] = a + b;
  }
  char* hb = nullptr;
  const size_t bytes = sizeof(Ctl) + (size_t)(K + 1) * P * 4 + 256;
  CK(hipHostMalloc((void**)&hb, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  memset(hb, 0, bytes);
  Ctl* ctl = (Ctl*)hb;
  float* hin = (float*)(hb + sizeof(Ctl));
  float* hout = hin + K * P;
  Ctl* dctl;
  CK(hipHostGetDevicePointer((void**)&dctl, ctl, 0));
  float* din = (float*)((char*)dctl + sizeof(Ctl));
  float* dout = din + K * P;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  volatile unsigned long long* vdone = &ctl->done;
  auto wait_done = [&](unsigned long long s) {  // spin with a 2 s limit
    auto t0 = std::chrono::steady_clock::now();
    while (*vdone != s) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        fprintf(stderr, "completion word never reached %llu (is %llu)\n", s, *vdone);
        ((volatile unsigned long long*)&ctl->stop)[0] = 1;
        exit(3);
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  };
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
  auto pack = [&] {
    memcpy(hin, x0.data(), P * 4);
    memcpy(hin + P, x1.data(), P * 4);
  };
  auto check = [&](const char* what) {
    if (memcmp(res.data(), ref.data(), P * 4)) {
      fprintf(stderr, "%s: result differs\n", what);
      exit(2);
    }
  };
  unsigned long long seq = 0;
  std::vector<double> t_ev, t_flag, t_bell, t_cold;
  // warm up
  for (int i = 0; i < 50; ++i) {
    pack();
    hipLaunchKernelGGL(k_once, dim3(1), dim3(kThreads), 0, st, din, dout, w0, w1, dctl, ++seq);
    CK(hipEventRecord(ev, st));
    CK(hipEventSynchronize(ev));
  }
  for (int i = 0; i < iters; ++i) {  // launch + event
    auto t0 = now();
    pack();
    hipLaunchKernelGGL(k_once, dim3(1), dim3(kThreads), 0, st, din, dout, w0, w1, dctl, ++seq);
    CK(hipEventRecord(ev, st));
    CK(hipEventSynchronize(ev));
    memcpy(res.data(), hout, P * 4);
    t_ev.push_back(us(t0, now()));
  }
  check("launch+event");
  for (int i = 0; i < iters; ++i) {  // launch + flag
    auto t0 = now();
    pack();
    const unsigned long long s = ++seq;
    hipLaunchKernelGGL(k_once, dim3(1), dim3(kThreads), 0, st, din, dout, w0, w1, dctl, s);
    wait_done(s);
    memcpy(res.data(), hout, P * 4);
    t_flag.push_back(us(t0, now()));
  }
  CK(hipStreamSynchronize(st));
  check("launch+flag");
  // G workgroups (16-byte loads, padded layout: client 1 at P + 2)
  unsigned* counter;
  CK(hipMalloc((void**)&counter, 4));
  CK(hipMemset(counter, 0, 4));
  auto pack2 = [&] {
    memcpy(hin, x0.data(), P * 4);
    memcpy(hin + P + 2, x1.data(), P * 4);
  };
  std::vector<std::pair<int, double>> t_multi;
  for (int G : {1, 2, 4, 8, 16, 32, 64}) {
    std::vector<double> t;
    for (int i = 0; i < iters / 3; ++i) {
      auto t0 = now();
      pack2();
      const unsigned long long s = ++seq;
      hipLaunchKernelGGL(k_multi, dim3(G), dim3(256), 0, st, din, dout + 4, w0, w1, dctl, s, counter);
      wait_done(s);
      memcpy(res.data(), hout + 4, P * 4);
      t.push_back(us(t0, now()));
    }
    CK(hipStreamSynchronize(st));
    check("multi");
    t_multi.push_back({G, med(t)});
  }
  // doorbell: one resident kernel; idle exit after 20 ms (100 MHz ticks)
  ctl->doorbell = seq;
  hipLaunchKernelGGL(k_resident, dim3(1), dim3(kThreads), 0, st, din, dout, w0, w1, dctl, seq, 2000000ull);
  for (int i = 0; i < iters; ++i) {
    auto t0 = now();
    pack();
    const unsigned long long s = ++seq;
    std::atomic_thread_fence(std::memory_order_release);
    ((volatile unsigned long long*)&ctl->doorbell)[0] = s;
    wait_done(s);
    memcpy(res.data(), hout, P * 4);
    t_bell.push_back(us(t0, now()));
  }
  check("doorbell");
  ((volatile unsigned long long*)&ctl->stop)[0] = 1;
  CK(hipStreamSynchronize(st));
  ctl->stop = 0;
  // cold doorbell: the kernel launched per round together with the ring (after its idle exit)
  for (int i = 0; i < 200; ++i) {
    auto t0 = now();
    pack();
    const unsigned long long s = ++seq;
    ((volatile unsigned long long*)&ctl->doorbell)[0] = s;
    hipLaunchKernelGGL(k_resident, dim3(1), dim3(kThreads), 0, st, din, dout, w0, w1, dctl, s - 1, 100000ull);
    wait_done(s);
    memcpy(res.data(), hout, P * 4);
    t_cold.push_back(us(t0, now()));
    ((volatile unsigned long long*)&ctl->stop)[0] = 1;
    CK(hipStreamSynchronize(st));
    ctl->stop = 0;
  }
  check("cold");
  auto pk = [&] {
    std::vector<double> v;
    for (int i = 0; i < iters; ++i) {
      auto t0 = now();
      pack();
      memcpy(res.data(), hout, P * 4);
      v.push_back(us(t0, now()));
    }
    return med(v);
  };
  printf("{\"launch_event_us\": %.2f, \"launch_flag_us\": %.2f, \"doorbell_us\": %.2f, \"doorbell_cold_us\": %.2f, "
         "\"pack_copy_only_us\": %.2f, \"iters\": %d, \"launch_flag_by_workgroups_us\": {",
         med(t_ev), med(t_flag), med(t_bell), med(t_cold), pk(), iters);
  for (size_t i = 0; i < t_multi.size(); ++i)
    printf("%s\"%d\": %.2f", i ? ", " : "", t_multi[i].first, t_multi[i].second);
  printf("}}\n");
  CK(hipHostFree(hb));
  return 0;
}
