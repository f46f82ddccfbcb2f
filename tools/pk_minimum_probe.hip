// Probe (r03al): does __builtin_elementwise_minimum / maximum on two-float16 vectors (gfx950:
// v_pk_minimum3_f16 / v_pk_maximum3_f16 with a repeated operand) compute the IEEE 754-2019 minimum /
// maximum of each half?  Random pairs of float16 bit patterns (finite, +-0, +-inf, NaN, subnormal);
// host reference per half; prints the mismatch count per op and the first few mismatches.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__global__ void k_pk(const h2* a, const h2* b, h2* mn, h2* mx, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  mn[i] = __builtin_elementwise_minimum(a[i], b[i]);
  mx[i] = __builtin_elementwise_maximum(a[i], b[i]);
}

// three distinct operands: the compiler fuses min(min(a, b), c) into one v_pk_minimum3_f16
__global__ void k_pk3(const h2* a, const h2* b, const h2* c, h2* mn, h2* mx, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  mn[i] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(a[i], b[i]), c[i]);
  mx[i] = __builtin_elementwise_maximum(__builtin_elementwise_maximum(a[i], b[i]), c[i]);
}

static float h2f(unsigned short u) {
  _Float16 h;
  memcpy(&h, &u, 2);
  return (float)h;
}
static bool isnan16(unsigned short u) { return (u & 0x7FFF) > 0x7C00; }
// IEEE minimum: NaN if either is NaN; -0 < +0; else the smaller
static bool ref(unsigned short x, unsigned short y, bool want_min, unsigned short got) {
  if (isnan16(x) || isnan16(y)) return isnan16(got);
  const float fx = h2f(x), fy = h2f(y);
  unsigned short e;
  if (fx == fy) {  // equal values: only +-0 differ in bits
    const bool xneg = x & 0x8000;
    e = want_min ? (xneg ? x : y) : (xneg ? y : x);
  } else {
    e = (want_min ? fx < fy : fx > fy) ? x : y;
  }
  return got == e;
}

int main() {
  const int n = 1 << 16;
  std::vector<unsigned short> A(2 * n), B(2 * n);
  const unsigned short pats[] = {0x0000, 0x8000, 0x3800, 0xB800, 0x7C00, 0xFC00, 0x7E00, 0x0001, 0x8001, 0x3C00};
  srand(1);
  for (int i = 0; i < 2 * n; ++i) {
    A[i] = rand() % 3 ? pats[rand() % 10] : (unsigned short)rand();
    B[i] = rand() % 3 ? pats[rand() % 10] : (unsigned short)rand();
  }
  void *da, *db, *dmn, *dmx;
  (void)hipMalloc(&da, 4 * n);
  (void)hipMalloc(&db, 4 * n);
  (void)hipMalloc(&dmn, 4 * n);
  (void)hipMalloc(&dmx, 4 * n);
  (void)hipMemcpy(da, A.data(), 4 * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, B.data(), 4 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_pk, dim3(n / 256), dim3(256), 0, 0, (const h2*)da, (const h2*)db, (h2*)dmn, (h2*)dmx, n);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::vector<unsigned short> MN(2 * n), MX(2 * n);
  (void)hipMemcpy(MN.data(), dmn, 4 * n, hipMemcpyDeviceToHost);
  (void)hipMemcpy(MX.data(), dmx, 4 * n, hipMemcpyDeviceToHost);
  int bad_mn = 0, bad_mx = 0, shown = 0;
  for (int i = 0; i < 2 * n; ++i) {
    const bool okn = ref(A[i], B[i], true, MN[i]), okx = ref(A[i], B[i], false, MX[i]);
    bad_mn += !okn;
    bad_mx += !okx;
    if ((!okn || !okx) && shown < 8) {
      printf("half %d: a=%04x b=%04x min=%04x max=%04x\n", i & 1, A[i], B[i], MN[i], MX[i]);
      ++shown;
    }
  }
  printf("{\"pairs\": %d, \"min_mismatch\": %d, \"max_mismatch\": %d}\n", 2 * n, bad_mn, bad_mx);
  // three operands: reference = two chained two-operand results (already checked above)
  std::vector<unsigned short> C(2 * n);
  for (int i = 0; i < 2 * n; ++i) C[i] = rand() % 3 ? pats[rand() % 10] : (unsigned short)rand();
  void *dc, *dmn3, *dmx3;
  (void)hipMalloc(&dc, 4 * n);
  (void)hipMalloc(&dmn3, 4 * n);
  (void)hipMalloc(&dmx3, 4 * n);
  (void)hipMemcpy(dc, C.data(), 4 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_pk3, dim3(n / 256), dim3(256), 0, 0, (const h2*)da, (const h2*)db, (const h2*)dc, (h2*)dmn3,
                     (h2*)dmx3, n);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::vector<unsigned short> MN3(2 * n), MX3(2 * n);
  (void)hipMemcpy(MN3.data(), dmn3, 4 * n, hipMemcpyDeviceToHost);
  (void)hipMemcpy(MX3.data(), dmx3, 4 * n, hipMemcpyDeviceToHost);
  int bad3n = 0, bad3x = 0;
  shown = 0;
  for (int i = 0; i < 2 * n; ++i) {
    const bool okn = ref(MN[i], C[i], true, MN3[i]), okx = ref(MX[i], C[i], false, MX3[i]);
    bad3n += !okn;
    bad3x += !okx;
    if ((!okn || !okx) && shown < 8) {
      printf("3-op half %d: a=%04x b=%04x c=%04x min3=%04x max3=%04x\n", i & 1, A[i], B[i], C[i], MN3[i], MX3[i]);
      ++shown;
    }
  }
  printf("{\"triples\": %d, \"min3_mismatch\": %d, \"max3_mismatch\": %d}\n", 2 * n, bad3n, bad3x);
  return 0;
}
