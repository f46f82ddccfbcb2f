// CPU check of fedml_amd/csrc/mt_poly.h (tests/test_mt_jump.py builds and runs it):
//   1. phi from Berlekamp-Massey has degree 19937 and annihilates every bit of the sequence;
//   2. the window J words ahead, from the correlation XOR_{i: g_i} x_{i+j} with g = x^J mod phi,
//      equals the sequentially generated window (words 1..623 exactly, word 0's top bit);
//   3. x^(cJ) from jump_polys() equals xpow(c*J);
// then prints the one-time host cost of the polynomials for the device path's chunk size.
// g++ -O2 -std=c++17 -I fedml_amd/csrc tools/mt_jump_check.cpp -o mt_jump_check
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include <thread>

#include "mt_poly.h"

using namespace fa_mt;

static bool check_window(uint32_t seed, uint64_t J) {
  std::vector<uint32_t> x;
  mt_sequence(seed, x, (size_t)(J + 624 + 19937 + 624));
  const Poly g = xpow(J);
  std::vector<uint32_t> w(624, 0);
  for (int i = 0; i < kDeg; ++i)
    if (get_bit(g, i))
      for (int j = 0; j < 624; ++j) w[j] ^= x[(size_t)(i + j)];
  if ((w[0] ^ x[J]) & 0x80000000u) return false;
  for (int j = 1; j < 624; ++j)
    if (w[j] != x[J + j]) return false;
  return true;
}

int main(int argc, char** argv) {
  auto t0 = std::chrono::steady_clock::now();
  const Poly& phi = charpoly();
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  auto t1 = std::chrono::steady_clock::now();
  if (phi.empty()) {
    printf("FAIL: Berlekamp-Massey did not find a degree-19937 polynomial\n");
    return 1;
  }
  int weight = 0;
  for (int k = 0; k <= kDeg; ++k) weight += get_bit(phi, k);
  // 1. phi annihilates all 32 bit planes of the sequence
  std::vector<uint32_t> x;
  mt_sequence(12345u, x, (size_t)(kDeg + 2000));
  for (int t = 1; t < 1000; t += 97) {  // x_0's low 31 bits are not state: from t = 1
    uint32_t acc = 0;
    for (int k = 0; k <= kDeg; ++k)
      if (get_bit(phi, k)) acc ^= x[(size_t)(t + k)];
    if (acc != 0) {
      printf("FAIL: phi does not annihilate the sequence at t=%d (0x%08x)\n", t, acc);
      return 1;
    }
  }
  // 2. jumps by J against sequential generation
  const uint64_t Js[] = {1, 623, 624, 1000, 624 * 3, 12345, 624 * 64};
  const uint32_t seeds[] = {0u, 1u, 5489u, 4294967295u, 2718281828u};
  for (uint64_t J : Js)
    for (uint32_t s : seeds)
      if (!check_window(s, J)) {
        printf("FAIL: window after J=%llu from seed %u\n", (unsigned long long)J, s);
        return 1;
      }
  // 3. both carry-less products agree; the cached multiples
  {
    const Poly a = xpow(123456789ull), b = xpow(987654321ull);
    std::vector<uint64_t> p1((size_t)(2 * kPolyWords + 2), 0), p2 = p1;
    clmul_table(a, b, p2.data());
    if (__builtin_cpu_supports("pclmul")) {
      clmul_pclmul(a, b, p1.data());
      if (p1 != p2) {
        printf("FAIL: pclmul and table carry-less products differ\n");
        return 1;
      }
    }
  }
  const uint64_t J = 624 * 7;
  const std::vector<Poly>& v = jump_polys(J, 5);
  for (int c = 1; c <= 5; ++c)
    if (v[(size_t)c - 1] != xpow((uint64_t)c * J)) {
      printf("FAIL: jump_polys(%llu)[%d] != x^(c J)\n", (unsigned long long)J, c);
      return 1;
    }
  // 4. two threads (two contexts' calls) growing the cache for different J at once: each gets its own
  //    copy, equal to the sequential powers (the copy is taken under the cache's lock)
  {
    const uint64_t Ja = 624 * 3, Jb = 624 * 11;
    std::vector<Poly> ra, rb;
    std::thread ta([&] { for (int c = 1; c <= 24; c += 3) ra = jump_polys(Ja, c); });
    std::thread tb([&] { for (int c = 1; c <= 24; c += 3) rb = jump_polys(Jb, c); });
    ta.join();
    tb.join();
    for (int c = 1; c <= 22; ++c)
      if (ra[(size_t)c - 1] != xpow((uint64_t)c * Ja) || rb[(size_t)c - 1] != xpow((uint64_t)c * Jb)) {
        printf("FAIL: concurrent jump_polys differ at c = %d\n", c);
        return 1;
      }
  }
  auto t2 = std::chrono::steady_clock::now();
  const int n = argc > 1 ? atoi(argv[1]) : 0;  // optional: time n polynomials of the device chunk size
  double tp = 0;
  if (n > 0) {
    auto a = std::chrono::steady_clock::now();
    jump_polys(624ull << 10, n);
    tp = ms(a, std::chrono::steady_clock::now());
  }
  printf("{\"ok\": true, \"phi_weight\": %d, \"charpoly_ms\": %.1f, \"checks_ms\": %.1f, \"polys\": %d, "
         "\"polys_ms\": %.1f}\n", weight, ms(t0, t1), ms(t1, t2), n, tp);
  return 0;
}
