// mt_poly.h -- host-side GF(2) polynomial arithmetic for MT19937 jump-ahead (plain C++, no HIP).
//
// numpy's legacy RandomState is MT19937: the 19,937-bit state advances by a fixed F2-linear map F
// (one 32-bit word of the output sequence x_t per step).  With phi the characteristic polynomial of F
// and g(x) = x^J mod phi, the state J steps ahead is g(F) applied to the current one; as the state
// after i steps is the window (x_i, ..., x_{i+623}) of the sequence, word j of the state J steps past
// the window at 0 is  XOR_{i : g_i = 1} x_{i+j}  (j = 0..623; only word 0's top bit is state).  The
// device computes that correlation (finite.hip, k_mt_jump); this header finds phi (Berlekamp-Massey
// on one bit of the sequence, computed once) and the jump polynomials x^(cJ) mod phi.
#pragma once

#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

namespace fa_mt {

constexpr int kDeg = 19937;                // degree of phi (the state dimension)
constexpr int kPolyWords = (kDeg + 64) / 64;  // 312 words hold a polynomial of degree <= 19937
using Poly = std::vector<uint64_t>;

inline int get_bit(const Poly& p, int i) { return (int)((p[(size_t)i >> 6] >> (i & 63)) & 1u); }
inline void flip_bit(Poly& p, int i) { p[(size_t)i >> 6] ^= 1ull << (i & 63); }

// numpy's mt19937 word sequence x_0, x_1, ... from init_genrand(seed): x_0..x_623 the seeded state,
// x_t = x_{t-227} ^ twist(x_{t-624}, x_{t-623}) after that.
inline void mt_sequence(uint32_t seed, std::vector<uint32_t>& x, size_t n) {
  x.resize(std::max<size_t>(n, 624));
  uint32_t v = seed;
  for (int i = 0; i < 624; ++i) {
    x[i] = v;
    v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)(i + 1);
  }
  for (size_t t = 624; t < n; ++t) {
    const uint32_t y = (x[t - 624] & 0x80000000u) | (x[t - 623] & 0x7fffffffu);
    x[t] = x[t - 227] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
}

// Berlekamp-Massey over GF(2) on the top bit of x_t (a linear function of the state at step t; the
// low 31 bits of x_0 are not state): the minimal polynomial of that bit sequence, which for MT19937
// (phi irreducible) is phi itself.  Returned as phi_k = coefficient of x^k.
inline Poly charpoly_compute() {
  const int N = 2 * kDeg + 128;
  std::vector<uint32_t> x;
  mt_sequence(5489u, x, (size_t)N);
  const int RW = (N + 63) / 64 + 2;
  std::vector<uint64_t> R((size_t)RW, 0);  // R[k] = s_{N-1-k}
  for (int k = 0; k < N; ++k)
    if (x[(size_t)(N - 1 - k)] >> 31) R[(size_t)k >> 6] |= 1ull << (k & 63);
  const int CW = (N + 63) / 64 + 2;
  std::vector<uint64_t> C((size_t)CW, 0), B((size_t)CW, 0), T;
  C[0] = B[0] = 1;
  int L = 0, m = 1;
  for (int n = 0; n < N; ++n) {
    // d = XOR_{i=0..L} c_i s_{n-i} = parity(C & (R >> base)), base = N-1-n
    const int base = N - 1 - n, bw = base >> 6, bs = base & 63;
    uint64_t acc = 0;
    const int words = (L >> 6) + 1;
    for (int w = 0; w < words; ++w) {
      uint64_t r = R[(size_t)(bw + w)] >> bs;
      if (bs) r |= R[(size_t)(bw + w + 1)] << (64 - bs);
      acc ^= C[(size_t)w] & r;
    }
    if (!__builtin_parityll(acc)) {
      ++m;
      continue;
    }
    const bool grow = 2 * L <= n;
    if (grow) T = C;
    // C ^= B << m
    const int ws = m >> 6, bsh = m & 63;
    for (int w = CW - 1; w >= ws; --w) {
      uint64_t v = B[(size_t)(w - ws)] << bsh;
      if (bsh && w - ws - 1 >= 0) v |= B[(size_t)(w - ws - 1)] >> (64 - bsh);
      C[(size_t)w] ^= v;
    }
    if (grow) {
      L = n + 1 - L;
      B = T;
      m = 1;
    } else {
      ++m;
    }
  }
  Poly phi((size_t)kPolyWords, 0);
  if (L != kDeg) return Poly();  // not MT19937's state dimension: refuse (caller reports)
  for (int k = 0; k <= L; ++k)  // phi_k = c_{L-k}
    if ((C[(size_t)(L - k) >> 6] >> ((L - k) & 63)) & 1u) flip_bit(phi, k);
  return phi;
}

inline const Poly& charpoly() {
  static std::once_flag once;
  static Poly phi;
  std::call_once(once, [] { phi = charpoly_compute(); });
  return phi;
}

// terms of phi below x^19937 (phi is sparse: reduction flips these bits per set high bit)
inline const std::vector<int>& charpoly_terms() {
  static std::once_flag once;
  static std::vector<int> t;
  std::call_once(once, [] {
    const Poly& p = charpoly();
    if (p.empty()) return;
    for (int k = 0; k < kDeg; ++k)
      if (get_bit(p, k)) t.push_back(k);
  });
  return t;
}

// a (degree < 2*19937) reduced mod phi in place; returns the low kPolyWords words
inline Poly reduce(std::vector<uint64_t>& a) {
  const std::vector<int>& terms = charpoly_terms();
  const int top = (int)a.size() * 64 - 1;
  for (int d = top; d >= kDeg; --d) {
    if (!((a[(size_t)d >> 6] >> (d & 63)) & 1u)) continue;
    a[(size_t)d >> 6] ^= 1ull << (d & 63);  // x^d = x^(d-19937) * (phi - x^19937)
    const int s = d - kDeg;
    for (int k : terms) {
      const int b = s + k;
      a[(size_t)b >> 6] ^= 1ull << (b & 63);
    }
  }
  a.resize((size_t)kPolyWords);
  return a;
}

// carry-less product of two kPolyWords-word polynomials into p (2 * kPolyWords + 1 words)
__attribute__((target("pclmul,sse2"))) inline void clmul_pclmul(const Poly& a, const Poly& b, uint64_t* p) {
  typedef long long v2di __attribute__((vector_size(16)));
  for (int i = 0; i < kPolyWords; ++i) {
    if (!a[(size_t)i]) continue;
    const v2di av = {(long long)a[(size_t)i], 0};
    for (int j = 0; j < kPolyWords; ++j) {
      if (!b[(size_t)j]) continue;
      const v2di bv = {(long long)b[(size_t)j], 0};
      const v2di r = __builtin_ia32_pclmulqdq128(av, bv, 0x00);
      p[i + j] ^= (uint64_t)r[0];
      p[i + j + 1] ^= (uint64_t)r[1];
    }
  }
}
inline void clmul_table(const Poly& a, const Poly& b, uint64_t* p) {  // 4-bit windows of a
  std::vector<uint64_t> t((size_t)16 * (kPolyWords + 1), 0);  // t[k] = b * k (k < 16)
  for (int k = 1; k < 16; ++k)
    for (int bit = 0; bit < 4; ++bit)
      if (k >> bit & 1)
        for (int w = 0; w <= kPolyWords; ++w) {
          uint64_t v = (w < kPolyWords ? b[(size_t)w] << bit : 0);
          if (bit && w > 0) v |= b[(size_t)w - 1] >> (64 - bit);
          t[(size_t)k * (kPolyWords + 1) + w] ^= v;
        }
  for (int i = 0; i < kPolyWords; ++i)
    for (int q = 0; q < 16; ++q) {
      const int k = (int)(a[(size_t)i] >> (4 * q) & 15u);
      if (!k) continue;
      const int sh = 4 * q;
      const uint64_t* tk = &t[(size_t)k * (kPolyWords + 1)];
      for (int w = 0; w <= kPolyWords; ++w) {
        p[i + w] ^= tk[w] << sh;
        if (sh) p[i + w + 1] ^= tk[w] >> (64 - sh);
      }
    }
}

inline Poly mulmod(const Poly& a, const Poly& b) {
  std::vector<uint64_t> p((size_t)(2 * kPolyWords + 2), 0);
  static const bool has_pclmul = __builtin_cpu_supports("pclmul");
  if (has_pclmul) clmul_pclmul(a, b, p.data());
  else clmul_table(a, b, p.data());
  return reduce(p);
}

// x^e mod phi by square-and-multiply (e >= 0)
inline Poly xpow(uint64_t e) {
  Poly r((size_t)kPolyWords, 0), base((size_t)kPolyWords, 0);
  r[0] = 1;
  base[0] = 2;  // x
  while (e) {
    if (e & 1) r = mulmod(r, base);
    e >>= 1;
    if (e) base = mulmod(base, base);
  }
  return r;
}

// Jump polynomials x^(c*J) mod phi for c = 1..count, cached per J (they depend on J only).  Returns a
// COPY of the first `count`, made under the lock: another context may grow the cache (and move its
// storage) while the caller reads them.
inline std::vector<Poly> jump_polys(uint64_t J, int count) {
  static std::mutex mu;
  static std::vector<std::pair<uint64_t, std::vector<Poly>>> cache;
  std::lock_guard<std::mutex> lk(mu);
  std::vector<Poly>* v = nullptr;
  for (auto& e : cache)
    if (e.first == J) v = &e.second;
  if (!v) {
    cache.emplace_back(J, std::vector<Poly>());
    v = &cache.back().second;
  }
  if ((int)v->size() < count) {
    if (v->empty()) v->push_back(xpow(J));
    const Poly g1 = (*v)[0];
    while ((int)v->size() < count) v->push_back(mulmod(v->back(), g1));
  }
  return std::vector<Poly>(v->begin(), v->begin() + std::max(0, count));
}

}  // namespace fa_mt
