// pairrot.hip -- k_pairdist_rot: Krum's pairwise squared distances (krum_defense.py:50-66,
// compute_euclidean_distance = (v_i - v_j).norm()) with the pair differences formed by DPP row
// rotation.  Launched by fa_pairwise_sqdist_rt (robust.hip) for float32-run dtypes.
//
// Built WITHOUT SLP vectorization (Makefile): the vectorizer pairs neighbouring scalar sub / fma into
// v_pk_add_f32 / v_pk_fma_f32, which take no DPP operand, and the rotation then costs a separate
// v_mov_b32_dpp per difference.  As scalars, the compiler folds the v_mov_b32_dpp into the v_sub_f32,
// so a pair-coordinate is exactly one v_sub_f32_dpp + one v_fmac_f32 -- the VALU floor of the metric.
//
// Why: the LDS tile kernels (robust.hip) stage [coordinate][client] tiles and spend most of their
// VALU issue on operand movement (r04d PMC: about 27% of the sub + fma floor at K = 32).
//
// Layout.  A wave is 4 rows x 16 lanes.  Lane r of every row holds client 16g + r of a client group
// g (16 clients), row q its own coordinates: per step (`unit`, 16 coordinates) lane (q, r) loads
// coordinates 4q..4q+3 of the unit, one 16-byte load per group.  row_ror:(16 - d) gives lane r the
// value of lane (r + d) & 15 of the same row inside the subtraction:
//   cross pair of groups (a, b), a < b:  t = rot_d(x_b) - x_a, d = 0..15 -> 256 pairs, 16 rotations;
//   within group g:                      t = rot_d(x_g) - x_g, d = 1..8  -> 120 pairs (d = 8: r < 8).
// A wave owns two SLOTS of 16 accumulators: a slot is one cross pair of groups or two groups' within
// pairs.  Tasks: G(G-1)/2 cross + ceil(G/2) within slots, G = ceil(K / 16) -- K = 32: 2 slots, one
// wave; K = 128: 32 slots, 16 waves.  The waves of a task set read the same lines (L1 / L2); `reps`
// replicas of the set split a workgroup's units.
//
// Precision: float32 runs of <= kPairRun coordinates per lane; at each flush the 4 rows' runs are
// added across rows (permlane16 / permlane32 swaps, so every row holds the same sum) and each row
// keeps a quarter of the slot accumulators in float64 -- 16 VGPRs of float64 sums instead of 64.
// Rows, replicas and workgroups are added in a fixed order: the result is deterministic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <utility>

#include "fa_internal.h"
#include "pair_seg.h"

namespace fa_detail {

RotSplit rot_split(int k) {
  RotSplit s;
  s.G = (k + 15) / 16;
  s.nslots = s.G * (s.G - 1) / 2 + (s.G + 1) / 2;
  s.wpt = (s.nslots + 1) / 2;
  // replicas of the task set per workgroup: about 4 waves at small K (FA_PAIR_ROT_R overrides)
  static const int ov = [] {
    const char* e = getenv("FA_PAIR_ROT_R");
    return e ? atoi(e) : 0;
  }();
  s.reps = ov >= 1 ? ov : std::max(1, 4 / s.wpt);
  while (s.reps > 1 && s.reps * s.wpt > 16) --s.reps;
  s.nthreads = 64 * s.wpt * s.reps;
  return s;
}

namespace {

__device__ __forceinline__ int64_t pair_index(int i, int j, int k) {  // i < j
  return (int64_t)i * k - (int64_t)i * (i + 1) / 2 + (j - i - 1);
}

template <int RT>
__device__ __forceinline__ float rdiff(float d) {
  if constexpr (RT == 1) return (float)(__bf16)d;
  else if constexpr (RT == 2) return (float)(_Float16)d;
  else return d;
}

// lane r of each 16-lane row <- lane (r + D) & 15 of the same row (row_ror:(16 - D))
template <int D>
__device__ __forceinline__ float rot16(float v) {
  if constexpr (D == 0) return v;
  else return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x120 + (16 - D), 0xf, 0xf, true));
}

// Software-pipelined: the next difference is formed before this one's fma, so v_sub_f32_dpp and
// v_fmac_f32 alternate and consecutive differences use two temporaries.  One temporary reused by
// back-to-back (sub_dpp, fma) pairs costs an s_nop per pair (the DPP instruction's tied destination
// was written by the previous VALU op); r04g/r04k probe (tools/dpp_rate_probe.hip): see DESIGN.md.
template <int RT, int O, int D, int N, int S>  // S: first rotation (0 cross, 1 within)
__device__ __forceinline__ void rot_pipe(float a, float b, float t, float* acc) {
  if constexpr (D + 1 < N) {
    const float tn = rdiff<RT>(rot16<S + D + 1>(b) - a);
    acc[O + D] = __builtin_fmaf(t, t, acc[O + D]);
    rot_pipe<RT, O, D + 1, N, S>(a, b, tn, acc);
  } else {
    acc[O + D] = __builtin_fmaf(t, t, acc[O + D]);
  }
}
// acc[O + d] += (rot_d(b) - a)^2, d = 0..15
template <int RT, int O>
__device__ __forceinline__ void rot_cross(float a, float b, float* acc) {
  rot_pipe<RT, O, 0, 16, 0>(a, b, rdiff<RT>(b - a), acc);
}
// acc[O + d - 1] += (rot_d(a) - a)^2, d = 1..8.  The rotated operand goes through an opaque copy: a
// group's rotations feed both its within and a cross slot, and a shared v_mov_b32_dpp (CSE) could no
// longer fold into either subtraction
template <int RT, int O>
__device__ __forceinline__ void rot_within(float a, float* acc) {
  float b;
  asm("" : "=v"(b) : "0"(a));
  rot_pipe<RT, O, 0, 8, 1>(a, b, rdiff<RT>(rot16<1>(b) - a), acc);
}

// slot s of the task list -> groups (a, b) and kind; a = -1: no task (the last wave's spare slot)
__device__ __forceinline__ void rot_slot(int s, int G, int& a, int& b, bool& cross) {
  const int nx = G * (G - 1) / 2;
  cross = s < nx;
  if (cross) {
    int i = 0, rem = s;
    while (rem >= G - 1 - i) { rem -= G - 1 - i; ++i; }
    a = i;
    b = i + 1 + rem;
  } else if (s < nx + (G + 1) / 2) {
    a = 2 * (s - nx);
    b = a + 1 < G ? a + 1 : -1;
  } else {
    a = b = -1;
  }
}

// accumulator m of slot (a, b, cross) on lane r -> pair (i, j), i < j; false: not a pair of this K
// (every pair i < j < K is produced by exactly one (slot, r, m): tests/test_pair_rot_map.py)
__device__ __forceinline__ bool rot_pair(int a, int b, bool cross, int r, int m, int k, int& i, int& j) {
  if (a < 0) return false;
  if (cross) {
    i = 16 * a + r;
    j = 16 * b + ((r + m) & 15);
    return j < k;
  }
  const int g = m < 8 ? a : b, d = m < 8 ? m + 1 : m - 7;
  if (g < 0 || (d == 8 && r >= 8)) return false;
  const int x = 16 * g + r, y = 16 * g + ((r + d) & 15);
  i = x < y ? x : y;
  j = x < y ? y : x;
  return j < k;
}

__device__ __forceinline__ float row_sum4(float v) {  // the sum over the wave's 4 rows, on every row
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  auto p2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(p2[0]) + __uint_as_float(p2[1]);
}

// SMALL: K <= 32 (G <= 2) -- every wave holds both groups (one 16-byte load per group and unit, no
// duplicate loads) and does all 32 accumulators (cross 0-1, within 0, within 1); P units in flight per
// wave (ring of P register buffers).  Otherwise the task slots above, two units in flight.
template <bool VEC, int RT, bool SMALL, int P>
__global__ void __launch_bounds__(1024)
k_pairdist_rot(const PSeg* __restrict__ segs, int nseg, const void* const* __restrict__ ptrs, int k, int G,
               int wpt, int64_t nunits, double* __restrict__ partial, int dbg) {
  extern __shared__ double red[];  // [waves][32 accumulators][16 lanes]
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  const int q = lane >> 4, r = lane & 15;
  const int R = (int)(blockDim.x >> 6) / wpt;
  const int rep = wid / wpt, wv = wid % wpt;
  int sa[2], sb[2];
  bool sx[2];
  rot_slot(2 * wv, G, sa[0], sb[0], sx[0]);
  rot_slot(2 * wv + 1, G, sa[1], sb[1], sx[1]);
  // groups this wave loads: NL = 2 (SMALL: groups 0, 1) or 4 (slot j: groups sa[j], sb[j]); a lane whose
  // client is past K, or whose slot has no group, reads client 0's data -- it only feeds accumulators
  // of pairs that are never written
  constexpr int NL = SMALL ? 2 : 4;
  int cl[NL];
#pragma unroll
  for (int g = 0; g < NL; ++g) {
    const int grp = SMALL ? g : (g & 1 ? sb[g >> 1] : sa[g >> 1]);
    cl[g] = grp >= 0 && 16 * grp + r < k ? 16 * grp + r : 0;
  }
  float acc[32];
  double accd[8];  // row q: accumulators 8q .. 8q + 7
#pragma unroll
  for (int m = 0; m < 32; ++m) acc[m] = 0.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i) accd[i] = 0.0;
  auto flush = [&]() {
    float s[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) {
      s[m] = row_sum4(acc[m]);
      acc[m] = 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float v = q == 0 ? s[i] : q == 1 ? s[8 + i] : q == 2 ? s[16 + i] : s[24 + i];
      accd[i] += (double)v;
    }
  };
  const bool act0 = sa[0] >= 0, act1 = sa[1] >= 0, two = G > 1;
  // accumulators: slot j at 16 j; a cross slot d = 0..15, a within slot group a d = 1..8 at 0..7 and
  // group b at 8..15 (the slot layout of rot_pair)
  auto compute = [&](const float (&x)[NL][4]) {
    if constexpr (SMALL) {
      if (two) {  // slot 0 = cross (0, 1), slot 1 = within (0, 1)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          rot_cross<RT, 0>(x[0][e], x[1][e], acc);
          rot_within<RT, 16>(x[0][e], acc);
          rot_within<RT, 24>(x[1][e], acc);
        }
      } else {  // K <= 16: slot 0 = within (0)
#pragma unroll
        for (int e = 0; e < 4; ++e) rot_within<RT, 0>(x[0][e], acc);
      }
    } else {
      auto slot = [&](auto J) {
        constexpr int j = decltype(J)::value;
        if (!(j == 0 ? act0 : act1)) return;
        if (sx[j]) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            rot_cross<RT, 16 * j>(x[2 * j][e], x[2 * j + 1][e], acc);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            rot_within<RT, 16 * j>(x[2 * j][e], acc);
            rot_within<RT, 16 * j + 8>(x[2 * j + 1][e], acc);
          }
        }
      };
      slot(std::integral_constant<int, 0>{});
      slot(std::integral_constant<int, 1>{});
    }
  };
  int run = 0;
  auto step = [&]() {
    run += 4;
    if (run + 4 > kPairRun) {
      flush();
      run = 0;
    }
  };
  typedef const __attribute__((address_space(1))) float* gptr;
  // each workgroup takes a contiguous run of units [u0, u1); replica `rep` the units u0 + rep + n R.
  // Per segment: client pointers once, the units wholly inside the segment by unconditional loads
  // P - 1 units ahead, then the segment's partial last unit with guarded loads.
  const int64_t u0 = nunits * blockIdx.x / gridDim.x, u1 = nunits * (blockIdx.x + 1) / gridDim.x;
  for (int si = nseg > 1 && u0 < u1 ? find_seg(segs, nseg, u0) : 0; si < nseg && u0 < u1; ++si) {
    const PSeg sg = segs[si];
    if (sg.tile_start >= u1) break;
    const int64_t nfull = sg.numel / kRotUnit, send = sg.tile_start + (sg.numel + kRotUnit - 1) / kRotUnit;
    const int64_t lo = std::max(u0, sg.tile_start), hi = std::min(u1, send);
    if (lo >= hi) continue;
    const float* pc[NL];
#pragma unroll
    for (int g = 0; g < NL; ++g) pc[g] = (const float*)ptrs[sg.ptr_base + cl[g]];
    const int64_t first = lo + (((rep - (lo - u0)) % R) + R) % R;  // my first unit in [lo, hi)
    const int64_t fend = std::min(hi, sg.tile_start + nfull);       // end of the whole units
    const int64_t n = first < fend ? (fend - 1 - first) / R + 1 : 0;
    auto load = [&](int64_t t, float (&x)[NL][4]) {  // my t-th whole unit (clamped to n - 1)
      t = t < n ? t : n - 1;
      const int64_t e0 = (first + (dbg == 1 ? 0 : t) * R - sg.tile_start) * kRotUnit + 4 * q;
#pragma unroll
      for (int g = 0; g < NL; ++g) {
        if constexpr (VEC) {
          typedef float f32x4 __attribute__((ext_vector_type(4)));
          const f32x4 v = *(const __attribute__((address_space(1))) f32x4*)(pc[g] + e0);
          x[g][0] = v.x;
          x[g][1] = v.y;
          x[g][2] = v.z;
          x[g][3] = v.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[g][e] = ((gptr)pc[g])[e0 + e];
        }
      }
    };
    if (n > 0) {
      // a ring of P register buffers, no load under a branch (exact vmcnt waits); the clamped index
      // re-reads the last unit (a cache hit) instead of branching
      float buf[P][NL][4];
#pragma unroll
      for (int s = 0; s < P - 1; ++s) load(s, buf[s]);
      for (int64_t t = 0; t < n; t += P) {
#pragma unroll
        for (int s = 0; s < P; ++s) {
          load(t + s + P - 1, buf[(s + P - 1) % P]);
          if (t + s < n) {
            if (dbg == 2) {
#pragma unroll
              for (int g = 0; g < NL; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[4 * g + e] += buf[s][g][e];
            } else {
              compute(buf[s]);
            }
            step();
          }
        }
      }
    }
    // the partial last unit of the segment, if it falls in [lo, hi) and to this replica
    const int64_t tail = sg.tile_start + nfull;
    if (nfull * kRotUnit < sg.numel && tail >= lo && tail < hi && (tail - u0) % R == rep) {
      const int64_t e0 = nfull * kRotUnit + 4 * q;
      float x[NL][4];
#pragma unroll
      for (int g = 0; g < NL; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool in = e0 + e < sg.numel;
          const float v = ((gptr)pc[g])[in ? e0 + e : sg.numel - 1];
          x[g][e] = in ? v : 0.0f;
        }
      compute(x);
      step();
    }
  }
  flush();
  // LDS [wave][accumulator 8q + i][lane r]; then per (slot, r, m) the replicas in order
#pragma unroll
  for (int i = 0; i < 8; ++i) red[((int64_t)wid * 32 + 8 * q + i) * 16 + r] = accd[i];
  __syncthreads();
  double* out = partial + (int64_t)blockIdx.x * ((int64_t)k * (k - 1) / 2);
  for (int idx = threadIdx.x; idx < wpt * 512; idx += (int)blockDim.x) {
    const int rr = idx & 15, m = (idx >> 4) & 15, js = idx >> 8;  // js = wave-in-set * 2 + slot
    int a, b, i, j;
    bool x;
    rot_slot(js, G, a, b, x);
    if (!rot_pair(a, b, x, rr, m, k, i, j)) continue;
    double s = 0.0;
    for (int p = 0; p < R; ++p) s += red[((int64_t)(p * wpt + (js >> 1)) * 32 + 16 * (js & 1) + m) * 16 + rr];
    out[pair_index(i, j, k)] = s;
  }
}

}  // namespace

int launch_pairdist_rot(int k, int rt, bool vec, int nblocks, const PSeg* segs, int nseg,
                        const void* const* ptrs, int64_t nunits, double* partial, hipStream_t st) {
  const RotSplit rs = rot_split(k);
  const size_t lds = sizeof(double) * 512 * (size_t)(rs.nthreads / 64);
  // K <= 32: units in flight per wave (FA_PAIR_ROT_P = 2 / 3 / 4 for float32 differences, A/B; r04i:
  // 2, 3 and 4 within 2% of each other)
  static const int pdepth = [] {
    const char* e = getenv("FA_PAIR_ROT_P");
    const int v = e ? atoi(e) : 0;
    return v >= 2 && v <= 4 ? v : 2;
  }();
  static const int dbg = [] {  // TEMPORARY measurement switch: 1 = cache-resident loads, 2 = no pair math
    const char* e = getenv("FA_PAIR_ROT_DBG");
    return e ? atoi(e) : 0;
  }();
#define FA_PDR(V, R, S, P) hipLaunchKernelGGL((k_pairdist_rot<V, R, S, P>), dim3((unsigned)nblocks), \
    dim3((unsigned)rs.nthreads), lds, st, segs, nseg, ptrs, k, rs.G, rs.wpt, nunits, partial, dbg)
  if (rs.G <= 2) {
    if (vec && rt == 0) {
      if (pdepth == 3) FA_PDR(true, 0, true, 3); else if (pdepth == 4) FA_PDR(true, 0, true, 4); else FA_PDR(true, 0, true, 2);
    } else if (vec) {
      if (rt == 1) FA_PDR(true, 1, true, 2); else FA_PDR(true, 2, true, 2);
    } else {
      if (rt == 1) FA_PDR(false, 1, true, 2); else if (rt == 2) FA_PDR(false, 2, true, 2); else FA_PDR(false, 0, true, 2);
    }
  } else if (vec) {
    if (rt == 1) FA_PDR(true, 1, false, 2); else if (rt == 2) FA_PDR(true, 2, false, 2); else FA_PDR(true, 0, false, 2);
  } else {
    if (rt == 1) FA_PDR(false, 1, false, 2); else if (rt == 2) FA_PDR(false, 2, false, 2); else FA_PDR(false, 0, false, 2);
  }
#undef FA_PDR
  return (int)hipGetLastError();
}

}  // namespace fa_detail
