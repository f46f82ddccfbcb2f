/*
 * fedagg_robust.h -- C ABI of the robust-aggregation kernels (libfedagg.so), same context,
 * memory, stream and error conventions as fedagg.h.  Entries and the reference code each replaces
 * (paths relative to liuliuliu0605/FedML python/fedml/):
 *
 *   fa_coord_median     core/security/defense/coordinate_wise_median_defense.py:26-31
 *                       torch.median(torch.cat(client vectors, -1), dim=-1).values
 *   fa_coord_median_tiled  the same over tile-interleaved arena rows
 *   fa_pairwise_sqdist  core/security/defense/krum_defense.py:52-66 (_compute_krum_score's
 *                       compute_euclidean_distance(v_i, v_j) ** 2 for every pair)
 *   fa_pairwise_sqdist_rt  the same for bfloat16 / float16 models (differences in the model dtype)
 *   fa_pairwise_sqdist_gram  the same for float32 models in the Gram form (matrix cores, kappa-guarded)
 *   fa_pairwise_sqdist_gram_limit  the kappa limit that guard applies to an input (its error model)
 *
 * Contract (bit-exact; pinned by tests/golden/g16_*): for every element e, out[e] is the input
 * element (bit pattern) that ATen's median selects: the first NaN in client order if any client
 * holds a NaN there; otherwise the element of rank (k-1)/2 when the k values are ordered by
 * (value, client index), -0.0 == +0.0.  dtype: F32, BF16, F16, F64.
 *
 * fa_pairwise_sqdist is floating-point work whose summation order differs from the reference's
 * float32 `norm()` (itself order-dependent): D[i][j] = sum_e (x_i[e] - x_j[e])^2 with float32
 * differences, float32 sums over <= 64 coordinates, float64 above; relative error <= 1e-6 vs the
 * exact sum (tests/test_gpu_robust.py).  The Krum selection built on it is checked bit-for-bit
 * against the reference (tests/golden/g18_*).
 */
#ifndef FEDAGG_ROBUST_H
#define FEDAGG_ROBUST_H

#include <stddef.h>

#include "fedagg.h"

#ifdef __cplusplus
extern "C" {
#endif

/*
 * A whole (vectorized) state_dict in one launch: d_in[s * k + i] = client i's tensor of segment s
 * (seg_numel[s] elements of `dtype`), d_out[s] the median tensor of segment s.
 */
int fa_coord_median(fa_ctx *ctx, int dtype, int32_t num_segments, const int64_t *seg_numel, int32_t k,
                    const void *const *d_in, void *const *d_out, void *hip_stream);
/*
 * The same over TILE-INTERLEAVED client rows (fedml_amd/arena.py ClientArena(tiled=True), the
 * layout fa_weighted_sum_tiled reads): element e of client i's segment s is at
 * d_in[s * k + i] + (e / E) * tile_stride + (e % E) * sizeof(dtype), E = FA_TILE_BYTES / sizeof(dtype);
 * every d_in pointer is the start of a tile; tile_stride a positive multiple of FA_TILE_BYTES.
 * Same results, bit for bit, as fa_coord_median over the logical rows.
 */
int fa_coord_median_tiled(fa_ctx *ctx, int dtype, int32_t num_segments, const int64_t *seg_numel, int32_t k,
                          const void *const *d_in, int64_t tile_stride, void *const *d_out, void *hip_stream);

/*
 * Pairwise squared Euclidean distances of k float32 client vectors (2 <= k <= 128), each given
 * as num_segments pieces (d_in[s * k + i], seg_numel[s] elements): d_dist = k x k float64 device
 * matrix (symmetric, zero diagonal).  d_scratch: device buffer of at least
 * fa_pairwise_sqdist_scratch_bytes(...) bytes (per-block partial sums; caller-owned, reusable).
 */
int fa_pairwise_sqdist(fa_ctx *ctx, int32_t num_segments, const int64_t *seg_numel, int32_t k,
                       const void *const *d_in, void *d_dist, void *d_scratch, size_t scratch_bytes,
                       void *hip_stream);
/*
 * As fa_pairwise_sqdist, with every difference x_i[e] - x_j[e] rounded to `diff_dtype` before it is
 * squared: FA_DTYPE_F32 (no rounding; = fa_pairwise_sqdist), FA_DTYPE_BF16 or FA_DTYPE_F16 (round
 * to nearest even, overflow to inf).  Replaces the same loop for bfloat16 / float16 models, where
 * the reference's vectorize_weight (core/security/common/utils.py:8-13) keeps the model's dtype and
 * `(v1 - v2)` (utils.py:24-27) rounds each difference to it; the inputs stay float32 (the clients'
 * values widened exactly).  The caller rounds sqrt(D) to the same dtype to reproduce the
 * reference's `.norm()` result (the norm of a bf16/f16 tensor is returned in that dtype).
 * FA_DTYPE_F64: float64 models -- the inputs are FLOAT64 vectors and every difference, square and
 * sum is computed in float64 (the reference's vectorize_weight keeps float64 and `(v1 - v2).norm()`
 * runs in it; krum_defense.py:50-66).
 */
int fa_pairwise_sqdist_rt(fa_ctx *ctx, int diff_dtype, int32_t num_segments, const int64_t *seg_numel, int32_t k,
                          const void *const *d_in, void *d_dist, void *d_scratch, size_t scratch_bytes,
                          void *hip_stream);
size_t fa_pairwise_sqdist_scratch_bytes(int32_t num_segments, const int64_t *seg_numel, int32_t k);
/*
 * fa_pairwise_sqdist for float32 vectors in the Gram form on the matrix cores (r05):
 * D_ij = A_i + A_j - 2 G_ij over y_i = x_i - c (c: the per-coordinate median of clients 0..4), G = Y Y^T
 * on the f32-input MFMA (k <= 32 with 16-byte aligned clients: v_mfma_f32_16x16x4_f32 over the three
 * upper 16x16 tiles, chunks streamed by LDS-DMA; otherwise v_mfma_f32_32x32x2_f32 over the upper
 * 32x32 tiles; k in (32, 128] with 16-byte aligned clients (FA_GRAM3=0: off): y split exactly into three bf16 parts on the
 * bf16 MFMA), float32 runs of n = 64-256 products summed in float64.
 * Same d_dist layout (k x k float64, symmetric, zero diagonal).  The form cancels: its relative error
 * is ~ 0.30 kappa_ij u n / sqrt(P) (one sigma, u = 2^-24, P = total coordinates), kappa_ij =
 * (A_i + A_j) / D_ij -- so it also writes kappa_max = max over pairs (one float64 at d_kappa_max; +inf
 * when some D_ij <= 0 or an input is not finite).  kappa_limit > 0: the direct kernels of
 * fa_pairwise_sqdist are queued behind it, guarded on the device -- they return at once when
 * kappa_max <= fa_pairwise_sqdist_gram_limit(..., kappa_limit) and otherwise recompute d_dist, so the
 * call stays asynchronous and every distance it returns is within 1e-6 relative of the exact value
 * (fedml_amd/engine.py passes 16); kappa_limit <= 0: the Gram result only, no guard.
 * d_scratch: fa_pairwise_sqdist_gram_scratch_bytes(...) bytes.
 */
int fa_pairwise_sqdist_gram(fa_ctx *ctx, int32_t num_segments, const int64_t *seg_numel, int32_t k,
                            const void *const *d_in, void *d_dist, void *d_kappa_max, double kappa_limit,
                            void *d_scratch, size_t scratch_bytes, void *hip_stream);
size_t fa_pairwise_sqdist_gram_scratch_bytes(int32_t num_segments, const int64_t *seg_numel, int32_t k);
/*
 * The kappa limit fa_pairwise_sqdist_gram's guard applies to this input: min(kappa_limit,
 * 1e-6 / (6 x 0.30 u n / sqrt(P) + b)) -- the largest kappa at which 6 sigma of the error model above
 * (plus, for the bf16x3 forms, a measured size-independent part b) stays <= 1e-6 relative (n, b of the
 * kernel the call would run; d_in only for its 16-byte alignment).  0 for
 * invalid arguments or kappa_limit <= 0.  Host only, no device work.
 */
double fa_pairwise_sqdist_gram_limit(int32_t num_segments, const int64_t *seg_numel, int32_t k,
                                     const void *const *d_in, double kappa_limit);

#ifdef __cplusplus
}
#endif

#endif /* FEDAGG_ROBUST_H */
