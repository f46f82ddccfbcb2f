/*
 * fedagg_finite.h -- C ABI of the finite-field secure-aggregation kernels (libfedagg.so).
 *
 * Second kernel family behind the same context as fedagg.h: the server side of the reference's
 * secure aggregation (SecAgg / LightSecAgg), which is an int64 reduction over clients in the
 * finite field Z_p plus the fixed-point quantisation around it.  Entries and the reference code
 * each replaces (paths relative to liuliuliu0605/FedML python/fedml/):
 *
 *   fa_finite_sum       core/mpc/lightsecagg.py:134-145, core/mpc/secagg.py:148-159
 *                         aggregate_models_in_finite                      (FA_FINITE_MOD_EACH)
 *                       cross_silo/lightsecagg/lsa_fedml_aggregator.py:130-166
 *                         aggregate_model_reconstruction: sum, - mask, mod (FA_FINITE_MOD_END),
 *                         transform_finite_to_tensor (lightsecagg.py:157-185), * 1/len(active)
 *                       cross_silo/secagg/sa_fedml_aggregator.py:138-184
 *                         (FA_FINITE_MOD_FIRST | FA_FINITE_MOD_EACH | FA_FINITE_MOD_END)
 *   fa_finite_quantize  core/mpc/lightsecagg.py:150-154, 187-192 my_q / transform_tensor_to_finite
 *                       core/mpc/lightsecagg.py:83-95 model_masking (when d_mask is given)
 *   fa_lcc_decode       core/mpc/lightsecagg.py:50-55 LCC_decoding_with_points (its np.dot + np.mod;
 *                       the U x U Lagrange coefficients are computed on the host, they are tiny)
 *                       as called by lsa_fedml_aggregator.py:101-128 aggregate_mask_reconstruction
 *
 * Arithmetic contract (bit-exact to the reference's numpy code; pinned by tests/golden/g11-g15):
 *   int64 +, -, * wrap (two's complement); mod(a) = np.mod(a, p) = floor remainder in [0, p), p > 0.
 *   dequantize (my_q_inv, float64): f = (double)v - (p-1)/2;  v' = (double)v - (f > 0 ? (double)p : 0);
 *     real = (float)(v' / 2^q), then real = real * (float)scale in float32 (torch's tensor * Python
 *     float).
 *   quantize (my_q): float32 input: t = rint(x * 2^q) (float32, half-to-even); t += (float)p if t < 0
 *     (float32 add; NaN stays NaN); float64 input: the same in float64 with (double)p; int64 input:
 *     t = x * 2^q (int64 wrap), then (double)t + (t < 0 ? (double)p : 0).  The result is cast to
 *     int64 by truncation; NaN, +-Inf and values outside [-2^63, 2^63) give INT64_MIN (numpy's
 *     astype on x86).  With d_mask: out = mod(out + mask).
 *   q_bits must be in [0, 62].
 *
 * Memory, streams and errors as in fedagg.h (device pointers, host tables, async on hip_stream,
 * FA_OK or a negative fa_status).
 */
#ifndef FEDAGG_FINITE_H
#define FEDAGG_FINITE_H

#include "fedagg.h"

#ifdef __cplusplus
extern "C" {
#endif

enum fa_finite_flags {
    FA_FINITE_MOD_FIRST = 1, /* acc = mod(x_0) before the first add (SecAgg's i == 0 branch) */
    FA_FINITE_MOD_EACH = 2,  /* acc = mod(acc + x_i) after every add                           */
    FA_FINITE_MOD_END = 4,   /* acc = mod(acc) after the mask subtraction (or the last add)     */
    FA_FINITE_REAL_F64 = 8   /* real output is my_q_inv's float64 itself (no float32, no scale)  */
};

/*
 * Per segment s (a state_dict tensor, int64) and element e, clients i = 0..k-1 in order:
 *   acc = x_0[e]; MOD_FIRST: acc = mod(acc);
 *   acc = acc + x_i[e] (MOD_EACH: then acc = mod(acc));
 *   d_mask && d_mask[s]: acc = acc - mask_s[e];   MOD_END: acc = mod(acc);
 *   d_out_finite[s][e] = acc                         (int64; if d_out_finite && d_out_finite[s])
 *   d_out_real[s][e]   = dequantize(acc) * scale     (float32; if d_out_real && d_out_real[s])
 *                        with REAL_F64: my_q_inv's float64 value, unscaled (my_q_inv itself)
 * d_in[s * k + i]: client i's int64 tensor for segment s.  At least one output per segment.
 */
int fa_finite_sum(fa_ctx *ctx, int32_t num_segments, const int64_t *seg_numel, int32_t k,
                  const void *const *d_in, const void *const *d_mask, int64_t prime, int flags,
                  void *const *d_out_finite, int32_t q_bits, double scale, void *const *d_out_real,
                  void *hip_stream);

/* fa_finite_sum for ONE flat segment over tile-interleaved client inputs (addressing as
 * fa_weighted_sum_tiled, include/fedagg.h: element e of client i at d_in[i] + (e / 512) *
 * tile_stride + (e % 512) * 8); mask and outputs flat.  All 16-byte aligned. */
int fa_finite_sum_tiled(fa_ctx *ctx, int64_t n, int32_t k, const void *const *d_in,
                        int64_t tile_stride, const void *d_mask, int64_t prime, int flags,
                        void *d_out_finite, int32_t q_bits, double scale, void *d_out_real,
                        void *hip_stream);

/*
 * my_q of every element of segment s (dtype FA_DTYPE_F32, FA_DTYPE_F64 or FA_DTYPE_I64), written
 * as int64 to d_out[s]; with d_mask && d_mask[s], model_masking's out = mod(out + mask_s[e]).
 */
int fa_finite_quantize(fa_ctx *ctx, int dtype, int32_t num_segments, const int64_t *seg_numel,
                       const void *const *d_x, const void *const *d_mask, int64_t prime, int32_t q_bits,
                       void *const *d_out, void *hip_stream);

/*
 * out[e] = mod(sum_{i<k} coef[j*k + i] * f[i*m + c]) for e = j*m + c < n_out (n_out <= rows*m):
 * the first n_out entries of np.mod(U_dec.dot(f_eval), p).reshape(-1), int64 wrap.  coef is a HOST
 * array (rows x k, row-major); d_f a device int64 array (k x m, row-major); d_out int64[n_out].
 */
int fa_lcc_decode(fa_ctx *ctx, int32_t rows, int32_t k, int64_t m, const int64_t *coef,
                  const void *d_f, int64_t prime, int64_t n_out, void *d_out, void *hip_stream);

/*
 * SecAgg's mask re-expansion (cross_silo/secagg/sa_fedml_aggregator.py:92-136): numpy's legacy
 *   np.random.seed(seed_s); R_s = np.random.randint(0, prime, size=n)
 * for every stream s (MT19937 seeded by init_genrand; each draw 32-bit masked rejection when
 * prime - 1 <= 0xFFFFFFFF, else 64-bit draws hi << 32 | lo with masked rejection -- numpy's
 * random_bounded_uint64_fill with use_masked), summed with signs and reduced:
 *   d_out[e] = mod(sum_s sign_s * R_s[e])    (in [0, prime), int64)
 * which is what the reference's loop of masks, `np.mod(mask + temp, p)` and `aggregated_mask +=`
 * leaves (modular sums; every intermediate stays below 2 p).  seeds / signs are HOST arrays of
 * num_streams entries (seed in [0, 2^32), sign +1 or -1).  d_scratch: at least
 * fa_mt_randint_sum_scratch_bytes(n) bytes of device memory.  Streams of at least two chunks
 * (chunk = 624 << k words, k chosen per call) are expanded by MT19937 jump-ahead: every chunk of
 * every stream starts from its own jumped state (x^(cJ) mod the characteristic polynomial, computed
 * and cached on the host at the first call for a chunk size) and runs in parallel; the context then
 * holds device work space for the chunk windows and one plane of n values per stream of a group (the
 * group sized to FA_MT_PLANE_MB, default 2048 MiB), kept for reuse until fa_ctx_destroy.  Shorter
 * streams: one wave per stream.  FA_MT_JUMP=0 forces the one-wave form (identical results).
 */
int fa_mt_randint_sum(fa_ctx *ctx, int32_t num_streams, const uint32_t *seeds, const int8_t *signs,
                      int64_t prime, int64_t n, void *d_out, void *d_scratch, size_t scratch_bytes,
                      void *hip_stream);
size_t fa_mt_randint_sum_scratch_bytes(int64_t n);

#ifdef __cplusplus
}
#endif

#endif /* FEDAGG_FINITE_H */
