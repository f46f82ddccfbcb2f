/*
 * finite_oracle.c -- CPU restatement of the reference's finite-field secure-aggregation arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY (same rules as fedagg_oracle.c): only tests/, smoke() and bench.py's
 * cpu_baseline leg load it, and only as the checker.
 *
 * Parity: pinned by the g11-g15 fixtures (tests/golden/make_golden.py, cases_secagg), which ran
 * the reference's own numpy code.  Restated (paths relative to python/fedml/):
 *   orc_finite_sum       core/mpc/lightsecagg.py:134-145 aggregate_models_in_finite (MOD_EACH),
 *                        cross_silo/lightsecagg/lsa_fedml_aggregator.py:130-160 (sum, - mask, MOD_END),
 *                        cross_silo/secagg/sa_fedml_aggregator.py:138-180 (MOD_FIRST|MOD_EACH, - mask, MOD_END)
 *                        + my_q_inv / transform_finite_to_tensor (lightsecagg.py:157-185) and the
 *                        "* (1 / len(active))" average (lsa_fedml_aggregator.py:163-166).
 *   orc_finite_quantize  my_q / transform_tensor_to_finite (lightsecagg.py:150-154, 187-192) and
 *                        model_masking (lightsecagg.py:83-95).
 *   orc_lcc_decode       LCC_decoding_with_points's np.mod(U_dec.dot(f_eval), p) (lightsecagg.py:50-55).
 * numpy semantics restated: int64 + - * wrap (two's complement); np.mod(a, p) with p > 0 is the
 * floor remainder in [0, p); float -> int64 casts truncate, and NaN / +-Inf / out-of-range give
 * INT64_MIN (x86 cvtts*2si, which numpy's astype compiles to); Python-int operands of float32
 * arrays are cast to float32 (NEP 50), of float64 arrays to float64.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

enum { ORC_F32 = 0, ORC_F64 = 3, ORC_I64 = 4 };
enum { ORC_MOD_FIRST = 1, ORC_MOD_EACH = 2, ORC_MOD_END = 4, ORC_REAL_F64 = 8 };

static inline int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
static inline int64_t wmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }

/* np.mod(a, p), p > 0 */
static inline int64_t fmod64(int64_t a, int64_t p) {
    int64_t r = a % p;
    return r < 0 ? r + p : r;
}

/* numpy astype(int64) of a double on x86 */
static inline int64_t d2i64(double v) {
    if (!(v >= -9223372036854775808.0 && v < 9223372036854775808.0)) return INT64_MIN;
    return (int64_t)v;
}

/* my_q_inv (lightsecagg.py:157-161), float64 */
static inline double dequant64(int64_t v, int64_t p, double half, double pow2q) {
    const double flag = (double)v - half;
    const double is_neg = flag > 0.0 ? 1.0 : 0.0;      /* (|sign(f)| + sign(f)) / 2 */
    const double xq = (double)v - (double)p * is_neg;
    return xq / pow2q;
}

/* out_real: float32 (torch.Tensor(my_q_inv(.)) * fp32(scale)) or, with ORC_REAL_F64, my_q_inv's float64 */
int orc_finite_sum(int64_t n, int32_t k, const int64_t *const *x, const int64_t *mask, int64_t p,
                   int flags, int64_t *out_finite, int32_t q_bits, double scale, void *out_real) {
    if (k <= 0 || p <= 0 || n < 0 || q_bits < 0 || q_bits > 62) return -1;
    const double half = (double)(p - 1) / 2.0;
    const double pow2q = ldexp(1.0, q_bits);
    const float s32 = (float)scale;
    for (int64_t e = 0; e < n; ++e) {
        int64_t acc = x[0][e];
        if (flags & ORC_MOD_FIRST) acc = fmod64(acc, p);
        for (int32_t i = 1; i < k; ++i) {
            acc = wadd(acc, x[i][e]);
            if (flags & ORC_MOD_EACH) acc = fmod64(acc, p);
        }
        if (mask) acc = wsub(acc, mask[e]);
        if (flags & ORC_MOD_END) acc = fmod64(acc, p);
        if (out_finite) out_finite[e] = acc;
        if (out_real) {
            const double r = dequant64(acc, p, half, pow2q);
            if (flags & ORC_REAL_F64) ((double *)out_real)[e] = r;
            else ((float *)out_real)[e] = (float)r * s32;
        }
    }
    return 0;
}

/* my_q (lightsecagg.py:150-154) on one element; dtype = the numpy array's dtype */
static inline int64_t quant_f32(float x, int64_t p, int32_t q) {
    const float xi = rintf(x * ldexpf(1.0f, q));
    const float s = isnan(xi) ? xi : (xi > 0.0f ? 1.0f : (xi < 0.0f ? -1.0f : 0.0f));
    const float is_neg = (fabsf(s) - s) / 2.0f;
    const float out = xi + (float)p * is_neg;
    return d2i64((double)out);
}
static inline int64_t quant_f64(double x, int64_t p, int32_t q) {
    const double xi = rint(x * ldexp(1.0, q));
    const double s = isnan(xi) ? xi : (xi > 0.0 ? 1.0 : (xi < 0.0 ? -1.0 : 0.0));
    const double is_neg = (fabs(s) - s) / 2.0;
    const double out = xi + (double)p * is_neg;
    return d2i64(out);
}
static inline int64_t quant_i64(int64_t x, int64_t p, int32_t q) {
    const int64_t xi = wmul(x, (int64_t)1 << q);
    const double is_neg = xi < 0 ? 1.0 : 0.0;          /* (|sign| - sign) / 2, true division */
    return d2i64((double)xi + (double)p * is_neg);
}

int orc_finite_quantize(int dtype, int64_t n, const void *x, const int64_t *mask, int64_t p, int32_t q_bits,
                        int64_t *out) {
    if (p <= 0 || n < 0 || q_bits < 0 || q_bits > 62) return -1;
    for (int64_t e = 0; e < n; ++e) {
        int64_t v;
        switch (dtype) {
            case ORC_F32: v = quant_f32(((const float *)x)[e], p, q_bits); break;
            case ORC_F64: v = quant_f64(((const double *)x)[e], p, q_bits); break;
            case ORC_I64: v = quant_i64(((const int64_t *)x)[e], p, q_bits); break;
            default: return -2;
        }
        if (mask) v = fmod64(wadd(v, mask[e]), p);
        out[e] = v;
    }
    return 0;
}

/* out[e] = np.mod(sum_i coef[j][i] * f[i][c], p) for e = j * m + c < n_out (int64 wrap). */
int orc_lcc_decode(int32_t rows, int32_t k, int64_t m, const int64_t *coef, const int64_t *f, int64_t p,
                   int64_t n_out, int64_t *out) {
    if (rows <= 0 || k <= 0 || m <= 0 || p <= 0 || n_out < 0 || n_out > (int64_t)rows * m) return -1;
    for (int64_t e = 0; e < n_out; ++e) {
        const int64_t j = e / m, c = e % m;
        int64_t acc = 0;
        for (int32_t i = 0; i < k; ++i) acc = wadd(acc, wmul(coef[j * k + i], f[(int64_t)i * m + c]));
        out[e] = fmod64(acc, p);
    }
    return 0;
}
