/*
 * robust_oracle.c -- CPU restatement of the reference's robust aggregation arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY (same rules as fedagg_oracle.c).
 *
 * Parity: pinned by the g16 / g18 fixtures (tests/golden/make_golden.py, cases_robust), which ran
 * the reference's defenses.  Restated (paths relative to python/fedml/):
 *   orc_coord_median   core/security/defense/coordinate_wise_median_defense.py:26-31:
 *                      torch.median(stack of the K client vectors, dim=-1).values, i.e. ATen's
 *                      median_with_indices_impl: if the K values hold a NaN, the FIRST NaN (in
 *                      client order); otherwise the element of rank (K-1)/2 when the values are
 *                      ordered by (value, client index) -- -0.0 and +0.0 compare equal, so the
 *                      client index decides which zero is returned.
 *   orc_pairwise_sqdist  core/security/defense/krum_defense.py:52-66 (compute_euclidean_distance
 *                      = (v_i - v_j).norm(), squared): the exact float64 sum of squared float32
 *                      differences -- the value the reference's float32 norm approximates; the
 *                      GPU kernel is checked against it with a stated tolerance (krum_defense's
 *                      own float32 norm is order-dependent), and the Krum SELECTION bit-for-bit
 *                      against the fixtures.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

enum { ORC_F32 = 0, ORC_BF16 = 1, ORC_F16 = 2, ORC_F64 = 3 };

float orc_bf16_to_f32(uint16_t h);
float orc_f16_to_f32(uint16_t h);

static double ld(int dt, const void *p, int64_t e) {
    switch (dt) {
        case ORC_F32: return ((const float *)p)[e];
        case ORC_BF16: return orc_bf16_to_f32(((const uint16_t *)p)[e]);
        case ORC_F16: return orc_f16_to_f32(((const uint16_t *)p)[e]);
        default: return ((const double *)p)[e];
    }
}

static void cp(int dt, void *dst, int64_t e, const void *src) {
    const size_t s = dt == ORC_F32 ? 4 : dt == ORC_F64 ? 8 : 2;
    memcpy((char *)dst + e * s, (const char *)src + e * s, s);
}

int orc_coord_median(int dtype, int64_t n, int32_t k, const void *const *in, void *out) {
    if (k <= 0 || k > 4096 || n < 0) return -1;
    if (dtype != ORC_F32 && dtype != ORC_BF16 && dtype != ORC_F16 && dtype != ORC_F64) return -2;
    int32_t idx[4096];
    double val[4096];
    const int32_t r = (k - 1) / 2;
    for (int64_t e = 0; e < n; ++e) {
        int32_t nan_at = -1;
        for (int32_t i = 0; i < k; ++i) {
            val[i] = ld(dtype, in[i], e);
            if (isnan(val[i]) && nan_at < 0) nan_at = i;
        }
        if (nan_at >= 0) { cp(dtype, out, e, in[nan_at]); continue; }
        /* insertion sort of client indices by (value, index): stable on the index */
        for (int32_t i = 0; i < k; ++i) {
            int32_t j = i;
            while (j > 0 && val[idx[j - 1]] > val[i]) { idx[j] = idx[j - 1]; --j; }
            idx[j] = i;
        }
        cp(dtype, out, e, in[idx[r]]);
    }
    return 0;
}

/* d[i*k + j] = sum_e (x_i[e] - x_j[e])^2 in float64 (float32 inputs), every ordered pair */
/* krum_defense.py:52-66 for bfloat16 / float16 models: vectorize_weight keeps the model dtype, so
 * `(v_i - v_j)` rounds every difference to it (ATen's CPU sub: float arithmetic, one rounding to the
 * storage type); the norm squares and sums those in float.  Here: the float32 difference rounded to
 * bf16 (rt = 1) or f16 (rt = 2) by this oracle's own RNE conversions, squared and summed exactly in
 * float64.  x: the clients' values widened to float32 (exact). */
uint16_t orc_f32_to_bf16(float f);
uint16_t orc_f32_to_f16(float f);
int orc_pairwise_sqdist_rt(int64_t n, int32_t k, const float *const *x, int rt, double *d) {
    if (k <= 0 || n < 0 || rt < 0 || rt > 2) return -1;
    for (int32_t i = 0; i < k; ++i)
        for (int32_t j = 0; j < k; ++j) {
            double s = 0.0;
            if (i != j)
                for (int64_t e = 0; e < n; ++e) {
                    float t = x[i][e] - x[j][e];
                    if (rt == 1) t = orc_bf16_to_f32(orc_f32_to_bf16(t));
                    else if (rt == 2) t = orc_f16_to_f32(orc_f32_to_f16(t));
                    s += (double)t * (double)t;
                }
            d[(int64_t)i * k + j] = s;
        }
    return 0;
}

int orc_pairwise_sqdist(int64_t n, int32_t k, const float *const *x, double *d) {
    if (k <= 0 || n < 0) return -1;
    /* one sequential float64 sum per unordered pair (the (j, i) entry is the same sum: the float32
       differences are exact in float64 and square to the same terms); pairs spread over threads */
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t p = 0; p < (int64_t)k * k; ++p) {
        const int32_t i = (int32_t)(p / k), j = (int32_t)(p % k);
        if (j <= i) continue;
        double s = 0.0;
        for (int64_t e = 0; e < n; ++e) {
            const double t = (double)x[i][e] - (double)x[j][e];
            s += t * t;
        }
        d[(int64_t)i * k + j] = s;
        d[(int64_t)j * k + i] = s;
    }
    for (int32_t i = 0; i < k; ++i) d[(int64_t)i * k + i] = 0.0;
    return 0;
}
