/*
 * sdmm_oracle_kmeans.c -- CPU ORACLE (test infrastructure only; see
 * sdmm_oracle.h): kMeansPPInit, mitsuba/src/integrators/dmm/jmm/
 * mixture_model_init.h:244-330, the k-means++ choice of the n_pos seed
 * positions / normals that uniformHemisphereInit (:79-242) expands into K = 8
 * n_pos components when kMeansPlusPlus is set (:130-138).
 *
 * Per draw i (rng() = u[i]):
 *   weight_j = metric_j                         i == 0   (:268-270)
 *            = 0 if minSpatialNormal_j < 0.2^2 and minSpatial_j < 0.02^2
 *              else minDist_j^5                 i > 0    (:271-284)
 *   weight_j *= metric_j, metric_j = clamp(w_j, 1e-3, 3)  (:120, :289)
 *   index = lower_bound of u in the normalised CDF (createCdfEigen,
 *           sampleDiscreteCdf, utils.h:133-183); no remaining position or a
 *           zero sum: the uniform CDF (:292-299)
 *   then every sample's min distances to the new position (:306-328):
 *   dist^2 = |x_j - p|^2 + (acos(clamp(n_j.n_p)) / pi)^2.
 *
 * mode 0 ("reference"): the reference's float arithmetic -- float pow, the
 *   float normalisation and the sequential float CDF, lower_bound + tie walk.
 * mode 1 ("device"): the rule the HIP kernel implements -- the same float
 *   distances, the weights and their running sums in fp64, index = the first
 *   j whose prefix sum >= u * S (S the total; none -> the last positive
 *   weight), uniform fallback j = ceil(u n) - 1.  It differs from mode 0 only
 *   where u falls within the float CDF's rounding (~1e-7 relative) of a
 *   boundary; the tests measure how often.
 * Distances follow the file-wide conventions of sdmm_oracle.c (no FMA
 * contraction; acos as (float) acos((double) x)).
 */
#include "sdmm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <xmmintrin.h>

static void ftz_restore_k(unsigned* s) { _mm_setcsr(*s); }
#define FTZ_SCOPE_K                                                          \
    unsigned ftz_saved_ __attribute__((cleanup(ftz_restore_k))) = _mm_getcsr(); \
    _mm_setcsr(ftz_saved_ | 0x8040u)

#define KM_PI 3.14159265358979323846
static const double NORMAL_T = 0.2 * 0.2;    /* NORMAL_DISTANCE_TRHESHOLD (:76) */
static const double SPATIAL_T = 2e-2 * 2e-2; /* SPATIAL_DISTANCE_THRESHOLD (:77) */

static float metric_of(float w) {
    float m = w > 1e-3f ? w : 1e-3f;
    return m < 3.0f ? m : 3.0f;
}

/* utils.h:150-183 on a float CDF */
static int64_t lower_bound_walk(const float* cdf, int64_t n, float u) {
    int64_t first = 0, count = n;
    while (count > 0) {
        int64_t step = count / 2, it = first + step;
        if (cdf[it] < u) { first = it + 1; count -= step + 1; }
        else count = step;
    }
    if (first == n) {
        --first;
        while (first > 0 && cdf[first] == cdf[first - 1]) --first;
    }
    return first;
}

int or_kmeanspp_select(const float* x0, const float* x1, const float* x2, const float* n0, const float* n1,
                       const float* n2, const float* w, int64_t n, int nPos, const float* u, int mode,
                       int64_t* out_idx) {
    FTZ_SCOPE_K;
    if (n <= 0 || nPos <= 0) return -1;
    float* md = (float*)malloc(sizeof(float) * (size_t)n);
    float* msd = (float*)malloc(sizeof(float) * (size_t)n);
    float* msnd = (float*)malloc(sizeof(float) * (size_t)n);
    float* cdf = (float*)malloc(sizeof(float) * (size_t)n);
    double* pd = (double*)malloc(sizeof(double) * (size_t)n);
    if (!md || !msd || !msnd || !cdf || !pd) {
        free(md); free(msd); free(msnd); free(cdf); free(pd);
        return -2;
    }
    for (int64_t j = 0; j < n; ++j) md[j] = msd[j] = msnd[j] = INFINITY;
    for (int pi = 0; pi < nPos; ++pi) {
        int64_t chosen;
        int64_t remaining = 0;
        if (mode == 0) {
            for (int64_t j = 0; j < n; ++j) {
                const float m = metric_of(w[j]);
                float c;
                if (pi == 0) {
                    c = m;
                    ++remaining;
                } else if ((double)msnd[j] < NORMAL_T && (double)msd[j] < SPATIAL_T) {
                    c = 0.0f;
                } else {
                    c = powf(md[j], 5.0f);
                    ++remaining;
                }
                cdf[j] = c * m;
            }
            int ok = remaining > 0;
            if (ok) {
                float s = 0.0f;
                for (int64_t j = 0; j < n; ++j) s += cdf[j];
                ok = s != 0.0f;
                if (ok) {
                    for (int64_t j = 0; j < n; ++j) cdf[j] /= s;
                    for (int64_t j = 1; j < n; ++j) cdf[j] = cdf[j - 1] + cdf[j];
                }
            }
            if (!ok) {
                for (int64_t j = 0; j < n; ++j) cdf[j] = 1.0f / (float)n;
                float s = 0.0f;
                for (int64_t j = 0; j < n; ++j) s += cdf[j];
                for (int64_t j = 0; j < n; ++j) cdf[j] /= s;
                for (int64_t j = 1; j < n; ++j) cdf[j] = cdf[j - 1] + cdf[j];
            }
            chosen = lower_bound_walk(cdf, n, u[pi]);
        } else {
            double S = 0.0;
            int64_t last_pos = -1;
            for (int64_t j = 0; j < n; ++j) {
                const double m = (double)metric_of(w[j]);
                double v;
                if (pi == 0) {
                    v = m * m;
                    ++remaining;
                } else if ((double)msnd[j] < NORMAL_T && (double)msd[j] < SPATIAL_T) {
                    v = 0.0;
                } else {
                    const double d = (double)md[j];
                    const double d2 = d * d;
                    v = d2 * d2 * d * m;
                    ++remaining;
                }
                pd[j] = v;
                S += v;
                if (v > 0.0) last_pos = j;
            }
            if (remaining > 0 && S > 0.0) {
                const double target = (double)u[pi] * S;
                double run = 0.0;
                chosen = -1;
                for (int64_t j = 0; j < n; ++j) {
                    run += pd[j];
                    if (run >= target) { chosen = j; break; }
                }
                if (chosen < 0) chosen = last_pos;
            } else {
                double c = ceil((double)u[pi] * (double)n) - 1.0;
                chosen = c < 0.0 ? 0 : (c > (double)(n - 1) ? n - 1 : (int64_t)c);
            }
        }
        out_idx[pi] = chosen;
        if (pi + 1 == nPos) break;
        /* min distances to the new position (:306-328) */
        const float p0 = x0[chosen], p1 = x1[chosen], p2 = x2[chosen];
        const float q0 = n0[chosen], q1 = n1[chosen], q2 = n2[chosen];
        for (int64_t j = 0; j < n; ++j) {
            float dot = n0[j] * q0 + n1[j] * q1 + n2[j] * q2;
            dot = dot > 1.0f ? 1.0f : (dot < -1.0f ? -1.0f : dot);
            const float nd = (float)((double)(float)acos((double)dot) / KM_PI);
            const float nd2 = nd * nd;
            const float d0 = x0[j] - p0, d1 = x1[j] - p1, d2 = x2[j] - p2;
            const float sd2 = d0 * d0 + d1 * d1 + d2 * d2;
            const float dist = sd2 + nd2;
            if (dist < md[j]) md[j] = dist;
            if ((double)nd2 < NORMAL_T && sd2 < msd[j]) {
                msnd[j] = nd2;
                msd[j] = sd2;
            }
        }
    }
    free(md); free(msd); free(msnd); free(cdf); free(pd);
    return 0;
}

/* uniformHemisphereInit with kMeansPlusPlus (:130-138): one PCG32 stream
 * (seeded as or_uniform_hemisphere_init) -- nPos draws for the k-means++
 * choices, then the direction jitter of the components (:199-232). */
int or_uniform_hemisphere_init_kmeanspp(or_mixture* m, or_em_state* st, const float* x0, const float* x1,
                                        const float* x2, const float* n0, const float* n1, const float* n2,
                                        const float* w, int64_t n, int nPositions, float depthPrior,
                                        float minAllowedSpatialDistance, uint64_t seed, int mode, int select_mode,
                                        int64_t* out_idx) {
    or_pcg32 rng;
    or_pcg32_seed(&rng, seed, 0xda3e39cb94b95bdbULL);
    float* u = (float*)malloc(sizeof(float) * (size_t)nPositions);
    float* pos = (float*)malloc(sizeof(float) * 3 * (size_t)nPositions);
    float* nrm = (float*)malloc(sizeof(float) * 3 * (size_t)nPositions);
    if (!u || !pos || !nrm) {
        free(u); free(pos); free(nrm);
        return -2;
    }
    for (int i = 0; i < nPositions; ++i) u[i] = or_pcg32_next_float(&rng);
    int r = or_kmeanspp_select(x0, x1, x2, n0, n1, n2, w, n, nPositions, u, select_mode, out_idx);
    if (!r) {
        for (int i = 0; i < nPositions; ++i) {
            const int64_t j = out_idx[i];
            pos[3 * i] = x0[j]; pos[3 * i + 1] = x1[j]; pos[3 * i + 2] = x2[j];
            nrm[3 * i] = n0[j]; nrm[3 * i + 1] = n1[j]; nrm[3 * i + 2] = n2[j];
        }
        /* configure() reports success as true (mixture_model.h) */
        r = or_uniform_hemisphere_init_rng(m, st, pos, nrm, nPositions, depthPrior, minAllowedSpatialDistance,
                                           &rng, mode) ? 0 : -3;
    }
    free(u); free(pos); free(nrm);
    return r;
}
