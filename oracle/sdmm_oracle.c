/*
 * sdmm_oracle.c -- CPU ORACLE (test infrastructure only; see sdmm_oracle.h).
 *
 * Restates jmm (mitsuba/src/integrators/dmm/jmm/) in plain C99.  Conventions
 * used where the C++ source leaves the rounding unspecified (the reference is
 * compiled with -ffp-contract=fast through Eigen's expression templates and
 * cannot be built here, so its exact rounding is unknowable):
 *   - float expressions are evaluated left to right with no FMA contraction
 *     (this file is compiled with -ffp-contract=off);
 *   - a float libm call f(x) (acosf, sinf, cosf, logf) is evaluated as
 *     (float) f((double) x), i.e. the correctly rounded float in practice;
 *     exp() in the pdfs is double in the reference itself (mvtn.h:359);
 *   - sqrt is the IEEE correctly rounded sqrtf (tsqrtf, utils.h:13-15);
 *   - the inverse of a triangular Cholesky factor is formed by forward
 *     substitution and its determinant as the product of the diagonal
 *     (Eigen uses PartialPivLU for the 5x5 `m_cholL.inverse()`, mvtn.cpp:61);
 *   - std::sort ties in MixtureModel::conditional are broken by ascending
 *     component index (the reference sort is unstable, mixture_model.h:264).
 * The HIP guided-query kernel follows exactly these conventions so that the
 * component indices it selects are bit-identical to this oracle's.
 */
#include "sdmm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <xmmintrin.h>

/* The plugin enables flush-to-zero / denormals-are-zero by default
 * (flushDenormals=true, volpath_sdmm.cpp:64,88-90: enoki::set_flush_denormals).
 * Every exported entry point runs under FTZ|DAZ and restores MXCSR on exit. */
static void ftz_restore(unsigned* s) { _mm_setcsr(*s); }
#define FTZ_SCOPE                                                          \
    unsigned ftz_saved_ __attribute__((cleanup(ftz_restore))) = _mm_getcsr(); \
    _mm_setcsr(ftz_saved_ | 0x8040u)

#define OR_PI 3.14159265358979323846
#define INV_SQRT_TWO_PI 0.39894228040143267793994605993438186847585863116492

/* constexpr static Scalar NORMALIZATION = std::pow(INV_SQRT_TWO_PI, d)
 * (mvtn.h:351-352, mvn.h:121-122): float base, double pow, rounded to float. */
static float norm_const(int d) {
    return (float)pow((double)(float)INV_SQRT_TWO_PI, (double)d);
}

static float fl_acos(float x) { return (float)acos((double)x); }
static float fl_cos(float x) { return (float)cos((double)x); }
static float fl_sin(float x) { return (float)sin((double)x); }
static float fl_log(float x) { return (float)log((double)x); }

/* ------------------------------------------------------------------------ */
/* PCG32 (M.E. O'Neill; the enoki::PCG32 used by the plugin, sdmm_proc.h:87) */
#define PCG32_MULT 0x5851f42d4c957f2dULL

void or_pcg32_seed(or_pcg32* r, uint64_t initstate, uint64_t initseq) {
    r->state = 0u;
    r->inc = (initseq << 1u) | 1u;
    or_pcg32_next_uint(r);
    r->state += initstate;
    or_pcg32_next_uint(r);
}

uint32_t or_pcg32_next_uint(or_pcg32* r) {
    uint64_t oldstate = r->state;
    r->state = oldstate * PCG32_MULT + r->inc;
    uint32_t xorshifted = (uint32_t)(((oldstate >> 18u) ^ oldstate) >> 27u);
    uint32_t rot = (uint32_t)(oldstate >> 59u);
    return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
}

float or_pcg32_next_float(or_pcg32* r) {
    union { uint32_t u; float f; } x;
    x.u = (or_pcg32_next_uint(r) >> 9) | 0x3f800000u;
    return x.f - 1.0f;
}

/* ------------------------------------------------------------------------ */
/* Coordinates (utils.h:32-48): row 2 = n. */
void or_coordinates(const float n[3], float to[9]) {
    FTZ_SCOPE;
    float sign = copysignf(1.0f, n[2]);
    const float a = -1.0f / (sign + n[2]);
    const float b = n[0] * n[1] * a;
    to[0] = 1.0f + sign * n[0] * n[0] * a; to[1] = sign * b; to[2] = -sign * n[0];
    to[3] = b; to[4] = sign + n[1] * n[1] * a; to[5] = -n[1];
    to[6] = n[0]; to[7] = n[1]; to[8] = n[2];
}

static void coordinates_d(const double n[3], double to[9]) {
    double sign = copysign(1.0, n[2]);
    const double a = -1.0 / (sign + n[2]);
    const double b = n[0] * n[1] * a;
    to[0] = 1.0 + sign * n[0] * n[0] * a; to[1] = sign * b; to[2] = -sign * n[0];
    to[3] = b; to[4] = sign + n[1] * n[1] * a; to[5] = -n[1];
    to[6] = n[0]; to[7] = n[1]; to[8] = n[2];
}

/* boost::math::sinc_pi for float (sinc.hpp): Taylor near 0. */
float or_sinc_pi(float x) {
    FTZ_SCOPE;
    const float taylor_0_bound = 1.1920928955078125e-07f; /* epsilon<float> */
    const float taylor_2_bound = sqrtf(taylor_0_bound);
    const float taylor_n_bound = sqrtf(taylor_2_bound);
    float ax = fabsf(x);
    if (ax >= taylor_n_bound) return fl_sin(x) / x;
    float result = 1.0f;
    if (ax >= taylor_0_bound) {
        float x2 = x * x;
        result -= x2 / 6.0f;
        if (ax >= taylor_2_bound) result += (x2 * x2) / 120.0f;
    }
    return result;
}

static double sinc_pi_d(double x) {
    const double taylor_0_bound = 2.220446049250313e-16;
    const double taylor_2_bound = sqrt(taylor_0_bound);
    const double taylor_n_bound = sqrt(taylor_2_bound);
    double ax = fabs(x);
    if (ax >= taylor_n_bound) return sin(x) / x;
    double result = 1.0;
    if (ax >= taylor_0_bound) {
        double x2 = x * x;
        result -= x2 / 6.0;
        if (ax >= taylor_2_bound) result += (x2 * x2) / 120.0;
    }
    return result;
}

/* TangentSpace::log (mvtn.h:146-177).  emb = sample - zeroedOutMean.
 * m_invRotation = to, so relToNorthPole = to * direction. */
int or_ts_log(const float to[9], const float emb[6], float tangent[5], float* jac) {
    FTZ_SCOPE;
    const float d0 = emb[3], d1 = emb[4], d2 = emb[5];
    if (d0 == 0.0f && d1 == 0.0f && d2 == 0.0f) return 0;
    float r0 = to[0] * d0 + to[1] * d1 + to[2] * d2;
    float r1 = to[3] * d0 + to[4] * d1 + to[5] * d2;
    float c = to[6] * d0 + to[7] * d1 + to[8] * d2;
    if (c <= -1.0f) return 0;
    c = (c < 1.0f) ? c : 1.0f; /* std::min(Scalar(1), cosAngle) */
    float angle = fl_acos(c);
    float s = sqrtf(1.0f - c * c);
    float a = ((double)s < 1e-3) ? 1.0f : (angle / s);
    tangent[0] = emb[0]; tangent[1] = emb[1]; tangent[2] = emb[2];
    tangent[3] = r0 * a;
    tangent[4] = r1 * a;
    *jac = a;
    return 1;
}

/* TangentSpace::exp (mvtn.h:93-120).  m_rotation = to^T. */
int or_ts_exp(const float to[9], const float tangent[5], float emb[6], float* jac) {
    FTZ_SCOPE;
    float t0 = tangent[3], t1 = tangent[4];
    float length = sqrtf(t0 * t0 + t1 * t1);
    if ((double)length >= OR_PI) {
        for (int i = 0; i < 6; ++i) emb[i] = 0.0f;
        return 0;
    }
    float s = or_sinc_pi(length);
    float rel0 = t0 * s, rel1 = t1 * s, rel2 = fl_cos(length);
    emb[0] = tangent[0]; emb[1] = tangent[1]; emb[2] = tangent[2];
    emb[3] = to[0] * rel0 + to[3] * rel1 + to[6] * rel2;
    emb[4] = to[1] * rel0 + to[4] * rel1 + to[7] * rel2;
    emb[5] = to[2] * rel0 + to[5] * rel1 + to[8] * rel2;
    *jac = s;
    return 1;
}

/* MVTN::pdfAndLog (mvtn.h:350-365). */
float or_mvtn_pdf_and_log(const or_mixture* m, int k, const float sample[6], float tangent[5]) {
    FTZ_SCOPE;
    const float* mean = m->mean + 6 * k;
    float emb[6] = {sample[0] - mean[0], sample[1] - mean[1], sample[2] - mean[2],
                    sample[3], sample[4], sample[5]};
    float jac;
    if (!or_ts_log(m->to + 9 * k, emb, tangent, &jac)) {
        for (int i = 0; i < 5; ++i) tangent[i] = 0.0f;
        return 0.0f;
    }
    const float* Li = m->cholLInv + 25 * k;
    float q = 0.0f;
    for (int i = 0; i < 5; ++i) {
        float s = 0.0f;
        for (int j = 0; j < 5; ++j) s += Li[5 * i + j] * tangent[j];
        q += s * s;
    }
    static float NORM5 = -1.0f;
    if (NORM5 < 0.0f) NORM5 = norm_const(5);
    float pdf = (float)((double)NORM5 * exp(-0.5 * (double)q));
    pdf *= m->detInv[k] * jac;
    tangent[0] += mean[0]; tangent[1] += mean[1]; tangent[2] += mean[2];
    return pdf;
}

/* MultivariateNormal<3,3>::pdf(x, isInside) (mvn.h:118-128): forward
 * substitution with L (m_cholesky.matrixL().solve). */
float or_marginal_pdf(const or_mixture* m, int k, const float c[3]) {
    FTZ_SCOPE;
    const float* L = m->margL + 9 * k;
    const float* mu = m->mean + 6 * k;
    float r0 = c[0] - mu[0], r1 = c[1] - mu[1], r2 = c[2] - mu[2];
    float s0 = r0 / L[0];
    r1 = r1 - s0 * L[3];
    r2 = r2 - s0 * L[6];
    float s1 = r1 / L[4];
    r2 = r2 - s1 * L[7];
    float s2 = r2 / L[8];
    float q = s0 * s0 + s1 * s1 + s2 * s2;
    static float NORM3 = -1.0f;
    if (NORM3 < 0.0f) NORM3 = norm_const(3);
    float pdf = (float)((double)NORM3 * exp(-0.5 * (double)q));
    return pdf * m->margDetInv[k];
}

/* ------------------------------------------------------------------------ */
/* small dense linear algebra, generic over float/double via macros          */

#define DEFINE_LINALG(T, SFX, SQRT)                                              \
/* Eigen LLT<Lower> unblocked (LLT.h llt_inplace::unblocked); reads lower. */   \
static int llt_##SFX(const T* A, int n, T* L) {                                  \
    for (int i = 0; i < n * n; ++i) L[i] = 0;                                    \
    for (int i = 0; i < n; ++i)                                                  \
        for (int j = 0; j <= i; ++j) L[i * n + j] = A[i * n + j];                \
    for (int k = 0; k < n; ++k) {                                                \
        T x = L[k * n + k];                                                      \
        for (int j = 0; j < k; ++j) x -= L[k * n + j] * L[k * n + j];            \
        if (!(x > (T)0)) return 0;                                               \
        x = SQRT(x);                                                             \
        L[k * n + k] = x;                                                        \
        for (int i = k + 1; i < n; ++i) {                                        \
            T v = L[i * n + k];                                                  \
            for (int j = 0; j < k; ++j) v -= L[i * n + j] * L[k * n + j];        \
            L[i * n + k] = v / x;                                                \
        }                                                                        \
    }                                                                            \
    return 1;                                                                    \
}                                                                                \
/* inverse of a lower-triangular matrix by forward substitution */              \
static void tri_inv_##SFX(const T* L, int n, T* Li) {                           \
    for (int i = 0; i < n * n; ++i) Li[i] = 0;                                   \
    for (int c = 0; c < n; ++c) {                                                \
        for (int i = c; i < n; ++i) {                                            \
            T v = (i == c) ? (T)1 : (T)0;                                        \
            for (int j = c; j < i; ++j) v -= L[i * n + j] * Li[j * n + c];       \
            Li[i * n + c] = v / L[i * n + i];                                    \
        }                                                                        \
    }                                                                            \
}                                                                                \
/* Eigen compute_inverse_size3 (InverseImpl.h): adjugate / det */               \
static void inv3_##SFX(const T* m, T* r) {                                       \
    T c00 = m[4] * m[8] - m[5] * m[7];                                           \
    T c10 = m[7] * m[2] - m[8] * m[1];                                           \
    T c20 = m[1] * m[5] - m[2] * m[4];                                           \
    T det = c00 * m[0] + c10 * m[3] + c20 * m[6];                                \
    T invdet = (T)1 / det;                                                       \
    r[0] = c00 * invdet; r[1] = c10 * invdet; r[2] = c20 * invdet;               \
    r[3] = (m[5] * m[6] - m[3] * m[8]) * invdet;                                 \
    r[4] = (m[8] * m[0] - m[6] * m[2]) * invdet;                                 \
    r[5] = (m[2] * m[3] - m[0] * m[5]) * invdet;                                 \
    r[6] = (m[3] * m[7] - m[4] * m[6]) * invdet;                                 \
    r[7] = (m[6] * m[1] - m[7] * m[0]) * invdet;                                 \
    r[8] = (m[0] * m[4] - m[1] * m[3]) * invdet;                                 \
}                                                                                \
/* cyclic Jacobi eigenvalues of the symmetric matrix read from the lower      \
 * triangle (SelfAdjointEigenSolver reads the lower triangle). */              \
static int is_pd_##SFX(const T* A, int n) {                                      \
    T a[25];                                                                     \
    for (int i = 0; i < n; ++i)                                                  \
        for (int j = 0; j < n; ++j)                                              \
            a[i * n + j] = (i >= j) ? A[i * n + j] : A[j * n + i];               \
    for (int i = 0; i < n * n; ++i) if (!isfinite((double)a[i])) return 0;       \
    for (int sweep = 0; sweep < 64; ++sweep) {                                   \
        T off = 0;                                                               \
        for (int p = 0; p < n; ++p)                                              \
            for (int q = p + 1; q < n; ++q) off += a[p * n + q] * a[p * n + q];  \
        if (off == (T)0) break;                                                  \
        for (int p = 0; p < n; ++p) {                                            \
            for (int q = p + 1; q < n; ++q) {                                    \
                T apq = a[p * n + q];                                            \
                if (apq == (T)0) continue;                                       \
                T app = a[p * n + p], aqq = a[q * n + q];                        \
                T theta = (aqq - app) / ((T)2 * apq);                            \
                T t = (theta >= 0 ? (T)1 : (T)-1) /                              \
                      (fabs((double)theta) + SQRT(theta * theta + (T)1));        \
                if (!isfinite((double)(theta * theta)))                          \
                    t = (T)1 / ((T)2 * theta);                                   \
                T cs = (T)1 / SQRT(t * t + (T)1), sn = t * cs;                   \
                for (int k = 0; k < n; ++k) {                                    \
                    T akp = a[k * n + p], akq = a[k * n + q];                    \
                    a[k * n + p] = cs * akp - sn * akq;                          \
                    a[k * n + q] = sn * akp + cs * akq;                          \
                }                                                                \
                for (int k = 0; k < n; ++k) {                                    \
                    T apk = a[p * n + k], aqk = a[q * n + k];                    \
                    a[p * n + k] = cs * apk - sn * aqk;                          \
                    a[q * n + k] = sn * apk + cs * aqk;                          \
                }                                                                \
            }                                                                    \
        }                                                                        \
    }                                                                            \
    for (int i = 0; i < n; ++i) if (!(a[i * n + i] > (T)0)) return 0;            \
    return 1;                                                                    \
}

DEFINE_LINALG(float, f32, sqrtf)
DEFINE_LINALG(double, f64, sqrt)

int or_is_positive_definite_f64(const double* A, int n) { FTZ_SCOPE; return is_pd_f64(A, n); }
int or_is_positive_definite_f32(const float* A, int n) { FTZ_SCOPE; return is_pd_f32(A, n); }

/* ------------------------------------------------------------------------ */
/* MVTN::set (mvtn.cpp:16-65) + precomputeConditioning (mvtn.h:386-408) +
 * marginal() (mvtn.h:446-454) + the conditional component's LLT, which the
 * reference recomputes on every conditional() call from the same matrix. */
int or_component_set(or_mixture* m, int k, const double mean[6], const double cov[25], int mode) {
    FTZ_SCOPE;
    float* fm = m->mean + 6 * k;
    float* fc = m->cov + 25 * k;
    for (int i = 0; i < 6; ++i) fm[i] = (float)mean[i];
    for (int i = 0; i < 25; ++i) fc[i] = (float)cov[i];
    int ok = 1;
    if (mode == 0) {
        or_coordinates(fm + 3, m->to + 9 * k);
        /* conditioning, float */
        float AA[9], AB[6], BA[6], BB[4], AAi[9], P[6], S[4];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) AA[3 * i + j] = fc[5 * i + j];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 2; ++j) AB[2 * i + j] = fc[5 * i + 3 + j];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 3; ++j) BA[3 * i + j] = fc[5 * (3 + i) + j];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j) BB[2 * i + j] = fc[5 * (3 + i) + 3 + j];
        inv3_f32(AA, AAi);
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 3; ++j) {
                float v = 0.0f;
                for (int l = 0; l < 3; ++l) v += BA[3 * i + l] * AAi[3 * l + j];
                P[3 * i + j] = v;
            }
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j) {
                float v = 0.0f;
                for (int l = 0; l < 3; ++l) v += P[3 * i + l] * AB[2 * l + j];
                S[2 * i + j] = BB[2 * i + j] - v;
            }
        memcpy(m->muPremult + 6 * k, P, sizeof(P));
        memcpy(m->condCov + 4 * k, S, sizeof(S));
        float L[25], Li[25];
        if (llt_f32(fc, 5, L)) {
            tri_inv_f32(L, 5, Li);
            memcpy(m->cholL + 25 * k, L, sizeof(L));
            memcpy(m->cholLInv + 25 * k, Li, sizeof(Li));
            float det = 1.0f;
            for (int i = 0; i < 5; ++i) det *= L[6 * i];
            m->detInv[k] = 1.0f / det;
        } else {
            ok = 0;
        }
        float L3[9];
        float A3[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) A3[3 * i + j] = fc[5 * i + j];
        if (llt_f32(A3, 3, L3)) {
            memcpy(m->margL + 9 * k, L3, sizeof(L3));
            m->margDetInv[k] = 1.0f / (L3[0] * L3[4] * L3[8]);
        }
        float L2[4], L2i[4];
        if (llt_f32(S, 2, L2)) {
            /* Eigen 2x2 inverse: [d -b; -c a] * (1/det), det = a*d - c*b */
            float det2 = L2[0] * L2[3] - L2[2] * L2[1];
            float invdet = 1.0f / det2;
            L2i[0] = L2[3] * invdet; L2i[1] = -L2[1] * invdet;
            L2i[2] = -L2[2] * invdet; L2i[3] = L2[0] * invdet;
            memcpy(m->condL + 4 * k, L2, sizeof(L2));
            memcpy(m->condLInv + 4 * k, L2i, sizeof(L2i));
            m->condDetInv[k] = 1.0f / (L2[0] * L2[3]);
        }
    } else {
        double md[3] = {(double)fm[3], (double)fm[4], (double)fm[5]};
        double tod[9];
        coordinates_d(md, tod);
        for (int i = 0; i < 9; ++i) m->to[9 * k + i] = (float)tod[i];
        double AA[9], AB[6], BA[6], BB[4], AAi[9], P[6], S[4];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) AA[3 * i + j] = cov[5 * i + j];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 2; ++j) AB[2 * i + j] = cov[5 * i + 3 + j];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 3; ++j) BA[3 * i + j] = cov[5 * (3 + i) + j];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j) BB[2 * i + j] = cov[5 * (3 + i) + 3 + j];
        inv3_f64(AA, AAi);
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 3; ++j) {
                double v = 0.0;
                for (int l = 0; l < 3; ++l) v += BA[3 * i + l] * AAi[3 * l + j];
                P[3 * i + j] = v;
            }
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j) {
                double v = 0.0;
                for (int l = 0; l < 3; ++l) v += P[3 * i + l] * AB[2 * l + j];
                S[2 * i + j] = BB[2 * i + j] - v;
            }
        for (int i = 0; i < 6; ++i) m->muPremult[6 * k + i] = (float)P[i];
        for (int i = 0; i < 4; ++i) m->condCov[4 * k + i] = (float)S[i];
        double L[25], Li[25];
        if (llt_f64(cov, 5, L)) {
            tri_inv_f64(L, 5, Li);
            double det = 1.0;
            for (int i = 0; i < 5; ++i) det *= L[6 * i];
            for (int i = 0; i < 25; ++i) {
                m->cholL[25 * k + i] = (float)L[i];
                m->cholLInv[25 * k + i] = (float)Li[i];
            }
            m->detInv[k] = (float)(1.0 / det);
        } else {
            ok = 0;
        }
        double A3[9], L3[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) A3[3 * i + j] = cov[5 * i + j];
        if (llt_f64(A3, 3, L3)) {
            for (int i = 0; i < 9; ++i) m->margL[9 * k + i] = (float)L3[i];
            m->margDetInv[k] = (float)(1.0 / (L3[0] * L3[4] * L3[8]));
        }
        double L2[4];
        if (llt_f64(S, 2, L2)) {
            double det2 = L2[0] * L2[3];
            m->condL[4 * k + 0] = (float)L2[0]; m->condL[4 * k + 1] = 0.0f;
            m->condL[4 * k + 2] = (float)L2[2]; m->condL[4 * k + 3] = (float)L2[3];
            m->condLInv[4 * k + 0] = (float)(L2[3] / det2);
            m->condLInv[4 * k + 1] = 0.0f;
            m->condLInv[4 * k + 2] = (float)(-L2[2] / det2);
            m->condLInv[4 * k + 3] = (float)(L2[0] / det2);
            m->condDetInv[k] = (float)(1.0 / det2);
        }
    }
    m->valid[k] = ok;
    return ok;
}

/* jmm::normalizePdf + createCdf (utils.h:64-102), float, sequential. */
static int create_cdf_f(float* w, int n, float* cdf, int normalize) {
    if (normalize) {
        float sum = 0.0f;
        for (int i = 0; i < n; ++i) sum += w[i];
        if (sum == 0.0f) return 0;
        for (int i = 0; i < n; ++i) w[i] = w[i] / sum;
    }
    float acc = 0.0f;
    for (int i = 0; i < n; ++i) { acc += w[i]; cdf[i] = acc; }
    return 1;
}

int or_mixture_configure(or_mixture* m) {
    FTZ_SCOPE;
    /* createMarginals() happens inside or_component_set. */
    return create_cdf_f(m->weights, m->K, m->cdf, 1);
}

/* ------------------------------------------------------------------------ */
/* posteriorAndLog (mixture_model.h:146-192) */
void or_posterior_and_log(const or_mixture* m, const float sample[6], int useHeuristic,
                          float heuristicPdf, float* pdf, float* posterior,
                          float* tangents, float* heuristicPosterior) {
    FTZ_SCOPE;
    const int K = m->K;
    const float h = m->heuristicWeight;
    *heuristicPosterior = 0.0f;
    for (int k = 0; k < K; ++k) {
        pdf[k] = or_mvtn_pdf_and_log(m, k, sample, tangents + 5 * k);
        posterior[k] = m->weights[k] * pdf[k];
    }
    float sum = 0.0f;
    for (int k = 0; k < K; ++k) sum += posterior[k];
    if (useHeuristic) sum = (1.0f - h) * sum + h * heuristicPdf;
    const float invSum = 1.0f / sum;
    if (isfinite(invSum)) {
        for (int k = 0; k < K; ++k) posterior[k] *= invSum;
        if (useHeuristic) {
            for (int k = 0; k < K; ++k) posterior[k] *= (1.0f - h);
            *heuristicPosterior = h * heuristicPdf * invSum;
            for (int k = 0; k < K; ++k) pdf[k] = h * heuristicPdf + (1.0f - h) * pdf[k];
        }
    } else {
        for (int k = 0; k < K; ++k) { posterior[k] = 0.0f; pdf[k] = 0.0f; }
        *heuristicPosterior = 0.0f;
    }
}

void or_responsibilities(const or_mixture* m, const or_samples* s, float* out) {
    FTZ_SCOPE;
    const int K = m->K;
    float* pdf = (float*)malloc(sizeof(float) * K);
    float* tan = (float*)malloc(sizeof(float) * K * 5);
    for (int64_t n = 0; n < s->n; ++n) {
        float x[6];
        for (int i = 0; i < 6; ++i) x[i] = s->x[i][n];
        int useH = s->isDiffuse ? (s->isDiffuse[n] != 0) : 0;
        float hp = s->hpdf ? s->hpdf[n] : 0.0f;
        float hpost;
        or_posterior_and_log(m, x, useH, hp, pdf, out + n * K, tan, &hpost);
    }
    free(pdf);
    free(tan);
}

/* ------------------------------------------------------------------------ */
/* "exact" E-step term: w_k * pdf_k(x) of mvtn.h:350-365 evaluated in double
 * from the float parameters, flushing where the reference's fp32 FTZ build
 * flushes (NORM*exp -> *detInv*J -> *w_k); tangent spatial part = p.        */
static double ftz_d(double v) { return (fabs(v) < (double)1.17549435082228750797e-38F) ? 0.0 : v; }

static double posterior_term_exact(const or_mixture* m, int k, const float xf[6], double tangent[5]) {
    const float* mf = m->mean + 6 * k;
    const float* tof = m->to + 9 * k;
    const double d0 = xf[3], d1 = xf[4], d2 = xf[5];
    for (int i = 0; i < 5; ++i) tangent[i] = 0.0;
    if (d0 == 0.0 && d1 == 0.0 && d2 == 0.0) return 0.0;
    const double r0 = (double)tof[0] * d0 + (double)tof[1] * d1 + (double)tof[2] * d2;
    const double r1 = (double)tof[3] * d0 + (double)tof[4] * d1 + (double)tof[5] * d2;
    double c = (double)tof[6] * d0 + (double)tof[7] * d1 + (double)tof[8] * d2;
    if (c <= -1.0) return 0.0;
    c = (c < 1.0) ? c : 1.0;
    const double angle = acos(c);
    const double sn = sqrt(1.0 - c * c);
    const double a = (sn < 1e-3) ? 1.0 : angle / sn;
    double t[5] = {(double)xf[0] - (double)mf[0], (double)xf[1] - (double)mf[1],
                   (double)xf[2] - (double)mf[2], r0 * a, r1 * a};
    const float* Li = m->cholLInv + 25 * k;
    double q = 0.0;
    for (int i = 0; i < 5; ++i) {
        double u = 0.0;
        for (int j = 0; j < 5; ++j) u += (double)Li[5 * i + j] * t[j];
        q += u * u;
    }
    static float NORM5 = -1.0f;
    if (NORM5 < 0.0f) NORM5 = norm_const(5);
    const double p1 = ftz_d((double)NORM5 * exp(-0.5 * q));
    const double p2 = ftz_d(p1 * ftz_d((double)m->detInv[k] * a));
    tangent[0] = xf[0]; tangent[1] = xf[1]; tangent[2] = xf[2];
    tangent[3] = t[3]; tangent[4] = t[4];
    return ftz_d((double)m->weights[k] * p2);
}

/* EM, instantiated three times: faithful (float), accurate (float per-pair
 * math, double accumulation and M-step), exact (double per-pair math too). */
#define ACC float
#define ACC_IS_FLOAT 1
#define EXACT_E 0
#define FN(x) x##_f32
#include "sdmm_oracle_em.inc"
#undef ACC
#undef ACC_IS_FLOAT
#undef EXACT_E
#undef FN

#define ACC double
#define ACC_IS_FLOAT 0
#define EXACT_E 0
#define FN(x) x##_f64
#include "sdmm_oracle_em.inc"
#undef ACC
#undef ACC_IS_FLOAT
#undef EXACT_E
#undef FN

#define ACC double
#define ACC_IS_FLOAT 0
#define EXACT_E 1
#define FN(x) x##_x64
#include "sdmm_oracle_em.inc"
#undef ACC
#undef ACC_IS_FLOAT
#undef EXACT_E
#undef FN

void or_em_state_init(or_em_state* st, int K, double alpha, const double bPrior5[5],
                      double niPriorMinusOne, double epsilon, int decreasePrior) {
    /* StepwiseTangentEM ctor (stepwise_tangent.h:221-252) */
    st->K = K;
    st->iterationsRun = 0;
    st->decreasePrior = decreasePrior;
    st->trainingCutoff = 32;
    st->alpha = (double)(float)alpha;
    st->niPriorMinusOne = (double)(float)niPriorMinusOne;
    st->heuristicTotalWeight = 0.0;
    st->sgH = 0.0;
    float eps = (float)epsilon; /* 1e-100 as float == 0 (appendix A.6) */
    for (int k = 0; k < K; ++k) {
        st->totalWeight[k] = 0.0;
        st->sgW[k] = 0.0;
        for (int i = 0; i < 5; ++i) st->sgM[5 * k + i] = 0.0;
        for (int i = 0; i < 25; ++i) st->sgC[25 * k + i] = 0.0;
        for (int i = 0; i < 25; ++i) st->bPriors[25 * k + i] = 0.0f;
        for (int i = 0; i < 5; ++i) st->bPriors[25 * k + 6 * i] = (float)bPrior5[i];
        for (int i = 0; i < 9; ++i) st->bDepth[9 * k + i] = 0.0f;
        for (int i = 0; i < 3; ++i) st->bDepth[9 * k + 4 * i] = eps;
    }
}

/* ------------------------------------------------------------------------ */
/* uniformHemisphereInit (mixture_model_init.h:79-242), positions/normals given
 * (the kMeansPlusPlus=false branch: positions = first samples). */
int or_uniform_hemisphere_init(or_mixture* m, or_em_state* st, const float* positions,
                               const float* normals, int nPositions, float depthPrior,
                               float minAllowedSpatialDistance, uint64_t seed, int mode) {
    or_pcg32 rng;
    or_pcg32_seed(&rng, seed, 0xda3e39cb94b95bdbULL);
    return or_uniform_hemisphere_init_rng(m, st, positions, normals, nPositions, depthPrior,
                                          minAllowedSpatialDistance, &rng, mode);
}

/* the same, drawing the direction jitter from a caller's PCG32 stream (the
 * kMeansPlusPlus branch shares one rng between the position choice and it) */
int or_uniform_hemisphere_init_rng(or_mixture* m, or_em_state* st, const float* positions,
                                   const float* normals, int nPositions, float depthPrior,
                                   float minAllowedSpatialDistance, or_pcg32* rngp, int mode) {
    FTZ_SCOPE;
    or_pcg32 rng = *rngp;
    const float maxRadiusSqr = (float)10.644640675668422; /* chi2(6).quantile(0.90) */
    const float widthVarSqr =
        (float)(0.5 * (double)minAllowedSpatialDistance * (double)minAllowedSpatialDistance /
                (double)maxRadiusSqr);
    const float depthVarSqr = depthPrior * depthPrior / maxRadiusSqr;
    const float nThetas = 2.0f, nPhis = 4.0f;
    const float directionalInit = 1.0f / (nThetas * nPhis);
    const int K = nPositions * 8;
    m->K = K;
    int k = 0;
    for (int pi = 0; pi < nPositions; ++pi) {
        const float* p = positions + 3 * pi;
        const float* n = normals + 3 * pi;
        float to[9];
        or_coordinates(n, to);
        const float* s = to;
        const float* t = to + 3;
        float cov[25];
        for (int i = 0; i < 25; ++i) cov[i] = 0.0f;
        for (int i = 0; i < 5; ++i) cov[6 * i] = 1.0f;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                cov[5 * i + j] = (s[i] * s[j] * widthVarSqr + t[i] * t[j] * widthVarSqr) +
                                 n[i] * n[j] * depthVarSqr;
        const float dcov = (float)(2.0 * OR_PI * (double)directionalInit);
        cov[18] = dcov; cov[24] = dcov;
        cov[19] = 0.0f; cov[23] = 0.0f;
        float bPrior[25];
        for (int i = 0; i < 25; ++i) bPrior[i] = 0.0f;
        for (int i = 0; i < 5; ++i) bPrior[6 * i] = 1.0f;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                bPrior[5 * i + j] = s[i] * s[j] * 1e-4f + t[i] * t[j] * 1e-4f + n[i] * n[j] * 1e-4f;
        bPrior[18] = 1e-5f; bPrior[24] = 1e-5f;
        float theta = 0.0f;
        for (int ti = 0; ti < (int)nThetas; ++ti) {
            float rn = (float)(((double)or_pcg32_next_float(&rng) - 0.5) * 2e-1);
            theta = (float)((double)theta + (0.5 * OR_PI / (double)(nThetas + 1.0f) + (double)rn));
            const float cosTheta = fl_cos(theta);
            const float sinTheta = sqrtf(1.0f - cosTheta * cosTheta);
            float phi = 0.0f;
            for (int fi = 0; fi < (int)nPhis; ++fi) {
                rn = (float)(((double)or_pcg32_next_float(&rng) - 0.5) * 1e-1);
                phi = (float)((double)phi + (2.0 * OR_PI / (double)nPhis + (double)rn));
                float sinPhi = fl_sin(phi), cosPhi = fl_cos(phi);
                float dl0 = sinTheta * cosPhi, dl1 = sinTheta * sinPhi, dl2 = cosTheta;
                double mean[6], covd[25];
                for (int i = 0; i < 3; ++i) mean[i] = p[i];
                for (int i = 0; i < 3; ++i) mean[3 + i] = (float)((s[i] * dl0 + t[i] * dl1) + n[i] * dl2);
                for (int i = 0; i < 25; ++i) covd[i] = cov[i];
                or_component_set(m, k, mean, covd, mode);
                m->weights[k] = 1.0f / (float)K;
                if (st) {
                    for (int i = 0; i < 25; ++i) st->bPriors[25 * k + i] = bPrior[i];
                    for (int i = 0; i < 3; ++i)
                        for (int j = 0; j < 3; ++j) st->bDepth[9 * k + 3 * i + j] = n[i] * n[j] * 1e-6f;
                }
                ++k;
            }
        }
    }
    *rngp = rng;
    return or_mixture_configure(m);
}

/* ------------------------------------------------------------------------ */
/* Guided bounce.                                                             */

int or_sample_discrete_cdf(const float* cdf, int n, float u) {
    FTZ_SCOPE;
    /* std::lower_bound then the tie walk of utils.h:108-113 */
    int lo = 0, count = n;
    while (count > 0) {
        int step = count / 2, it = lo + step;
        if (cdf[it] < u) { lo = it + 1; count -= step + 1; }
        else count = step;
    }
    if (lo == n) {
        --lo;
        while (lo > 0 && cdf[lo] == cdf[lo - 1]) --lo;
    }
    return lo;
}

/* MVTN::conditional (mvtn.h:417-439) for joint component k at condition c:
 * conditional mean direction (conditionalExp, mvtn.h:122-144). */
static int cond_mean_dir(const or_mixture* m, int k, const float c[3], float e[3]) {
    const float* P = m->muPremult + 6 * k;
    const float* mu = m->mean + 6 * k;
    float d0 = c[0] - mu[0], d1 = c[1] - mu[1], d2 = c[2] - mu[2];
    float t0 = P[0] * d0 + P[1] * d1 + P[2] * d2;
    float t1 = P[3] * d0 + P[4] * d1 + P[5] * d2;
    float tan5[5] = {0.0f, 0.0f, 0.0f, t0, t1};
    float emb[6], jac;
    int ok = or_ts_exp(m->to + 9 * k, tan5, emb, &jac);
    e[0] = emb[3]; e[1] = emb[4]; e[2] = emb[5];
    return ok;
}

int or_conditional_create(const or_mixture* m, const float c[3], or_conditional* out) {
    FTZ_SCOPE;
    const int K = m->K;
    float* w = (float*)malloc(sizeof(float) * K);
    char* taken = (char*)calloc(K, 1);
    float totalMass = 0.0f;
    for (int k = 0; k < K; ++k) {
        float mp = or_marginal_pdf(m, k, c);
        w[k] = m->weights[k] * mp;
        totalMass += w[k];
    }
    float totalMassCutoff = (float)(0.99 * (double)totalMass);
    float accum = 0.0f;
    int lastIdx = K; /* reference leaves it uninitialised if never reached */
    for (int i = 0; i < K; ++i) {
        /* i-th element of a descending sort, ties -> lowest index */
        int best = -1;
        for (int k = 0; k < K; ++k) {
            if (taken[k]) continue;
            if (best < 0 || w[k] > w[best]) best = k;
        }
        taken[best] = 1;
        out->index[i] = best;
        out->weights[i] = w[best];
        int ok = cond_mean_dir(m, best, c, out->mean + 3 * i);
        if (!ok) { out->weights[i] = 0.0f; } /* stale component in the reference */
        or_coordinates(out->mean + 3 * i, out->to + 9 * i);
        accum += out->weights[i];
        if (accum >= totalMassCutoff) { lastIdx = i + 1; break; }
    }
    out->lastIdx = lastIdx;
    float sum = 0.0f;
    for (int i = 0; i < lastIdx; ++i) sum += out->weights[i];
    const float invSum = 1.0f / sum;
    out->heuristicConditionalWeight = 0.0f;
    if (isfinite(invSum)) {
        out->heuristicConditionalWeight = m->heuristicWeight * 1.0f * invSum;
        for (int i = 0; i < lastIdx; ++i) out->weights[i] = out->weights[i] * invSum;
    }
    out->valid = create_cdf_f(out->weights, lastIdx, out->cdf, 1);
    free(w);
    free(taken);
    return out->valid;
}

int or_conditional_sample(const or_mixture* m, const or_conditional* cd, const float u[3],
                          float dir[3]) {
    FTZ_SCOPE;
    int slot = or_sample_discrete_cdf(cd->cdf, cd->lastIdx, u[0]);
    int k = cd->index[slot];
    /* boxMullerTransform (mvtn.h:667-676) */
    float radius = sqrtf(-2.0f * fl_log(1.0f - u[1]));
    float theta = (float)(2.0 * OR_PI * (double)u[2]);
    double res0 = sin((double)theta), res1 = cos((double)theta);
    float z0 = radius * (float)res0, z1 = radius * (float)res1;
    const float* L = m->condL + 4 * k;
    float v0 = L[0] * z0 + L[1] * z1;
    float v1 = L[2] * z0 + L[3] * z1;
    float tan5[5] = {0.0f, 0.0f, 0.0f, v0, v1};
    float emb[6], jac;
    if (!or_ts_exp(cd->to + 9 * slot, tan5, emb, &jac)) {
        dir[0] = dir[1] = dir[2] = 0.0f;
    } else {
        dir[0] = emb[3]; dir[1] = emb[4]; dir[2] = emb[5];
    }
    return slot;
}

float or_conditional_pdf(const or_mixture* m, const or_conditional* cd, const float dir[3]) {
    FTZ_SCOPE;
    static float NORM2 = -1.0f;
    if (NORM2 < 0.0f) NORM2 = norm_const(2);
    float acc = 0.0f;
    for (int i = 0; i < cd->lastIdx; ++i) {
        if (cd->weights[i] == 0.0f) continue;
        int k = cd->index[i];
        float emb[6] = {0.0f, 0.0f, 0.0f, dir[0], dir[1], dir[2]};
        float tan5[5], jac;
        float p = 0.0f;
        if (or_ts_log(cd->to + 9 * i, emb, tan5, &jac)) {
            const float* Li = m->condLInv + 4 * k;
            float s0 = Li[0] * tan5[3] + Li[1] * tan5[4];
            float s1 = Li[2] * tan5[3] + Li[3] * tan5[4];
            float q = s0 * s0 + s1 * s1;
            p = (float)((double)NORM2 * exp(-0.5 * (double)q));
            p *= m->condDetInv[k] * jac;
        }
        acc += cd->weights[i] * p;
    }
    return acc;
}

static void cond_alloc(or_conditional* cd, int K) {
    cd->index = (int*)malloc(sizeof(int) * K);
    cd->weights = (float*)malloc(sizeof(float) * K);
    cd->cdf = (float*)malloc(sizeof(float) * K);
    cd->mean = (float*)malloc(sizeof(float) * K * 3);
    cd->to = (float*)malloc(sizeof(float) * K * 9);
}
static void cond_free(or_conditional* cd) {
    free(cd->index); free(cd->weights); free(cd->cdf); free(cd->mean); free(cd->to);
}

void or_guide_batch(const or_mixture* m, int64_t nq, const float* c, const float* u, float* dir,
                    float* pdf, int32_t* comp, int32_t* slot) {
    FTZ_SCOPE;
    or_conditional cd;
    cond_alloc(&cd, m->K);
    for (int64_t q = 0; q < nq; ++q) {
        if (!or_conditional_create(m, c + 3 * q, &cd)) {
            dir[3 * q] = dir[3 * q + 1] = dir[3 * q + 2] = 0.0f;
            pdf[q] = 0.0f;
            comp[q] = -1;
            if (slot) slot[q] = -1;
            continue;
        }
        int s = or_conditional_sample(m, &cd, u + 3 * q, dir + 3 * q);
        comp[q] = cd.index[s];
        if (slot) slot[q] = s;
        pdf[q] = or_conditional_pdf(m, &cd, dir + 3 * q);
    }
    cond_free(&cd);
}

void or_pdf_batch(const or_mixture* m, int64_t nq, const float* c, const float* d, float* pdf) {
    FTZ_SCOPE;
    or_conditional cd;
    cond_alloc(&cd, m->K);
    for (int64_t q = 0; q < nq; ++q) {
        if (!or_conditional_create(m, c + 3 * q, &cd)) { pdf[q] = 0.0f; continue; }
        pdf[q] = or_conditional_pdf(m, &cd, d + 3 * q);
    }
    cond_free(&cd);
}

#include "sdmm_oracle_product.inc"
#include "sdmm_oracle_li.inc"
