// guide.hip -- per-bounce guided conditional / sample / pdf on gfx950.
//
// Replaces, for a batch (wavefront) of guided queries against one mixture:
//   MixtureModel::conditional   mixture_model.h:235-304  (marginal weights,
//                               descending sort, 0.99-mass cutoff, normalise)
//   MultivariateNormal::pdf     multivariate_normal.h:118-128
//   MVTN::conditional           multivariate_tangent_normal.h:417-439, :122-144
//   MixtureModel::sample        mixture_model.h:72-75 + utils.h:104-115
//   MVTN::sample / Box-Muller   multivariate_tangent_normal.h:321-339, :667-676
//   MixtureModel::pdf           mixture_model.h:113-121 (+ MVTN::pdf :367-381)
// as called per bounce by SDMMRenderer::sampleSurface / pdfSurface
// (sdmm_proc.cpp:368, :411-421, :539-545).
//
// One thread per query.  The per-query marginal weights live in LDS laid out
// [k][thread] (conflict-free); the sort is an incremental selection that stops
// at the 0.99-mass cutoff, so only the kept prefix is ever ordered.  Every
// floating-point step follows oracle/sdmm_oracle.c operation for operation
// (no FMA contraction, double-precision transcendentals rounded to float, IEEE
// division/sqrt), which makes the selected component index bit-identical.
#include "sdmm_device.h"

#pragma clang fp contract(off)

namespace sdmm {

struct GuideConsts {
    float norm2, norm3;
};

__device__ __forceinline__ float gp_ld(const float* gp, int Kp, int f, int k) {
    return ((cfloat_p)gp)[f * Kp + k];
}

__device__ __forceinline__ float fl_acos(float x) { return (float)acos((double)x); }
__device__ __forceinline__ float fl_cos(float x) { return (float)cos((double)x); }
__device__ __forceinline__ float fl_sin(float x) { return (float)sin((double)x); }
__device__ __forceinline__ float fl_log(float x) { return (float)log((double)x); }

__device__ __forceinline__ void coordinates_f(const float n[3], float to[9]) {
    float sign = copysignf(1.0f, n[2]);
    const float a = -1.0f / (sign + n[2]);
    const float b = n[0] * n[1] * a;
    to[0] = 1.0f + sign * n[0] * n[0] * a; to[1] = sign * b; to[2] = -sign * n[0];
    to[3] = b; to[4] = sign + n[1] * n[1] * a; to[5] = -n[1];
    to[6] = n[0]; to[7] = n[1]; to[8] = n[2];
}

__device__ __forceinline__ float sinc_pi_f(float x) {
    const float taylor_0_bound = 1.1920928955078125e-07f;
    const float taylor_2_bound = 3.4526698300124393e-04f;  // sqrtf(eps)
    const float taylor_n_bound = 1.8581361171917516e-02f;  // sqrtf(sqrtf(eps))
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

// TangentSpace::exp restricted to the directional part; to = m_invRotation.
__device__ __forceinline__ bool ts_exp_dir(const float to[9], float t0, float t1, float e[3]) {
    float length = sqrtf(t0 * t0 + t1 * t1);
    if ((double)length >= kPi) { e[0] = e[1] = e[2] = 0.0f; return false; }
    float s = sinc_pi_f(length);
    float rel0 = t0 * s, rel1 = t1 * s, rel2 = fl_cos(length);
    e[0] = to[0] * rel0 + to[3] * rel1 + to[6] * rel2;
    e[1] = to[1] * rel0 + to[4] * rel1 + to[7] * rel2;
    e[2] = to[2] * rel0 + to[5] * rel1 + to[8] * rel2;
    return true;
}

// MVN<3,3>::pdf with the forward substitution of LLT::matrixL().solve.
__device__ __forceinline__ float marginal_pdf(const float* gp, int Kp, int k, const float c[3],
                                              float norm3) {
    float r0 = c[0] - gp_ld(gp, Kp, GP_MU0, k);
    float r1 = c[1] - gp_ld(gp, Kp, GP_MU1, k);
    float r2 = c[2] - gp_ld(gp, Kp, GP_MU2, k);
    float s0 = r0 / gp_ld(gp, Kp, GP_ML00, k);
    r1 = r1 - s0 * gp_ld(gp, Kp, GP_ML10, k);
    r2 = r2 - s0 * gp_ld(gp, Kp, GP_ML20, k);
    float s1 = r1 / gp_ld(gp, Kp, GP_ML11, k);
    r2 = r2 - s1 * gp_ld(gp, Kp, GP_ML21, k);
    float s2 = r2 / gp_ld(gp, Kp, GP_ML22, k);
    float q = s0 * s0 + s1 * s1 + s2 * s2;
    float pdf = (float)((double)norm3 * exp(-0.5 * (double)q));
    return pdf * gp_ld(gp, Kp, GP_MDI, k);
}

// MVTN::conditional: mean direction of joint component k's conditional at c.
__device__ __forceinline__ bool cond_mean_dir(const float* gp, int Kp, int k, const float c[3],
                                              float e[3]) {
    float d0 = c[0] - gp_ld(gp, Kp, GP_MU0, k);
    float d1 = c[1] - gp_ld(gp, Kp, GP_MU1, k);
    float d2 = c[2] - gp_ld(gp, Kp, GP_MU2, k);
    float t0 = gp_ld(gp, Kp, GP_P00, k) * d0 + gp_ld(gp, Kp, GP_P01, k) * d1 + gp_ld(gp, Kp, GP_P02, k) * d2;
    float t1 = gp_ld(gp, Kp, GP_P10, k) * d0 + gp_ld(gp, Kp, GP_P11, k) * d1 + gp_ld(gp, Kp, GP_P12, k) * d2;
    float to[9];
    for (int i = 0; i < 9; ++i) to[i] = gp_ld(gp, Kp, GP_T00 + i, k);
    return ts_exp_dir(to, t0, t1, e);
}

// MVTN<3,3>::pdf(d) for the conditional component of joint component k whose
// conditional mean direction is e (log map in the frame Coordinates(e)).
__device__ __forceinline__ float cond_component_pdf(const float* gp, int Kp, int k, const float e[3],
                                                    const float d[3], float norm2) {
    if (d[0] == 0.0f && d[1] == 0.0f && d[2] == 0.0f) return 0.0f;
    float to[9];
    coordinates_f(e, to);
    float r0 = to[0] * d[0] + to[1] * d[1] + to[2] * d[2];
    float r1 = to[3] * d[0] + to[4] * d[1] + to[5] * d[2];
    float cth = to[6] * d[0] + to[7] * d[1] + to[8] * d[2];
    if (cth <= -1.0f) return 0.0f;
    cth = (cth < 1.0f) ? cth : 1.0f;
    float angle = fl_acos(cth);
    float s = sqrtf(1.0f - cth * cth);
    float a = ((double)s < 1e-3) ? 1.0f : (angle / s);
    float t0 = r0 * a, t1 = r1 * a;
    float s0 = gp_ld(gp, Kp, GP_CI00, k) * t0 + gp_ld(gp, Kp, GP_CI01, k) * t1;
    float s1 = gp_ld(gp, Kp, GP_CI10, k) * t0 + gp_ld(gp, Kp, GP_CI11, k) * t1;
    float q = s0 * s0 + s1 * s1;
    float p = (float)((double)norm2 * exp(-0.5 * (double)q));
    p *= gp_ld(gp, Kp, GP_CDI, k) * a;
    return p;
}

// Shared per-query conditional construction.  Returns lastIdx (0 if the
// conditional is invalid); fills the LDS slot list.  wl: [K][T] weights whose
// sign bit marks "taken"; sl: [K][T] slot -> component.
struct CondInfo {
    int lastIdx;
    float invSum;   // 1/sum if finite else 1 (no scaling)
    bool scaled;
    float sum2;
};

__device__ __forceinline__ CondInfo build_conditional(const float* gp, int Kp, int K, const float c[3],
                                                      float* wl, int* sl, int T, int tid, float norm3) {
    float total = 0.0f;
    for (int k = 0; k < K; ++k) {
        const float mp = marginal_pdf(gp, Kp, k, c, norm3);
        const float wk = gp_ld(gp, Kp, GP_W, k) * mp;
        wl[k * T + tid] = wk;
        total += wk;
    }
    const float cutoff = (float)(0.99 * (double)total);
    float accum = 0.0f;
    int lastIdx = K;
    for (int i = 0; i < K; ++i) {
        int best = -1;
        float bw = 0.0f;
        for (int k = 0; k < K; ++k) {
            const float x = wl[k * T + tid];
            if (__builtin_signbit(x)) continue;
            if (best < 0 || x > bw) { best = k; bw = x; }
        }
        if (best < 0) { lastIdx = i; break; }
        wl[best * T + tid] = -bw;
        sl[i * T + tid] = best;
        float e[3];
        float wi = bw;
        if (!cond_mean_dir(gp, Kp, best, c, e)) wi = 0.0f;  // oracle convention
        accum += wi;
        if (accum >= cutoff) { lastIdx = i + 1; break; }
    }
    CondInfo ci;
    ci.lastIdx = lastIdx;
    // sum of the kept weights (std::accumulate) == accum (same values, same order)
    const float invSum = 1.0f / accum;
    ci.scaled = __builtin_isfinite(invSum);
    ci.invSum = invSum;
    float sum2 = 0.0f;
    for (int i = 0; i < lastIdx; ++i) {
        const int k = sl[i * T + tid];
        float wi = -wl[k * T + tid];
        float e[3];
        if (!cond_mean_dir(gp, Kp, k, c, e)) wi = 0.0f;
        if (ci.scaled) wi = wi * invSum;
        sum2 += wi;
    }
    ci.sum2 = sum2;
    return ci;
}

// normalised conditional weight of slot i (createCdf(true) after the 1/sum scale)
__device__ __forceinline__ float slot_weight(const float* gp, int Kp, const float c[3], const CondInfo& ci,
                                             const float* wl, const int* sl, int T, int tid, int i,
                                             int& k, float e[3]) {
    k = sl[i * T + tid];
    float wi = -wl[k * T + tid];
    if (!cond_mean_dir(gp, Kp, k, c, e)) wi = 0.0f;
    if (ci.scaled) wi = wi * ci.invSum;
    return wi / ci.sum2;
}

__global__ void __launch_bounds__(64)
guide_kernel(const float* __restrict__ gp, int Kp, int K, int64_t nq, const float* __restrict__ c0,
             const float* __restrict__ c1, const float* __restrict__ c2, const float* __restrict__ u0,
             const float* __restrict__ u1, const float* __restrict__ u2, float* __restrict__ d0,
             float* __restrict__ d1, float* __restrict__ d2, float* __restrict__ pdf,
             int32_t* __restrict__ comp, GuideConsts gc) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int T = blockDim.x;
    const int tid = threadIdx.x;
    float* wl = lds;
    int* sl = (int*)(lds + (size_t)K * T);
    const int64_t q = (int64_t)blockIdx.x * T + tid;
    if (q >= nq) return;
    const float c[3] = {c0[q], c1[q], c2[q]};
    const float u[3] = {u0[q], u1[q], u2[q]};
    const CondInfo ci = build_conditional(gp, Kp, K, c, wl, sl, T, tid, gc.norm3);
    if (ci.lastIdx == 0 || ci.sum2 == 0.0f) {
        d0[q] = 0.0f; d1[q] = 0.0f; d2[q] = 0.0f; pdf[q] = 0.0f; comp[q] = -1;
        return;
    }
    // sampleDiscreteCdf: lower_bound == first slot with cdf >= u, else tie walk
    float cdf = 0.0f, prev = 0.0f;
    int slot = -1, runStart = 0;
    int ksel = -1;
    float esel[3] = {0.0f, 0.0f, 0.0f};
    for (int i = 0; i < ci.lastIdx; ++i) {
        int k;
        float e[3];
        const float f = slot_weight(gp, Kp, c, ci, wl, sl, T, tid, i, k, e);
        cdf += f;
        if (i == 0 || cdf != prev) runStart = i;
        prev = cdf;
        if (cdf >= u[0]) { slot = i; ksel = k; esel[0] = e[0]; esel[1] = e[1]; esel[2] = e[2]; break; }
    }
    if (slot < 0) {
        slot = runStart;
        float e[3];
        int k;
        slot_weight(gp, Kp, c, ci, wl, sl, T, tid, slot, k, e);
        ksel = k; esel[0] = e[0]; esel[1] = e[1]; esel[2] = e[2];
    }
    // MVTN::sample of the conditional component (Box-Muller, L z, exp map)
    const float radius = sqrtf(-2.0f * fl_log(1.0f - u[1]));
    const float theta = (float)(2.0 * kPi * (double)u[2]);
    const double res0 = sin((double)theta), res1 = cos((double)theta);
    const float z0 = radius * (float)res0, z1 = radius * (float)res1;
    const float L00 = gp_ld(gp, Kp, GP_CL00, ksel), L10 = gp_ld(gp, Kp, GP_CL10, ksel);
    const float L11 = gp_ld(gp, Kp, GP_CL11, ksel);
    const float v0 = L00 * z0 + 0.0f * z1;
    const float v1 = L10 * z0 + L11 * z1;
    float tof[9];
    coordinates_f(esel, tof);
    float dir[3];
    ts_exp_dir(tof, v0, v1, dir);
    // MixtureModel::pdf over the conditional (the gmmPdf of pdfSurface)
    float acc = 0.0f;
    for (int i = 0; i < ci.lastIdx; ++i) {
        int k;
        float e[3];
        const float f = slot_weight(gp, Kp, c, ci, wl, sl, T, tid, i, k, e);
        if (f == 0.0f) continue;
        acc += f * cond_component_pdf(gp, Kp, k, e, dir, gc.norm2);
    }
    d0[q] = dir[0]; d1[q] = dir[1]; d2[q] = dir[2];
    pdf[q] = acc;
    comp[q] = ksel;
}

// gmmPdf of a given direction (BSDF-sampled bounce): conditional + pdf.
__global__ void __launch_bounds__(64)
guide_pdf_kernel(const float* __restrict__ gp, int Kp, int K, int64_t nq, const float* __restrict__ c0,
                 const float* __restrict__ c1, const float* __restrict__ c2, const float* __restrict__ e0,
                 const float* __restrict__ e1, const float* __restrict__ e2, float* __restrict__ pdf,
                 GuideConsts gc) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int T = blockDim.x;
    const int tid = threadIdx.x;
    float* wl = lds;
    int* sl = (int*)(lds + (size_t)K * T);
    const int64_t q = (int64_t)blockIdx.x * T + tid;
    if (q >= nq) return;
    const float c[3] = {c0[q], c1[q], c2[q]};
    const float dir[3] = {e0[q], e1[q], e2[q]};
    const CondInfo ci = build_conditional(gp, Kp, K, c, wl, sl, T, tid, gc.norm3);
    if (ci.lastIdx == 0 || ci.sum2 == 0.0f) { pdf[q] = 0.0f; return; }
    float acc = 0.0f;
    for (int i = 0; i < ci.lastIdx; ++i) {
        int k;
        float e[3];
        const float f = slot_weight(gp, Kp, c, ci, wl, sl, T, tid, i, k, e);
        if (f == 0.0f) continue;
        acc += f * cond_component_pdf(gp, Kp, k, e, dir, gc.norm2);
    }
    pdf[q] = acc;
}

// lower_bound + tie walk on caller-provided CDFs (the bit-exact index KAT).
__global__ void sample_cdf_kernel(const float* __restrict__ cdf, int n, const float* __restrict__ u,
                                  int64_t nq, int32_t* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const float x = u[q];
    int lo = 0, count = n;
    while (count > 0) {
        int step = count / 2, it = lo + step;
        if (cdf[it] < x) { lo = it + 1; count -= step + 1; }
        else count = step;
    }
    if (lo == n) {
        --lo;
        while (lo > 0 && cdf[lo] == cdf[lo - 1]) --lo;
    }
    out[q] = lo;
}

static int guide_threads() { return 64; }

hipError_t launch_guide(const float* gp, int Kp, int K, int64_t nq, const float* const c[3],
                        const float* const u[3], float* const d[3], float* pdf, int32_t* comp,
                        float norm2, float norm3, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    const int T = guide_threads();
    const size_t lds = (size_t)K * T * (sizeof(float) + sizeof(int));
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    GuideConsts gc{norm2, norm3};
    const int64_t blocks = (nq + T - 1) / T;
    hipLaunchKernelGGL(guide_kernel, dim3((unsigned)blocks), dim3(T), lds, st, gp, Kp, K, nq, c[0], c[1],
                       c[2], u[0], u[1], u[2], d[0], d[1], d[2], pdf, comp, gc);
    return hipGetLastError();
}

hipError_t launch_guide_pdf(const float* gp, int Kp, int K, int64_t nq, const float* const c[3],
                            const float* const d[3], float* pdf, float norm2, float norm3,
                            hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    const int T = guide_threads();
    const size_t lds = (size_t)K * T * (sizeof(float) + sizeof(int));
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    GuideConsts gc{norm2, norm3};
    const int64_t blocks = (nq + T - 1) / T;
    hipLaunchKernelGGL(guide_pdf_kernel, dim3((unsigned)blocks), dim3(T), lds, st, gp, Kp, K, nq, c[0],
                       c[1], c[2], d[0], d[1], d[2], pdf, gc);
    return hipGetLastError();
}

hipError_t launch_sample_cdf(const float* cdf, int n, const float* u, int64_t nq, int32_t* out,
                             hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    hipLaunchKernelGGL(sample_cdf_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, cdf, n, u,
                       nq, out);
    return hipGetLastError();
}

}  // namespace sdmm
