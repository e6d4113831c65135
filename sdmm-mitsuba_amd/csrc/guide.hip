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
// at the 0.99-mass cutoff, so only the kept prefix is ever ordered.
//
// Precision split.  Everything the selected component index depends on -- the
// marginal weights, the validity of each conditional, the normalisation and
// the CDF -- follows oracle/sdmm_oracle.c operation for operation (no FMA
// contraction, the double-precision exp of mvtn.h:359 rounded to float, IEEE
// division/sqrt), which makes the index bit-identical.  A marginal weight whose
// exponent argument puts NORM3 exp(-q/2) below FLT_MIN is exactly 0 under the
// plugin's FTZ (volpath_sdmm.cpp:88-90) and skips the double exp.  The sampled
// direction and the mixture pdf (tolerances 1e-5 / 1e-4) use the float
// transcendentals.
#include "sdmm_device.h"
#include <cstdlib>

#include <hipcub/hipcub.hpp>

#pragma clang fp contract(off)

namespace sdmm {

// (diagnostic SDMM_WAVE_CLOCK: per-phase shader clocks of the one-wave full-K
// product path, summed by workgroups 0..3 and printed at their end)
#ifdef SDMM_WAVE_CLOCK
__shared__ unsigned long long g_wclk[12];
__shared__ unsigned long long g_wlast;
#define WCLK(i)                                                          \
    do {                                                                 \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();   \
        if (threadIdx.x == 0) { g_wclk[i] += now_ - g_wlast; g_wlast = now_; } \
    } while (0)
#else
#define WCLK(i) do {} while (0)
#endif

struct GuideConsts {
    float norm2, norm3;
    // product path: a candidate-served query with more than this many pairs
    // (kept slots x table lobes) goes to the one-wave path instead (the
    // same bits; its pairs then run 64 at a time)
    int route_pairs = 0x7fffffff;
};
// The threshold above: 160 pairs (Kitchen product, 8 lobes, capacity 40:
// 8.75 -> 8.32 ms a call, profiles/round6_ab_route.log; the Cornell products'
// candidate queries stay below it).  SDMM_PRODUCT_ROUTE_PAIRS overrides.
static int product_route_pairs() {
    static const int v = [] {
        const char* e = std::getenv("SDMM_PRODUCT_ROUTE_PAIRS");
        return e && *e ? std::atoi(e) : 160;
    }();
    return v;
}

// A Gaussian weight as the reference forms it: (float)((double)norm *
// exp(-0.5 * (double)q)) (multivariate_normal.h:126, mvtn.h:359).  Round 5
// measured a table-driven double exp decided by a Ziv rounding test in its
// place: no faster (the device double exp is ~30 instructions, 14 of them
// DFMA, about what the table path costs) and the LDS table cost occupancy --
// Cornell K = 128 guided pass 12.0 vs 11.3 ms, K = 512 product 91 vs 86 ms.
__device__ __forceinline__ float gauss_w(float norm, float q) {
    return (float)((double)norm * exp(-0.5 * (double)q));
}

__device__ __forceinline__ float gp_ld(const float* gp, int Kp, int f, int k) {
    return ((cfloat_p)gp)[k * GP_STRIDE + f];   // AoS record (sdmm_device.h)
}

// q above this gives NORM3 exp(-q/2) < 2^-126: the float weight flushes to 0
// (2 (126 ln 2 + ln NORM3) = 169.16, with margin)
constexpr float kMarginalZeroQ = 170.0f;

__device__ __forceinline__ float sinc_pi_f(float x) {
    const float taylor_0_bound = 1.1920928955078125e-07f;
    const float taylor_2_bound = 3.4526698300124393e-04f;  // sqrtf(eps)
    const float taylor_n_bound = 1.8581361171917516e-02f;  // sqrtf(sqrtf(eps))
    float ax = fabsf(x);
    if (ax >= taylor_n_bound) return sinf(x) / x;
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
    float rel0 = t0 * s, rel1 = t1 * s, rel2 = cosf(length);
    e[0] = to[0] * rel0 + to[3] * rel1 + to[6] * rel2;
    e[1] = to[1] * rel0 + to[4] * rel1 + to[7] * rel2;
    e[2] = to[2] * rel0 + to[5] * rel1 + to[8] * rel2;
    return true;
}

// IEEE float division x / d as (float)((double)x * RN64(1 / d)), bit for bit.
// Why exact: write x / d = (A / B) 2^e with A, B < 2^24 integer significands.
// A float rounding midpoint near it is N / 2^s with N odd of 25 bits; then
// A / B - N / 2^s = (A 2^s - N B) / (B 2^s) with a NONZERO integer numerator
// (N odd and > A cannot divide A 2^s), so the exact quotient is at least
// 2^-49 / |A/B| ~ 2^-50 (relative) away from every midpoint, while the double
// product is within 2^-52 of it (two roundings to 53 bits).  Rounding the
// product to float therefore lands on the same float as rounding the exact
// quotient; exact quotients stay exact.  (The usual "double rounding is
// innocuous for >= 2p + 2 bits" argument, applied to a reciprocal product.)
// Replaces the ~11-instruction v_div_scale/fmas/fixup expansion and its two
// s_setreg denormal-mode switches per division.
__device__ __forceinline__ float div_exact(float x, const float* gp, int f, int k) {
    const uint32_t lo = __builtin_bit_cast(uint32_t, ((cfloat_p)gp)[k * GP_STRIDE + f]);
    const uint32_t hi = __builtin_bit_cast(uint32_t, ((cfloat_p)gp)[k * GP_STRIDE + f + 1]);
    const double r = __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
    return (float)((double)x * r);
}

// x / d for many x and one d, bit for bit as the float division (the same
// argument as div_exact: RN64(1 / d) once, then one double product per
// quotient rounded to float; FTZ flushes a denormal quotient in both).  The
// float division is ~10 instructions with two denormal-mode switches.
struct DivBy {
    double r;
    __device__ explicit DivBy(float d) : r(1.0 / (double)d) {}
    __device__ float operator()(float x) const { return (float)((double)x * r); }
};

// MVN<3,3>::pdf with the forward substitution of LLT::matrixL().solve:
// marginal_q is the squared Mahalanobis distance, marginal_pdf_q the pdf.
__device__ __forceinline__ float marginal_q(const float* gp, int Kp, int k, const float c[3]) {
    float r0 = c[0] - gp_ld(gp, Kp, GP_MU0, k);
    float r1 = c[1] - gp_ld(gp, Kp, GP_MU1, k);
    float r2 = c[2] - gp_ld(gp, Kp, GP_MU2, k);
    float s0 = div_exact(r0, gp, GP_RML00, k);   // r0 / ML00
    r1 = r1 - s0 * gp_ld(gp, Kp, GP_ML10, k);
    r2 = r2 - s0 * gp_ld(gp, Kp, GP_ML20, k);
    float s1 = div_exact(r1, gp, GP_RML11, k);   // r1 / ML11
    r2 = r2 - s1 * gp_ld(gp, Kp, GP_ML21, k);
    float s2 = div_exact(r2, gp, GP_RML22, k);   // r2 / ML22
    return s0 * s0 + s1 * s1 + s2 * s2;
}
__device__ __forceinline__ float marginal_pdf_q(const float* gp, int Kp, int k, float q, float norm3) {
    if (q > kMarginalZeroQ) return 0.0f;   // flushes to 0 in the reference (FTZ)
    float pdf = gauss_w(norm3, q);
    return pdf * gp_ld(gp, Kp, GP_MDI, k);
}
__device__ __forceinline__ float marginal_pdf(const float* gp, int Kp, int k, const float c[3], float norm3) {
    return marginal_pdf_q(gp, Kp, k, marginal_q(gp, Kp, k, c), norm3);
}

// The marginal fields of component k's record (weight, mean, the Cholesky
// entries the forward substitution reads, detInv, the three exact-division
// reciprocals), loaded together so that a loop over components can fetch
// component k + 1's while it evaluates k (the record loads of a per-lane
// mixture pointer are vector loads with L2 latency).  Same operations as
// marginal_q / marginal_pdf_q above.
struct MargRec {
    float w, mu0, mu1, mu2, ml10, ml20, ml21, mdi;
    uint32_t r[6];
};
__device__ __forceinline__ MargRec load_marg(const float* gp, int k) {
    const cfloat_p b = (cfloat_p)gp + k * GP_STRIDE;
    MargRec m;
    m.w = b[GP_W]; m.mu0 = b[GP_MU0]; m.mu1 = b[GP_MU1]; m.mu2 = b[GP_MU2];
    m.ml10 = b[GP_ML10]; m.ml20 = b[GP_ML20]; m.ml21 = b[GP_ML21]; m.mdi = b[GP_MDI];
#pragma unroll
    for (int i = 0; i < 6; ++i) m.r[i] = __builtin_bit_cast(uint32_t, b[GP_RML00 + i]);
    return m;
}
__device__ __forceinline__ double marg_rcp(const MargRec& m, int i) {
    return __builtin_bit_cast(double, (uint64_t)m.r[2 * i] | ((uint64_t)m.r[2 * i + 1] << 32));
}
__device__ __forceinline__ float marginal_weight_rec(const MargRec& m, const float c[3], float norm3) {
    float r0 = c[0] - m.mu0;
    float r1 = c[1] - m.mu1;
    float r2 = c[2] - m.mu2;
    float s0 = (float)((double)r0 * marg_rcp(m, 0));   // r0 / ML00
    r1 = r1 - s0 * m.ml10;
    r2 = r2 - s0 * m.ml20;
    float s1 = (float)((double)r1 * marg_rcp(m, 1));   // r1 / ML11
    r2 = r2 - s1 * m.ml21;
    float s2 = (float)((double)r2 * marg_rcp(m, 2));   // r2 / ML22
    const float q = s0 * s0 + s1 * s1 + s2 * s2;
    float pdf = 0.0f;
    if (!(q > kMarginalZeroQ)) pdf = gauss_w(norm3, q) * m.mdi;
    return m.w * pdf;
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
    float angle = acosf(cth);
    float s = sqrtf(1.0f - cth * cth);
    float a = ((double)s < 1e-3) ? 1.0f : (angle / s);
    float t0 = r0 * a, t1 = r1 * a;
    float s0 = gp_ld(gp, Kp, GP_CI00, k) * t0 + gp_ld(gp, Kp, GP_CI01, k) * t1;
    float s1 = gp_ld(gp, Kp, GP_CI10, k) * t0 + gp_ld(gp, Kp, GP_CI11, k) * t1;
    float q = s0 * s0 + s1 * s1;
    float p = norm2 * expf(-0.5f * q);
    p *= gp_ld(gp, Kp, GP_CDI, k) * a;
    return p;
}
// validity of joint component k's conditional at c (cond_mean_dir's
// TangentSpace::exp check, same float operations) without the sin/cos
__device__ __forceinline__ bool cond_valid(const float* gp, int Kp, int k, const float c[3]) {
    float d0 = c[0] - gp_ld(gp, Kp, GP_MU0, k);
    float d1 = c[1] - gp_ld(gp, Kp, GP_MU1, k);
    float d2 = c[2] - gp_ld(gp, Kp, GP_MU2, k);
    float t0 = gp_ld(gp, Kp, GP_P00, k) * d0 + gp_ld(gp, Kp, GP_P01, k) * d1 + gp_ld(gp, Kp, GP_P02, k) * d2;
    float t1 = gp_ld(gp, Kp, GP_P10, k) * d0 + gp_ld(gp, Kp, GP_P11, k) * d1 + gp_ld(gp, Kp, GP_P12, k) * d2;
    float length = sqrtf(t0 * t0 + t1 * t1);
    return !((double)length >= kPi);
}

// ---------------------------------------------------------------------------
// The part of a query after the kept (sorted, cut-off) prefix is known:
// normalisation, sampleDiscreteCdf, Box-Muller + exp map, and the conditional
// mixture pdf (mixture_model.h:286-303, :72-75, :113-121; utils.h:64-115;
// mvtn.h:321-339, :367-381).  Slots supplies slot i -> (component, raw
// weight, valid); weights of invalid conditionals count as 0 (oracle
// convention, oracle/sdmm_oracle.c or_conditional_create).
struct QueryOut {
    float d[3];
    float pdf;
    int comp;
};
// comp of a query evaluated at a given direction (the mixed wavefront's pdf
// queries) whose conditional is valid; -1 stays "no valid conditional".
constexpr int kCompPdfValid = -2;

template <class Slots>
__device__ __forceinline__ QueryOut finish_query(const float* gp, int Kp, const float c[3], const float u[3],
                                                 int lastIdx, float accum, const Slots& S,
                                                 const float* dir_in, GuideConsts gc) {
    QueryOut o{{0.0f, 0.0f, 0.0f}, 0.0f, -1};
    // sum of the kept weights (std::accumulate) == accum (same values, same order)
    const float invSum = 1.0f / accum;
    const bool scaled = __builtin_isfinite(invSum);
    float sum2 = 0.0f;
    for (int i = 0; i < lastIdx; ++i) {
        float wi = S.valid(i) ? S.weight(i) : 0.0f;
        if (scaled) wi = wi * invSum;
        sum2 += wi;
    }
    if (lastIdx == 0 || sum2 == 0.0f) return o;   // createCdf(true) fails: BSDF only
    const DivBy by_sum2(sum2);
    auto slot_w = [&](int i) {
        float wi = S.valid(i) ? S.weight(i) : 0.0f;
        if (scaled) wi = wi * invSum;
        return by_sum2(wi);
    };
    float dir[3];
    if (!dir_in) {
        // sampleDiscreteCdf: lower_bound == first slot with cdf >= u, else tie walk
        float cdf = 0.0f, prev = 0.0f;
        int slot = -1, runStart = 0;
        for (int i = 0; i < lastIdx; ++i) {
            cdf += slot_w(i);
            if (i == 0 || cdf != prev) runStart = i;
            prev = cdf;
            if (cdf >= u[0]) { slot = i; break; }
        }
        if (slot < 0) slot = runStart;
        const int ksel = S.comp(slot);
        float esel[3];
        cond_mean_dir(gp, Kp, ksel, c, esel);
        // MVTN::sample of the conditional component (Box-Muller, L z, exp map)
        const float radius = sqrtf(-2.0f * logf(1.0f - u[1]));
        const float theta = (float)(2.0 * kPi * (double)u[2]);
        float res0, res1;
        sincosf(theta, &res0, &res1);
        const float z0 = radius * res0, z1 = radius * res1;
        const float L00 = gp_ld(gp, Kp, GP_CL00, ksel), L10 = gp_ld(gp, Kp, GP_CL10, ksel);
        const float L11 = gp_ld(gp, Kp, GP_CL11, ksel);
        const float v0 = L00 * z0 + 0.0f * z1;
        const float v1 = L10 * z0 + L11 * z1;
        float tof[9];
        coordinates_f(esel, tof);
        ts_exp_dir(tof, v0, v1, dir);
        o.comp = ksel;
    } else {
        dir[0] = dir_in[0]; dir[1] = dir_in[1]; dir[2] = dir_in[2];
        o.comp = kCompPdfValid;
    }
    // MixtureModel::pdf over the conditional (the gmmPdf of pdfSurface)
    float acc = 0.0f;
    for (int i = 0; i < lastIdx; ++i) {
        const float f = slot_w(i);
        if (f == 0.0f) continue;
        const int k = S.comp(i);
        float e[3];
        cond_mean_dir(gp, Kp, k, c, e);
        acc += f * cond_component_pdf(gp, Kp, k, e, dir, gc.norm2);
    }
    o.d[0] = dir[0]; o.d[1] = dir[1]; o.d[2] = dir[2];
    o.pdf = acc;
    return o;
}

// ---------------------------------------------------------------------------
// Fast path: per-query candidate list.
//
// Pass 1 forms totalMass exactly as the reference (sequential float sum in
// component order, mixture_model.h:248-261).  No component with weight
// w < tau = (totalMass - cutoff) / K * 0.999 can be in the kept prefix: all
// of them together hold less than totalMass - cutoff, so the sorted
// accumulation reaches the cutoff before the first of them (the 0.999 covers
// the float rounding of the sums, |error| <= K eps << 1e-3).  Pass 2
// recomputes the weights and keeps those >= tau in an LDS list sorted
// (weight desc, index asc) -- the order of the reference's std::sort with
// ties broken towards the lower index -- together with the validity of their
// conditionals.  The cutoff walk then runs over that list.  A query falls back
// to the full-K path (guide_fallback_kernel) when totalMass is not finite,
// the list overflows, or the list runs out before the cutoff (only possible
// when invalid conditionals zero out kept weights).  With K = 128 the list
// holds a median of ~10 and a 99th percentile of ~34 entries.
#ifndef SDMM_GUIDE_CAP_MAX
#define SDMM_GUIDE_CAP_MAX 64
#endif
constexpr int kGuideCap = SDMM_GUIDE_CAP_MAX;
// lists of at least this capacity are built in registers (build_candidates_reg)
constexpr int kGuideRegCap = 40;

struct CandSlots {
    const float* cw;
    const unsigned short* ck;
    int T, tid;
    __device__ float weight(int i) const { return cw[i * T + tid]; }
    __device__ int comp(int i) const { return ck[i * T + tid] & 0x7fff; }
    __device__ bool valid(int i) const { return (ck[i * T + tid] >> 15) != 0; }
};

// A query whose marginal weights are all exactly zero (totalMass 0, e.g. a
// point far from every component of a narrow, young mixture): the
// reference's scan takes one zero weight (accum 0 >= cutoff 0), createCdf
// then fails on the zero sum and the bounce is BSDF only -- what the full-K
// path computes for it too.  The candidate kernels answer it directly
// (round 4: optimizeAsync's guided passes sent 99-145 K such queries per pass
// down the full-K path).
constexpr int kNoMass = -2;

// returns lastIdx >= 0, or -1: needs the full-K fallback.
//
// ONE pass over the components: it forms totalMass exactly as the reference
// (sequential float sum in component order, mixture_model.h:248-261) and, in
// the same loop, keeps every LIVE component (weight > 0) in the LDS list
// sorted (weight desc, index asc) by stable insertion, at most `cap` of them.
// When the list is full a newcomer either displaces the last entry or is
// dropped.  A dropped weight never exceeds the final last entry (the last
// entry of a full list only grows), and a skipped weight (below the running
// bound, hence below the final tau) is below every candidate, so the list
// prefix with w >= tau is exactly the first ncand entries of the reference's
// selection order.  The cutoff walk runs over it; when it reaches the cutoff
// inside the list the kept prefix is that of the full-K scan, whatever was
// dropped.  Only a walk that exhausts the candidates without reaching the
// cutoff (a full list, or invalid conditionals zeroing kept weights) needs
// the full-K fallback -- unless the candidates are all K components.  tau > 0
// whenever totalMass > 0, so a weight of exactly 0 (all components with q >
// kMarginalZeroQ, most of K) can never be a candidate and never enters the
// list.  Validity of the conditionals is only evaluated for the candidates.
__device__ __forceinline__ int build_candidates(const float* gp, int Kp, int K, const float c[3], float* cw,
                                                unsigned short* ck, int T, int tid, float norm3, int cap,
                                                float& accum) {
    float total = 0.0f;
    int cnt = 0;
    // 0.0089 / K (< the 0.009 / K of the bound below; the float product's
    // rounding, 2^-24 relative, stays far inside the margin): one multiply per
    // component instead of a double division
    const float skip_f = 0.0089f / (float)K;
    MargRec nx = load_marg(gp, 0);   // (K >= 1)
    for (int k = 0; k < K; ++k) {
        const MargRec rec = nx;
        if (k + 1 < K) nx = load_marg(gp, k + 1);   // next component's fields in flight
        const float w = marginal_weight_rec(rec, c, norm3);
        total += w;
        // the float sum of non-negative terms never decreases, so the final
        // tau >= (0.01 total - ulp) 0.999 / K > 0.009 total_so_far / K: a weight
        // below that is never a candidate
        if (!(w > 0.0f) || w < total * skip_f) continue;
        if (cnt == cap) {
            // full: w joins only if it sorts before the last entry (ties keep
            // the lower index, which arrived first)
            if (cap == 0 || !(w > cw[(cap - 1) * T + tid])) continue;
            --cnt;
        }
        int pos = cnt;
        while (pos > 0 && cw[(pos - 1) * T + tid] < w) {
            cw[pos * T + tid] = cw[(pos - 1) * T + tid];
            ck[pos * T + tid] = ck[(pos - 1) * T + tid];
            --pos;
        }
        cw[pos * T + tid] = w;
        ck[pos * T + tid] = (unsigned short)k;
        ++cnt;
    }
    if (!__builtin_isfinite(total)) return -1;
    if (total == 0.0f) return kNoMass;   // every marginal weight zero: BSDF only (below)
    const float cutoff = (float)(0.99 * (double)total);
    const double tau = ((double)total - (double)cutoff) / (double)K * 0.999;
    if (!(tau > 0.0)) return -1;
    int ncand = 0;
    while (ncand < cnt && (double)cw[ncand * T + tid] >= tau) ++ncand;
    accum = 0.0f;
    for (int i = 0; i < ncand; ++i) {
        const int k = ck[i * T + tid];
        const bool ok = cond_valid(gp, Kp, k, c);
        ck[i * T + tid] = (unsigned short)(k | (ok ? 0x8000 : 0));
        accum += ok ? cw[i * T + tid] : 0.0f;
        if (accum >= cutoff) return i + 1;
    }
    // cutoff never reached inside the candidates: exact only if they are all of K
    return (ncand == K) ? K : -1;
}

// The same list built in REGISTERS (LCAP entries, static indices), the
// finished list written to the LDS slots once for the walk and finish.
// Measured (A/B, one box): the tree wavefront over K = 128 leaves (wide,
// long lists) 21.1 -> 17.6 ms per guided pass as a (weight, index)
// compare-and-swap ripple; the K = 16 leaves and the single trained K = 128
// mixture (short lists, where the ripple's fixed LCAP-step cost and its
// registers outweigh the LDS shifts) 466 -> 489 us and 618 -> 692 us -- so
// only the LCAP = 40 instances use it.
// Each (weight, index) entry is one orderable
// 64-bit key held as a double: bits 63..32 = the weight's bits + 1 (weights
// here are positive normal floats, so the pattern is a positive normal double
// and the doubles order as the keys), bits 31..0 = 2^32 - 1 - index (a larger
// key comes first: weight desc, index asc -- the selection order; keys are
// unique).  0 marks an empty slot.  One insertion step is then
// slot' = max(slot, x), x' = min(slot, x): full-rate f64 operations (three
// with the compiler's canonicalising max of the loop-carried slot; inline asm
// saves nothing, the in-place update then costs a move) instead of the
// compare and four selects of the (weight, index) pair ripple (287 VALU per
// live weight for LCAP = 40).  The list is walked in chunks of
// eight slots, and a chunk none of whose slots can change in any lane (x not
// above its smallest slot: x sorts after it, or nothing left to carry) is
// skipped on a wave-uniform branch.  The list is the top LCAP live weights
// seen; a capacity cap < LCAP is its first cap entries (the top cap), so the
// results are those of the cap-entry list above.
__device__ __forceinline__ double cand_key(float w, int k) {
    const uint64_t b = ((uint64_t)(__builtin_bit_cast(uint32_t, w) + 1u) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)k);
    return __builtin_bit_cast(double, b);
}
template <int LCAP>
__device__ __forceinline__ int build_candidates_key(const float* gp, int Kp, int K, const float c[3], float* cw,
                                                    unsigned short* ck, int T, int tid, float norm3, int cap,
                                                    float& accum) {
    constexpr int CH = 8;   // slots per skippable chunk (round 4: chunks of 4 / 20 measured the same)
    static_assert(LCAP % CH == 0, "whole chunks");
    double L[LCAP];
#pragma unroll
    for (int i = 0; i < LCAP; ++i) L[i] = 0.0;
    float total = 0.0f;
    const float skip_f = 0.0089f / (float)K;
    MargRec nx = load_marg(gp, 0);
    for (int k = 0; k < K; ++k) {
        const MargRec rec = nx;
        if (k + 1 < K) nx = load_marg(gp, k + 1);
        const float w = marginal_weight_rec(rec, c, norm3);
        total += w;
        if (!(w > 0.0f) || w < total * skip_f) continue;
        double x = cand_key(w, k);
#pragma unroll
        for (int c0 = 0; c0 < LCAP; c0 += CH) {
            if (!__any(x > L[c0 + CH - 1])) continue;
#pragma unroll
            for (int i = c0; i < c0 + CH; ++i) {
                const double hi = __builtin_fmax(L[i], x);
                x = __builtin_fmin(L[i], x);
                L[i] = hi;
            }
        }
    }
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < LCAP; ++i) {
        const uint64_t b = __builtin_bit_cast(uint64_t, L[i]);
        if (i < cap && b != 0) {
            cw[i * T + tid] = __builtin_bit_cast(float, (uint32_t)(b >> 32) - 1u);
            ck[i * T + tid] = (unsigned short)(0xFFFFFFFFu - (uint32_t)b);
            cnt = i + 1;
        }
    }
    if (!__builtin_isfinite(total)) return -1;
    if (total == 0.0f) return kNoMass;   // every marginal weight zero: BSDF only (below)
    const float cutoff = (float)(0.99 * (double)total);
    const double tau = ((double)total - (double)cutoff) / (double)K * 0.999;
    if (!(tau > 0.0)) return -1;
    int ncand = 0;
    while (ncand < cnt && (double)cw[ncand * T + tid] >= tau) ++ncand;
    accum = 0.0f;
    for (int i = 0; i < ncand; ++i) {
        const int k = ck[i * T + tid];
        const bool ok = cond_valid(gp, Kp, k, c);
        ck[i * T + tid] = (unsigned short)(k | (ok ? 0x8000 : 0));
        accum += ok ? cw[i * T + tid] : 0.0f;
        if (accum >= cutoff) return i + 1;
    }
    return (ncand == K) ? K : -1;
}

template <int LCAP>
__device__ __forceinline__ int build_candidates_reg(const float* gp, int Kp, int K, const float c[3], float* cw,
                                                    unsigned short* ck, int T, int tid, float norm3, int cap,
                                                    float& accum) {
    return build_candidates_key<LCAP>(gp, Kp, K, c, cw, ck, T, tid, norm3, cap, accum);
}

// Plane pointers of one guided batch (inputs c, u or given directions e;
// outputs d, pdf, comp).
struct GuideIO {
    const float *c0, *c1, *c2, *u0, *u1, *u2, *e0, *e1, *e2;
    float *d0, *d1, *d2, *pdf;
    int32_t* comp;
    // mixed wavefront (sampling kernels only): pmode[q] != 0 makes query q a
    // pdf query at the given direction e[q] (d[q] = e[q], comp -2 / -1)
    const uint8_t* pmode;
};

// One mixture's guide record as the wavefront kernels see it (per tree node;
// K = 0: the node has no trained mixture -> BSDF only, sdmm_proc.cpp:316-323).
struct GuideMix {
    const float* gp;
    int Kp, K;
};
static_assert(sizeof(GuideMix) == 16, "GuideMix");
// A mixture record known wave-uniform (a uniform-leaf wave): its fields moved
// to SGPRs, so that the record loads of a uniform component index compile to
// scalar loads (the compiler cannot see the uniformity through the table
// load and the branch structure).
__device__ __forceinline__ GuideMix uniform_mix(const GuideMix& m) {
    const uint64_t p = (uint64_t)(uintptr_t)m.gp;
    const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32));
    return GuideMix{(const float*)(uintptr_t)(lo | (hi << 32)), __builtin_amdgcn_readfirstlane(m.Kp),
                    __builtin_amdgcn_readfirstlane(m.K)};
}

// Query q with no valid conditional: the reference falls back to BSDF
// sampling (comp -1, gmmPdf 0).
template <bool PDF_ONLY>
__device__ __forceinline__ void write_invalid(const GuideIO& io, int64_t q) {
    io.pdf[q] = 0.0f;
    if constexpr (!PDF_ONLY) {
        io.d0[q] = 0.0f; io.d1[q] = 0.0f; io.d2[q] = 0.0f;
        io.comp[q] = -1;
    }
}

template <bool PDF_ONLY, class Slots>
__device__ __forceinline__ void finish_and_write(const float* gp, int Kp, const float c[3], int lastIdx,
                                                 float accum, const Slots& S, const GuideIO& io, int64_t q,
                                                 GuideConsts gc) {
    if constexpr (PDF_ONLY) {
        const float dir[3] = {io.e0[q], io.e1[q], io.e2[q]};
        io.pdf[q] = finish_query(gp, Kp, c, nullptr, lastIdx, accum, S, dir, gc).pdf;
    } else {
        const float u[3] = {io.u0[q], io.u1[q], io.u2[q]};
        const float dg[3] = {io.pmode && io.pmode[q] ? io.e0[q] : 0.0f, io.pmode && io.pmode[q] ? io.e1[q] : 0.0f,
                             io.pmode && io.pmode[q] ? io.e2[q] : 0.0f};
        const QueryOut o = finish_query(gp, Kp, c, u, lastIdx, accum, S, (io.pmode && io.pmode[q]) ? dg : nullptr, gc);
        io.d0[q] = o.d[0]; io.d1[q] = o.d[1]; io.d2[q] = o.d[2];
        io.pdf[q] = o.pdf;
        io.comp[q] = o.comp;
    }
}

// Candidate path of query q against one mixture; true: q needs the full-K
// fallback (appended to fb_list).
template <bool PDF_ONLY, int LCAP, bool REG = false>
__device__ __forceinline__ bool serve_cand(const float* gp, int Kp, int K, const GuideIO& io, int64_t q,
                                           const float c[3], float* cw, unsigned short* ck, int tid, int cap,
                                           GuideConsts gc, int* fb_count, int32_t* fb_list) {
    float accum = 0.0f;
    const int lastIdx = REG ? build_candidates_reg<LCAP>(gp, Kp, K, c, cw, ck, 64, tid, gc.norm3, cap, accum)
                            : build_candidates(gp, Kp, K, c, cw, ck, 64, tid, gc.norm3, cap, accum);
    if (lastIdx == kNoMass) {
        write_invalid<PDF_ONLY>(io, q);
        return false;
    }
    if (lastIdx < 0) {
        fb_list[atomicAdd(fb_count, 1)] = (int32_t)q;
        return true;
    }
    finish_and_write<PDF_ONLY>(gp, Kp, c, lastIdx, accum, CandSlots{cw, ck, 64, tid}, io, q, gc);
    return false;
}

// LDS list capacity LCAP (24 or 40): the lists are 6 B per entry per thread,
// so the capacity sets the workgroups per CU (LDS-limited occupancy).
template <bool PDF_ONLY, int LCAP>
__global__ void __launch_bounds__(64)
guide_cand_kernel(const float* __restrict__ gp, int Kp, int K, int64_t nq, GuideIO io, GuideConsts gc, int cap,
                  int* __restrict__ fb_count, int32_t* __restrict__ fb_list, const int32_t* __restrict__ perm) {
    __shared__ float cw[LCAP * 64];
    __shared__ unsigned short ck[LCAP * 64];
    const int tid = threadIdx.x;
    const int64_t t = (int64_t)blockIdx.x * 64 + tid;
    if (t >= nq) return;
    // coherent order: thread t serves query perm[t] (Morton order of c)
    const int64_t q = perm ? (int64_t)perm[t] : t;
    const float c[3] = {io.c0[q], io.c1[q], io.c2[q]};
    serve_cand<PDF_ONLY, LCAP>(gp, Kp, K, io, q, c, cw, ck, tid, cap, gc, fb_count, fb_list);
}

// Wavefront over the spatial tree's leaves (SDMMRenderer::sampleSurface,
// sdmm_proc.cpp:309-368): node = STree.find(c) (:314), that node's mixture
// (tab[node]; none -> BSDF only), then the query exactly as
// guide_cand_kernel serves it against that one mixture.  The waves are
// Morton-ordered, so a wave's queries mostly share a leaf; the waterfall loop
// serves one distinct mixture per trip with its record address uniform
// (readfirstlane), keeping the record loads scalar.
template <bool PDF_ONLY, int LCAP>
__global__ void __launch_bounds__(64)
guide_tree_cand_kernel(const STNodeDev* __restrict__ nodes, const GuideMix* __restrict__ tab, int64_t nq,
                       GuideIO io, GuideConsts gc, int cap, int* __restrict__ fb_count,
                       int32_t* __restrict__ fb_list, const int32_t* __restrict__ perm,
                       int32_t* __restrict__ node_out, const uint32_t* __restrict__ skeys, int mb) {
    __shared__ float cw[LCAP * 64];
    __shared__ unsigned short ck[LCAP * 64];
    const int tid = threadIdx.x;
    const int64_t t = (int64_t)blockIdx.x * 64 + tid;
    if (t >= nq) return;
    const int64_t q = perm ? (int64_t)perm[t] : t;
    const float c[3] = {io.c0[q], io.c1[q], io.c2[q]};
    // leaf-major order: the sorted key holds the node (tree_keys_kernel)
    const int node = skeys ? (int)(skeys[t] >> mb) - 1 : stree_find_point(nodes, c[0], c[1], c[2]);
    if (node_out) node_out[q] = node;
    {
        // the common case (Morton order): every lane of the wave in one leaf,
        // served in uniform control flow (a ballot), without the waterfall
        // loop (-4 %).  The record fields behind mx.gp still compile to vector
        // loads here (ISA: 54 global_load, 21 s_load; the single-mixture
        // kernel, whose gp is a kernel argument, reads them with s_load) --
        // see DESIGN.md, guided wavefront.
        const int n0 = __builtin_amdgcn_readfirstlane(node);
        if (__builtin_amdgcn_ballot_w64(node != n0) == 0) {
            const GuideMix mx = uniform_mix((n0 >= 0) ? tab[n0] : GuideMix{nullptr, 0, 0});
            if (mx.K <= 0) {
                write_invalid<PDF_ONLY>(io, q);
            } else {
                serve_cand<PDF_ONLY, LCAP, (LCAP >= kGuideRegCap)>(mx.gp, mx.Kp, mx.K, io, q, c, cw, ck, tid, cap, gc,
                                                                 fb_count, fb_list);
            }
            return;
        }
    }
    for (;;) {
        const int n0 = __builtin_amdgcn_readfirstlane(node);
        if (node != n0) continue;
        const GuideMix mx = (n0 >= 0) ? tab[n0] : GuideMix{nullptr, 0, 0};
        if (mx.K <= 0)
            write_invalid<PDF_ONLY>(io, q);
        else
            serve_cand<PDF_ONLY, LCAP, (LCAP >= kGuideRegCap)>(mx.gp, mx.Kp, mx.K, io, q, c, cw, ck, tid, cap, gc,
                                                             fb_count, fb_list);
        break;
    }
}

// ---------------------------------------------------------------------------
// Fallback: the full-K conditional of one query, as the reference forms it
// (mixture_model.h:248-284; oracle or_conditional_create):
//
//   total = sum_k w_k in component order;  cutoff = (float)(0.99 total);
//   repeat: take the largest untaken w (lowest index among equals; the scan
//   replaces only on a strictly larger value), accum += valid ? w : 0,
//   stop once accum >= cutoff (lastIdx = K if never reached).
//
// build_full_wave below evaluates exactly this with a whole wave per query.
// ---------------------------------------------------------------------------
// Full-K queries, ONE query per wave (the fallback of the plain guide and of
// the product path).  A full-K query costs O(K x kept) selection steps and,
// with a learned BSDF, kept x M product pairs; served by a single thread it
// was the long pole of a batch (round 1: 97 % of a Kitchen K = 512 product
// call).  Same results as the selection above / finish_query / finish_product,
// bit for bit:
//   * lane l holds the weights of components l, l + 64, ... (K <= 512) in
//     registers, by the same expression;
//   * every order-dependent float reduction -- the total in component order,
//     the kept weights' sum2 (createCdf), the product mass, the CDF walks, the
//     pdf accumulations -- is formed in the reference order from v_readlane
//     broadcasts, uniformly in every lane (no LDS round trip per term); a term
//     the reference skips is added as -0.0f, an exact no-op (x + -0 == x for
//     every x, NaN included);
//   * each selection step picks what the reference scan picks -- among the
//     untaken entries (sign bit clear) the largest, the lowest index among
//     equals -- as a wave max then a wave min of the candidate indices; with a
//     NaN among the untaken entries the scan's rule is order-dependent, so the
//     scan itself runs (uniformly, in component order);
//   * per-slot and per-pair quantities are evaluated by the lanes in parallel.
// Needs all 64 lanes active (workgroup = one wave).

__device__ __forceinline__ float rl(float x, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}
// acc += x of lanes 0 .. n-1, in lane order (uniform result).  The wave's
// values go through a 64-float LDS stage (st, 16-B aligned, this wave's own)
// and come back as 16 broadcast ds_read_b128, so each term is ONE dependent
// VGPR add; lanes >= n stage -0.0f, an exact no-op (x + -0 == x for every x,
// NaN included).  (Round 6; was a v_readlane + SALU-counted loop per term:
// 5 instructions and a taken branch, ~37 wall cycles a term at 3 waves per
// SIMD.)
__device__ __forceinline__ void stage64(float* st, float x, bool live) {
    st[__lane_id()] = live ? x : -0.0f;
}
__device__ __forceinline__ float seq_sum(float acc, float x, int n, float* st) {
    stage64(st, x, __lane_id() < n);
    const float4* s4 = (const float4*)st;
#pragma unroll
    for (int p = 0; p < 16; ++p) {
        const float4 v = s4[p];
        acc += v.x;
        acc += v.y;
        acc += v.z;
        acc += v.w;
    }
    return acc;
}
template <int CTRL>
__device__ __forceinline__ int dppi(int x) { return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false); }
constexpr int kWaveKMax = 512;            // components per wave query: 8 per lane
constexpr int kWaveSlots = kWaveKMax / 64;

struct WaveLds {
    int* sl;         // K   kept slot -> component | (conditional valid) << 31
    float* fw;       // K   slot weights: raw, then slot_w(i)
    float* se;       // 3K  conditional mean direction of each kept slot (product)
    float* lobe;     // 20M world-frame learned-BSDF lobes of the query's material (product),
                     // then M ints: the nonzero-weight lobes' indices in order
    float* pc;       // this workgroup's global scratch: kPcStride x pcap floats, the product
                     // pairs of pass 1 {w, included, mean, Linv, detInv} (when they fit)
    int pcap;
    float* st;       // 64  the serial sums' broadcast stage (seq_sum), 16-B aligned
};
constexpr int kPcStride = 10;
// pair f = base + lane's record in the pair scratch: field j at r[64 j] (each
// 64-pair chunk field-major, so a chunk's field is one coalesced 256-B access)
constexpr int kProductPairCap = 1024;   // kept x lobes per full-K product query kept in scratch

// LDS carve-up of a one-wave workgroup (+ its slice of the pair scratch).
__device__ __forceinline__ WaveLds wave_lds(float* lds, int K, float* pscratch = nullptr, int pcap = 0, int M = 0) {
    WaveLds L;
    L.sl = (int*)lds;
    L.fw = lds + K;
    L.se = lds + 2 * K;
    L.lobe = L.se + 3 * K;
    L.pc = pscratch ? pscratch + (size_t)blockIdx.x * kPcStride * pcap : nullptr;
    L.pcap = pscratch ? pcap : 0;
    L.st = lds + ((5 * K + 21 * M + 3) & ~3);
    return L;
}
__device__ __forceinline__ float* pc_rec(const WaveLds& L, int base, int lane) {
    return L.pc + (size_t)base * kPcStride + lane;
}
static size_t wave_lds_bytes(int K, int M = 0) {
    return sizeof(float) * ((5 * (size_t)K + 21 * (size_t)M + 3) / 4 * 4 + 64) + 16;
}

// lane ^ J of a wave-uniform compile-time J (DPP inside rows, ds_bpermute across)
template <int J>
__device__ __forceinline__ uint32_t xor_lane_u(uint32_t x) {
    const int xi = (int)x;
    if constexpr (J == 1) return (uint32_t)dppi<0xB1>(xi);         // quad_perm [1,0,3,2]
    else if constexpr (J == 2) return (uint32_t)dppi<0x4E>(xi);    // quad_perm [2,3,0,1]
    else if constexpr (J == 4) {                                   // row_shl:4 / row_shr:4 by bank
        int t = __builtin_amdgcn_update_dpp(xi, xi, 0x104, 0xF, 0x5, false);
        return (uint32_t)__builtin_amdgcn_update_dpp(t, xi, 0x114, 0xF, 0xA, false);
    } else if constexpr (J == 8) return (uint32_t)dppi<0x128>(xi); // row_ror:8
    else return (uint32_t)__shfl_xor(xi, J);
}

// Bitonic networks over the 64 S elements of a wave (W = 64) or the 16 S
// elements of a 16-lane group (W = 16), element e = W i + (lane mod W), in
// the order the reference's selection scan takes weights: largest first, the
// lowest index among equals.  One packed 64-bit key per element, (weight key
// << 32) | (2^32 - 1 - index), makes that order a single unsigned compare
// (a larger key comes first).  Stage (KS, J): element e pairs with e ^ J; the
// KS-block of e runs "up" (larger first) when (e & KS) == 0.
template <int J>
__device__ __forceinline__ uint64_t xor_lane_u64(uint64_t x) {
    const uint32_t lo = xor_lane_u<J>((uint32_t)x), hi = xor_lane_u<J>((uint32_t)(x >> 32));
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ uint64_t sel_key(uint32_t wkey, uint32_t idx) {
    return ((uint64_t)wkey << 32) | (uint64_t)(0xFFFFFFFFu - idx);
}
__device__ __forceinline__ uint32_t sel_idx(uint64_t k) { return 0xFFFFFFFFu - (uint32_t)k; }
__device__ __forceinline__ uint32_t sel_wkey(uint64_t k) { return (uint32_t)(k >> 32); }

template <int W, int S, int KS, int J>
__device__ __forceinline__ void bsort_step(uint64_t (&v)[S], int gl) {
    if constexpr (J >= W) {
        constexpr int JJ = J / W;
#pragma unroll
        for (int i = 0; i < S; ++i) {
            if (i & JJ) continue;
            const int i2 = i | JJ;
            const bool up = ((W * i) & KS) == 0;   // lanes do not reach bit KS >= 2W
            const bool b = v[i] > v[i2];
            const bool sw = up ? !b : b;
            const uint64_t a = v[i];
            v[i] = sw ? v[i2] : a;
            v[i2] = sw ? a : v[i2];
        }
    } else {
        const bool lower = (gl & J) == 0;
#pragma unroll
        for (int i = 0; i < S; ++i) {
            const uint64_t o = xor_lane_u64<J>(v[i]);
            const bool up = ((W * i + gl) & KS) == 0;
            const bool b = v[i] > o;
            const bool keep = (lower == up) ? b : !b;
            v[i] = keep ? v[i] : o;
        }
    }
}
template <int W, int S, int KS, int J>
__device__ __forceinline__ void bsort_stage(uint64_t (&v)[S], int gl) {
    bsort_step<W, S, KS, J>(v, gl);
    if constexpr (J > 1) bsort_stage<W, S, KS, J / 2>(v, gl);
}
template <int W, int S, int KS = 2>
__device__ __forceinline__ void bsort(uint64_t (&v)[S], int gl) {
    bsort_stage<W, S, KS, KS / 2>(v, gl);
    if constexpr (KS < W * S) bsort<W, S, 2 * KS>(v, gl);
}

// The kept prefix from sorted entries (build_full_wave_s): sorted element
// p = 64 i + lane, its slot record written by its own lane, its term of the
// kept mass (0 for an invalid conditional); accum in the selection order up
// to the first slot that reaches the cutoff.  Returns true with lastIdx =
// that slot + 1; false when every live entry was taken without reaching it
// (lastIdx = n_live: the scan finds nothing left, K when every weight is live).
template <int S2>
__device__ __forceinline__ bool kept_prefix(const uint32_t (&key)[S2], const uint32_t (&idx)[S2], unsigned vmask,
                                            float cutoff, const WaveLds& L, int lane, float& accum, int& lastIdx) {
    int n_live = 0;   // entries with a weight (sorted first)
    float term[S2];
#pragma unroll
    for (int i = 0; i < S2; ++i) {
        n_live += __builtin_popcountll(__builtin_amdgcn_ballot_w64(key[i] != 0u));
        const unsigned vm = (unsigned)__shfl((int)vmask, (int)(idx[i] & 63u));
        const bool ok = (vm >> (idx[i] >> 6)) & 1u;
        const float w = __builtin_bit_cast(float, key[i] - 1u);
        term[i] = ok ? w : 0.0f;
        if (key[i] != 0u) {
            L.sl[64 * i + lane] = (int)idx[i] | (ok ? (int)0x80000000 : 0);
            L.fw[64 * i + lane] = w;
        }
    }
    // accum in the selection order, up to the first slot that reaches the
    // cutoff; all live entries taken without reaching it: lastIdx = n_live
    // (the scan finds nothing left), which is K when every weight is live
    lastIdx = n_live;
    bool done = false;
#pragma unroll
    for (int i = 0; i < S2; ++i) {
        if (done) break;
        const int n = min(64, n_live - 64 * i);
        if (n <= 0) break;
        // the terms through the broadcast stage (seq_sum); a padded
        // lane's -0.0f cannot cross the cutoff (accum unchanged)
        stage64(L.st, term[i], lane < n);
        const float4* s4 = (const float4*)L.st;
#pragma unroll 1
        for (int p = 0; 4 * p < n && !done; ++p) {
            const float4 v = s4[p];
            const float e4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                accum += e4[e];
                if (accum >= cutoff) { lastIdx = 64 * i + 4 * p + e + 1; done = true; break; }
            }
        }
    }
    return done;
}

// The kept prefix of query c's full-K conditional (above): slots
// i < lastIdx in L.sl / L.fw (raw weight); returns lastIdx and accum.
//
// S = 64-lane slots per component index (K <= 64 S).  Without a NaN weight the
// selection order is a strict total order -- (weight desc, index asc) -- so the
// wave sorts all K weights once (a bitonic network in registers: 21..45
// compare-exchange steps for K = 64..512) and walks the sorted sequence,
// instead of one wave max + min reduction per kept component (O(K x kept));
// accum and the cutoff test run in that same order, so lastIdx, the slots and
// accum are those of the reference's scan bit for bit.  Keys: the weight's bits
// + 1 (non-negative floats order as unsigned integers; +0.0 -> 1), 0 for an
// absent entry (sign bit set: never taken).  With a NaN present the scan's
// choice depends on the order of comparisons, so the scan itself runs.
template <int S>
__device__ __forceinline__ int build_full_wave_s(const float* gp, int Kp, int K, const float c[3], const WaveLds& L,
                                                 int lane, float norm3, float& accum) {
    float wr[S];
    unsigned vmask = 0;   // bit i: the conditional of component lane + 64 i is valid
    bool nan_seen = false;
#pragma unroll
    for (int i = 0; i < S; ++i) {
        const int k = lane + 64 * i;
        wr[i] = -0.0f;    // absent: never a candidate
        if (k < K) {
            wr[i] = gp_ld(gp, Kp, GP_W, k) * marginal_pdf(gp, Kp, k, c, norm3);
            vmask |= (cond_valid(gp, Kp, k, c) ? 1u : 0u) << i;
        }
        nan_seen |= (wr[i] != wr[i]);
    }
    WCLK(1);
    float total = 0.0f;   // component order
#pragma unroll
    for (int i = 0; i < S; ++i)
        if (64 * i < K) total = seq_sum(total, wr[i], min(64, K - 64 * i), L.st);
    WCLK(8);
    const float cutoff = (float)(0.99 * (double)total);
    accum = 0.0f;
    int lastIdx = K;   // the reference leaves it uninitialised if never reached
    if (!__any(nan_seen)) {
        if constexpr (S >= 4) {
            // K > 128: the kept prefix is usually far shorter than K (~90 of
            // 512 at the Cornell K = 512 leaves).  The entries with key >= T,
            // T the smallest 16-bit-prefix threshold leaving at most 128 of
            // them, are exactly the first entries of the full sorted order
            // (every other key is smaller), so sorting only them (two per
            // lane) gives the same prefix, slots and accum -- when the
            // cutoff is reached inside them; otherwise the full sort below.
            uint32_t wk[S];
#pragma unroll
            for (int i = 0; i < S; ++i)
                wk[i] = __builtin_signbit(wr[i]) ? 0u : __builtin_bit_cast(uint32_t, wr[i]) + 1u;
            auto count_ge = [&](uint32_t t) __attribute__((always_inline)) {
                int cnt = 0;
#pragma unroll
                for (int i = 0; i < S; ++i) cnt += __builtin_popcountll(__builtin_amdgcn_ballot_w64(wk[i] >= t));
                return cnt;
            };
            constexpr int kSub = 128;
            uint32_t T = 1u;
            if (count_ge(1u) > kSub) {
                // keys are at most 0x7F800001 (+inf + 1): prefix 0x7F81 leaves none
                uint32_t lo = 0u, hi = 0x7F81u;
                while (hi - lo > 1u) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (count_ge(mid << 16) <= kSub) hi = mid;
                    else lo = mid;
                }
                T = hi << 16;
            }
            // their valid mass (any order) against the cutoff: a cheap test
            // that the prefix ends inside them (kept_prefix decides exactly)
            float part = 0.0f;
#pragma unroll
            for (int i = 0; i < S; ++i)
                if (wk[i] >= T && ((vmask >> i) & 1u)) part += wr[i];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o);
            if (part >= cutoff) {
                uint64_t* sc = (uint64_t*)(((uintptr_t)L.se + 7u) & ~(uintptr_t)7u);   // (se: unused until prep)
                int base = 0;
#pragma unroll
                for (int i = 0; i < S; ++i) {
                    const bool in = wk[i] >= T;
                    const uint64_t m = __builtin_amdgcn_ballot_w64(in);
                    const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    if (in) sc[pos] = sel_key(wk[i], (uint32_t)(lane + 64 * i));
                    base += __builtin_popcountll(m);
                }
                __builtin_amdgcn_wave_barrier();
                uint64_t v2[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int q = lane + 64 * j;
                    v2[j] = q < base ? sc[q] : sel_key(0u, (uint32_t)lane);   // padding: absent
                }
                __builtin_amdgcn_wave_barrier();
                bsort<64, 2>(v2, lane);
                uint32_t key2[2], idx2[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) { key2[j] = sel_wkey(v2[j]); idx2[j] = sel_idx(v2[j]); }
                if (kept_prefix<2>(key2, idx2, vmask, cutoff, L, lane, accum, lastIdx)) {
                    __syncthreads();
                    return lastIdx;
                }
                accum = 0.0f;   // (the cutoff lies past them: the full sort)
            }
        }
        uint32_t key[S], idx[S];
        {
            uint64_t v[S];
#pragma unroll
            for (int i = 0; i < S; ++i)
                v[i] = sel_key(__builtin_signbit(wr[i]) ? 0u : __builtin_bit_cast(uint32_t, wr[i]) + 1u,
                               (uint32_t)(lane + 64 * i));
            bsort<64, S>(v, lane);
#pragma unroll
            for (int i = 0; i < S; ++i) { key[i] = sel_wkey(v[i]); idx[i] = sel_idx(v[i]); }
        }
        WCLK(9);
        kept_prefix<S>(key, idx, vmask, cutoff, L, lane, accum, lastIdx);
        __syncthreads();
        WCLK(10);
        return lastIdx;
    }
    for (int it = 0; it < K; ++it) {
        // the reference scan itself, in component order (a NaN is present)
        int best = -1;
        float bw = 0.0f;
#pragma unroll
        for (int i = 0; i < S; ++i)
            for (int l = 0; l < 64 && 64 * i + l < K; ++l) {
                const float x = rl(wr[i], l);
                if (__builtin_signbit(x)) continue;
                if (best < 0 || x > bw) { best = 64 * i + l; bw = x; }
            }
        if (best < 0) { lastIdx = it; break; }
#pragma unroll
        for (int i = 0; i < S; ++i)
            if (best == lane + 64 * i) wr[i] = -bw;
        const bool ok = ((unsigned)__builtin_amdgcn_readlane((int)vmask, best & 63) >> (best >> 6)) & 1u;
        if (lane == 0) {
            L.sl[it] = best | (ok ? (int)0x80000000 : 0);
            L.fw[it] = bw;
        }
        accum += ok ? bw : 0.0f;
        if (accum >= cutoff) { lastIdx = it + 1; break; }
    }
    __syncthreads();
    return lastIdx;
}

__device__ __forceinline__ int build_full_wave(const float* gp, int Kp, int K, const float c[3], const WaveLds& L,
                                               int lane, float norm3, float& accum) {
    if (K <= 64) return build_full_wave_s<1>(gp, Kp, K, c, L, lane, norm3, accum);
    if (K <= 128) return build_full_wave_s<2>(gp, Kp, K, c, L, lane, norm3, accum);
    if (K <= 256) return build_full_wave_s<4>(gp, Kp, K, c, L, lane, norm3, accum);
    return build_full_wave_s<kWaveSlots>(gp, Kp, K, c, L, lane, norm3, accum);
}

__device__ __forceinline__ int slot_comp(const WaveLds& L, int i) { return L.sl[i] & 0x7fffffff; }

// L.fw[i] = slot_w(i) (finish_query's normalisation) for i < lastIdx;
// returns sum2 (uniform).
__device__ __forceinline__ float wave_slot_weights(int lastIdx, float accum, const WaveLds& L, int lane) {
    const float invSum = 1.0f / accum;
    const bool scaled = __builtin_isfinite(invSum);
    float sum2 = 0.0f;
    for (int base = 0; base < lastIdx; base += 64) {
        const int i = base + lane;
        float wi = -0.0f;
        if (i < lastIdx) {
            wi = (L.sl[i] < 0) ? L.fw[i] : 0.0f;   // bit 31: valid conditional
            if (scaled) wi = wi * invSum;
            L.fw[i] = wi;
        }
        sum2 = seq_sum(sum2, wi, min(64, lastIdx - base), L.st);
    }
    if (lastIdx > 0 && sum2 != 0.0f) {
        const DivBy by_sum2(sum2);
        for (int i = lane; i < lastIdx; i += 64) L.fw[i] = by_sum2(L.fw[i]);
    }
    __syncthreads();
    return sum2;
}

// finish_query with the lanes sharing the slots (the plain conditional: the
// guide's fallback, and the product path's h = 0.5 case).  Uniform result.
template <bool PDF_ONLY>
__device__ QueryOut finish_query_wave(const float* gp, int Kp, const float c[3], const float u[3],
                                      const float* dir_in, int lastIdx, float sum2, const WaveLds& L, int lane,
                                      GuideConsts gc) {
    QueryOut o{{0.0f, 0.0f, 0.0f}, 0.0f, -1};
    if (lastIdx == 0 || sum2 == 0.0f) return o;   // createCdf(true) fails: BSDF only
    float dir[3];
    if constexpr (!PDF_ONLY) {
        // sampleDiscreteCdf: lower_bound == first slot with cdf >= u, else the tie walk
        float cdf = 0.0f, prev = 0.0f;
        int slot = -1, runStart = 0;
        for (int base = 0; base < lastIdx && slot < 0; base += 64) {
            const float x = (base + lane < lastIdx) ? L.fw[base + lane] : 0.0f;
            const int n = min(64, lastIdx - base);
            stage64(L.st, x, true);   // (broadcast stage, as seq_sum)
            const float4* s4 = (const float4*)L.st;
#pragma unroll 1
            for (int q4 = 0; 4 * q4 < n && slot < 0; ++q4) {
                const float4 v = s4[q4];
                const float e4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int l = 4 * q4 + e;
                    if (l >= n) break;
                    cdf += e4[e];
                    if (base + l == 0 || cdf != prev) runStart = base + l;
                    prev = cdf;
                    if (cdf >= u[0]) { slot = base + l; break; }
                }
            }
        }
        if (slot < 0) slot = runStart;
        const int ksel = slot_comp(L, slot);
        float esel[3];
        cond_mean_dir(gp, Kp, ksel, c, esel);
        const float radius = sqrtf(-2.0f * logf(1.0f - u[1]));
        const float theta = (float)(2.0 * kPi * (double)u[2]);
        float res0, res1;
        sincosf(theta, &res0, &res1);
        const float z0 = radius * res0, z1 = radius * res1;
        const float L00 = gp_ld(gp, Kp, GP_CL00, ksel), L10 = gp_ld(gp, Kp, GP_CL10, ksel);
        const float L11 = gp_ld(gp, Kp, GP_CL11, ksel);
        const float v0 = L00 * z0 + 0.0f * z1;
        const float v1 = L10 * z0 + L11 * z1;
        float tof[9];
        coordinates_f(esel, tof);
        ts_exp_dir(tof, v0, v1, dir);
        o.comp = ksel;
    } else {
        dir[0] = dir_in[0]; dir[1] = dir_in[1]; dir[2] = dir_in[2];
        o.comp = kCompPdfValid;
    }
    // MixtureModel::pdf over the conditional: terms in parallel, summed in slot order
    float acc = 0.0f;
    for (int base = 0; base < lastIdx; base += 64) {
        const int i = base + lane;
        float term = -0.0f;
        if (i < lastIdx) {
            const float f = L.fw[i];
            if (f != 0.0f) {
                const int k = slot_comp(L, i);
                float e[3];
                cond_mean_dir(gp, Kp, k, c, e);
                term = f * cond_component_pdf(gp, Kp, k, e, dir, gc.norm2);
            }
        }
        acc = seq_sum(acc, term, min(64, lastIdx - base), L.st);
    }
    o.d[0] = dir[0]; o.d[1] = dir[1]; o.d[2] = dir[2];
    o.pdf = acc;
    return o;
}

template <bool PDF_ONLY>
__device__ __forceinline__ void serve_full_wave(const float* gp, int Kp, int K, const GuideIO& io, int64_t q,
                                                const float c[3], const WaveLds& L, int lane, GuideConsts gc) {
    float accum = 0.0f;
    const int lastIdx = build_full_wave(gp, Kp, K, c, L, lane, gc.norm3, accum);
    const float sum2 = wave_slot_weights(lastIdx, accum, L, lane);
    float u[3] = {0.0f, 0.0f, 0.0f}, dg[3] = {0.0f, 0.0f, 0.0f};
    bool pdf_q = PDF_ONLY;
    if constexpr (!PDF_ONLY) pdf_q = io.pmode && io.pmode[q];   // uniform: one query per wave
    if (pdf_q) { dg[0] = io.e0[q]; dg[1] = io.e1[q]; dg[2] = io.e2[q]; }
    else { u[0] = io.u0[q]; u[1] = io.u1[q]; u[2] = io.u2[q]; }
    const QueryOut o = pdf_q ? finish_query_wave<true>(gp, Kp, c, u, dg, lastIdx, sum2, L, lane, gc)
                             : finish_query_wave<false>(gp, Kp, c, u, dg, lastIdx, sum2, L, lane, gc);
    if (lane == 0) {
        io.pdf[q] = o.pdf;
        if constexpr (!PDF_ONLY) {
            io.d0[q] = o.d[0]; io.d1[q] = o.d[1]; io.d2[q] = o.d[2];
            io.comp[q] = o.comp;
        }
    }
    __syncthreads();   // the LDS is reused by the wave's next query
}

// The fallback queries listed by the candidate kernel, one per workgroup
// (one wave), grid-stride.
template <bool PDF_ONLY>
__global__ void __launch_bounds__(64)
guide_fallback_kernel(const float* __restrict__ gp, int Kp, int K, GuideIO io, GuideConsts gc,
                      const int* __restrict__ fb_count, const int32_t* __restrict__ fb_list) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x;
    const int count = *fb_count;
    const WaveLds L = wave_lds(lds, K);
    for (int idx = blockIdx.x; idx < count; idx += gridDim.x) {
        const int64_t q = fb_list[idx];
        const float c[3] = {io.c0[q], io.c1[q], io.c2[q]};
        serve_full_wave<PDF_ONLY>(gp, Kp, K, io, q, c, L, lane, gc);
    }
}

// Fallback queries of the tree wavefront (each against its own leaf's mixture;
// kmax = the largest K in tab sizes the LDS).
template <bool PDF_ONLY>
__global__ void __launch_bounds__(64)
guide_tree_fallback_kernel(const STNodeDev* __restrict__ nodes, const GuideMix* __restrict__ tab, int kmax,
                           GuideIO io, GuideConsts gc, const int* __restrict__ fb_count,
                           const int32_t* __restrict__ fb_list, const int32_t* __restrict__ node_of) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x;
    const int count = *fb_count;
    const WaveLds L = wave_lds(lds, kmax);
    for (int idx = blockIdx.x; idx < count; idx += gridDim.x) {
        const int64_t q = fb_list[idx];
        const float c[3] = {io.c0[q], io.c1[q], io.c2[q]};
        // uniform: a listed query has a mixture; node_of: the candidate kernel's find
        const int node = node_of ? node_of[q] : stree_find_point(nodes, c[0], c[1], c[2]);
        const GuideMix mx = uniform_mix(tab[node]);   // (one query per wave: uniform)
        serve_full_wave<PDF_ONLY>(mx.gp, mx.Kp, mx.K, io, q, c, L, lane, gc);
    }
}

// ---------------------------------------------------------------------------
// Full-K queries of SMALL mixtures (K <= 128; the tree's wide leaves), FOUR
// per wave: a 16-lane group per query, lane l of a group holding components
// l, l + 16, ... (S slots, K <= 16 S).  Same arithmetic, same order, same
// bits as serve_full_wave; what changes is that every instruction of the
// serial float chains (total, the cutoff walk, sum2, the CDF walk, the pdf
// sum) serves four queries, the per-slot values stay in registers (no LDS),
// and the sort's cross-lane steps are DPP moves inside the group's row.  A
// group's broadcasts never leave its own 16 lanes (ds_swizzle, DPP row
// patterns, bpermute inside the group) and its control flow is uniform
// across its lanes, so the groups of a wave may diverge freely.  A query
// with a NaN weight goes to the one-wave kernel (list fb2), whose scan
// reproduces the reference's order-dependent NaN comparisons.
constexpr int kGroupKMax = 128;

template <int L>
__device__ __forceinline__ float gbc_t(float x) {   // lane L of this lane's 16-lane group
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, x), 0x10 | (L << 5)));
}
// (l is a constant after unrolling: the switch folds to one swizzle)
__device__ __forceinline__ float gbc(float x, int l) {
    switch (l) {
        case 0: return gbc_t<0>(x);   case 1: return gbc_t<1>(x);   case 2: return gbc_t<2>(x);
        case 3: return gbc_t<3>(x);   case 4: return gbc_t<4>(x);   case 5: return gbc_t<5>(x);
        case 6: return gbc_t<6>(x);   case 7: return gbc_t<7>(x);   case 8: return gbc_t<8>(x);
        case 9: return gbc_t<9>(x);   case 10: return gbc_t<10>(x); case 11: return gbc_t<11>(x);
        case 12: return gbc_t<12>(x); case 13: return gbc_t<13>(x); case 14: return gbc_t<14>(x);
        default: return gbc_t<15>(x);
    }
}
// acc += x of this group's elements p = 16 i + l < n, in p order (n uniform
// inside a group; a skipped term adds -0.0, an exact no-op)
template <int S>
__device__ __forceinline__ float gseq_sum(float acc, const float (&x)[S], int n) {
#pragma unroll
    for (int i = 0; i < S; ++i) {
        if (!__any(16 * i < n)) break;
        // all 16 broadcasts in flight first, then the add chain (one wait)
        float b[16];
#pragma unroll
        for (int l = 0; l < 16; ++l) b[l] = gbc(x[i], l);
#pragma unroll
        for (int l = 0; l < 16; ++l) acc += (16 * i + l < n) ? b[l] : -0.0f;
    }
    return acc;
}
// One full-K query on this lane's group; false: a NaN weight (the caller
// hands the query to the one-wave kernel).  Outputs written by group lane 0.
template <bool PDF_ONLY, int S>
__device__ __forceinline__ bool serve_full_group(const float* gp, int Kp, int K, const GuideIO& io, int64_t q,
                                                 int lane, GuideConsts gc) {
    const int gl = lane & 15;
    const int gbase = lane & 48;
    const float c[3] = {io.c0[q], io.c1[q], io.c2[q]};
    float wr[S];
    unsigned vmask = 0;   // bit i: the conditional of component 16 i + gl is valid
    bool nan_l = false;
#pragma unroll
    for (int i = 0; i < S; ++i) {
        const int k = 16 * i + gl;
        wr[i] = -0.0f;    // absent: never a candidate
        if (k < K) {
            wr[i] = gp_ld(gp, Kp, GP_W, k) * marginal_pdf(gp, Kp, k, c, gc.norm3);
            vmask |= (cond_valid(gp, Kp, k, c) ? 1u : 0u) << i;
        }
        nan_l |= (wr[i] != wr[i]);
    }
    if (((__builtin_amdgcn_ballot_w64(nan_l) >> gbase) & 0xFFFFull) != 0) return false;
    // totalMass in component order (element k = 16 i + l)
    const float total = gseq_sum<S>(0.0f, wr, K);
    const float cutoff = (float)(0.99 * (double)total);
    // the selection order: (weight desc, index asc), absent entries last
    uint32_t key[S], idx[S];
    {
        uint64_t v[S];
#pragma unroll
        for (int i = 0; i < S; ++i)
            v[i] = sel_key(__builtin_signbit(wr[i]) ? 0u : __builtin_bit_cast(uint32_t, wr[i]) + 1u,
                           (uint32_t)(16 * i + gl));
        bsort<16, S>(v, gl);
#pragma unroll
        for (int i = 0; i < S; ++i) { key[i] = sel_wkey(v[i]); idx[i] = sel_idx(v[i]); }
    }
    int n_live = 0;
    float w[S];
    bool ok[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
        n_live += __builtin_popcountll((__builtin_amdgcn_ballot_w64(key[i] != 0u) >> gbase) & 0xFFFFull);
        const unsigned vm = (unsigned)__shfl((int)vmask, gbase | (int)(idx[i] & 15u));
        ok[i] = (vm >> (idx[i] >> 4)) & 1u;
        w[i] = __builtin_bit_cast(float, key[i] - 1u);
    }
    // the cutoff walk: accum of the valid weights in selection order
    float accum = 0.0f;
    int lastIdx = n_live;   // (K when every weight is live and the cutoff is never reached)
    bool done = false;
#pragma unroll
    for (int i = 0; i < S; ++i) {
        if (!__any(!done && 16 * i < n_live)) break;
        const float t = ok[i] ? w[i] : 0.0f;
        float bt[16];
#pragma unroll
        for (int l = 0; l < 16; ++l) bt[l] = gbc(t, l);
#pragma unroll
        for (int l = 0; l < 16; ++l) {
            const int p = 16 * i + l;
            if (!done && p < n_live) {
                accum += bt[l];
                if (accum >= cutoff) { lastIdx = p + 1; done = true; }
            }
        }
    }
    // finish_query: slot weights, createCdf, sample / given direction, pdf
    const float invSum = 1.0f / accum;
    const bool scaled = __builtin_isfinite(invSum);
    float f[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
        float wi = ok[i] ? w[i] : 0.0f;
        if (scaled) wi = wi * invSum;
        f[i] = wi;
    }
    const float sum2 = gseq_sum<S>(0.0f, f, lastIdx);
    bool pdf_q = PDF_ONLY;
    if constexpr (!PDF_ONLY) pdf_q = io.pmode && io.pmode[q];   // uniform in the group
    float outd[3] = {0.0f, 0.0f, 0.0f};
    float outpdf = 0.0f;
    int outcomp = -1;
    if (lastIdx > 0 && sum2 != 0.0f) {
        const DivBy by_sum2(sum2);
#pragma unroll
        for (int i = 0; i < S; ++i) f[i] = by_sum2(f[i]);
        float dir[3];
        if (!pdf_q) {
            // sampleDiscreteCdf: lower_bound == first slot with cdf >= u, else the tie walk
            const float u0 = io.u0[q], u1 = io.u1[q], u2 = io.u2[q];
            float cdf = 0.0f, prev = 0.0f;
            int slot = -1, runStart = 0;
#pragma unroll
            for (int i = 0; i < S; ++i) {
                if (!__any(slot < 0 && 16 * i < lastIdx)) break;
                float bf[16];
#pragma unroll
                for (int l = 0; l < 16; ++l) bf[l] = gbc(f[i], l);
#pragma unroll
                for (int l = 0; l < 16; ++l) {
                    const float b = bf[l];
                    const int p = 16 * i + l;
                    if (slot < 0 && p < lastIdx) {
                        cdf += b;
                        if (p == 0 || cdf != prev) runStart = p;
                        prev = cdf;
                        if (cdf >= u0) slot = p;
                    }
                }
            }
            if (slot < 0) slot = runStart;
            int mine = 0;
#pragma unroll
            for (int i = 0; i < S; ++i) mine = (i == (slot >> 4)) ? (int)idx[i] : mine;
            const int ksel = __shfl(mine, gbase | (slot & 15));
            float esel[3];
            cond_mean_dir(gp, Kp, ksel, c, esel);
            const float radius = sqrtf(-2.0f * logf(1.0f - u1));
            const float theta = (float)(2.0 * kPi * (double)u2);
            float res0, res1;
            sincosf(theta, &res0, &res1);
            const float z0 = radius * res0, z1 = radius * res1;
            const float L00 = gp_ld(gp, Kp, GP_CL00, ksel), L10 = gp_ld(gp, Kp, GP_CL10, ksel);
            const float L11 = gp_ld(gp, Kp, GP_CL11, ksel);
            const float v0 = L00 * z0 + 0.0f * z1;
            const float v1 = L10 * z0 + L11 * z1;
            float tof[9];
            coordinates_f(esel, tof);
            ts_exp_dir(tof, v0, v1, dir);
            outcomp = ksel;
        } else {
            dir[0] = io.e0[q]; dir[1] = io.e1[q]; dir[2] = io.e2[q];
            outcomp = kCompPdfValid;
        }
        // MixtureModel::pdf over the conditional: terms per own slot, summed in slot order
        float term[S];
#pragma unroll
        for (int i = 0; i < S; ++i) {
            term[i] = -0.0f;
            if (16 * i + gl < lastIdx && f[i] != 0.0f) {
                float e[3];
                cond_mean_dir(gp, Kp, (int)idx[i], c, e);
                term[i] = f[i] * cond_component_pdf(gp, Kp, (int)idx[i], e, dir, gc.norm2);
            }
        }
        outpdf = gseq_sum<S>(0.0f, term, lastIdx);
        outd[0] = dir[0]; outd[1] = dir[1]; outd[2] = dir[2];
    }
    if (gl == 0) {
        io.pdf[q] = outpdf;
        if constexpr (!PDF_ONLY) {
            io.d0[q] = outd[0]; io.d1[q] = outd[1]; io.d2[q] = outd[2];
            io.comp[q] = outcomp;
        }
    }
    return true;
}

// ---------------------------------------------------------------------------
// The same full-K query on a G-lane group, G = 4 (an A/B option) or 16: lane l
// of a group holds components l, l + G, ... (S slots, K <= G S).  Same
// arithmetic and order as serve_full_group (G = 16 reproduces it); with G = 4
// sixteen queries share every instruction of the serial float chains (four
// times as many as with 16-lane groups), the broadcasts inside a group are
// DPP quad permutes (no LDS pipe), and the sort's cross-lane steps are the
// two quad steps (J = 1, 2) -- the rest of the bitonic network is
// compare-exchange inside a lane's registers.  The per-slot values stay in
// registers as keys (weight bits + 1, index) plus a validity bit mask; the
// slot weights and pdf terms are re-derived from them where consumed.
template <int G>
__device__ __forceinline__ float gbcast(float x, int l) {   // lane l of this lane's G-lane group
    if constexpr (G == 16) {
        return gbc(x, l);
    } else {
        static_assert(G == 4, "groups of 4 or 16 lanes");
        const int xi = __builtin_bit_cast(int, x);
        int r;
        switch (l) {   // quad_perm [l, l, l, l]
            case 0: r = dppi<0x00>(xi); break;
            case 1: r = dppi<0x55>(xi); break;
            case 2: r = dppi<0xAA>(xi); break;
            default: r = dppi<0xFF>(xi); break;
        }
        return __builtin_bit_cast(float, r);
    }
}
// acc += v(i) of this group's elements p = G i + l < n, in p order (n uniform
// inside a group; a skipped term adds -0.0, an exact no-op); v(i) is this
// lane's value of slot i
template <int G, int S, class V>
__device__ __forceinline__ float gseq_stream(float acc, int n, V&& v) {
#pragma unroll
    for (int i = 0; i < S; ++i) {
        if (!__any(G * i < n)) break;
        const float x = v(i);
        float b[G];
#pragma unroll
        for (int l = 0; l < G; ++l) b[l] = gbcast<G>(x, l);
#pragma unroll
        for (int l = 0; l < G; ++l) acc += (G * i + l < n) ? b[l] : -0.0f;
    }
    return acc;
}

template <bool PDF_ONLY, int G, int S>
__device__ __forceinline__ bool serve_full_group_g(const float* gp, int Kp, int K, const GuideIO& io, int64_t q,
                                                   int lane, GuideConsts gc) {
    static_assert(S <= 32, "validity masks are 32-bit");
    constexpr uint64_t GM = (1ull << G) - 1;
    const int gl = lane & (G - 1);
    const int gbase = lane & ~(G - 1);
    const float c[3] = {io.c0[q], io.c1[q], io.c2[q]};
    uint32_t key[S], idx[S];
    uint32_t vmask = 0;   // bit i: the conditional of component G i + gl is valid
    float total;
    {
        float wr[S];
        bool nan_l = false;
#pragma unroll
        for (int i = 0; i < S; ++i) {
            const int k = G * i + gl;
            wr[i] = -0.0f;    // absent: never a candidate
            if (k < K) {
                wr[i] = gp_ld(gp, Kp, GP_W, k) * marginal_pdf(gp, Kp, k, c, gc.norm3);
                vmask |= (cond_valid(gp, Kp, k, c) ? 1u : 0u) << i;
            }
            nan_l |= (wr[i] != wr[i]);
        }
        if (((__builtin_amdgcn_ballot_w64(nan_l) >> gbase) & GM) != 0) return false;
        // totalMass in component order (element k = G i + l)
        total = gseq_stream<G, S>(0.0f, K, [&](int i) { return wr[i]; });
        // the selection order: (weight desc, index asc), absent entries last
        uint64_t v[S];
#pragma unroll
        for (int i = 0; i < S; ++i)
            v[i] = sel_key(__builtin_signbit(wr[i]) ? 0u : __builtin_bit_cast(uint32_t, wr[i]) + 1u,
                           (uint32_t)(G * i + gl));
        bsort<G, S>(v, gl);
#pragma unroll
        for (int i = 0; i < S; ++i) { key[i] = sel_wkey(v[i]); idx[i] = sel_idx(v[i]); }
    }
    const float cutoff = (float)(0.99 * (double)total);
    int n_live = 0;
    uint32_t okm = 0;   // bit i: sorted element G i + gl has a valid conditional
#pragma unroll
    for (int i = 0; i < S; ++i) {
        n_live += __builtin_popcountll((__builtin_amdgcn_ballot_w64(key[i] != 0u) >> gbase) & GM);
        const unsigned vm = (unsigned)__shfl((int)vmask, gbase | (int)(idx[i] & (G - 1)));
        okm |= ((vm >> (idx[i] / G)) & 1u) << i;
    }
    auto wk = [&](int i) { return __builtin_bit_cast(float, key[i] - 1u); };
    auto kept = [&](int i) { return ((okm >> i) & 1u) ? wk(i) : 0.0f; };
    // the cutoff walk: accum of the valid weights in selection order
    float accum = 0.0f;
    int lastIdx = n_live;   // (K when every weight is live and the cutoff is never reached)
    bool done = false;
#pragma unroll
    for (int i = 0; i < S; ++i) {
        if (!__any(!done && G * i < n_live)) break;
        const float t = kept(i);
        float bt[G];
#pragma unroll
        for (int l = 0; l < G; ++l) bt[l] = gbcast<G>(t, l);
#pragma unroll
        for (int l = 0; l < G; ++l) {
            const int p = G * i + l;
            if (!done && p < n_live) {
                accum += bt[l];
                if (accum >= cutoff) { lastIdx = p + 1; done = true; }
            }
        }
    }
    // finish_query: slot weights, createCdf, sample / given direction, pdf
    const float invSum = 1.0f / accum;
    const bool scaled = __builtin_isfinite(invSum);
    auto fs = [&](int i) {   // the slot weight before the sum2 normalisation
        float wi = kept(i);
        if (scaled) wi = wi * invSum;
        return wi;
    };
    const float sum2 = gseq_stream<G, S>(0.0f, lastIdx, fs);
    bool pdf_q = PDF_ONLY;
    if constexpr (!PDF_ONLY) pdf_q = io.pmode && io.pmode[q];   // uniform in the group
    float outd[3] = {0.0f, 0.0f, 0.0f};
    float outpdf = 0.0f;
    int outcomp = -1;
    if (lastIdx > 0 && sum2 != 0.0f) {
        const DivBy by_sum2(sum2);
        auto f = [&](int i) { return by_sum2(fs(i)); };
        float dir[3];
        if (!pdf_q) {
            // sampleDiscreteCdf: lower_bound == first slot with cdf >= u, else the tie walk
            const float u0 = io.u0[q], u1 = io.u1[q], u2 = io.u2[q];
            float cdf = 0.0f, prev = 0.0f;
            int slot = -1, runStart = 0;
#pragma unroll
            for (int i = 0; i < S; ++i) {
                if (!__any(slot < 0 && G * i < lastIdx)) break;
                const float fi = f(i);
                float bf[G];
#pragma unroll
                for (int l = 0; l < G; ++l) bf[l] = gbcast<G>(fi, l);
#pragma unroll
                for (int l = 0; l < G; ++l) {
                    const float b = bf[l];
                    const int p = G * i + l;
                    if (slot < 0 && p < lastIdx) {
                        cdf += b;
                        if (p == 0 || cdf != prev) runStart = p;
                        prev = cdf;
                        if (cdf >= u0) slot = p;
                    }
                }
            }
            if (slot < 0) slot = runStart;
            int mine = 0;
#pragma unroll
            for (int i = 0; i < S; ++i) mine = (i == slot / G) ? (int)idx[i] : mine;
            const int ksel = __shfl(mine, gbase | (slot & (G - 1)));
            float esel[3];
            cond_mean_dir(gp, Kp, ksel, c, esel);
            const float radius = sqrtf(-2.0f * logf(1.0f - u1));
            const float theta = (float)(2.0 * kPi * (double)u2);
            float res0, res1;
            sincosf(theta, &res0, &res1);
            const float z0 = radius * res0, z1 = radius * res1;
            const float L00 = gp_ld(gp, Kp, GP_CL00, ksel), L10 = gp_ld(gp, Kp, GP_CL10, ksel);
            const float L11 = gp_ld(gp, Kp, GP_CL11, ksel);
            const float v0 = L00 * z0 + 0.0f * z1;
            const float v1 = L10 * z0 + L11 * z1;
            float tof[9];
            coordinates_f(esel, tof);
            ts_exp_dir(tof, v0, v1, dir);
            outcomp = ksel;
        } else {
            dir[0] = io.e0[q]; dir[1] = io.e1[q]; dir[2] = io.e2[q];
            outcomp = kCompPdfValid;
        }
        // MixtureModel::pdf over the conditional: terms per own slot, summed in slot order
        outpdf = gseq_stream<G, S>(0.0f, lastIdx, [&](int i) {
            float term = -0.0f;
            const float fi = f(i);
            if (G * i + gl < lastIdx && fi != 0.0f) {
                float e[3];
                cond_mean_dir(gp, Kp, (int)idx[i], c, e);
                term = fi * cond_component_pdf(gp, Kp, (int)idx[i], e, dir, gc.norm2);
            }
            return term;
        });
        outd[0] = dir[0]; outd[1] = dir[1]; outd[2] = dir[2];
    }
    if (gl == 0) {
        io.pdf[q] = outpdf;
        if constexpr (!PDF_ONLY) {
            io.d0[q] = outd[0]; io.d1[q] = outd[1]; io.d2[q] = outd[2];
            io.comp[q] = outcomp;
        }
    }
    return true;
}

// The listed full-K queries, a G-lane group each (grid-stride over groups);
// TREE: each against its own leaf's mixture.  NaN queries -> fb2 (count at
// fb2[0], list from fb2 + 1) for the one-wave kernel.
// 16 (default) or 4 lanes per query.  Round 4 A/B, Cornell K=128 tree
// wavefront: 12.4 ms per guided pass with 16-lane groups, 13.1 ms with 4-lane
// groups (32 slots per lane: 256 VGPRs with a spill, 2 waves per SIMD)
// 16-lane groups (round 4: 4-lane groups, 16 queries per wave, spilled and
// lost: 13.1 against 12.0 ms per K = 128 guided pass)
constexpr int kGroupLanes = 16;
#ifndef SDMM_GROUP_WPE   // (A/B: tools/build_variant.sh)
#define SDMM_GROUP_WPE 4
#endif
constexpr int kGroupWpe = SDMM_GROUP_WPE;   // 128 VGPRs, no spill; K=128 guided pass 17.6 -> 15.2 ms (2: 189 VGPRs)
// (4-lane groups with 16 or 32 slots: 256 VGPRs, 2 waves per SIMD, no spill)
template <bool PDF_ONLY, bool TREE, int S>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(S >= 16 ? 2 : kGroupWpe)))
guide_group_fallback_kernel(const float* __restrict__ gp1, int Kp1, int K1, const STNodeDev* __restrict__ nodes,
                            const GuideMix* __restrict__ tab, GuideIO io, GuideConsts gc,
                            const int* __restrict__ fb_count, const int32_t* __restrict__ fb_list,
                            int* __restrict__ fb2, const int32_t* __restrict__ node_of) {
    constexpr int G = kGroupLanes, GPW = 64 / G;
    const int lane = threadIdx.x;
    const int count = *fb_count;
    const int64_t groups = (int64_t)gridDim.x * GPW;
    const int64_t g0 = (int64_t)blockIdx.x * GPW + lane / G;
    // With node_of (tree wavefront), the chain list entry -> node -> mixture
    // record of a query is fetched in a three-stage pipeline across this
    // group's iterations (entry three ahead, node two ahead, record one
    // ahead), so no iteration starts by waiting on three dependent loads.
    const bool piped = TREE && node_of != nullptr;
    int64_t qa = 0, qb = 0, qc = 0;   // entries of iterations i + 1, i + 2 (and i + 3 in flight)
    int nb = 0;                       // node of iteration i + 1
    GuideMix mc{gp1, Kp1, K1};        // record of iteration i
    if (piped) {
        if (g0 < count) {
            const int64_t q0 = fb_list[g0];
            mc = tab[node_of[q0]];
            qc = q0;
        }
        if (g0 + groups < count) { qa = fb_list[g0 + groups]; nb = node_of[qa]; }
        if (g0 + 2 * groups < count) qb = fb_list[g0 + 2 * groups];
    }
    for (int64_t gi = g0; gi < count; gi += groups) {
        int64_t q;
        const float* gp = gp1;
        int Kp = Kp1, K = K1;
        if (piped) {
            q = qc;
            gp = mc.gp; Kp = mc.Kp; K = mc.K;
            // advance the pipeline: record of i + 1, node of i + 2, entry of i + 3
            const bool h1 = gi + groups < count, h2 = gi + 2 * groups < count, h3 = gi + 3 * groups < count;
            if (h1) mc = tab[nb];
            qc = qa;
            if (h2) nb = node_of[qb];
            qa = qb;
            if (h3) qb = fb_list[gi + 3 * groups];
        } else {
            q = fb_list[gi];
            if constexpr (TREE) {
                // a listed query has a mixture
                const int node = stree_find_point(nodes, io.c0[q], io.c1[q], io.c2[q]);
                const GuideMix mx = tab[node];
                gp = mx.gp; Kp = mx.Kp; K = mx.K;
            }
        }
        bool ok;
        if constexpr (G == 16) ok = serve_full_group<PDF_ONLY, S>(gp, Kp, K, io, q, lane, gc);
        else ok = serve_full_group_g<PDF_ONLY, G, S>(gp, Kp, K, io, q, lane, gc);
        if (!ok && (lane & (G - 1)) == 0) fb2[1 + atomicAdd(fb2, 1)] = (int32_t)q;
    }
}

// S = slots per lane: kmax <= G S
template <bool PDF_ONLY, bool TREE>
static void launch_group_fallback(int kmax, int blocks, hipStream_t st, const float* gp, int Kp, int K,
                                  const STNodeDev* nd, const GuideMix* tb, const GuideIO& io, GuideConsts gc,
                                  const int* fb_count, const int32_t* fb_list, int* fb2,
                                  const int32_t* node_of = nullptr) {
    constexpr int G = kGroupLanes;
    if (kmax <= G)
        hipLaunchKernelGGL((guide_group_fallback_kernel<PDF_ONLY, TREE, 1>), dim3(blocks), dim3(64), 0, st, gp, Kp,
                           K, nd, tb, io, gc, fb_count, fb_list, fb2, node_of);
    else if (kmax <= 2 * G)
        hipLaunchKernelGGL((guide_group_fallback_kernel<PDF_ONLY, TREE, 2>), dim3(blocks), dim3(64), 0, st, gp, Kp,
                           K, nd, tb, io, gc, fb_count, fb_list, fb2, node_of);
    else if (kmax <= 4 * G)
        hipLaunchKernelGGL((guide_group_fallback_kernel<PDF_ONLY, TREE, 4>), dim3(blocks), dim3(64), 0, st, gp, Kp,
                           K, nd, tb, io, gc, fb_count, fb_list, fb2, node_of);
    else if (kmax <= 8 * G)
        hipLaunchKernelGGL((guide_group_fallback_kernel<PDF_ONLY, TREE, 8>), dim3(blocks), dim3(64), 0, st, gp, Kp,
                           K, nd, tb, io, gc, fb_count, fb_list, fb2, node_of);
}
static_assert(kGroupKMax <= 8 * kGroupLanes, "group slots");

// ---------------------------------------------------------------------------
// Product with a learned BSDF (the plugin's sampleProduct path,
// sdmm_proc.cpp:327-392, :474-486): MixtureModel::multiply of the query's
// conditional with a learned-BSDF lobe set (mixture_model.h:345-370,
// multivariate_tangent_normal.h:555-617), then sample / pdf of the product.
// Follows oracle/sdmm_oracle_product.inc operation for operation (contract
// off, the oracle's correctly rounded float transcendentals as
// (float)f((double)x), IEEE division / sqrt), so the product weights -- and
// with them the selected (joint component, lobe) index -- are bit-identical.
// The product is never materialised: one pass sums the weights, a second
// walks the CDF to the sampled pair, a third accumulates the pdf at the
// sampled direction, each recomputing the pairs (a pair is ~40 small
// matrix/vector ops; the kept conditional x lobes is tens of pairs).

// Per-query cache of the product pairs formed by the mass pass (pass 1), so
// the CDF walk and the pdf pass read them instead of re-forming every pair
// (each ~40 small ops with fp64-rounded transcendentals).  Pair p of the
// query in cache column `col`: fields f (weight, slot | lobe << 16, mean 3,
// Linv 4, detInv) at base[(p * kPairFields + f) * stride + col] -- coalesced
// across a wave's queries.  A query with more than cap pairs re-forms them.
constexpr int kPairFields = 10;
constexpr int kPairCacheCap = 16;
struct PairCacheDev {
    float* base;
    int64_t stride;
    int cap;
};

// heuristicConditionalWeight with a usable product (sdmm_proc.cpp:386-387)
constexpr float kProductH = 0.3f;

struct BsdfTab {
    const float* w;      // [B][M]
    const float* mean;   // [B][M][3]  local shading frame
    const float* cov;    // [B][M][4]  2x2 in the lobe's own tangent frame
    int B, M;
    // per material (nullable): a diffuse BSDF -- the plugin's diffuse case
    // (sdmm_proc.cpp:335-339) only re-centres slice 0 on the shading normal
    // (set_mean: mean n, frame Coordinates(n)); slices >= 1 are used as stored
    const uint8_t* diffuse;
};

struct ProductIO {
    const int32_t* material;   // per query; < 0: no learned BSDF
    const float* F[9];         // per-query to-world frame, row-major [s t n]
    float* h;                  // heuristicConditionalWeight per query
    // mixed wavefront (nullable; sampling kernels): query q is a pdf query at
    // its given direction io.e[q] when choice[q] <= h, h being the query's own
    // heuristic weight (0.3 product / 0.5 conditional), the reference's
    // rRec.nextSample1D() <= heuristicConditionalWeight (:392)
    const float* choice;
    PairCacheDev cache;        // the thread path's pair cache (base null: none)
};

__device__ __forceinline__ float acos_x(float x) { return (float)acos((double)x); }
__device__ __forceinline__ float sin_x(float x) { return (float)sin((double)x); }
__device__ __forceinline__ float cos_x(float x) { return (float)cos((double)x); }
__device__ __forceinline__ float log_x(float x) { return (float)log((double)x); }

__device__ __forceinline__ float sinc_pi_x(float x) {
    const float taylor_0_bound = 1.1920928955078125e-07f;
    const float taylor_2_bound = 3.4526698300124393e-04f;
    const float taylor_n_bound = 1.8581361171917516e-02f;
    const float ax = fabsf(x);
    if (ax >= taylor_n_bound) return sin_x(x) / x;
    float result = 1.0f;
    if (ax >= taylor_0_bound) {
        const float x2 = x * x;
        result -= x2 / 6.0f;
        if (ax >= taylor_2_bound) result += (x2 * x2) / 120.0f;
    }
    return result;
}

// or_ts_log (TangentSpace::log, mvtn.h:146-177), directional part
__device__ __forceinline__ bool ts_log_x(const float to[9], const float d[3], float& t0, float& t1,
                                         float& jac) {
    if (d[0] == 0.0f && d[1] == 0.0f && d[2] == 0.0f) return false;
    const float r0 = to[0] * d[0] + to[1] * d[1] + to[2] * d[2];
    const float r1 = to[3] * d[0] + to[4] * d[1] + to[5] * d[2];
    float c = to[6] * d[0] + to[7] * d[1] + to[8] * d[2];
    if (c <= -1.0f) return false;
    c = (c < 1.0f) ? c : 1.0f;
    const float angle = acos_x(c);
    const float s = sqrtf(1.0f - c * c);
    const float a = ((double)s < 1e-3) ? 1.0f : (angle / s);
    t0 = r0 * a;
    t1 = r1 * a;
    jac = a;
    return true;
}

// or_ts_exp (TangentSpace::exp, mvtn.h:93-120), directional part
__device__ __forceinline__ bool ts_exp_x(const float to[9], float t0, float t1, float e[3]) {
    const float length = sqrtf(t0 * t0 + t1 * t1);
    if ((double)length >= kPi) { e[0] = e[1] = e[2] = 0.0f; return false; }
    const float s = sinc_pi_x(length);
    const float rel0 = t0 * s, rel1 = t1 * s, rel2 = cos_x(length);
    e[0] = to[0] * rel0 + to[3] * rel1 + to[6] * rel2;
    e[1] = to[1] * rel0 + to[4] * rel1 + to[7] * rel2;
    e[2] = to[2] * rel0 + to[5] * rel1 + to[8] * rel2;
    return true;
}

// the conditional mean direction of joint component k with the oracle's
// transcendentals (cond_mean_dir uses the fast float ones)
__device__ __forceinline__ void cond_mean_dir_x(const float* gp, int Kp, int k, const float c[3], float e[3]) {
    const float d0 = c[0] - gp_ld(gp, Kp, GP_MU0, k);
    const float d1 = c[1] - gp_ld(gp, Kp, GP_MU1, k);
    const float d2 = c[2] - gp_ld(gp, Kp, GP_MU2, k);
    const float t0 = gp_ld(gp, Kp, GP_P00, k) * d0 + gp_ld(gp, Kp, GP_P01, k) * d1 + gp_ld(gp, Kp, GP_P02, k) * d2;
    const float t1 = gp_ld(gp, Kp, GP_P10, k) * d0 + gp_ld(gp, Kp, GP_P11, k) * d1 + gp_ld(gp, Kp, GP_P12, k) * d2;
    float to[9];
    for (int i = 0; i < 9; ++i) to[i] = gp_ld(gp, Kp, GP_T00 + i, k);
    ts_exp_x(to, t0, t1, e);
}

__device__ __forceinline__ void m22_mul(const float* a, const float* b, float* r) {
    r[0] = a[0] * b[0] + a[1] * b[2];
    r[1] = a[0] * b[1] + a[1] * b[3];
    r[2] = a[2] * b[0] + a[3] * b[2];
    r[3] = a[2] * b[1] + a[3] * b[3];
}
__device__ __forceinline__ void m22_mul_t(const float* a, const float* b, float* r) {
    r[0] = a[0] * b[0] + a[1] * b[1];
    r[1] = a[0] * b[2] + a[1] * b[3];
    r[2] = a[2] * b[0] + a[3] * b[1];
    r[3] = a[2] * b[2] + a[3] * b[3];
}
__device__ __forceinline__ void m22_inv(const float* m, float* r) {
    const float invdet = 1.0f / (m[0] * m[3] - m[2] * m[1]);
    r[0] = m[3] * invdet;
    r[1] = -m[1] * invdet;
    r[2] = -m[2] * invdet;
    r[3] = m[0] * invdet;
}
__device__ __forceinline__ bool llt22(const float* A, float* L) {
    float x = A[0];
    if (!(x > 0.0f)) return false;
    const float l00 = sqrtf(x);
    const float l10 = A[2] / l00;
    x = A[3] - l10 * l10;
    if (!(x > 0.0f)) return false;
    L[0] = l00; L[1] = 0.0f; L[2] = l10; L[3] = sqrtf(x);
    return true;
}
__device__ __forceinline__ void m23_33(const float* a, const float* b, float* r) {
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j)
            r[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}
__device__ __forceinline__ void m23_32(const float* a, const float* b, float* r) {
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            r[2 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[2 + j] + a[3 * i + 2] * b[4 + j];
}
// TangentSpace::logJacobian (mvtn.h:211-246), 2x3
__device__ __forceinline__ void log_jacobian(const float to[9], const float mean[3], const float x[3],
                                             float J[6]) {
    const float r0 = to[0] * x[0] + to[1] * x[1] + to[2] * x[2];
    const float r1 = to[3] * x[0] + to[4] * x[1] + to[5] * x[2];
    float c = to[6] * x[0] + to[7] * x[1] + to[8] * x[2];
    c = (c < 1.0f) ? c : 1.0f;
    for (int i = 0; i < 6; ++i) J[i] = 0.0f;
    if (c <= -1.0f) return;
    if (c == 1.0f || (x[0] == mean[0] && x[1] == mean[1] && x[2] == mean[2])) {
        J[0] = 1.0f; J[4] = 1.0f;
        return;
    }
    const float angle = acos_x(c);
    const float aos = 1.0f / sinc_pi_x(angle);
    J[0] = aos; J[4] = aos;
    const float iss = 1.0f / (1.0f - c * c);
    J[2] = r0 * c * aos * iss - r0 * iss;
    J[5] = r1 * c * aos * iss - r1 * iss;
}
// TangentSpace::expJacobian (mvtn.h:179-209), 3x2
__device__ __forceinline__ void exp_jacobian(float t0, float t1, float J[6]) {
    const float length = sqrtf(t0 * t0 + t1 * t1);
    for (int i = 0; i < 6; ++i) J[i] = 0.0f;
    if (length == 0.0f) {
        J[0] = 1.0f; J[3] = 1.0f;
        return;
    }
    const float lsq = length * length;
    const float cs = cos_x(length);
    const float sinc = sinc_pi_x(length);
    const float cms = (cs - sinc) / lsq;
    J[0] = sinc + t0 * t0 * cms;
    J[3] = sinc + t1 * t1 * cms;
    const float off = t0 * t1 * cms;
    J[2] = off;
    J[1] = off;
    J[4] = -t0 * sinc;
    J[5] = -t1 * sinc;
}

// One product component: the conditional slot (e, to_i, ci) times the world
// lobe (mj, to_j, cj).  Returns the weight factor newWeight (0: dropped).
struct ProdComp {
    float mean[3];
    float L[4];
    float Linv[4];
    float detInv;
};
__device__ __forceinline__ float mvtn_multiply(const float e[3], const float to_i[9], const float ci[4],
                                            const float mj[3], const float to_j[9], const float cj[4],
                                            float norm2, ProdComp& out, bool lazy) {
    // ts_log_x(to_i, mj), keeping acos(c): logJacobian(to_i, e, mj) below forms
    // the same r0, r1, clamped c and acos(c) (the same float expressions), so
    // both share one evaluation -- bitwise what the two separate calls give
    if (mj[0] == 0.0f && mj[1] == 0.0f && mj[2] == 0.0f) return 0.0f;
    const float r0 = to_i[0] * mj[0] + to_i[1] * mj[1] + to_i[2] * mj[2];
    const float r1 = to_i[3] * mj[0] + to_i[4] * mj[1] + to_i[5] * mj[2];
    float c = to_i[6] * mj[0] + to_i[7] * mj[1] + to_i[8] * mj[2];
    if (c <= -1.0f) return 0.0f;
    c = (c < 1.0f) ? c : 1.0f;
    const float angle = acos_x(c);
    const float sang = sqrtf(1.0f - c * c);
    const float jac = ((double)sang < 1e-3) ? 1.0f : (angle / sang);
    const float om0 = r0 * jac, om1 = r1 * jac;
    float lj[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if (c == 1.0f || (mj[0] == e[0] && mj[1] == e[1] && mj[2] == e[2])) {
        lj[0] = 1.0f; lj[4] = 1.0f;
    } else {
        const float aos = 1.0f / sinc_pi_x(angle);
        lj[0] = aos; lj[4] = aos;
        const float iss = 1.0f / (1.0f - c * c);
        lj[2] = r0 * c * aos * iss - r0 * iss;
        lj[5] = r1 * c * aos * iss - r1 * iss;
    }
    float a[6], from_j[9], b[6], ej[6], J[4], t[4], ocov[4];
    m23_33(lj, to_i, a);
    for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc) from_j[3 * r + cc] = to_j[3 * cc + r];
    m23_33(a, from_j, b);
    exp_jacobian(0.0f, 0.0f, ej);
    m23_32(b, ej, J);
    m22_mul(J, cj, t);
    m22_mul_t(t, J, ocov);
    float csum[4], icsum[4], ci_ics[4], cnt[4];
    for (int i = 0; i < 4; ++i) csum[i] = ci[i] + ocov[i];
    m22_inv(csum, icsum);
    m22_mul(ci, icsum, ci_ics);
    const float mt0 = 0.0f + (ci_ics[0] * om0 + ci_ics[1] * om1);
    const float mt1 = 0.0f + (ci_ics[2] * om0 + ci_ics[3] * om1);
    m22_mul(ci_ics, ocov, cnt);
    // The weight depends only on om, csum and jac.  Evaluated first: a pair
    // whose weight is exactly 0 (FTZ) contributes nothing to a mass or a pdf
    // whatever the rest gives (every later exit also returns 0), so with
    // `lazy` it stops here.  The sampled pair is evaluated in full (a
    // zero-weight pair is sampled only by u = 0 on the first pair).
    float Ls[4];
    if (!llt22(csum, Ls)) return 0.0f;
    const float invDet = 1.0f / (Ls[0] * Ls[3]);
    const float s0 = om0 / Ls[0];
    const float s1 = (om1 - Ls[2] * s0) / Ls[3];
    float w = gauss_w(norm2, s0 * s0 + s1 * s1);
    w = w * (invDet * jac);
    if (lazy && w == 0.0f) return 0.0f;
    // ts_exp_x(to_i, mt) and expJacobian(mt) share |mt|, its sinc and cos
    const float length = sqrtf(mt0 * mt0 + mt1 * mt1);
    if ((double)length >= kPi) { out.mean[0] = out.mean[1] = out.mean[2] = 0.0f; return 0.0f; }
    // sinc_pi_x(length) and cos_x(length) from one double sincos (one argument
    // reduction; the same double values as the separate sin and cos)
    double sd, cd;
    sincos((double)length, &sd, &cd);
    const float cs = (float)cd;
    float sinc = 1.0f;
    if (length >= 1.8581361171917516e-02f) {
        sinc = (float)sd / length;
    } else if (length >= 1.1920928955078125e-07f) {
        const float x2 = length * length;
        sinc -= x2 / 6.0f;
        if (length >= 3.4526698300124393e-04f) sinc += (x2 * x2) / 120.0f;
    }
    {
        const float rel0 = mt0 * sinc, rel1 = mt1 * sinc, rel2 = cs;
        out.mean[0] = to_i[0] * rel0 + to_i[3] * rel1 + to_i[6] * rel2;
        out.mean[1] = to_i[1] * rel0 + to_i[4] * rel1 + to_i[7] * rel2;
        out.mean[2] = to_i[2] * rel0 + to_i[5] * rel1 + to_i[8] * rel2;
    }
    float to_n[9];
    coordinates_f(out.mean, to_n);
    float ln[6], a2[6], from_i[9], b2[6], ei[6], J2[4], t2[4], cov_n[4];
    log_jacobian(to_n, out.mean, out.mean, ln);
    m23_33(ln, to_n, a2);
    for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc) from_i[3 * r + cc] = to_i[3 * cc + r];
    m23_33(a2, from_i, b2);
    for (int i = 0; i < 6; ++i) ei[i] = 0.0f;
    if (length == 0.0f) {
        ei[0] = 1.0f; ei[3] = 1.0f;
    } else {
        const float lsq = length * length;
        const float cms = (cs - sinc) / lsq;
        ei[0] = sinc + mt0 * mt0 * cms;
        ei[3] = sinc + mt1 * mt1 * cms;
        const float off = mt0 * mt1 * cms;
        ei[2] = off;
        ei[1] = off;
        ei[4] = -mt0 * sinc;
        ei[5] = -mt1 * sinc;
    }
    m23_32(b2, ei, J2);
    m22_mul(J2, cnt, t2);
    m22_mul_t(t2, J2, cov_n);
    if (!llt22(cov_n, out.L)) return 0.0f;
    m22_inv(out.L, out.Linv);
    out.detInv = 1.0f / (out.L[0] * out.L[3]);
    return w;
}

// the world-frame lobe j of material b: mean F m, frame Coordinates(m) F^T
__device__ __forceinline__ void bsdf_world(const float F[9], const BsdfTab& bt, int b, int j, float mw[3],
                                           float tw[9], float cj[4], float& wj) {
    const int idx = b * bt.M + j;
    wj = bt.w[idx];
    const float ml[3] = {bt.mean[3 * idx], bt.mean[3 * idx + 1], bt.mean[3 * idx + 2]};
    for (int i = 0; i < 4; ++i) cj[i] = bt.cov[4 * idx + i];
    if (bt.diffuse && bt.diffuse[b]) {
        // slice 0: mean = the shading normal (F's third column), frame
        // Coordinates(mean); the other slices as stored (world)
        if (j == 0) { mw[0] = F[2]; mw[1] = F[5]; mw[2] = F[8]; }
        else { mw[0] = ml[0]; mw[1] = ml[1]; mw[2] = ml[2]; }
        coordinates_f(mw, tw);
        return;
    }
    float tl[9];
    coordinates_f(ml, tl);
    for (int i = 0; i < 3; ++i) mw[i] = F[3 * i] * ml[0] + F[3 * i + 1] * ml[1] + F[3 * i + 2] * ml[2];
    for (int i = 0; i < 3; ++i)
        for (int jj = 0; jj < 3; ++jj)
            tw[3 * i + jj] = tl[3 * i] * F[3 * jj] + tl[3 * i + 1] * F[3 * jj + 1] + tl[3 * i + 2] * F[3 * jj + 2];
}

// Walk the product pairs in the reference's order (slot i asc, lobe j asc)
// calling fn(pair_index, slot, k, j, weight, comp) for every kept pair.
template <class Slots, class Fn>
__device__ __forceinline__ void for_each_pair(const float* gp, int Kp, const float* condCov, const float c[3],
                                              int lastIdx, float invSum, bool scaled, float sum2,
                                              const Slots& S, const BsdfTab& bt, int b, const float F[9],
                                              float norm2, bool lazy, Fn&& fn) {
    int p = 0;
    const DivBy by_sum2(sum2);
    for (int i = 0; i < lastIdx; ++i) {
        float wi = S.valid(i) ? S.weight(i) : 0.0f;
        if (scaled) wi = wi * invSum;
        wi = by_sum2(wi);
        if (wi == 0.0f) continue;
        const int k = S.comp(i);
        float e[3], to_i[9], ci[4];
        cond_mean_dir_x(gp, Kp, k, c, e);
        coordinates_f(e, to_i);
        for (int l = 0; l < 4; ++l) ci[l] = condCov[4 * k + l];
        for (int j = 0; j < bt.M; ++j) {
            if (bt.w[b * bt.M + j] == 0.0f) continue;   // (a skipped lobe: no world transform)
            float mw[3], tw[9], cj[4], wj;
            bsdf_world(F, bt, b, j, mw, tw, cj, wj);
            if (e[0] * mw[0] + e[1] * mw[1] + e[2] * mw[2] < 0.0f) continue;
            ProdComp pc;
            const float nw = mvtn_multiply(e, to_i, ci, mw, tw, cj, norm2, pc, lazy);
            if (fn(p, i, k, j, wi * wj * nw, pc)) return;
            ++p;
        }
    }
}

// Product pair (slot i, lobe j) evaluated on its own, exactly as
// for_each_pair forms it (the same expressions): its weight wi * wj * nw and
// component.  Used to re-form the one pair a cached walk selected.
template <class Slots>
__device__ __forceinline__ float eval_pair(const float* gp, int Kp, const float* condCov, const float c[3],
                                           float invSum, bool scaled, float sum2, const Slots& S, int i,
                                           const BsdfTab& bt, int b, int j, const float F[9], float norm2,
                                           ProdComp& pc) {
    float wi = S.valid(i) ? S.weight(i) : 0.0f;
    if (scaled) wi = wi * invSum;
    wi = DivBy(sum2)(wi);
    const int k = S.comp(i);
    float e[3], to_i[9], ci[4];
    cond_mean_dir_x(gp, Kp, k, c, e);
    coordinates_f(e, to_i);
    for (int l = 0; l < 4; ++l) ci[l] = condCov[4 * k + l];
    float mw[3], tw[9], cj[4], wj;
    bsdf_world(F, bt, b, j, mw, tw, cj, wj);
    const float nw = mvtn_multiply(e, to_i, ci, mw, tw, cj, norm2, pc, false);
    return wi * wj * nw;
}


// MVTN<3,3>::pdf of a product component at d
__device__ __forceinline__ float prod_comp_pdf(const ProdComp& pc, const float d[3], float norm2) {
    float to[9];
    coordinates_f(pc.mean, to);
    float t0, t1, jac;
    if (!ts_log_x(to, d, t0, t1, jac)) return 0.0f;
    const float s0 = pc.Linv[0] * t0 + pc.Linv[1] * t1;
    const float s1 = pc.Linv[2] * t0 + pc.Linv[3] * t1;
    float v = gauss_w(norm2, s0 * s0 + s1 * s1);
    v *= pc.detInv * jac;
    return v;
}

// Query q after its conditional's kept prefix is known.  Returns false when
// the product is unusable (no learned BSDF, no pair, zero mass): the caller
// then serves the plain conditional (h = 0.5).
// choice: the mixed wavefront's BSDF/guide draw (> 1 when none): a query
// whose product is usable becomes a pdf query at dir_in when choice <= 0.3.
template <bool PDF_ONLY, class Slots>
__device__ bool finish_product(const float* gp, int Kp, const float* condCov, const float c[3], int lastIdx,
                               float accum, const Slots& S, const BsdfTab& bt, int b, const float F[9],
                               const float* u, const float* dir_in, float choice, GuideConsts gc, QueryOut& o,
                               const PairCacheDev& pcd, int64_t col) {
    const float invSum = 1.0f / accum;
    const bool scaled = __builtin_isfinite(invSum);
    float sum2 = 0.0f;
    for (int i = 0; i < lastIdx; ++i) {
        float wi = S.valid(i) ? S.weight(i) : 0.0f;
        if (scaled) wi = wi * invSum;
        sum2 += wi;
    }
    // pass 1: the product mass (createCdf(true)'s sum), each pair cached
    float total = 0.0f;
    int P = 0;
    bool cached = pcd.base != nullptr;
    auto cf = [&](int p, int f) -> float& { return pcd.base[((int64_t)p * kPairFields + f) * pcd.stride + col]; };
    for_each_pair(gp, Kp, condCov, c, lastIdx, invSum, scaled, sum2, S, bt, b, F, gc.norm2, true,
                  [&](int p, int i, int, int j, float w, const ProdComp& pc) {
                      total += w;
                      ++P;
                      if (cached) {
                          if (p >= pcd.cap) {
                              cached = false;
                          } else {
                              cf(p, 0) = w;
                              cf(p, 1) = __builtin_bit_cast(float, i | (j << 16));
                              if (w != 0.0f) {   // (a zero-weight pair is never read back)
                                  cf(p, 2) = pc.mean[0]; cf(p, 3) = pc.mean[1]; cf(p, 4) = pc.mean[2];
                                  cf(p, 5) = pc.Linv[0]; cf(p, 6) = pc.Linv[1]; cf(p, 7) = pc.Linv[2];
                                  cf(p, 8) = pc.Linv[3]; cf(p, 9) = pc.detInv;
                              }
                          }
                      }
                      return false;
                  });
    if (P == 0 || total == 0.0f) return false;
    float dir[3];
    o.comp = kCompPdfValid;
    if (!PDF_ONLY && !(choice <= kProductH)) {
        // pass 2: sampleDiscreteCdf over the normalised weights (lower_bound,
        // then the tie walk), keeping the selected pair
        float cdf = 0.0f, prev = 0.0f;
        int runStart = 0, sel = -1, selComp = -1, runComp = -1;
        ProdComp pcs{}, runPc{};
        if (cached) {
            int selCode = -1, runCode = -1;
            for (int p = 0; p < P; ++p) {
                cdf += cf(p, 0) / total;
                const int code = __builtin_bit_cast(int, cf(p, 1));
                if (p == 0 || cdf != prev) { runStart = p; runCode = code; }
                prev = cdf;
                if (cdf >= u[0]) { sel = p; selCode = code; break; }
            }
            if (sel < 0) selCode = runCode;
            const int si = selCode & 0xffff, sj = selCode >> 16;
            (void)eval_pair(gp, Kp, condCov, c, invSum, scaled, sum2, S, si, bt, b, sj, F, gc.norm2, pcs);
            selComp = S.comp(si) * bt.M + sj;
        } else {
            for_each_pair(gp, Kp, condCov, c, lastIdx, invSum, scaled, sum2, S, bt, b, F, gc.norm2, false,
                          [&](int p, int, int k, int j, float w, const ProdComp& pc) {
                              cdf += w / total;
                              if (p == 0 || cdf != prev) { runStart = p; runComp = k * bt.M + j; runPc = pc; }
                              prev = cdf;
                              if (cdf >= u[0]) { sel = p; selComp = k * bt.M + j; pcs = pc; return true; }
                              return false;
                          });
            if (sel < 0) { sel = runStart; selComp = runComp; pcs = runPc; }
        }
        const float radius = sqrtf(-2.0f * log_x(1.0f - u[1]));
        const float theta = (float)(2.0 * kPi * (double)u[2]);
        const float z0 = radius * sin_x(theta), z1 = radius * cos_x(theta);
        const float v0 = pcs.L[0] * z0 + pcs.L[1] * z1;
        const float v1 = pcs.L[2] * z0 + pcs.L[3] * z1;
        float to[9];
        coordinates_f(pcs.mean, to);
        if (!ts_exp_x(to, v0, v1, dir)) dir[0] = dir[1] = dir[2] = 0.0f;
        o.comp = selComp;
    } else {
        dir[0] = dir_in[0]; dir[1] = dir_in[1]; dir[2] = dir_in[2];
    }
    // pass 3: the product mixture pdf at dir
    float acc = 0.0f;
    if (cached) {
        for (int p = 0; p < P; ++p) {
            const float wn = cf(p, 0) / total;
            if (wn == 0.0f) continue;
            ProdComp pc{};
            pc.mean[0] = cf(p, 2); pc.mean[1] = cf(p, 3); pc.mean[2] = cf(p, 4);
            pc.Linv[0] = cf(p, 5); pc.Linv[1] = cf(p, 6); pc.Linv[2] = cf(p, 7); pc.Linv[3] = cf(p, 8);
            pc.detInv = cf(p, 9);
            acc += wn * prod_comp_pdf(pc, dir, gc.norm2);
        }
    } else {
        for_each_pair(gp, Kp, condCov, c, lastIdx, invSum, scaled, sum2, S, bt, b, F, gc.norm2, true,
                      [&](int, int, int, int, float w, const ProdComp& pc) {
                          const float wn = w / total;
                          if (wn != 0.0f) acc += wn * prod_comp_pdf(pc, dir, gc.norm2);
                          return false;
                      });
    }
    o.d[0] = dir[0]; o.d[1] = dir[1]; o.d[2] = dir[2];
    o.pdf = acc;
    return true;
}

// One thread per query over the full-K conditional (LDS K x blockDim).
// Everything after the kept prefix of query q's conditional is known
// (slots S, lastIdx, accum): the product with the query's learned BSDF, or the
// plain conditional, and the outputs.
template <bool PDF_ONLY, class Slots>
__device__ __forceinline__ void product_tail(const float* gp, int Kp, const float* condCov, const float c[3],
                                             int lastIdx, float accum, const Slots& S, const GuideIO& io,
                                             const ProductIO& pio, const BsdfTab& bt, int64_t q, GuideConsts gc,
                                             int64_t col) {
    int b = pio.material ? pio.material[q] : -1;
    if (b >= bt.B) b = -1;
    const bool mixed = !PDF_ONLY && pio.choice != nullptr;
    const float choice = mixed ? pio.choice[q] : 2.0f;
    // createCdf(true) of the conditional (finish_query's validity test)
    float sum2 = 0.0f;
    {
        const float invSum = 1.0f / accum;
        const bool scaled = __builtin_isfinite(invSum);
        for (int i = 0; i < lastIdx; ++i) {
            float wi = S.valid(i) ? S.weight(i) : 0.0f;
            if (scaled) wi = wi * invSum;
            sum2 += wi;
        }
    }
    const bool cvalid = lastIdx > 0 && sum2 != 0.0f;
    QueryOut o{{0.0f, 0.0f, 0.0f}, 0.0f, -1};
    float h = 1.0f;                       // no valid conditional: BSDF only
    if (cvalid) {
        float u[3] = {0.0f, 0.0f, 0.0f}, dg[3] = {0.0f, 0.0f, 0.0f};
        if (PDF_ONLY || mixed) { dg[0] = io.e0[q]; dg[1] = io.e1[q]; dg[2] = io.e2[q]; }
        if constexpr (!PDF_ONLY) { u[0] = io.u0[q]; u[1] = io.u1[q]; u[2] = io.u2[q]; }
        bool used = false;
        if (b >= 0 && bt.M > 0) {
            float F[9];
            for (int i = 0; i < 9; ++i) F[i] = pio.F[i][q];
            used = finish_product<PDF_ONLY>(gp, Kp, condCov, c, lastIdx, accum, S, bt, b, F, u, dg, choice, gc, o,
                                            pio.cache, col);
        }
        if (used) {
            h = kProductH;
        } else {
            h = 0.5f;
            const bool pdfq = PDF_ONLY || choice <= 0.5f;
            o = finish_query(gp, Kp, c, pdfq ? nullptr : u, lastIdx, accum, S, pdfq ? dg : nullptr, gc);
        }
    }
    if constexpr (PDF_ONLY) {
        io.pdf[q] = o.pdf;
    } else {
        io.d0[q] = o.d[0]; io.d1[q] = o.d[1]; io.d2[q] = o.d[2];
        io.pdf[q] = o.pdf;
        io.comp[q] = o.comp;
    }
    if (pio.h) pio.h[q] = h;
}

// no valid conditional: BSDF only, h = 1 (sdmm_proc.cpp:316-323)
template <bool PDF_ONLY>
__device__ __forceinline__ void product_invalid(const GuideIO& io, const ProductIO& pio, int64_t q) {
    write_invalid<PDF_ONLY>(io, q);
    if (pio.h) pio.h[q] = 1.0f;
}

// A candidate-served product query whose pair walk (kept slots x lobes) is
// long goes to the one-wave path (gc.route_pairs; the results are the same)
__device__ __forceinline__ bool routed_to_wave(int lastIdx, const ProductIO& pio, const BsdfTab& bt, int64_t q,
                                               const GuideConsts& gc) {
    if (lastIdx * bt.M <= gc.route_pairs) return false;
    const int b = pio.material ? pio.material[q] : -1;
    return b >= 0 && b < bt.B;
}

// Candidate path (as guide_cand_kernel: the kept prefix from the per-query LDS
// list, bit-identical to the full-K selection); queries the list cannot serve
// exactly go to fb_list for guide_product_wave_kernel.  perm: coherent order.
template <bool PDF_ONLY, int LCAP>
__global__ void __launch_bounds__(64)
guide_product_cand_kernel(const float* __restrict__ gp, int Kp, int K, const float* __restrict__ condCov,
                          int64_t nq, GuideIO io, ProductIO pio, BsdfTab bt, GuideConsts gc, int cap,
                          int* __restrict__ fb_count, int32_t* __restrict__ fb_list,
                          const int32_t* __restrict__ perm) {
    __shared__ float cw[LCAP * 64];
    __shared__ unsigned short ck[LCAP * 64];
    const int tid = threadIdx.x;
    const int64_t t = (int64_t)blockIdx.x * 64 + tid;
    if (t >= nq) return;
    const int64_t q = perm ? (int64_t)perm[t] : t;
    const float c[3] = {io.c0[q], io.c1[q], io.c2[q]};
    float accum = 0.0f;
    // (the register list: K = 512 x 8 lobes 10.81 -> 10.61 ms per 2^18 queries)
    const int lastIdx = build_candidates_reg<LCAP>(gp, Kp, K, c, cw, ck, 64, tid, gc.norm3, cap, accum);
    if (lastIdx == kNoMass) {   // every marginal weight zero: BSDF only, as the full-K path finds
        product_invalid<PDF_ONLY>(io, pio, q);
        return;
    }
    if (lastIdx < 0 || routed_to_wave(lastIdx, pio, bt, q, gc)) {
        fb_list[atomicAdd(fb_count, 1)] = (int32_t)q;
        return;
    }
    product_tail<PDF_ONLY>(gp, Kp, condCov, c, lastIdx, accum, CandSlots{cw, ck, 64, tid}, io, pio, bt, q, gc, t);
}

// ---------------------------------------------------------------------------
// Product path, full-K queries one per wave (the section above for the
// selection; the product terms follow finish_product / for_each_pair).
//
// Per query, before the pair passes (lanes in parallel): the conditional
// mean direction of every kept slot with nonzero weight (cond_mean_dir_x) and
// the world-frame lobes of the query's material (bsdf_world) -- the values
// for_each_pair forms inside its loops, evaluated once instead of per pair.
__device__ __forceinline__ void wave_prepare_product(const float* gp, int Kp, const float c[3], int lastIdx,
                                                     const WaveLds& L, const BsdfTab& bt, int b, const float F[9],
                                                     int lane) {
    for (int i = lane; i < lastIdx; i += 64) {
        if (L.fw[i] == 0.0f) continue;
        float e[3];
        cond_mean_dir_x(gp, Kp, slot_comp(L, i), c, e);
        L.se[3 * i] = e[0]; L.se[3 * i + 1] = e[1]; L.se[3 * i + 2] = e[2];
    }
    for (int j = lane; j < bt.M; j += 64) {
        float* lb = L.lobe + 20 * j;
        bsdf_world(F, bt, b, j, lb, lb + 3, lb + 12, lb[16]);
    }
    // the nonzero-weight lobes in order (M <= 64: one lane each): the pair
    // walk skips the others, so it runs over kept x nonzero pairs only (a
    // table padded to a common lobe count costs no chunks)
    {
        const bool nzl = lane < bt.M && bt.w[b * bt.M + lane] != 0.0f;
        const uint64_t m = __builtin_amdgcn_ballot_w64(nzl);
        if (nzl) ((int*)(L.lobe + 20 * bt.M))[__builtin_popcountll(m & ((1ull << lane) - 1ull))] = lane;
    }
    __syncthreads();
}

// Product pair (slot i, lobe j) of for_each_pair: false when the walk skips
// it (zero slot weight, zero lobe weight, opposite hemisphere); else its
// weight wi * wj * nw and product component.
__device__ __forceinline__ bool pair_eval(const float* condCov, const WaveLds& L, int i, int j, float norm2,
                                          float& w, ProdComp& pc, int& k, bool lazy = true) {
    const float wi = L.fw[i];
    if (wi == 0.0f) return false;
    k = slot_comp(L, i);
    const float e[3] = {L.se[3 * i], L.se[3 * i + 1], L.se[3 * i + 2]};
    const float* lb = L.lobe + 20 * j;
    const float wj = lb[16];
    if (wj == 0.0f) return false;
    if (e[0] * lb[0] + e[1] * lb[1] + e[2] * lb[2] < 0.0f) return false;
    float to_i[9], ci[4];
    coordinates_f(e, to_i);
    for (int l = 0; l < 4; ++l) ci[l] = condCov[4 * k + l];
    const float nw = mvtn_multiply(e, to_i, ci, lb, lb + 3, lb + 12, norm2, pc, lazy);
    w = wi * wj * nw;
    return true;
}

// finish_product with the pairs spread over the lanes (64 per chunk, flat
// index f = slot * M + lobe: the reference's walk order).  When the kept x M
// pairs fit L.pcap, pass 1 keeps each pair's {w, mean, Linv, detInv} in the
// workgroup's scratch (written and re-read by the same wave: L2-resident) and
// the CDF walk and the pdf read them; otherwise they are recomputed.
// Returns false when the product is unusable (no pair / zero mass).
// (diagnostic SDMM_PW_STOP = 4 / 1 / 2 / 3: return after the slot weights /
// the preparation / pass 1 / pass 2 -- stage costs by difference; the outputs
// are not the product's)
#ifndef SDMM_PW_STOP
#define SDMM_PW_STOP 0
#endif
template <bool PDF_ONLY>
__device__ bool finish_product_wave(const float* gp, int Kp, const float* condCov, const float c[3], int lastIdx,
                                    const WaveLds& L, const BsdfTab& bt, int b, const float F[9], const float* u,
                                    const float* dir_in, float choice, int lane, GuideConsts gc, QueryOut& o) {
    if (SDMM_PW_STOP == 4) return true;
    wave_prepare_product(gp, Kp, c, lastIdx, L, bt, b, F, lane);
    if (SDMM_PW_STOP == 1) return true;
    WCLK(3);
    // pair f = (kept slot f / M, nonzero lobe nzj[f % M]) -- the reference's
    // walk order with the zero-weight lobes (which it skips) left out
    const int M = __builtin_popcountll(__builtin_amdgcn_ballot_w64(lane < bt.M && bt.w[b * bt.M + lane] != 0.0f));
    const int* nzj = (const int*)(L.lobe + 20 * bt.M);
    const int NP = lastIdx * M;
    const bool keep = NP <= L.pcap;
    // pass 1: the product mass (createCdf(true)'s sum) and the pair count
    float total = 0.0f;
    int P = 0;
    for (int base = 0; base < NP; base += 64) {
        const int f = base + lane;
        float w = 0.0f;
        bool inc = false;
        if (f < NP) {
            ProdComp pc{};
            int k;
            inc = pair_eval(condCov, L, f / M, nzj[f % M], gc.norm2, w, pc, k);
            if (keep) {
                float* r = pc_rec(L, base, lane);
                r[0] = w;
                r[64] = inc ? 1.0f : 0.0f;
                r[2 * 64] = pc.mean[0]; r[3 * 64] = pc.mean[1]; r[4 * 64] = pc.mean[2];
                r[5 * 64] = pc.Linv[0]; r[6 * 64] = pc.Linv[1]; r[7 * 64] = pc.Linv[2]; r[8 * 64] = pc.Linv[3];
                r[9 * 64] = pc.detInv;
            }
        }
        total = seq_sum(total, inc ? w : -0.0f, min(64, NP - base), L.st);
        P += __builtin_popcountll(__builtin_amdgcn_ballot_w64(inc));
    }
    __syncthreads();
    WCLK(4);
    if (SDMM_PW_STOP == 2) return true;
    if (P == 0 || total == 0.0f) return false;
    float dir[3];
    o.comp = kCompPdfValid;
    if (!PDF_ONLY && !(choice <= kProductH)) {
        // pass 2: sampleDiscreteCdf over w / total (lower_bound + tie walk)
        float cdf = 0.0f, prev = 0.0f;
        int p = 0, run_f = -1, sel_f = -1;
        for (int base = 0; base < NP && sel_f < 0; base += 64) {
            const int f = base + lane;
            float x = 0.0f;
            bool inc = false;
            if (f < NP) {
                float w = 0.0f;
                if (keep) {
                    const float* r = pc_rec(L, base, lane);
                    inc = r[64] != 0.0f;
                    w = r[0];
                } else {
                    ProdComp pc{};
                    int k;
                    inc = pair_eval(condCov, L, f / M, nzj[f % M], gc.norm2, w, pc, k);
                }
                if (inc) x = w / total;
            }
            const uint64_t incm = __builtin_amdgcn_ballot_w64(inc);
            const int n = min(64, NP - base);
            stage64(L.st, x, true);   // (broadcast stage, as seq_sum)
            const float4* s4 = (const float4*)L.st;
#pragma unroll 1
            for (int q4 = 0; 4 * q4 < n && sel_f < 0; ++q4) {
                const float4 v = s4[q4];
                const float e4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int l = 4 * q4 + e;
                    if (l >= n) break;
                    if (!((incm >> l) & 1)) continue;
                    cdf += e4[e];
                    if (p == 0 || cdf != prev) run_f = base + l;
                    prev = cdf;
                    ++p;
                    if (cdf >= u[0]) { sel_f = base + l; break; }
                }
            }
        }
        if (sel_f < 0) sel_f = run_f;
        // the selected pair's product component, evaluated in full (uniform)
        ProdComp pcs{};
        int ksel = 0;
        float wsel = 0.0f;
        (void)pair_eval(condCov, L, sel_f / M, nzj[sel_f % M], gc.norm2, wsel, pcs, ksel, false);
        const float radius = sqrtf(-2.0f * log_x(1.0f - u[1]));
        const float theta = (float)(2.0 * kPi * (double)u[2]);
        const float z0 = radius * sin_x(theta), z1 = radius * cos_x(theta);
        const float v0 = pcs.L[0] * z0 + pcs.L[1] * z1;
        const float v1 = pcs.L[2] * z0 + pcs.L[3] * z1;
        float to[9];
        coordinates_f(pcs.mean, to);
        if (!ts_exp_x(to, v0, v1, dir)) dir[0] = dir[1] = dir[2] = 0.0f;
        o.comp = ksel * bt.M + nzj[sel_f % M];
    } else {
        dir[0] = dir_in[0]; dir[1] = dir_in[1]; dir[2] = dir_in[2];
    }
    WCLK(5);
    if (SDMM_PW_STOP == 3) return true;
    // pass 3: the product mixture pdf at dir (a cached chunk's ten fields
    // loaded at once, coalesced; fetching the next chunk's ahead measured no
    // gain and 18 more spilled VGPRs)
    float acc = 0.0f;
    for (int base = 0; base < NP; base += 64) {
        const int f = base + lane;
        float term = -0.0f;
        float r[kPcStride];
        if (keep && f < NP) {
            const float* rr = pc_rec(L, base, lane);
#pragma unroll
            for (int j = 0; j < kPcStride; ++j) r[j] = rr[64 * j];
        }
        if (f < NP) {
            if (keep) {
                if (r[1] != 0.0f) {
                    const float wn = r[0] / total;
                    if (wn != 0.0f) {
                        ProdComp pc{};
                        pc.mean[0] = r[2]; pc.mean[1] = r[3]; pc.mean[2] = r[4];
                        pc.Linv[0] = r[5]; pc.Linv[1] = r[6]; pc.Linv[2] = r[7]; pc.Linv[3] = r[8];
                        pc.detInv = r[9];
                        term = wn * prod_comp_pdf(pc, dir, gc.norm2);
                    }
                }
            } else {
                ProdComp pc{};
                int k;
                float w = 0.0f;
                if (pair_eval(condCov, L, f / M, nzj[f % M], gc.norm2, w, pc, k)) {
                    const float wn = w / total;
                    if (wn != 0.0f) term = wn * prod_comp_pdf(pc, dir, gc.norm2);
                }
            }
        }
        acc = seq_sum(acc, term, min(64, NP - base), L.st);
    }
    WCLK(6);
    o.d[0] = dir[0]; o.d[1] = dir[1]; o.d[2] = dir[2];
    o.pdf = acc;
    return true;
}

// product_tail for one query served by a whole wave; lane 0 writes.
template <bool PDF_ONLY>
__device__ void product_tail_wave(const float* gp, int Kp, const float* condCov, const float c[3], int lastIdx,
                                  float accum, const WaveLds& L, const GuideIO& io, const ProductIO& pio,
                                  const BsdfTab& bt, int64_t q, int lane, GuideConsts gc) {
    int b = pio.material ? pio.material[q] : -1;
    if (b >= bt.B) b = -1;
    const bool mixed = !PDF_ONLY && pio.choice != nullptr;
    const float choice = mixed ? pio.choice[q] : 2.0f;
    const float sum2 = wave_slot_weights(lastIdx, accum, L, lane);
    WCLK(2);
    const bool cvalid = lastIdx > 0 && sum2 != 0.0f;
    QueryOut o{{0.0f, 0.0f, 0.0f}, 0.0f, -1};
    float h = 1.0f;                       // no valid conditional: BSDF only
    float u[3] = {0.0f, 0.0f, 0.0f}, dg[3] = {0.0f, 0.0f, 0.0f};
    if (PDF_ONLY || mixed) { dg[0] = io.e0[q]; dg[1] = io.e1[q]; dg[2] = io.e2[q]; }
    if constexpr (!PDF_ONLY) { u[0] = io.u0[q]; u[1] = io.u1[q]; u[2] = io.u2[q]; }
    if (cvalid) {
        bool used = false;
        if (b >= 0 && bt.M > 0) {
            float F[9];
            for (int i = 0; i < 9; ++i) F[i] = pio.F[i][q];
            used = finish_product_wave<PDF_ONLY>(gp, Kp, condCov, c, lastIdx, L, bt, b, F, u, dg, choice, lane, gc,
                                                 o);
        }
        if (used) {
            h = kProductH;
        } else {
            h = 0.5f;
            // uniform: one query per wave
            if (PDF_ONLY || choice <= 0.5f)
                o = finish_query_wave<true>(gp, Kp, c, u, dg, lastIdx, sum2, L, lane, gc);
            else
                o = finish_query_wave<false>(gp, Kp, c, u, dg, lastIdx, sum2, L, lane, gc);
        }
    }
    if (lane == 0) {
        if constexpr (PDF_ONLY) {
            io.pdf[q] = o.pdf;
        } else {
            io.d0[q] = o.d[0]; io.d1[q] = o.d[1]; io.d2[q] = o.d[2];
            io.pdf[q] = o.pdf;
            io.comp[q] = o.comp;
        }
        if (pio.h) pio.h[q] = h;
    }
}

// The product path's full-K queries (listed by guide_product_cand_kernel):
// one wave per query, grid-stride.
// Waves per SIMD the one-wave product kernels' register budget is sized for.
// Round 5 (A/B: 2: 10.57, 3: 9.93, 4 (spills): 13.4 ms a Kitchen call) kept 3
// with ~65 VGPRs spilled; after round 6's serial-sum and partial-sort changes
// 2 (256 VGPRs, no spill) wins: Kitchen 8.33 -> 7.59 ms a call, K = 512
// Cornell product pass 62.9 -> 60.5 ms (4: 13.7 ms / 92 ms;
// profiles/round6_ab_product_wpe.log).
#ifndef SDMM_PRODUCT_WPE   // (A/B: tools/build_variant.sh)
#define SDMM_PRODUCT_WPE 2
#endif
constexpr int kProductWpe = SDMM_PRODUCT_WPE;
template <bool PDF_ONLY>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kProductWpe)))
guide_product_wave_kernel(const float* __restrict__ gp, int Kp, int K, const float* __restrict__ condCov,
                          GuideIO io, ProductIO pio, BsdfTab bt, GuideConsts gc, float* __restrict__ pscratch,
                          int pcap, const int* __restrict__ fb_count, const int32_t* __restrict__ fb_list) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x;
    const WaveLds L = wave_lds(lds, K, pscratch, pcap, bt.M);
    const int n = *fb_count;
    for (int idx = blockIdx.x; idx < n; idx += gridDim.x) {
        const int64_t q = fb_list[idx];
        const float c[3] = {io.c0[q], io.c1[q], io.c2[q]};
        float accum = 0.0f;
        const int lastIdx = build_full_wave(gp, Kp, K, c, L, lane, gc.norm3, accum);
        product_tail_wave<PDF_ONLY>(gp, Kp, condCov, c, lastIdx, accum, L, io, pio, bt, q, lane, gc);
        __syncthreads();   // the LDS is reused by the next query
    }
}

// ---------------------------------------------------------------------------
// Product sampling over the spatial tree's leaves (sampleSurface with
// sampleProduct for a wavefront of bounces, sdmm_proc.cpp:309-392): per query,
// node = STree.find(c) (:314), that node's mixture (none: BSDF only, h = 1,
// :316-323), then exactly what guide_product_cand_kernel /
// guide_product_wave_kernel do against that one mixture.  cctab[node] is the
// node mixture's conditional covariances (condCov).
template <bool PDF_ONLY, int LCAP>
__device__ __forceinline__ bool serve_product_cand(const float* gp, int Kp, int K, const float* condCov,
                                                   const GuideIO& io, const ProductIO& pio, const BsdfTab& bt,
                                                   int64_t q, const float c[3], float* cw, unsigned short* ck,
                                                   int tid, int cap, GuideConsts gc, int* fb_count,
                                                   int32_t* fb_list, int64_t t) {
    float accum = 0.0f;
    const int lastIdx = build_candidates_reg<LCAP>(gp, Kp, K, c, cw, ck, 64, tid, gc.norm3, cap, accum);
    if (lastIdx == kNoMass) {   // every marginal weight zero: BSDF only, as the full-K path finds
        product_invalid<PDF_ONLY>(io, pio, q);
        return false;
    }
    if (lastIdx < 0 || routed_to_wave(lastIdx, pio, bt, q, gc)) {
        fb_list[atomicAdd(fb_count, 1)] = (int32_t)q;
        return true;
    }
    product_tail<PDF_ONLY>(gp, Kp, condCov, c, lastIdx, accum, CandSlots{cw, ck, 64, tid}, io, pio, bt, q, gc, t);
    return false;
}


// Two waves per SIMD: left free the sampling form took 256 VGPRs + 10 AGPRs,
// ONE wave per SIMD for a latency-bound thread-per-query kernel; bounded to
// 256 registers it spills 11 (32 B of scratch) and the K = 512 product pass
// runs 85.5 -> 71.1 ms (first guided pass 111 -> 95 ms; round 5)
template <bool PDF_ONLY, int LCAP>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
guide_tree_product_cand_kernel(const STNodeDev* __restrict__ nodes, const GuideMix* __restrict__ tab,
                               const float* const* __restrict__ cctab, int64_t nq, GuideIO io, ProductIO pio,
                               BsdfTab bt, GuideConsts gc, int cap, int* __restrict__ fb_count,
                               int32_t* __restrict__ fb_list, const int32_t* __restrict__ perm,
                               int32_t* __restrict__ node_out, const uint32_t* __restrict__ skeys,
                               int mb) {
    __shared__ float cw[LCAP * 64];
    __shared__ unsigned short ck[LCAP * 64];
    const int tid = threadIdx.x;
    const int64_t t = (int64_t)blockIdx.x * 64 + tid;
    if (t >= nq) return;
    const int64_t q = perm ? (int64_t)perm[t] : t;
    const float c[3] = {io.c0[q], io.c1[q], io.c2[q]};
    // leaf-major order: the sorted key holds the node (tree_keys_kernel)
    const int node = skeys ? (int)(skeys[t] >> mb) - 1 : stree_find_point(nodes, c[0], c[1], c[2]);
    if (node_out) node_out[q] = node;
    // one leaf for the whole wave (the Morton-ordered common case): uniform
    // control flow; else one distinct leaf per trip (waterfall)
    const int n0 = __builtin_amdgcn_readfirstlane(node);
    const bool uniform = __builtin_amdgcn_ballot_w64(node != n0) == 0;
    if (uniform) {
        // uniform-leaf wave: the record in SGPRs (scalar record loads)
        const GuideMix mx = uniform_mix((n0 >= 0) ? tab[n0] : GuideMix{nullptr, 0, 0});
        if (mx.K <= 0) {
            product_invalid<PDF_ONLY>(io, pio, q);
        } else {
            serve_product_cand<PDF_ONLY, LCAP>(mx.gp, mx.Kp, mx.K, cctab[n0], io, pio, bt, q, c, cw, ck, tid, cap,
                                               gc, fb_count, fb_list, t);
        }
        return;
    }
    for (;;) {
        const int nw = __builtin_amdgcn_readfirstlane(node);
        if (node != nw) continue;
        const GuideMix mx = (nw >= 0) ? tab[nw] : GuideMix{nullptr, 0, 0};
        if (mx.K <= 0)
            product_invalid<PDF_ONLY>(io, pio, q);
        else
            serve_product_cand<PDF_ONLY, LCAP>(mx.gp, mx.Kp, mx.K, cctab[nw], io, pio, bt, q, c, cw, ck, tid, cap,
                                               gc, fb_count, fb_list, t);
        break;
    }
}

// the tree product path's full-K queries, one wave per query (grid-stride);
// kmax sizes the LDS
template <bool PDF_ONLY>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kProductWpe)))
guide_tree_product_wave_kernel(const STNodeDev* __restrict__ nodes, const GuideMix* __restrict__ tab,
                               const float* const* __restrict__ cctab, int kmax, GuideIO io, ProductIO pio,
                               BsdfTab bt, GuideConsts gc, float* __restrict__ pscratch, int pcap,
                               const int* __restrict__ fb_count, const int32_t* __restrict__ fb_list,
                               const int32_t* __restrict__ node_of) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x;
    const WaveLds L = wave_lds(lds, kmax, pscratch, pcap, bt.M);
    const int n = *fb_count;
#ifdef SDMM_WAVE_CLOCK
    if (lane < 12) g_wclk[lane] = 0;
    if (lane == 0) g_wlast = __builtin_amdgcn_s_memtime();
    __syncthreads();
    unsigned nq = 0, npairs = 0, nkept = 0;
#endif
    for (int idx = blockIdx.x; idx < n; idx += gridDim.x) {
        const int64_t q = fb_list[idx];
        const float c[3] = {io.c0[q], io.c1[q], io.c2[q]};
        // uniform: a listed query has a mixture; node_of: the candidate kernel's find
        const int node = node_of ? node_of[q] : stree_find_point(nodes, c[0], c[1], c[2]);
        const GuideMix mx = uniform_mix(tab[node]);   // (one query per wave: uniform)
        WCLK(0);
        float accum = 0.0f;
        const int lastIdx = build_full_wave(mx.gp, mx.Kp, mx.K, c, L, lane, gc.norm3, accum);
#ifdef SDMM_WAVE_CLOCK
        ++nq;
        nkept += lastIdx;
#endif
        product_tail_wave<PDF_ONLY>(mx.gp, mx.Kp, cctab[node], c, lastIdx, accum, L, io, pio, bt, q, lane, gc);
        __syncthreads();   // the LDS is reused by the next query
        WCLK(7);
    }
#ifdef SDMM_WAVE_CLOCK
    if (lane == 0 && blockIdx.x < 4)
        printf("WCLK blk %d q %u kept %u fetch %llu weights %llu sum2 %llu prep %llu pass1 %llu pass2 %llu pass3 %llu "
               "tail %llu total %llu sort %llu accum %llu\n",
               blockIdx.x, nq, nkept, g_wclk[0], g_wclk[1], g_wclk[2], g_wclk[3], g_wclk[4], g_wclk[5], g_wclk[6],
               g_wclk[7], g_wclk[8], g_wclk[9], g_wclk[10]);
#endif
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

// ---------------------------------------------------------------------------
// Coherent query order.  A wave's 64 queries run the candidate loop and the
// kept-component loops in lockstep, so their cost is that of the union of
// their live components; queries from all over the scene make every
// component live in every wave.  Sorting the batch along a 30-bit Morton
// curve of the condition position c (10 bits per axis of the normalised
// scene box) makes waves spatially coherent: 2.8x fewer cycles at Q = 2^20,
// K = 128 (tools/guide_coherence.py).  Every query is computed exactly as
// before -- only the thread that serves it changes -- and its outputs go to
// its own index.
__device__ __forceinline__ uint32_t spread3(uint32_t v) {   // 10 bits -> every third bit
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}
// bits per axis (<= 10): the key has 3 * bits bits
__device__ __forceinline__ uint32_t quantb(float x, int bits) {
    x = fminf(fmaxf(x, 0.0f), 1.0f);                          // NaN -> 0
    const uint32_t m = (1u << bits) - 1u;
    const uint32_t q = (uint32_t)(x * (float)(1u << bits));
    return q > m ? m : q;
}
__global__ void morton_keys_kernel(const float* __restrict__ c0, const float* __restrict__ c1,
                                   const float* __restrict__ c2, int n, int bits, uint32_t* __restrict__ keys,
                                   int32_t* __restrict__ idx) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    keys[q] = spread3(quantb(c0[q], bits)) | (spread3(quantb(c1[q], bits)) << 1) |
              (spread3(quantb(c2[q], bits)) << 2);
    idx[q] = q;
}

// bits per axis of the coherent order's key (round 4: 8 bits, one radix
// pass fewer, measured the same)
static int morton_bits() { return 10; }

size_t guide_sort_temp_bytes(int n) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, n, 0, 32);
    return bytes;
}

// keys/idx: 2 x n each; returns the sorted permutation in idx_out
static hipError_t coherent_order(const float* const c[3], int n, uint32_t* keys_in, uint32_t* keys_out,
                                 int32_t* idx_in, int32_t* idx_out, void* temp, size_t temp_bytes,
                                 hipStream_t st) {
    const int bits = morton_bits();
    hipLaunchKernelGGL(morton_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, c[0], c[1], c[2], n,
                       bits, keys_in, idx_in);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, idx_in, idx_out, n, 0, 3 * bits,
                                              st);
}

// Leaf-major coherent order for the tree wavefronts: key = (node + 1) in the
// high bits, the Morton code of c (mb / 3 bits per axis) in the low ones, so
// a wave's queries share ONE leaf except at the seams between leaves (plain
// Morton runs cross leaf boxes, whose planes sit at sample means, wherever
// the Z-curve does).  The sorted keys then carry every query's node: the
// candidate kernel reads node = (key >> mb) - 1 instead of walking the tree.
// The key is 32 bits: the Morton code at (32 - node bits) / 3 bits per axis
// (round 4: 24 / 28-bit keys over the Morton levels that vary inside a leaf
// measured within noise, K = 16 slower).
__global__ void tree_keys_kernel(const STNodeDev* __restrict__ nodes, const float* __restrict__ c0,
                                 const float* __restrict__ c1, const float* __restrict__ c2, int n, int mb,
                                 uint32_t* __restrict__ keys, int32_t* __restrict__ idx) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const float x = c0[q], y = c1[q], z = c2[q];
    const int node = stree_find_point(nodes, x, y, z);
    const int b = mb / 3;
    const uint32_t m = spread3(quantb(x, b)) | (spread3(quantb(y, b)) << 1) | (spread3(quantb(z, b)) << 2);
    keys[q] = ((uint32_t)(node + 1) << mb) | m;
    idx[q] = q;
}
// node bits for a tree of nn nodes (node + 1 < 2^nb); 0: no leaf-major order
static int leaf_key_bits(int nn) {
    int nb = 1;
    while (nb < 32 && (1ll << nb) <= (long long)nn) ++nb;
    return nb <= 20 ? nb : 0;
}
static hipError_t leaf_order(const STNodeDev* nodes, int nn, const float* const c[3], int n, uint32_t* keys_in,
                             uint32_t* keys_out, int32_t* idx_in, int32_t* idx_out, void* temp, size_t temp_bytes,
                             hipStream_t st, int* mb_out) {
    const int nb = leaf_key_bits(nn);
    const int mb = 32 - nb;
    *mb_out = mb;
    hipLaunchKernelGGL(tree_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, nodes, c[0], c[1], c[2],
                       n, mb, keys_in, idx_in);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, idx_in, idx_out, n, 0, nb + mb,
                                              st);
}
// (round 4: the plain Morton order instead: K = 128 guided pass 11.95
// against 11.37 ms, K = 512 product 88.6 against 85.6)
static bool leaf_order_on() { return true; }

static GuideIO make_io(const float* const c[3], const float* const u[3], const float* const dgiven[3],
                       float* const d[3], float* pdf, int32_t* comp, const uint8_t* pmode = nullptr) {
    // pdf only: dgiven without pmode; mixed: dgiven with pmode (sampling kernels)
    const bool pdf_only = dgiven != nullptr && pmode == nullptr;
    GuideIO io{};
    io.c0 = c[0]; io.c1 = c[1]; io.c2 = c[2];
    if (dgiven) {
        io.e0 = dgiven[0]; io.e1 = dgiven[1]; io.e2 = dgiven[2];
    }
    if (!pdf_only) {
        io.u0 = u[0]; io.u1 = u[1]; io.u2 = u[2];
        io.d0 = d[0]; io.d1 = d[1]; io.d2 = d[2];
        io.comp = comp;
        io.pmode = pmode;
    }
    io.pdf = pdf;
    return io;
}

// The candidate kernels' LDS list is sized by the template capacity LCAP
// (6 B per entry per thread), which sets the workgroups per CU.  A list never
// holds more than K entries, so the launch uses the smallest LCAP >= min(cap,
// K): identical results (no overflow can occur that the larger list would
// avoid), fewer LDS bytes for small mixtures (the tree's K=16 leaves).
template <bool PDF_ONLY>
static hipError_t launch_cand(int cap, dim3 grid, hipStream_t st, const float* gp, int Kp, int K, int64_t nq,
                              const GuideIO& io, GuideConsts gc, int* fb_count, int32_t* fb_list,
                              const int32_t* perm) {
    if (cap <= 16)
        hipLaunchKernelGGL((guide_cand_kernel<PDF_ONLY, 16>), grid, dim3(64), 0, st, gp, Kp, K, nq, io, gc, cap,
                           fb_count, fb_list, perm);
    else if (cap <= 24)
        hipLaunchKernelGGL((guide_cand_kernel<PDF_ONLY, 24>), grid, dim3(64), 0, st, gp, Kp, K, nq, io, gc, cap,
                           fb_count, fb_list, perm);
    else if (cap <= 40)
        hipLaunchKernelGGL((guide_cand_kernel<PDF_ONLY, 40>), grid, dim3(64), 0, st, gp, Kp, K, nq, io, gc, cap,
                           fb_count, fb_list, perm);
    else
        hipLaunchKernelGGL((guide_cand_kernel<PDF_ONLY, kGuideCap>), grid, dim3(64), 0, st, gp, Kp, K, nq, io, gc,
                           cap, fb_count, fb_list, perm);
    return hipGetLastError();
}
template <bool PDF_ONLY>
static hipError_t launch_tree_cand(int cap, dim3 grid, hipStream_t st, const STNodeDev* nd, const GuideMix* tb,
                                   int64_t nq, const GuideIO& io, GuideConsts gc, int* fb_count, int32_t* fb_list,
                                   const int32_t* perm, int32_t* node_out, const uint32_t* skeys, int mb) {
    if (cap <= 16)
        hipLaunchKernelGGL((guide_tree_cand_kernel<PDF_ONLY, 16>), grid, dim3(64), 0, st, nd, tb, nq, io, gc, cap,
                           fb_count, fb_list, perm, node_out, skeys, mb);
    else if (cap <= 24)
        hipLaunchKernelGGL((guide_tree_cand_kernel<PDF_ONLY, 24>), grid, dim3(64), 0, st, nd, tb, nq, io, gc, cap,
                           fb_count, fb_list, perm, node_out, skeys, mb);
    else if (cap <= 40)
        hipLaunchKernelGGL((guide_tree_cand_kernel<PDF_ONLY, 40>), grid, dim3(64), 0, st, nd, tb, nq, io, gc, cap,
                           fb_count, fb_list, perm, node_out, skeys, mb);
    else
        hipLaunchKernelGGL((guide_tree_cand_kernel<PDF_ONLY, kGuideCap>), grid, dim3(64), 0, st, nd, tb, nq, io,
                           gc, cap, fb_count, fb_list, perm, node_out, skeys, mb);
    return hipGetLastError();
}

// Candidate pass over all queries, then the fallback queries (listed by the
// candidate kernel) through the full-K path; both on stream st.
// fb_count: one device int, fb_list: nq device ints (scratch).
hipError_t launch_guide(const float* gp, int Kp, int K, int64_t nq, const float* const c[3],
                        const float* const u[3], const float* const dgiven[3], float* const d[3], float* pdf,
                        int32_t* comp, float norm2, float norm3, int cap, int* fb_count, int32_t* fb_list,
                        int cus, hipStream_t st, const GuideSortScratch* sort, int* fb2) {
    if (nq <= 0) return hipSuccess;
    cap = (cap < 0) ? 0 : (cap > kGuideCap ? kGuideCap : cap);
    if (nq > INT32_MAX) return hipErrorInvalidValue;
    const int T = 64;
    if (K > kWaveKMax) return hipErrorInvalidValue;
    const int Tfb = 64;
    const size_t lds_fb = wave_lds_bytes(K);
    GuideConsts gc{norm2, norm3};
    hipError_t e = hipMemsetAsync(fb_count, 0, sizeof(int), st);
    if (e != hipSuccess) return e;
    const int32_t* perm = nullptr;
    if (sort) {
        e = coherent_order(c, (int)nq, sort->keys[0], sort->keys[1], sort->idx[0], sort->idx[1], sort->temp,
                           sort->temp_bytes, st);
        if (e != hipSuccess) return e;
        perm = sort->idx[1];
    }
    const dim3 grid((unsigned)((nq + T - 1) / T));
    const int fb_blocks = cus * 16;
    const GuideIO io = make_io(c, u, dgiven, d, pdf, comp);
    cap = cap < K ? cap : K;
    e = dgiven ? launch_cand<true>(cap, grid, st, gp, Kp, K, nq, io, gc, fb_count, fb_list, perm)
               : launch_cand<false>(cap, grid, st, gp, Kp, K, nq, io, gc, fb_count, fb_list, perm);
    if (e != hipSuccess) return e;
    if (fb2 && K <= kGroupKMax) {
        // four full-K queries per wave; the NaN ones (if any) then one per wave
        e = hipMemsetAsync(fb2, 0, sizeof(int), st);
        if (e != hipSuccess) return e;
        if (dgiven)
            launch_group_fallback<true, false>(K, fb_blocks, st, gp, Kp, K, nullptr, nullptr, io, gc, fb_count,
                                               fb_list, fb2);
        else
            launch_group_fallback<false, false>(K, fb_blocks, st, gp, Kp, K, nullptr, nullptr, io, gc, fb_count,
                                                fb_list, fb2);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        fb_count = fb2;
        fb_list = fb2 + 1;
    }
    if (dgiven)
        hipLaunchKernelGGL(guide_fallback_kernel<true>, dim3(fb_blocks), dim3(Tfb), lds_fb, st, gp, Kp, K, io, gc,
                           fb_count, fb_list);
    else
        hipLaunchKernelGGL(guide_fallback_kernel<false>, dim3(fb_blocks), dim3(Tfb), lds_fb, st, gp, Kp, K, io,
                           gc, fb_count, fb_list);
    return hipGetLastError();
}

// The tree wavefront: every query against its own node's mixture (tab, one
// GuideMix per tree node; kmax = the largest K in it).  Same two-pass shape
// and the same per-query arithmetic as launch_guide.  sort: always used
// (Morton order keeps a wave inside one leaf) unless null.
hipError_t launch_guide_tree(const void* nodes, const void* tab, int kmax, int64_t nq, const float* const c[3],
                             const float* const u[3], const float* const dgiven[3], float* const d[3],
                             float* pdf, int32_t* comp, int32_t* node_out, float norm2, float norm3, int cap,
                             int* fb_count, int32_t* fb_list, int cus, hipStream_t st,
                             const GuideSortScratch* sort, const uint8_t* pmode, int* fb2, int nn) {
    if (nq <= 0) return hipSuccess;
    cap = (cap < 0) ? 0 : (cap > kGuideCap ? kGuideCap : cap);
    if (nq > INT32_MAX) return hipErrorInvalidValue;
    const int T = 64;
    if (kmax < 1) kmax = 1;
    if (kmax > kWaveKMax) return hipErrorInvalidValue;
    const int Tfb = 64;
    const size_t lds_fb = wave_lds_bytes(kmax);
    GuideConsts gc{norm2, norm3};
    hipError_t e = hipMemsetAsync(fb_count, 0, sizeof(int), st);
    if (e != hipSuccess) return e;
    const STNodeDev* nd = (const STNodeDev*)nodes;
    const int32_t* perm = nullptr;
    const uint32_t* skeys = nullptr;   // leaf-major sorted keys (node in the high bits)
    int mb = 0;
    if (sort) {
        if (leaf_order_on() && leaf_key_bits(nn) > 0) {
            e = leaf_order(nd, nn, c, (int)nq, sort->keys[0], sort->keys[1], sort->idx[0], sort->idx[1], sort->temp,
                           sort->temp_bytes, st, &mb);
            skeys = sort->keys[1];
        } else {
            e = coherent_order(c, (int)nq, sort->keys[0], sort->keys[1], sort->idx[0], sort->idx[1], sort->temp,
                               sort->temp_bytes, st);
        }
        if (e != hipSuccess) return e;
        perm = sort->idx[1];
    }
    const GuideMix* tb = (const GuideMix*)tab;
    const dim3 grid((unsigned)((nq + T - 1) / T));
    const int fb_blocks = cus * 16;
    const GuideIO io = make_io(c, u, dgiven, d, pdf, comp, pmode);
    if (pmode) dgiven = nullptr;   // mixed: the sampling kernels, pdf queries per pmode
    cap = cap < kmax ? cap : kmax;
    // every query's node as the candidate kernel finds it (the caller's
    // node_out, else a sort buffer free once the order is built: the sorted
    // keys with the plain Morton order, the sort's index input with the
    // leaf-major one): the fallback kernels read it instead of walking the tree
    int32_t* const node_of = node_out ? node_out
                                      : (sort ? (skeys ? sort->idx[0] : (int32_t*)sort->keys[1]) : nullptr);
    e = dgiven ? launch_tree_cand<true>(cap, grid, st, nd, tb, nq, io, gc, fb_count, fb_list, perm, node_of, skeys,
                                        mb)
               : launch_tree_cand<false>(cap, grid, st, nd, tb, nq, io, gc, fb_count, fb_list, perm, node_of, skeys,
                                         mb);
    if (e != hipSuccess) return e;
    if (fb2 && kmax <= kGroupKMax) {
        e = hipMemsetAsync(fb2, 0, sizeof(int), st);
        if (e != hipSuccess) return e;
        if (dgiven)
            launch_group_fallback<true, true>(kmax, fb_blocks, st, nullptr, 0, 0, nd, tb, io, gc, fb_count, fb_list,
                                              fb2, node_of);
        else
            launch_group_fallback<false, true>(kmax, fb_blocks, st, nullptr, 0, 0, nd, tb, io, gc, fb_count,
                                               fb_list, fb2, node_of);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        fb_count = fb2;
        fb_list = fb2 + 1;
    }
    if (dgiven)
        hipLaunchKernelGGL(guide_tree_fallback_kernel<true>, dim3(fb_blocks), dim3(Tfb), lds_fb, st, nd, tb, kmax,
                           io, gc, fb_count, fb_list, node_of);
    else
        hipLaunchKernelGGL(guide_tree_fallback_kernel<false>, dim3(fb_blocks), dim3(Tfb), lds_fb, st, nd, tb,
                           kmax, io, gc, fb_count, fb_list, node_of);
    return hipGetLastError();
}

// The product launches' scratch in the handle's grow-only buffer: the thread
// path's pair cache for `threads` query columns (640 B per column), then the
// wave kernel's pair slices (fblocks workgroups, mandatory).  Regrowth (rare:
// grow-only) syncs the stream, frees the old buffer and allocates the larger
// one with hipMalloc -- not from the stream-ordered pool: plugin threads call
// this on many handles at once (sdmm_api.cpp copy_prefix_many).  The cache is optional: when the buffer with
// it cannot be allocated, the slices alone are, and the thread path
// recomputes its pairs (the same values; pc->base = null), so a wavefront too
// large for a cache still runs.  sdmm_destroy (or the tree's destruction)
// releases the buffer.
static hipError_t product_scratch(ProductScratch* ps, int64_t threads, unsigned fblocks, hipStream_t st,
                                  PairCacheDev* pc, float** pairs) {
    if (!ps) return hipErrorInvalidValue;
    const size_t cb = kPairCacheCap > 0 ? sizeof(float) * kPairFields * (size_t)kPairCacheCap * (size_t)threads : 0;
    const size_t ca = (cb + 255) / 256 * 256;
    const size_t slices = sizeof(float) * kPcStride * (size_t)kProductPairCap * fblocks;
    auto grow = [&](size_t need) -> hipError_t {
        if (ps->bytes >= need) return hipSuccess;
        if (ps->base) {
            const hipError_t f = hipStreamSynchronize(st);   // every earlier use is on this stream
            if (f != hipSuccess) return f;
            (void)hipFree(ps->base);
        }
        ps->base = nullptr;
        ps->bytes = 0;
        const size_t grown = need + need / 4;
        hipError_t e = hipMalloc((void**)&ps->base, grown);
        if (e != hipSuccess) {
            (void)hipGetLastError();   // clear the sticky allocation error; try the exact size
            e = hipMalloc((void**)&ps->base, need);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                ps->base = nullptr;
                return e;
            }
            ps->bytes = need;
            return hipSuccess;
        }
        ps->bytes = grown;
        return hipSuccess;
    };
    if (ca > 0 && grow(ca + slices) == hipSuccess) {
        *pc = PairCacheDev{ps->base, threads, kPairCacheCap};
        *pairs = (float*)((char*)ps->base + ca);
        return hipSuccess;
    }
    const hipError_t e = grow(slices);   // no room for the cache: the slices alone
    if (e != hipSuccess) return e;
    *pc = PairCacheDev{nullptr, threads, kPairCacheCap};
    *pairs = ps->base;
    return hipSuccess;
}

// Product sampling (or its pdf, dgiven != null) against one mixture: the
// candidate kernel (thread per query), then its full-K queries one per wave.
hipError_t launch_guide_product(const float* gp, int Kp, int K, const float* condCov, int64_t nq,
                                const float* const c[3], const float* const u[3], const float* const dgiven[3],
                                float* const d[3], float* pdf, int32_t* comp, const int32_t* material,
                                const float* const frame[9], float* h, const float* bw, const float* bmean,
                                const float* bcov, const uint8_t* diffuse, int B, int M, float norm2, float norm3,
                                int cap, int* fb_count, int32_t* fb_list, int cus, hipStream_t st,
                                const GuideSortScratch* sort, ProductScratch* scratch) {
    if (nq <= 0) return hipSuccess;
    if (nq > INT32_MAX) return hipErrorInvalidValue;
    if (K > kWaveKMax || M > 64) return hipErrorInvalidValue;
    const size_t lds = wave_lds_bytes(K, M);
    cap = (cap < 0) ? 0 : (cap > kGuideCap ? kGuideCap : cap);
    cap = cap < K ? cap : K;
    GuideConsts gc{norm2, norm3};
    gc.route_pairs = product_route_pairs();
    const GuideIO io = make_io(c, u, dgiven, d, pdf, comp);
    ProductIO pio{};
    pio.material = material;
    for (int i = 0; i < 9; ++i) pio.F[i] = frame[i];
    pio.h = h;
    const BsdfTab bt{bw, bmean, bcov, B, M, diffuse};
    hipError_t e = hipMemsetAsync(fb_count, 0, sizeof(int), st);
    if (e != hipSuccess) return e;
    const int32_t* perm = nullptr;
    if (sort) {
        e = coherent_order(c, (int)nq, sort->keys[0], sort->keys[1], sort->idx[0], sort->idx[1], sort->temp,
                           sort->temp_bytes, st);
        if (e != hipSuccess) return e;
        perm = sort->idx[1];
    }
    const dim3 grid((unsigned)((nq + 63) / 64));
    // the full-K queries' product pairs (up to kProductPairCap per query): one
    // scratch slice per workgroup of the wave kernel
    const unsigned fblocks = (unsigned)(cus * 4 * kProductWpe);
    float* pscratch = nullptr;
    e = product_scratch(scratch, (int64_t)grid.x * 64, fblocks, st, &pio.cache, &pscratch);
    if (e != hipSuccess) return e;
#define SDMM_PRODUCT_CAND(P, L)                                                                           \
    hipLaunchKernelGGL((guide_product_cand_kernel<P, L>), grid, dim3(64), 0, st, gp, Kp, K, condCov, nq, io, pio, \
                       bt, gc, cap, fb_count, fb_list, perm)
    if (dgiven) {
        if (cap <= 16) SDMM_PRODUCT_CAND(true, 16);
        else if (cap <= 24) SDMM_PRODUCT_CAND(true, 24);
        else if (cap <= 40) SDMM_PRODUCT_CAND(true, 40);
        else SDMM_PRODUCT_CAND(true, kGuideCap);
    } else {
        if (cap <= 16) SDMM_PRODUCT_CAND(false, 16);
        else if (cap <= 24) SDMM_PRODUCT_CAND(false, 24);
        else if (cap <= 40) SDMM_PRODUCT_CAND(false, 40);
        else SDMM_PRODUCT_CAND(false, kGuideCap);
    }
#undef SDMM_PRODUCT_CAND
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (dgiven)
        hipLaunchKernelGGL(guide_product_wave_kernel<true>, dim3(fblocks), dim3(64), lds, st, gp, Kp, K, condCov, io,
                           pio, bt, gc, pscratch, kProductPairCap, fb_count, fb_list);
    else
        hipLaunchKernelGGL(guide_product_wave_kernel<false>, dim3(fblocks), dim3(64), lds, st, gp, Kp, K, condCov,
                           io, pio, bt, gc, pscratch, kProductPairCap, fb_count, fb_list);
    return hipGetLastError();
}

// The product wavefront over the tree (tab / cctab per node, kmax the largest
// K): candidate pass, then the full-K queries one per wave.  Modes: sampling
// (dgiven null), pdf only (dgiven, no choice), mixed (dgiven + choice: a pdf
// query where choice <= the query's h).
hipError_t launch_guide_product_tree(const void* nodes, const void* tab, const void* cctab, int kmax, int64_t nq,
                                     const float* const c[3], const float* const u[3], const float* choice,
                                     const float* const dgiven[3], float* const d[3], float* pdf, int32_t* comp,
                                     int32_t* node_out, const int32_t* material, const float* const frame[9],
                                     float* h, const float* bw, const float* bmean, const float* bcov,
                                     const uint8_t* diffuse, int B, int M, float norm2, float norm3, int cap,
                                     int* fb_count, int32_t* fb_list, int cus, hipStream_t st,
                                     const GuideSortScratch* sort, ProductScratch* scratch, int nn) {
    if (nq <= 0) return hipSuccess;
    if (nq > INT32_MAX) return hipErrorInvalidValue;
    if (kmax < 1) kmax = 1;
    if (kmax > kWaveKMax || M > 64) return hipErrorInvalidValue;
    const size_t lds = wave_lds_bytes(kmax, M);
    cap = (cap < 0) ? 0 : (cap > kGuideCap ? kGuideCap : cap);
    cap = cap < kmax ? cap : kmax;
    GuideConsts gc{norm2, norm3};
    gc.route_pairs = product_route_pairs();
    const bool pdf_only = dgiven != nullptr && choice == nullptr;
    // mixed: the sampling kernels also read the given directions (io.e);
    // the per-query mode comes from pio.choice, not io.pmode
    GuideIO iox{};
    iox.c0 = c[0]; iox.c1 = c[1]; iox.c2 = c[2];
    if (dgiven) { iox.e0 = dgiven[0]; iox.e1 = dgiven[1]; iox.e2 = dgiven[2]; }
    if (!pdf_only) {
        iox.u0 = u[0]; iox.u1 = u[1]; iox.u2 = u[2];
        iox.d0 = d[0]; iox.d1 = d[1]; iox.d2 = d[2];
        iox.comp = comp;
    }
    iox.pdf = pdf;
    ProductIO pio{};
    pio.material = material;
    for (int i = 0; i < 9; ++i) pio.F[i] = frame[i];
    pio.h = h;
    pio.choice = choice;
    const BsdfTab bt{bw, bmean, bcov, B, M, diffuse};
    hipError_t e = hipMemsetAsync(fb_count, 0, sizeof(int), st);
    if (e != hipSuccess) return e;
    const STNodeDev* nd = (const STNodeDev*)nodes;
    const int32_t* perm = nullptr;
    const uint32_t* skeys = nullptr;   // leaf-major sorted keys (see launch_guide_tree)
    int mb = 0;
    if (sort) {
        if (leaf_order_on() && leaf_key_bits(nn) > 0) {
            e = leaf_order(nd, nn, c, (int)nq, sort->keys[0], sort->keys[1], sort->idx[0], sort->idx[1], sort->temp,
                           sort->temp_bytes, st, &mb);
            skeys = sort->keys[1];
        } else {
            e = coherent_order(c, (int)nq, sort->keys[0], sort->keys[1], sort->idx[0], sort->idx[1], sort->temp,
                               sort->temp_bytes, st);
        }
        if (e != hipSuccess) return e;
        perm = sort->idx[1];
    }
    const GuideMix* tb = (const GuideMix*)tab;
    const float* const* cc = (const float* const*)cctab;
    const dim3 grid((unsigned)((nq + 63) / 64));
    const unsigned fblocks = (unsigned)(cus * 4 * kProductWpe);
    float* pscratch = nullptr;
    e = product_scratch(scratch, (int64_t)grid.x * 64, fblocks, st, &pio.cache, &pscratch);
    if (e != hipSuccess) return e;
    // every query's node from the candidate kernel (see launch_guide_tree)
    int32_t* const node_of = node_out ? node_out
                                      : (sort ? (skeys ? sort->idx[0] : (int32_t*)sort->keys[1]) : nullptr);
#define SDMM_TREE_PRODUCT_CAND(P, L)                                                                         \
    hipLaunchKernelGGL((guide_tree_product_cand_kernel<P, L>), grid, dim3(64), 0, st, nd, tb, cc, nq, iox, pio, \
                       bt, gc, cap, fb_count, fb_list, perm, node_of, skeys, mb)
    if (pdf_only) {
        if (cap <= 16) SDMM_TREE_PRODUCT_CAND(true, 16);
        else if (cap <= 24) SDMM_TREE_PRODUCT_CAND(true, 24);
        else if (cap <= 40) SDMM_TREE_PRODUCT_CAND(true, 40);
        else SDMM_TREE_PRODUCT_CAND(true, kGuideCap);
    } else {
        if (cap <= 16) SDMM_TREE_PRODUCT_CAND(false, 16);
        else if (cap <= 24) SDMM_TREE_PRODUCT_CAND(false, 24);
        else if (cap <= 40) SDMM_TREE_PRODUCT_CAND(false, 40);
        else SDMM_TREE_PRODUCT_CAND(false, kGuideCap);
    }
#undef SDMM_TREE_PRODUCT_CAND
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (pdf_only)
        hipLaunchKernelGGL(guide_tree_product_wave_kernel<true>, dim3(fblocks), dim3(64), lds, st, nd, tb, cc, kmax,
                           iox, pio, bt, gc, pscratch, kProductPairCap, fb_count, fb_list, node_of);
    else
        hipLaunchKernelGGL(guide_tree_product_wave_kernel<false>, dim3(fblocks), dim3(64), lds, st, nd, tb, cc,
                           kmax, iox, pio, bt, gc, pscratch, kProductPairCap, fb_count, fb_list, node_of);
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
