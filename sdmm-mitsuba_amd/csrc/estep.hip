// estep.hip -- E-step of the stepwise tangent-space EM on gfx950.
//
// Replaces the N x K hot loop of jmm::StepwiseTangentEM::calculateStats
// (mitsuba/src/integrators/dmm/jmm/opt/stepwise_tangent.h:270-353) and
// MixtureModel::posteriorAndLog (mixture_model.h:146-192) with
// MultivariateTangentNormal::pdfAndLog / TangentSpace::log
// (multivariate_tangent_normal.h:146-177, :350-365).
//
// Work mapping (MI355X-first, not the reference's sample-outer loop):
//   * a group of LPS lanes owns ALL K components: lane j holds components
//     j*CPL .. j*CPL+CPL-1 (CPL even) with their 29 parameters in VGPRs for
//     the whole kernel (loaded once, coalesced, from the SoA record
//     ep[f*Kp + k]);
//   * a lane evaluates its components two at a time with packed fp32
//     (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 on float2), halving the
//     VALU issue of the pair math; the sample operands are SGPR broadcasts;
//   * samples are staged in blocks of 64 (one coalesced vector load per plane,
//     a block ahead of use) and broadcast to the lanes per sample (with
//     LPS == 64 by v_readlane into SGPRs: the pair math reads them as scalar
//     operands);
//   * the posterior normaliser sum_k pi_k pdf_k is a DPP row reduction plus
//     v_readlane across rows (group_sum), one per sample;
//   * STATS: each lane accumulates the 21 sufficient statistics of its own
//     components in registers over the whole chunk (no cross-lane traffic in
//     the loop), then the workgroup folds its waves through LDS in a fixed
//     order and writes one fp32 partial row; reduce_partials sums rows in fp64.
//   * RESP: the normalised responsibilities are stored row-major [N][K]; a
//     group writes one contiguous K*4-byte row per sample (CPL*4 B per lane,
//     non-temporal vector stores).
#include "sdmm_device.h"

#include <cstdlib>

namespace sdmm {

// log2(NORMALIZATION) of mvtn.h:351-352, NORMALIZATION = (float)pow(0.39894228f, 5)
constexpr float kLog2Norm5 = -6.628740082514092f;

// ---- float / float2 arithmetic -------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef f2 V;   // two components per packed operation

__device__ __forceinline__ V sp(float x) { return (V)(x); }
__device__ __forceinline__ V vfma(V a, V b, V c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ V vrsq(V x) { return V{__builtin_amdgcn_rsqf(x.x), __builtin_amdgcn_rsqf(x.y)}; }
__device__ __forceinline__ V vexp2(V x) { return V{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)}; }
__device__ __forceinline__ V vabs(V x) { return __builtin_elementwise_abs(x); }

// theta / sin(theta) for cos(theta) = c in [-1, 1], with the reference's quirk
// `(sinAngle < 1e-3) ? 1 : angle / sinAngle` (mvtn.h:163-164).
//
// The reference computes acos and sqrt separately (~40 VALU ops with the
// libm-grade acosf and the IEEE sqrt expansion).  For c >= 0, with
// u = (1-c)/2, theta/sin(theta) = asin(sqrt u) / (sqrt u sqrt(1-u)) =: h(u) is
// analytic on [0, 1/2] and is a degree-9 polynomial here (8.5e-8 rel.,
// tools/fit_angle_over_sin.py).  For c < 0, theta = pi - theta' with
// theta' = acos|c| gives pi / sin(theta) - h(u).  Overall <= 2.9e-7 relative
// against float64; the reference's own fp32 acos/sqrt form is 1.8e-7 from it.
// Cost: 9 FMA + one v_rsq per component.
__device__ __forceinline__ V angle_over_sin(V c) {
    const V u = vfma(sp(-0.5f), vabs(c), sp(0.5f));
    V h = sp(5.659248352050781f);
    h = vfma(h, u, sp(-8.219043731689453f));
    h = vfma(h, u, sp(6.410147190093994f));
    h = vfma(h, u, sp(-2.090447187423706f));
    h = vfma(h, u, sp(0.9454659819602966f));
    h = vfma(h, u, sp(0.32539111375808716f));
    h = vfma(h, u, sp(0.46356001496315f));
    h = vfma(h, u, sp(0.533078670501709f));
    h = vfma(h, u, sp(0.666670560836792f));
    h = vfma(h, u, sp(1.0f));
    const V s2 = vfma(-c, c, sp(1.0f));
    const V fneg = vfma(sp(3.14159265358979f), vrsq(s2), -h);
    const V f = (c < sp(0.0f)) ? fneg : h;
    return (s2 < sp(1e-6f)) ? sp(1.0f) : f;
}

// ---- cancellation-free 1 + cos(theta) (the statistics kernels) -----------
// Near a component's antipode (c -> -1) theta/sin(theta) ~ pi / sqrt(1 - c^2)
// amplifies the rounding of c: fl(R2.d) + 1 carries an absolute error ~2^-24,
// a relative error 2^-24 / (1 + c) of 1 + c.  Rounding R2.d to fp32 alone puts
// the K = 128 EM parameters ~2e-4 from the exact evaluation of the same float
// parameters, twice the north-star 1e-4.  The statistics kernels
// therefore form delta = 1 + c without the cancellation:
//   n.d = (|n + d|^2 - |n|^2 - |d|^2) / 2   (n = R2, the mean direction)
//   1 + n.d = |n + d|^2 / 2 + (1 - |n|^2) / 2 + (1 - |d|^2) / 2,
// where n_i + d_i is exact near the antipode (Sterbenz) and the two defect
// halves are fp64-rounded constants (EP_CN per component, half_defect per
// sample): delta carries a few ulps of RELATIVE error everywhere.  The
// responsibility kernels (the metric) keep fl(R2.d), within their bound.
__device__ __forceinline__ float half_defect(float d0, float d1, float d2) {
    const double n2 = (double)d0 * (double)d0 + (double)d1 * (double)d1 + (double)d2 * (double)d2;
    return (float)(0.5 * (1.0 - n2));
}
__device__ __forceinline__ V one_plus_c(const V* __restrict__ P, float d0, float d1, float d2, float cd) {
    const V e0 = P[EP_R20] + d0, e1 = P[EP_R21] + d1, e2 = P[EP_R22] + d2;
    return vfma(sp(0.5f), vfma(e2, e2, vfma(e1, e1, e0 * e0)), P[EP_CN] + cd);
}
// u = (1 - |c|)/2 = min(delta, 2 - delta)/2 and s^2 = 1 - c^2 = delta (2 - delta)
__device__ __forceinline__ V half_gap(V dl, V om) { return sp(0.5f) * V{fminf(dl.x, om.x), fminf(dl.y, om.y)}; }

// angle_over_sin (degree-9 polynomial, quirks included) from delta = 1 + c
__device__ __forceinline__ V angle_over_sin_d(V dl) {
    const V om = sp(2.0f) - dl;
    const V u = half_gap(dl, om);
    V h = sp(5.659248352050781f);
    h = vfma(h, u, sp(-8.219043731689453f));
    h = vfma(h, u, sp(6.410147190093994f));
    h = vfma(h, u, sp(-2.090447187423706f));
    h = vfma(h, u, sp(0.9454659819602966f));
    h = vfma(h, u, sp(0.32539111375808716f));
    h = vfma(h, u, sp(0.46356001496315f));
    h = vfma(h, u, sp(0.533078670501709f));
    h = vfma(h, u, sp(0.666670560836792f));
    h = vfma(h, u, sp(1.0f));
    const V s2 = dl * om;
    const V fneg = vfma(sp(3.14159265358979f), vrsq(s2), -h);
    const V f = (dl < sp(1.0f)) ? fneg : h;     // c < 0
    return (s2 < sp(1e-6f)) ? sp(1.0f) : f;
}

// pair_pdf<true> with delta: pi_k pdf_k and the directional tangent (t0, t1);
// dfail = 0 (the log map fails at c <= -1, i.e. delta <= 0) or +inf (d == 0).
__device__ __forceinline__ V pair_pdf_stats(const V* __restrict__ P, float p0, float p1, float p2, float d0,
                                            float d1, float d2, float cd, float dfail, V& t0, V& t1) {
    const V tp0 = p0 - P[EP_MU0], tp1 = p1 - P[EP_MU1], tp2 = p2 - P[EP_MU2];
    const V dl = one_plus_c(P, d0, d1, d2, cd);
    const V a = angle_over_sin_d(dl);
    const V u0 = P[EP_L00] * tp0;
    const V u1 = vfma(P[EP_L11], tp1, P[EP_L10] * tp0);
    const V u2 = vfma(P[EP_L22], tp2, vfma(P[EP_L21], tp1, P[EP_L20] * tp0));
    const V s3 = vfma(P[EP_L32], tp2, vfma(P[EP_L31], tp1, P[EP_L30] * tp0));
    const V s4 = vfma(P[EP_L42], tp2, vfma(P[EP_L41], tp1, P[EP_L40] * tp0));
    const V r0 = vfma(P[EP_R02], sp(d2), vfma(P[EP_R01], sp(d1), P[EP_R00] * d0));
    const V r1 = vfma(P[EP_R12], sp(d2), vfma(P[EP_R11], sp(d1), P[EP_R10] * d0));
    const V ta = r0 * a, tb = r1 * a;
    const V u3 = vfma(P[EP_L33], ta, s3);
    const V u4 = vfma(P[EP_L44], tb, vfma(P[EP_L43], ta, s4));
    const auto ok = dl > sp(dfail);
    t0 = ok ? ta : sp(0.0f);
    t1 = ok ? tb : sp(0.0f);
    const V q = vfma(u4, u4, vfma(u3, u3, vfma(u2, u2, vfma(u1, u1, u0 * u0))));
    const V e = vexp2(vfma(q, sp(-0.72134752044448170368f), sp(kLog2Norm5)));
    const V pdf = e * (P[EP_DIPI] * a);
    return ok ? pdf : sp(0.0f);
}

// pi_k * pdf_k(x) (unnormalised posterior) of two components and the
// directional tangent of the sample in their frames.  p: sample position,
// d: sample direction.  cfail: -1 for a valid sample, +inf when d == 0
// (log map fails for d == 0 or c <= -1, mvtn.h:152-159: pdf = 0).
// q = |L^-1 t|^2 with t = (p - mu, a R0.d, a R1.d), a = theta/sin(theta);
// pdf = NORM5 exp(-q/2) * detInv * a (mvtn.h:350-365), times pi_k.
template <bool WANT_T>
__device__ __forceinline__ V pair_pdf(const V* __restrict__ P, float p0, float p1, float p2,
                                      float d0, float d1, float d2, float cfail, V& t0, V& t1) {
    const V tp0 = p0 - P[EP_MU0], tp1 = p1 - P[EP_MU1], tp2 = p2 - P[EP_MU2];
    const V c = vfma(P[EP_R22], sp(d2), vfma(P[EP_R21], sp(d1), P[EP_R20] * d0));
    const V a = angle_over_sin(__builtin_elementwise_min(c, sp(1.0f)));
    const V u0 = P[EP_L00] * tp0;
    const V u1 = vfma(P[EP_L11], tp1, P[EP_L10] * tp0);
    const V u2 = vfma(P[EP_L22], tp2, vfma(P[EP_L21], tp1, P[EP_L20] * tp0));
    const V s3 = vfma(P[EP_L32], tp2, vfma(P[EP_L31], tp1, P[EP_L30] * tp0));
    const V s4 = vfma(P[EP_L42], tp2, vfma(P[EP_L41], tp1, P[EP_L40] * tp0));
    V u3, u4;
    if constexpr (WANT_T) {
        // the statistics need the tangent vector itself
        const V r0 = vfma(P[EP_R02], sp(d2), vfma(P[EP_R01], sp(d1), P[EP_R00] * d0));
        const V r1 = vfma(P[EP_R12], sp(d2), vfma(P[EP_R11], sp(d1), P[EP_R10] * d0));
        const V ta = r0 * a, tb = r1 * a;
        u3 = vfma(P[EP_L33], ta, s3);
        u4 = vfma(P[EP_L44], tb, vfma(P[EP_L43], ta, s4));
        const auto okt = c > sp(cfail);
        t0 = okt ? ta : sp(0.0f);
        t1 = okt ? tb : sp(0.0f);
    } else {
        // folded: L33 a R0.d = a (A.d), L43 a R0.d + L44 a R1.d = a (B.d)
        const V ad = vfma(P[EP_A2], sp(d2), vfma(P[EP_A1], sp(d1), P[EP_A0] * d0));
        const V bd = vfma(P[EP_B2], sp(d2), vfma(P[EP_B1], sp(d1), P[EP_B0] * d0));
        u3 = vfma(a, ad, s3);
        u4 = vfma(a, bd, s4);
    }
    const V q = vfma(u4, u4, vfma(u3, u3, vfma(u2, u2, vfma(u1, u1, u0 * u0))));
    // NORM5 * exp(-q/2) as one v_exp_f32: 2^(q * -log2(e)/2 + log2(NORM5))
    const V e = vexp2(vfma(q, sp(-0.72134752044448170368f), sp(kLog2Norm5)));
    const V pdf = e * (P[EP_DIPI] * a);   // * detInv * jacobian * pi_k (mvtn.h:361, mixture_model.h:164)
    return (c > sp(cfail)) ? pdf : sp(0.0f);
}

struct SampleVals {
    float x0, x1, x2, x3, x4, x5, w, h;
    float cd;   // half_defect of the direction (statistics kernels)
    bool diffuse;
    // c > cfail selects valid log maps; d == 0 fails for every component
    __device__ float cfail() const {
        return (x3 == 0.0f && x4 == 0.0f && x5 == 0.0f) ? __builtin_inff() : -1.0f;
    }
    // the same on delta = 1 + c
    __device__ float dfail() const { return (x3 == 0.0f && x4 == 0.0f && x5 == 0.0f) ? __builtin_inff() : 0.0f; }
};

// Sample staging.  The wave walks its chunk in blocks of 64 consecutive
// samples: lane j loads sample base + j of every plane with one coalesced
// vector load (256 B per plane), one block ahead of use, and the per-sample
// values are broadcast from the block registers (v_readlane into SGPRs for
// LPS == 64, ds_bpermute for smaller groups).  Scalar (SMEM) loads per sample
// left the waves parked on HBM latency every 16 samples (one 64-B scalar line).
struct SampleBlock {
    float x0, x1, x2, x3, x4, x5, w, h;
    int diff;
    float cd;   // half_defect of this lane's sample (set when consumed, statistics kernels)
};

__device__ __forceinline__ SampleBlock load_block(const SamplesDev& s, int64_t base, int64_t s1, int lane) {
    const int64_t i = (base + lane < s1) ? base + lane : s1 - 1;
    SampleBlock b;
    b.x0 = __builtin_nontemporal_load(s.x[0] + i);
    b.x1 = __builtin_nontemporal_load(s.x[1] + i);
    b.x2 = __builtin_nontemporal_load(s.x[2] + i);
    b.x3 = __builtin_nontemporal_load(s.x[3] + i);
    b.x4 = __builtin_nontemporal_load(s.x[4] + i);
    b.x5 = __builtin_nontemporal_load(s.x[5] + i);
    b.w = __builtin_nontemporal_load(s.w + i);
    // optional planes: always issue the load (from a valid plane when absent)
    // so the number of loads in flight is static and the compiler's vmcnt
    // waits before each block stay partial
    const float* hp = s.hpdf ? s.hpdf : s.x[0];
    const uint8_t* dp = s.isDiffuse ? s.isDiffuse : (const uint8_t*)s.x[0];
    // (raw values: take_sample applies "absent -> 0" after the broadcast, so
    // nothing consumes the loaded registers before the block is used)
    b.h = __builtin_nontemporal_load(hp + i);
    // the flag byte travels inside its aligned dword (a u8 load's zero
    // extension would be re-applied right after the load, forcing the wait);
    // the dword never leaves the 4-byte word that holds byte i
    b.diff = *(const __attribute__((address_space(1))) int*)((uintptr_t)(dp + i) & ~(uintptr_t)3);
    return b;
}

template <int LPS>
__device__ __forceinline__ float bcast(float v, int src) {
    if constexpr (LPS == 64)
        return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
    else
        return __shfl(v, src);
}

// sample t + g of the block (t: wave-uniform offset, g: this lane's group)
template <int LPS, bool WANT_CD = false>
__device__ __forceinline__ SampleVals take_sample(const SampleBlock& b, int t, int g, bool has_h,
                                                  bool has_d, uintptr_t dpos) {
    const int src = (LPS == 64) ? t : t + g;
    SampleVals v;
    v.x0 = bcast<LPS>(b.x0, src); v.x1 = bcast<LPS>(b.x1, src); v.x2 = bcast<LPS>(b.x2, src);
    v.x3 = bcast<LPS>(b.x3, src); v.x4 = bcast<LPS>(b.x4, src); v.x5 = bcast<LPS>(b.x5, src);
    v.w = bcast<LPS>(b.w, src);
    v.cd = WANT_CD ? bcast<LPS>(b.cd, src) : 0.0f;
    v.h = has_h ? bcast<LPS>(b.h, src) : 0.0f;
    int word;
    if constexpr (LPS == 64)
        word = __builtin_amdgcn_readlane(b.diff, src);
    else
        word = __shfl(b.diff, src);
    v.diffuse = has_d && ((word >> (8 * (int)(dpos & 3))) & 0xff) != 0;
    return v;
}

// Walk samples [s0, s1) of this wave: body(sample, index, in_range) for each
// group's sample.  Two block buffers, each reloaded right after the block it
// holds has been consumed, so the loads of block b+1 fly during block b and
// no register copy (which would force an early vmcnt wait) is needed.
template <int LPS, bool WANT_CD, class F>
__device__ __forceinline__ void run_block(SampleBlock b, int64_t blk, int64_t s1, int g,
                                          const SamplesDev& s, F& body) {
    constexpr int SPW = 64 / LPS;
    const int cnt = (s1 - blk < 64) ? (int)(s1 - blk) : 64;
    const bool has_h = s.hpdf != nullptr, has_d = s.isDiffuse != nullptr;
    if constexpr (WANT_CD) b.cd = half_defect(b.x3, b.x4, b.x5);   // once per sample (its own lane)
    for (int t = 0; t < cnt; t += SPW) {
        // block lane t+g held sample blk+t+g (clamped to s1-1 past the end)
        int64_t si = blk + t + g;
        si = (si < s1) ? si : s1 - 1;
        const SampleVals sv = take_sample<LPS, WANT_CD>(b, t, g, has_h, has_d, (uintptr_t)(s.isDiffuse + si));
        body(sv, blk + t + g, t + g < cnt);
    }
}

template <int LPS, bool WANT_CD = false, class F>
__device__ __forceinline__ void walk_samples(const SamplesDev& s, int64_t s0, int64_t s1, int lane, int g,
                                             F&& body) {
    if (s0 >= s1) return;
    SampleBlock A = load_block(s, s0, s1, lane);
    for (int64_t blk = s0; blk < s1; blk += 128) {
        const SampleBlock B = load_block(s, blk + 64, s1, lane);   // clamped past the end
        run_block<LPS, WANT_CD>(A, blk, s1, g, s, body);
        A = load_block(s, blk + 128, s1, lane);
        if (blk + 64 < s1) run_block<LPS, WANT_CD>(B, blk + 64, s1, g, s, body);
    }
}

// Posterior normalisation of one sample (mixture_model.h:170-191):
// S' = (1-h) S + h hpdf for diffuse samples, gamma_k = q_k / S' (x (1-h)),
// gamma_h = h hpdf / S'; everything zero when 1/S' is not finite.
struct Norm {
    float gsc;     // gamma_k = q_k * gsc
    float hpost;   // gamma_h
    bool fin;      // 1/S' finite
};
template <int LPS>
__device__ __forceinline__ Norm normalise(float local, const SampleVals& sv) {
    const float S = group_sum<LPS>(local);
    const float S2 = sv.diffuse ? fmaf(1.0f - kHeuristicWeight, S, kHeuristicWeight * sv.h) : S;
    const float inv = __builtin_amdgcn_rcpf(S2);
    Norm n;
    n.fin = __builtin_isfinite(inv);
    n.gsc = n.fin ? (sv.diffuse ? inv * (1.0f - kHeuristicWeight) : inv) : 0.0f;
    n.hpost = (n.fin && sv.diffuse) ? kHeuristicWeight * sv.h * inv : 0.0f;
    return n;
}

template <int CPL>
__device__ __forceinline__ void load_params(const float* __restrict__ ep, int Kp, int kbase,
                                            V (&P)[CPL / 2][EP_FIELDS]) {
#pragma unroll
    for (int c = 0; c < CPL / 2; ++c)
#pragma unroll
        for (int f = 0; f < EP_FIELDS; ++f) P[c][f] = *(const V*)(ep + f * Kp + kbase + 2 * c);
}

// ---------------------------------------------------------------------------
// Responsibility E-step: resp[n*K + k] = posterior_k(x_n) exactly as
// posteriorAndLog returns it (zeros when 1/sum is not finite).
template <int CPL, int LPS>
__global__ void __launch_bounds__(256)
estep_resp_kernel(const float* __restrict__ ep, int Kp, int K, SamplesDev s, int64_t n,
                  int64_t chunk, float* __restrict__ resp) {
    static_assert(CPL % 2 == 0, "components are processed in packed pairs");
    constexpr int SPW = 64 / LPS;
    constexpr int NP = CPL / 2;
    const int lane = threadIdx.x & 63;
    const int g = lane / LPS;
    const int j = lane % LPS;
    // wave-uniform in an SGPR so that sample addresses stay scalar
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
    const int64_t s0 = wave * chunk;
    if (s0 >= n) return;
    const int64_t s1 = (s0 + chunk < n) ? s0 + chunk : n;

    const int kbase = j * CPL;
    V P[NP][EP_FIELDS];
    load_params<CPL>(ep, Kp, kbase, P);

    const bool full = ((kbase + CPL) <= K) && (K % CPL == 0);  // aligned vector row store
    walk_samples<LPS>(s, s0, s1, lane, g, [&](const SampleVals& sv, int64_t i, bool in)
                                              __attribute__((always_inline)) {
        const float cf = sv.cfail();
        V q[NP];
        V acc = sp(0.0f);
#pragma unroll
        for (int c = 0; c < NP; ++c) {
            V t0, t1;
            q[c] = pair_pdf<false>(P[c], sv.x0, sv.x1, sv.x2, sv.x3, sv.x4, sv.x5, cf, t0, t1);
            acc += q[c];
        }
        const Norm nm = normalise<LPS>(acc.x + acc.y, sv);
        if (!in) return;
        float* row = resp + i * (int64_t)K + kbase;
        V o[NP];
#pragma unroll
        for (int c = 0; c < NP; ++c) o[c] = nm.fin ? q[c] * nm.gsc : sp(0.0f);
        if (full) {
            if constexpr (NP == 1) {
                __builtin_nontemporal_store(o[0], (V*)row);
            } else {
#pragma unroll
                for (int c = 0; c < NP; c += 2) {
                    const f4 o4 = {o[c].x, o[c].y, o[c + 1].x, o[c + 1].y};
                    __builtin_nontemporal_store(o4, (f4*)(row + 2 * c));
                }
            }
        } else {
#pragma unroll
            for (int c = 0; c < NP; ++c) {
                if (kbase + 2 * c < K) __builtin_nontemporal_store(o[c].x, row + 2 * c);
                if (kbase + 2 * c + 1 < K) __builtin_nontemporal_store(o[c].y, row + 2 * c + 1);
            }
        }
    });
}

// ---------------------------------------------------------------------------
// Tiled responsibility E-step for 64 < K <= 128 (one packed component pair per
// lane, the wave holds all K components).
//
// The per-sample overheads of estep_resp_kernel (sample broadcast, a full
// wave reduction and the normalisation for every sample) are ~30 % of its
// VALU issue.  Here:
//   * the wave stages 64 samples in its own LDS slot (lane = sample, one
//     coalesced load per plane, a block ahead) and every lane reads a sample
//     with two broadcast ds_read_b128 (LDS pipe, no VALU);
//   * samples are taken in tiles of kTile = 16: each lane keeps its 16
//     unnormalised pairs q in registers and the 16 per-lane partial sums are
//     reduced across the wave in ONE transposed butterfly (each step halves the
//     values per lane), ~4 VALU per sample;
//   * the lane that ends up holding sample t's sum normalises it and hands the
//     scale back through LDS (one broadcast read per 4 samples);
//   * the pair math is pair_pdf<false> with a degree-7 angle polynomial, the
//     reference's rare angle cases folded into one select, and d == 0 handled
//     once per sample in the normalisation.
constexpr int kTile = 16;

// theta/sin(theta) of two components, the reference's quirks included
// (mvtn.h:157-164): with s2 = 1 - c^2,
//   s2 >= 1e-6:  h(u) for c >= 0, pi/sqrt(s2) - h(u) for c < 0 (theta = pi -
//                theta'), h a degree-7 fit (5.5e-7 relative on [0, 1/2],
//                tools/fit_angle_over_sin.py);
//   s2 <  1e-6:  1 (sin < 1e-3; also c > 1 by rounding, clamped to 1), or 0
//                when c <= -1 (the log map fails: pdf = 0).
// The last case is clamp(2^30 (c + 1)) -- one packed FMA with the clamp bit.
__device__ __forceinline__ V angle_over_sin_fast(V c) {
    const V s2 = vfma(-c, c, sp(1.0f));
    const V u = V{fmaf(-0.5f, fabsf(c.x), 0.5f), fmaf(-0.5f, fabsf(c.y), 0.5f)};
    V h = sp(3.3755881786346436f);
    h = vfma(h, u, sp(-3.17423415184021f));
    h = vfma(h, u, sp(2.1241207122802734f));
    h = vfma(h, u, sp(-0.04515757039189339f));
    h = vfma(h, u, sp(0.5178175568580627f));
    h = vfma(h, u, sp(0.5294308066368103f));
    h = vfma(h, u, sp(0.6667603850364685f));
    h = vfma(h, u, sp(0.9999996423721313f));
    const V fneg = vfma(sp(3.14159265358979f), vrsq(s2), -h);
    V one;
    const V big = sp(1073741824.0f);
    asm("v_pk_fma_f32 %0, %1, %2, %2 clamp" : "=v"(one) : "v"(c), "s"(big));
    const V f = V{c.x < 0.0f ? fneg.x : h.x, c.y < 0.0f ? fneg.y : h.y};
    return V{s2.x < 1e-6f ? one.x : f.x, s2.y < 1e-6f ? one.y : f.y};
}

// pi_k pdf_k of a component pair (the folded form of pair_pdf<false>; d == 0
// is handled per sample by the caller).
__device__ __forceinline__ V pair_q_fast(const V* __restrict__ P, float p0, float p1, float p2, float d0,
                                         float d1, float d2) {
    const V tp0 = p0 - P[EP_MU0], tp1 = p1 - P[EP_MU1], tp2 = p2 - P[EP_MU2];
    const V c = vfma(P[EP_R22], sp(d2), vfma(P[EP_R21], sp(d1), P[EP_R20] * d0));
    const V a = angle_over_sin_fast(c);
    const V u0 = P[EP_L00] * tp0;
    const V u1 = vfma(P[EP_L11], tp1, P[EP_L10] * tp0);
    const V u2 = vfma(P[EP_L22], tp2, vfma(P[EP_L21], tp1, P[EP_L20] * tp0));
    const V s3 = vfma(P[EP_L32], tp2, vfma(P[EP_L31], tp1, P[EP_L30] * tp0));
    const V s4 = vfma(P[EP_L42], tp2, vfma(P[EP_L41], tp1, P[EP_L40] * tp0));
    const V ad = vfma(P[EP_A2], sp(d2), vfma(P[EP_A1], sp(d1), P[EP_A0] * d0));
    const V bd = vfma(P[EP_B2], sp(d2), vfma(P[EP_B1], sp(d1), P[EP_B0] * d0));
    const V u3 = vfma(a, ad, s3);
    const V u4 = vfma(a, bd, s4);
    const V q = vfma(u4, u4, vfma(u3, u3, vfma(u2, u2, vfma(u1, u1, u0 * u0))));
    const V e = vexp2(vfma(q, sp(-0.72134752044448170368f), sp(kLog2Norm5)));
    return e * (P[EP_DIPI] * a);
}

// theta/sin(theta) without the sin < 1e-3 quirks (mvtn.h:157-164): h(u) for
// c >= 0 (h is within 1.7e-7 of the reference's exact 1 when sin < 1e-3), and
// pi/sqrt(1 - c^2) - h(u) for c < 0.  Tiles where some c < -0.9999995 (the
// quirk: J = 1, or a failed log map at c <= -1) are redone with
// angle_over_sin_fast by the caller.  u = (1 - |c|)/2 in plain VOP3 fmas with
// the |.| source modifier (packed ops have no abs).
__device__ __forceinline__ V angle_over_sin_main(V c) {
    const V s2 = vfma(-c, c, sp(1.0f));
    const V u = V{fmaf(-0.5f, fabsf(c.x), 0.5f), fmaf(-0.5f, fabsf(c.y), 0.5f)};
    V h = vfma(sp(3.3755881786346436f), u, sp(-3.17423415184021f));
    h = vfma(h, u, sp(2.1241207122802734f));
    h = vfma(h, u, sp(-0.04515757039189339f));
    h = vfma(h, u, sp(0.5178175568580627f));
    h = vfma(h, u, sp(0.5294308066368103f));
    h = vfma(h, u, sp(0.6667603850364685f));
    h = vfma(h, u, sp(0.9999996423721313f));
    const V fneg = vfma(sp(3.14159265358979f), vrsq(s2), -h);
    return V{c.x < 0.0f ? fneg.x : h.x, c.y < 0.0f ? fneg.y : h.y};
}

// pi_k pdf_k of a component pair for the responsibility tiles: origin-shifted
// spatial rows (p0..p2 are p - kOrigin; EP_NC* fold -L (mu - kOrigin)), folded
// directional rows, and the main-path angle (RARE selects the quirk path).
template <bool RARE>
__device__ __forceinline__ V pair_q_tile(const V* __restrict__ P, float p0, float p1, float p2, float d0,
                                         float d1, float d2, V& c) {
    c = vfma(P[EP_R22], sp(d2), vfma(P[EP_R21], sp(d1), P[EP_R20] * d0));
    const V a = RARE ? angle_over_sin_fast(c) : angle_over_sin_main(c);
    const V u0 = vfma(P[EP_L00], sp(p0), P[EP_NC0]);
    const V u1 = vfma(P[EP_L11], sp(p1), vfma(P[EP_L10], sp(p0), P[EP_NC1]));
    const V u2 = vfma(P[EP_L22], sp(p2), vfma(P[EP_L21], sp(p1), vfma(P[EP_L20], sp(p0), P[EP_NC2])));
    const V s3 = vfma(P[EP_L32], sp(p2), vfma(P[EP_L31], sp(p1), vfma(P[EP_L30], sp(p0), P[EP_NC3])));
    const V s4 = vfma(P[EP_L42], sp(p2), vfma(P[EP_L41], sp(p1), vfma(P[EP_L40], sp(p0), P[EP_NC4])));
    const V ad = vfma(P[EP_A2], sp(d2), vfma(P[EP_A1], sp(d1), P[EP_A0] * d0));
    const V bd = vfma(P[EP_B2], sp(d2), vfma(P[EP_B1], sp(d1), P[EP_B0] * d0));
    const V u3 = vfma(a, ad, s3);
    const V u4 = vfma(a, bd, s4);
    const V q = vfma(u4, u4, vfma(u3, u3, vfma(u2, u2, vfma(u1, u1, u0 * u0))));
    const V e = vexp2(vfma(q, sp(-0.72134752044448170368f), sp(kLog2Norm5)));
    return e * (P[EP_DIPI] * a);
}

// lane ^ 4 within each row of 16 (row_shl:4 on banks 0 and 2, row_shr:4 on
// banks 1 and 3: a disabled bank keeps the `old` operand)
__device__ __forceinline__ float xor4(float x) {
    const int xi = __builtin_bit_cast(int, x);
    int t = __builtin_amdgcn_update_dpp(xi, xi, 0x104, 0xF, 0x5, false);
    t = __builtin_amdgcn_update_dpp(t, xi, 0x114, 0xF, 0xA, false);
    return __builtin_bit_cast(float, t);
}

// Transposed butterfly over the wave: v[16] per lane in, out: the wave-wide
// sum of v[lane & 15] (every row of 16 lanes holds all 16 sums).  Step s
// pairs lane L with L ^ 2^s; L keeps the half of its values whose index bit
// equals its lane bit and receives the partner's copy of the same half.
__device__ __forceinline__ float transpose_sum16(const float (&v)[kTile], int lane) {
    const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4, b3 = lane & 8;
    float a[8], b[4], c[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float keep = b0 ? v[2 * i + 1] : v[2 * i];
        const float send = b0 ? v[2 * i] : v[2 * i + 1];
        a[i] = keep + dpp<0xB1>(send);   // quad_perm [1,0,3,2]: lane ^ 1
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float keep = b1 ? a[2 * i + 1] : a[2 * i];
        const float send = b1 ? a[2 * i] : a[2 * i + 1];
        b[i] = keep + dpp<0x4E>(send);   // quad_perm [2,3,0,1]: lane ^ 2
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const float keep = b2 ? b[2 * i + 1] : b[2 * i];
        const float send = b2 ? b[2 * i] : b[2 * i + 1];
        c[i] = keep + xor4(send);
    }
    const float keep = b3 ? c[1] : c[0];
    const float send = b3 ? c[0] : c[1];
    float x = keep + dpp<0x128>(send);  // row_ror:8: lane ^ 8
    x += __shfl_xor(x, 16);
    x += __shfl_xor(x, 32);
    return x;
}

// lane ^ M within the wave (DPP inside rows of 16, ds_bpermute across rows)
template <int M>
__device__ __forceinline__ float lane_xor(float x) {
    if constexpr (M == 1) return dpp<0xB1>(x);        // quad_perm [1,0,3,2]
    else if constexpr (M == 2) return dpp<0x4E>(x);   // quad_perm [2,3,0,1]
    else if constexpr (M == 4) return xor4(x);
    else if constexpr (M == 8) return dpp<0x128>(x);  // row_ror:8
    else return __shfl_xor(x, M);
}

// transposed butterfly, generic KT (power of two <= 16): out = the wave-wide
// sum of v[lane & (KT-1)]
template <int KT, int S = 0>
__device__ __forceinline__ float transpose_sum_step(const float* v, int lane) {
    constexpr int M = 1 << S;
    if constexpr (KT == 1) {
        float x = v[0];
        if constexpr (M <= 1) x += lane_xor<1>(x);
        if constexpr (M <= 2) x += lane_xor<2>(x);
        if constexpr (M <= 4) x += lane_xor<4>(x);
        if constexpr (M <= 8) x += lane_xor<8>(x);
        if constexpr (M <= 16) x += lane_xor<16>(x);
        x += lane_xor<32>(x);
        return x;
    } else {
        const bool bit = lane & M;
        float nxt[KT / 2];
#pragma unroll
        for (int i = 0; i < KT / 2; ++i) {
            const float keep = bit ? v[2 * i + 1] : v[2 * i];
            const float send = bit ? v[2 * i] : v[2 * i + 1];
            nxt[i] = keep + lane_xor<M>(send);
        }
        return transpose_sum_step<KT / 2, S + 1>(nxt, lane);
    }
}

template <int WPB, int SB, int KT, int OCC>
__global__ void __launch_bounds__(64 * WPB, OCC)
estep_resp_tile_kernel(const float* __restrict__ ep, int Kp, int K, SamplesDev s, int64_t n,
                       int64_t chunk, float* __restrict__ resp) {
    // per wave: the staged sample block (x0 x1 x2 x3 | x4 x5 hpdf diffuse) and
    // the tile's normalisation scales
    __shared__ float4 sblk[WPB][64][2];
    __shared__ __attribute__((aligned(16))) float sg[WPB][KT];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wave = (int64_t)blockIdx.x * WPB + wid;
    const int64_t s0 = wave * chunk;
    if (s0 >= n) return;
    const int64_t s1 = (s0 + chunk < n) ? s0 + chunk : n;

    const int kbase = 2 * lane;
    V P[EP_FIELDS];
#pragma unroll
    for (int f = 0; f < EP_FIELDS; ++f) P[f] = *(const V*)(ep + f * Kp + kbase);
    const bool full = (kbase + 2 <= K);
    const bool has_h = s.hpdf != nullptr, has_d = s.isDiffuse != nullptr;
    float4 (*blk_lds)[2] = sblk[wid];
    float* g_lds = sg[wid];

    SampleBlock A = load_block(s, s0, s1, lane);
    for (int64_t blk = s0; blk < s1; blk += 64) {
        {
            // stage the block (lane = sample); the flag byte comes out of its dword
            const int64_t si = (blk + lane < s1) ? blk + lane : s1 - 1;
            const int sh = 8 * (int)((uintptr_t)(s.isDiffuse + si) & 3);
            const bool dif = has_d && ((A.diff >> sh) & 0xff) != 0;
            // positions relative to kOrigin (the EP_NC* rows fold -L (mu - kOrigin))
            blk_lds[lane][0] = float4{A.x0 - kOrigin, A.x1 - kOrigin, A.x2 - kOrigin, A.x3};
            blk_lds[lane][1] = float4{A.x4, A.x5, has_h ? A.h : 0.0f, dif ? 1.0f : 0.0f};
        }
        A = load_block(s, blk + 64, s1, lane);   // next block in flight (clamped past the end)
        const int cnt = (s1 - blk < 64) ? (int)(s1 - blk) : 64;
        for (int tb = 0; tb < cnt; tb += KT) {
            V q[KT];
            // rare-angle detector: c < -0.9999995 <=> its bits, unsigned, exceed
            // those of -0.9999995f (integer max, no NaN canonicalisation)
            uint32_t cbits = 0;
#pragma unroll
            for (int t = 0; t < KT; ++t) {
                const float4 a = blk_lds[tb + t][0];
                const float4 b = blk_lds[tb + t][1];
                V c;
                q[t] = pair_q_tile<false>(P, a.x, a.y, a.z, a.w, b.x, b.y, c);
                cbits = __builtin_elementwise_max(cbits, __builtin_elementwise_max(fbits(c.x), fbits(c.y)));
                // keep the scheduler from hoisting every sample's LDS reads
                // (and their registers) to the top of the tile
                if (t % SB == SB - 1) __builtin_amdgcn_sched_barrier(0);
            }
            {
                // rare angle case in the tile (c < -0.9999995 somewhere): redo it
                // with the reference's quirks.  The test also reads the fast
                // path's values (a NaN -- NaN input -- takes the redo too,
                // harmlessly) so that the fast path is not sunk below the branch.
                V qs = q[0];
#pragma unroll
                for (int t = 1; t < KT; ++t) qs += q[t];
                const bool odd = cbits > __builtin_bit_cast(uint32_t, -0.9999995f) || !(qs.x + qs.y >= 0.0f);
                if (__builtin_amdgcn_ballot_w64(odd) != 0) {
#pragma unroll 1
                    for (int t = 0; t < KT; ++t) {
                        const float4 a = blk_lds[tb + t][0];
                        const float4 b = blk_lds[tb + t][1];
                        V c;
                        const V qt = pair_q_tile<true>(P, a.x, a.y, a.z, a.w, b.x, b.y, c);
#pragma unroll
                        for (int u = 0; u < KT; ++u) q[u] = (u == t) ? qt : q[u];
                    }
                }
            }
            float ps[KT];
#pragma unroll
            for (int t = 0; t < KT; ++t) ps[t] = q[t].x + q[t].y;
            const float S = transpose_sum_step<KT>(ps, lane);
            // posterior normalisation of sample tb + (lane & (KT - 1)) (mixture_model.h:170-191);
            // d == 0 fails every log map (mvtn.h:152-154): all pdfs 0, 1/S' not finite
            {
                const int t = tb + (lane & (KT - 1));
                const float4 a = blk_lds[t][0];
                const float4 b = blk_lds[t][1];
                const bool dzero = (a.w == 0.0f && b.x == 0.0f && b.y == 0.0f);
                const bool dif = b.w != 0.0f;
                const float S2 = dif ? fmaf(1.0f - kHeuristicWeight, S, kHeuristicWeight * b.z) : S;
                const float inv = __builtin_amdgcn_rcpf(S2);
                const bool fin = __builtin_isfinite(inv) && !dzero;
                const float g = fin ? (dif ? inv * (1.0f - kHeuristicWeight) : inv) : 0.0f;
                if (lane < KT) g_lds[lane] = g;
            }
            // a non-finite sum means a non-finite q (NaN input): zero by select
            const bool bad = __builtin_amdgcn_ballot_w64(!__builtin_isfinite(S)) != 0;
            const int tcnt = (cnt - tb < KT) ? cnt - tb : KT;
            float* row0 = resp + (blk + tb) * (int64_t)K + kbase;
            if (tcnt == KT && !bad && K == Kp) {
                // the common tile: straight-line stores, the scales read four at a time
#pragma unroll
                for (int t = 0; t < KT; t += 4) {
                    const float4 g4 = *(const float4*)&g_lds[t];
                    __builtin_nontemporal_store(q[t] * g4.x, (V*)(row0 + (int64_t)t * K));
                    __builtin_nontemporal_store(q[t + 1] * g4.y, (V*)(row0 + (int64_t)(t + 1) * K));
                    __builtin_nontemporal_store(q[t + 2] * g4.z, (V*)(row0 + (int64_t)(t + 2) * K));
                    __builtin_nontemporal_store(q[t + 3] * g4.w, (V*)(row0 + (int64_t)(t + 3) * K));
                }
            } else {
#pragma unroll
                for (int t = 0; t < KT; ++t) {
                    if (t >= tcnt) break;
                    const float g = g_lds[t];
                    V o = q[t] * g;
                    if (bad) o = (g != 0.0f) ? o : sp(0.0f);
                    float* row = row0 + (int64_t)t * K;
                    if (full) {
                        __builtin_nontemporal_store(o, (V*)row);
                    } else {
                        if (kbase < K) __builtin_nontemporal_store(o.x, row);
                    }
                }
            }
        }
    }
}

// Batched launches (sdmm_em_step_batched): workgroup b runs block items[b].y
// of leaf items[b].x, i.e. exactly the workgroup of the single-mixture launch
// over that leaf's samples, and writes its partial row at the leaf's rows.
__device__ __forceinline__ SamplesDev shift_samples(SamplesDev s, int64_t s0) {
    for (int i = 0; i < 6; ++i) s.x[i] += s0;
    s.w += s0;
    if (s.hpdf) s.hpdf += s0;
    if (s.isDiffuse) s.isDiffuse += s0;
    return s;
}

// ---------------------------------------------------------------------------
// Fused E-step + sufficient statistics (calculateStats + sumWeights).
// partial row layout (component-major): [ST_FIELDS k + f] for f < ST_FIELDS
// (W, M0..M4, C00..C44: the compact order), then [21Kp] = H, [21Kp+1] = wsum.
template <int CPL, int LPS>
__global__ void __launch_bounds__(256)
estep_stats_kernel(const float* __restrict__ ep, int Kp, int K, SamplesDev s, int64_t n,
                   int64_t chunk, float* __restrict__ partials, int pstride,
                   const LeafDesc* __restrict__ leaves, const int2* __restrict__ items) {
    int64_t bid = blockIdx.x;
    float* prow = partials + bid * pstride;
    if (leaves) {
        const int2 it = items[blockIdx.x];
        const LeafDesc& L = leaves[it.x];
        ep = L.ep;
        s = shift_samples(s, L.s0);
        n = L.n;
        chunk = L.chunk;
        bid = it.y;
        prow = partials + (int64_t)(L.row0 + it.y) * pstride;
    }
    static_assert(CPL % 2 == 0, "components are processed in packed pairs");
    constexpr int SPW = 64 / LPS;
    constexpr int NP = CPL / 2;
    extern __shared__ __attribute__((aligned(16))) float red[];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    const int g = lane / LPS;
    const int j = lane % LPS;
    const int64_t wave = bid * nw + wid;
    const int64_t s0 = wave * chunk;
    const int64_t s1 = (s0 + chunk < n) ? s0 + chunk : n;  // s1 <= s0: no samples

    const int kbase = j * CPL;
    V P[NP][EP_FIELDS];
    load_params<CPL>(ep, Kp, kbase, P);

    V acc[NP][ST_FIELDS];
#pragma unroll
    for (int c = 0; c < NP; ++c)
#pragma unroll
        for (int f = 0; f < ST_FIELDS; ++f) acc[c][f] = sp(0.0f);
    float accH = 0.0f, accWs = 0.0f;

    walk_samples<LPS, true>(s, s0, s1, lane, g, [&](const SampleVals& sv, int64_t, bool in)
                                                    __attribute__((always_inline)) {
        const bool finite_w = __builtin_isfinite(sv.w);
        // sumWeights counts every finite weight (stepwise_tangent.h:462-475)
        accWs += (in && finite_w) ? sv.w : 0.0f;
        // calculateStats skips non-finite and zero weights (:288-293)
        const bool use = in && finite_w && (sv.w != 0.0f);
        const float df = sv.dfail();
        V q[NP], ta[NP], tb[NP];
        V qs = sp(0.0f);
#pragma unroll
        for (int c = 0; c < NP; ++c) {
            q[c] = pair_pdf_stats(P[c], sv.x0, sv.x1, sv.x2, sv.x3, sv.x4, sv.x5, sv.cd, df, ta[c], tb[c]);
            qs += q[c];
        }
        const Norm nm = normalise<LPS>(qs.x + qs.y, sv);
        const float w = use ? sv.w : 0.0f;
        accH = fmaf(w, nm.hpost, accH);
        // posterior < 1e-10 is skipped (:312).  With thr = +inf when 1/S' is not
        // finite (posterior set to zero, mixture_model.h:182-191) nothing passes.
        const float thr = nm.fin ? 1e-10f : __builtin_inff();
        // Spatial statistics are accumulated centred on the component's mean
        // position (tp = p - mu_k) and un-centred in fp64 by
        // reduce_uncenter_kernel: the M-step's C/W - mu mu^T then does not
        // amplify fp32 accumulation error by |p|^2 / sigma^2.
#pragma unroll
        for (int c = 0; c < NP; ++c) {
            const V gam = q[c] * nm.gsc;
            const V v = (gam >= sp(thr)) ? gam * w : sp(0.0f);   // unused samples have w == 0
            const V tp0 = sv.x0 - P[c][EP_MU0];
            const V tp1 = sv.x1 - P[c][EP_MU1];
            const V tp2 = sv.x2 - P[c][EP_MU2];
            V* A = acc[c];
            A[ST_W] += v;
            const V v0 = v * tp0, v1 = v * tp1, v2 = v * tp2;
            A[ST_M0] += v0;
            A[ST_M1] += v1;
            A[ST_M2] += v2;
            const V v3 = v * ta[c], v4 = v * tb[c];
            A[ST_M3] += v3;
            A[ST_M4] += v4;
            A[ST_C00] = vfma(v0, tp0, A[ST_C00]);
            A[ST_C10] = vfma(v1, tp0, A[ST_C10]);
            A[ST_C11] = vfma(v1, tp1, A[ST_C11]);
            A[ST_C20] = vfma(v2, tp0, A[ST_C20]);
            A[ST_C21] = vfma(v2, tp1, A[ST_C21]);
            A[ST_C22] = vfma(v2, tp2, A[ST_C22]);
            A[ST_C30] = vfma(v3, tp0, A[ST_C30]);
            A[ST_C31] = vfma(v3, tp1, A[ST_C31]);
            A[ST_C32] = vfma(v3, tp2, A[ST_C32]);
            A[ST_C33] = vfma(v3, ta[c], A[ST_C33]);
            A[ST_C40] = vfma(v4, tp0, A[ST_C40]);
            A[ST_C41] = vfma(v4, tp1, A[ST_C41]);
            A[ST_C42] = vfma(v4, tp2, A[ST_C42]);
            A[ST_C43] = vfma(v4, ta[c], A[ST_C43]);
            A[ST_C44] = vfma(v4, tb[c], A[ST_C44]);
        }
    });

    // fold the lane groups of this wave holding the same components
    if constexpr (SPW > 1) {
#pragma unroll
        for (int off = LPS; off < 64; off <<= 1) {
#pragma unroll
            for (int c = 0; c < NP; ++c)
#pragma unroll
                for (int f = 0; f < ST_FIELDS; ++f) {
                    acc[c][f].x += __shfl_xor(acc[c][f].x, off);
                    acc[c][f].y += __shfl_xor(acc[c][f].y, off);
                }
        }
    }
    // H and wsum are group-uniform: keep one copy per group, then sum groups
    accH = (j == 0) ? accH : 0.0f;
    accWs = (j == 0) ? accWs : 0.0f;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        accH += __shfl_xor(accH, off);
        accWs += __shfl_xor(accWs, off);
    }

    // fold the workgroup's waves in a fixed order through LDS
    const int rowlen = ST_FIELDS * Kp + 2;
    for (int w = 0; w < nw; ++w) {
        if (wid == w && g == 0) {
#pragma unroll
            for (int c = 0; c < NP; ++c)
#pragma unroll
                for (int f = 0; f < ST_FIELDS; ++f) {
                    float* d0 = &red[ST_FIELDS * (kbase + 2 * c) + f];
                    float* d1 = d0 + ST_FIELDS;
                    *d0 = (w == 0) ? acc[c][f].x : *d0 + acc[c][f].x;
                    *d1 = (w == 0) ? acc[c][f].y : *d1 + acc[c][f].y;
                }
            if (lane == 0) {
                red[ST_FIELDS * Kp] = (w == 0) ? accH : red[ST_FIELDS * Kp] + accH;
                red[ST_FIELDS * Kp + 1] = (w == 0) ? accWs : red[ST_FIELDS * Kp + 1] + accWs;
            }
        }
        __syncthreads();
    }
    for (int idx = threadIdx.x; idx < rowlen; idx += blockDim.x) prow[idx] = red[idx];
}

// ---------------------------------------------------------------------------
// Tiled fused E-step + statistics for 64 < K <= 128 (one packed pair per
// lane), the estep_resp_tile_kernel scheme applied to calculateStats
// (stepwise_tangent.h:270-353): tiles of kStatTile = 4 samples keep q and the
// directional tangent (ta, tb) of the lane's pair in registers, the
// normaliser comes from a transposed butterfly, and the lane holding sample t
// publishes {gamma scale, weight, threshold} through LDS for the accumulation.

constexpr int kStatTile = 4;

// theta/sin(theta) from delta = 1 + c for the statistics tiles: the degree-7
// main-path polynomial of angle_over_sin_main; RARE adds the quirks of
// angle_over_sin_fast (s^2 < 1e-6: 1, or 0 when the log map fails, delta <= 0).
template <bool RARE>
__device__ __forceinline__ V angle_over_sin_tile_d(V dl) {
    const V om = sp(2.0f) - dl;
    const V u = half_gap(dl, om);
    V h = vfma(sp(3.3755881786346436f), u, sp(-3.17423415184021f));
    h = vfma(h, u, sp(2.1241207122802734f));
    h = vfma(h, u, sp(-0.04515757039189339f));
    h = vfma(h, u, sp(0.5178175568580627f));
    h = vfma(h, u, sp(0.5294308066368103f));
    h = vfma(h, u, sp(0.6667603850364685f));
    h = vfma(h, u, sp(0.9999996423721313f));
    const V s2 = dl * om;
    const V fneg = vfma(sp(3.14159265358979f), vrsq(s2), -h);
    const V f = V{dl.x < 1.0f ? fneg.x : h.x, dl.y < 1.0f ? fneg.y : h.y};
    if constexpr (!RARE) return f;
    const V one = V{dl.x > 0.0f ? 1.0f : 0.0f, dl.y > 0.0f ? 1.0f : 0.0f};
    return V{s2.x < 1e-6f ? one.x : f.x, s2.y < 1e-6f ? one.y : f.y};
}

// pi_k pdf_k and the directional tangent (mvtn.h:146-177; a = 0 when the log
// map fails, so ta = tb = 0 then) with the cancellation-free delta = 1 + c,
// returned in dl for the tile's rare-angle detector.
template <bool RARE>
__device__ __forceinline__ V pair_qt_fast(const V* __restrict__ P, float p0, float p1, float p2, float d0,
                                          float d1, float d2, float cd, V& ta, V& tb, V& dl) {
    const V tp0 = p0 - P[EP_MU0], tp1 = p1 - P[EP_MU1], tp2 = p2 - P[EP_MU2];
    dl = one_plus_c(P, d0, d1, d2, cd);
    const V a = angle_over_sin_tile_d<RARE>(dl);
    const V r0 = vfma(P[EP_R02], sp(d2), vfma(P[EP_R01], sp(d1), P[EP_R00] * d0));
    const V r1 = vfma(P[EP_R12], sp(d2), vfma(P[EP_R11], sp(d1), P[EP_R10] * d0));
    ta = r0 * a;
    tb = r1 * a;
    const V u0 = P[EP_L00] * tp0;
    const V u1 = vfma(P[EP_L11], tp1, P[EP_L10] * tp0);
    const V u2 = vfma(P[EP_L22], tp2, vfma(P[EP_L21], tp1, P[EP_L20] * tp0));
    const V s3 = vfma(P[EP_L32], tp2, vfma(P[EP_L31], tp1, P[EP_L30] * tp0));
    const V s4 = vfma(P[EP_L42], tp2, vfma(P[EP_L41], tp1, P[EP_L40] * tp0));
    const V u3 = vfma(P[EP_L33], ta, s3);
    const V u4 = vfma(P[EP_L44], tb, vfma(P[EP_L43], ta, s4));
    const V q = vfma(u4, u4, vfma(u3, u3, vfma(u2, u2, vfma(u1, u1, u0 * u0))));
    const V e = vexp2(vfma(q, sp(-0.72134752044448170368f), sp(kLog2Norm5)));
    return e * (P[EP_DIPI] * a);
}

// Transposed butterfly for 4 values: out = wave-wide sum of v[lane & 3].
__device__ __forceinline__ float transpose_sum4(const float (&v)[kStatTile], int lane) {
    const bool b0 = lane & 1, b1 = lane & 2;
    float a[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const float keep = b0 ? v[2 * i + 1] : v[2 * i];
        const float send = b0 ? v[2 * i] : v[2 * i + 1];
        a[i] = keep + dpp<0xB1>(send);
    }
    const float keep = b1 ? a[1] : a[0];
    const float send = b1 ? a[0] : a[1];
    float x = keep + dpp<0x4E>(send);
    x += xor4(x);
    x += dpp<0x128>(x);   // lane ^ 8
    x += __shfl_xor(x, 16);
    x += __shfl_xor(x, 32);
    return x;
}

// GROUP = false: each of the WPB waves walks its own sample chunk against all
// K <= 128 components (one packed pair per lane).  GROUP = true (128 < K <=
// 128 WPB: Pool K = 256 with WPB = 2, Kitchen K = 512 with WPB = 4): the waves
// of a workgroup walk the SAME chunk, wave w holding components 128 w ..
// 128 w + 127 -- the K = 128 register budget per lane at any K (round 1 kept
// 4 / 8 components per lane: 265 / 512 VGPRs with spills, one wave per SIMD).
// Per 4-sample tile each wave's partial normaliser goes through LDS and one
// workgroup barrier; every wave then sums the partials in wave order.  The
// waves' component ranges are disjoint, so the partial row needs no fold.
template <int WPB, int OCC, bool GROUP = false>
__global__ void __launch_bounds__(64 * WPB, OCC)
estep_stats_tile_kernel(const float* __restrict__ ep, int Kp, int K, SamplesDev s, int64_t n,
                        int64_t chunk, float* __restrict__ partials, int pstride,
                        const LeafDesc* __restrict__ leaves, const int2* __restrict__ items) {
    int64_t bid = blockIdx.x;
    float* prow = partials + bid * pstride;
    if (leaves) {
        const int2 it = items[blockIdx.x];
        const LeafDesc& L = leaves[it.x];
        ep = L.ep;
        s = shift_samples(s, L.s0);
        n = L.n;
        chunk = L.chunk;
        bid = it.y;
        prow = partials + (int64_t)(L.row0 + it.y) * pstride;
    }
    __shared__ float4 sblk[WPB][64][2];      // x0 x1 x2 x3 | x4 x5 hpdf diffuse
    __shared__ float2 sw[WPB][64];           // weight, half_defect of the direction
    __shared__ float4 sg[WPB][kStatTile];    // {gamma scale, weight, threshold, -}
    __shared__ float spart[2][WPB][kStatTile];   // GROUP: per-wave partial normalisers (tile parity)
    extern __shared__ __attribute__((aligned(16))) float red[];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wave = GROUP ? bid : bid * WPB + wid;
    const int64_t s0 = wave * chunk;
    const int64_t s1 = (s0 + chunk < n) ? s0 + chunk : n;   // s1 <= s0: no samples

    const int kbase = (GROUP ? 128 * wid : 0) + 2 * lane;
    int parity = 0;
    V P[EP_FIELDS];
#pragma unroll
    for (int f = 0; f < EP_FIELDS; ++f) P[f] = *(const V*)(ep + f * Kp + kbase);
    V acc[ST_FIELDS];
#pragma unroll
    for (int f = 0; f < ST_FIELDS; ++f) acc[f] = sp(0.0f);
    float accH = 0.0f, accWs = 0.0f;   // lanes < kStatTile: their samples' H and sumWeights terms
    const bool has_h = s.hpdf != nullptr, has_d = s.isDiffuse != nullptr;
    float4 (*blk_lds)[2] = sblk[wid];
    float2* w_lds = sw[wid];
    float4* g_lds = sg[wid];

    if (s0 < s1) {
        SampleBlock A = load_block(s, s0, s1, lane);
        for (int64_t blk = s0; blk < s1; blk += 64) {
            {
                const int64_t si = (blk + lane < s1) ? blk + lane : s1 - 1;
                const int sh = 8 * (int)((uintptr_t)(s.isDiffuse + si) & 3);
                const bool dif = has_d && ((A.diff >> sh) & 0xff) != 0;
                blk_lds[lane][0] = float4{A.x0, A.x1, A.x2, A.x3};
                blk_lds[lane][1] = float4{A.x4, A.x5, has_h ? A.h : 0.0f, dif ? 1.0f : 0.0f};
                w_lds[lane] = float2{A.w, half_defect(A.x3, A.x4, A.x5)};
            }
            A = load_block(s, blk + 64, s1, lane);
            const int cnt = (s1 - blk < 64) ? (int)(s1 - blk) : 64;
            for (int tb = 0; tb < cnt; tb += kStatTile) {
                V q[kStatTile], ta[kStatTile], tb2[kStatTile];
                float dmin = 1.0f;   // rare-angle detector: the smallest 1 + c of the tile
#pragma unroll
                for (int t = 0; t < kStatTile; ++t) {
                    const float4 a = blk_lds[tb + t][0];
                    const float4 b = blk_lds[tb + t][1];
                    V dl;
                    q[t] = pair_qt_fast<false>(P, a.x, a.y, a.z, a.w, b.x, b.y, w_lds[tb + t].y, ta[t], tb2[t], dl);
                    dmin = fminf(dmin, fminf(dl.x, dl.y));
                }
                {
                    // 1 + c < 1e-6 somewhere in the tile (sin < 1e-3 near the
                    // antipode, or a failed log map): redo it with the reference's
                    // angle quirks (a NaN sum takes the redo too)
                    const V qs = (q[0] + q[1]) + (q[2] + q[3]);
                    const bool odd = dmin < 1e-6f || !(qs.x + qs.y >= 0.0f);
                    if (__builtin_amdgcn_ballot_w64(odd) != 0) {
                        // (a loop, so that the compiler does not speculate it)
#pragma unroll 1
                        for (int t = 0; t < kStatTile; ++t) {
                            const float4 a = blk_lds[tb + t][0];
                            const float4 b = blk_lds[tb + t][1];
                            V ta1, tb1, dl1;
                            const V q1 = pair_qt_fast<true>(P, a.x, a.y, a.z, a.w, b.x, b.y, w_lds[tb + t].y, ta1,
                                                            tb1, dl1);
#pragma unroll
                            for (int u = 0; u < kStatTile; ++u) {
                                q[u] = (u == t) ? q1 : q[u];
                                ta[u] = (u == t) ? ta1 : ta[u];
                                tb2[u] = (u == t) ? tb1 : tb2[u];
                            }
                        }
                    }
                }
                float ps[kStatTile];
#pragma unroll
                for (int t = 0; t < kStatTile; ++t) ps[t] = q[t].x + q[t].y;
                float S = transpose_sum4(ps, lane);
                if constexpr (GROUP) {
                    // the workgroup's partial sums of sample tb + (lane & 3), in wave order
                    if (lane < kStatTile) spart[parity][wid][lane] = S;
                    __syncthreads();
                    S = spart[parity][0][lane & 3];
#pragma unroll
                    for (int w = 1; w < WPB; ++w) S += spart[parity][w][lane & 3];
                    parity ^= 1;
                }
                {
                    // posteriorAndLog normalisation (mixture_model.h:170-191) and the
                    // weight guards of calculateStats / sumWeights (:288-293, :462-475)
                    // for sample tb + (lane & 3); d == 0: every pdf is 0 (mvtn.h:152-154)
                    const int t = tb + (lane & 3);
                    const bool in = t < cnt;
                    const float4 a = blk_lds[t][0];
                    const float4 b = blk_lds[t][1];
                    const float w = w_lds[t].x;
                    const bool dzero = (a.w == 0.0f && b.x == 0.0f && b.y == 0.0f);
                    const bool dif = b.w != 0.0f;
                    const float Se = dzero ? 0.0f : S;
                    const float S2 = dif ? fmaf(1.0f - kHeuristicWeight, Se, kHeuristicWeight * b.z) : Se;
                    const float inv = __builtin_amdgcn_rcpf(S2);
                    const bool fin = __builtin_isfinite(inv);
                    const bool finite_w = __builtin_isfinite(w);
                    const bool use = in && finite_w && w != 0.0f;
                    const float g = (fin && !dzero) ? (dif ? inv * (1.0f - kHeuristicWeight) : inv) : 0.0f;
                    const float hpost = (fin && dif) ? kHeuristicWeight * b.z * inv : 0.0f;
                    const float weff = use ? w : 0.0f;
                    if (lane < kStatTile) {
                        // (GROUP: every wave sees the same samples; H and sumWeights
                        // are counted by wave 0's lanes only)
                        if (!GROUP || wid == 0) {
                            accWs += (in && finite_w) ? w : 0.0f;
                            accH = fmaf(weff, hpost, accH);
                        }
                        // gamma < 1e-10 is skipped (:312); nothing passes when 1/S' is
                        // not finite (posterior zeroed, mixture_model.h:182-191)
                        g_lds[lane] = float4{g, weff, (fin && !dzero) ? 1e-10f : __builtin_inff(), 0.0f};
                    }
                }
#pragma unroll
                for (int t = 0; t < kStatTile; ++t) {
                    const float4 gw = g_lds[t];
                    const float4 a = blk_lds[tb + t][0];
                    const V gam = q[t] * gw.x;
                    const V v = V{gam.x >= gw.z ? gam.x : 0.0f, gam.y >= gw.z ? gam.y : 0.0f} * gw.y;
                    const V tp0 = a.x - P[EP_MU0];
                    const V tp1 = a.y - P[EP_MU1];
                    const V tp2 = a.z - P[EP_MU2];
                    acc[ST_W] += v;
                    const V v0 = v * tp0, v1 = v * tp1, v2 = v * tp2;
                    acc[ST_M0] += v0;
                    acc[ST_M1] += v1;
                    acc[ST_M2] += v2;
                    const V v3 = v * ta[t], v4 = v * tb2[t];
                    acc[ST_M3] += v3;
                    acc[ST_M4] += v4;
                    acc[ST_C00] = vfma(v0, tp0, acc[ST_C00]);
                    acc[ST_C10] = vfma(v1, tp0, acc[ST_C10]);
                    acc[ST_C11] = vfma(v1, tp1, acc[ST_C11]);
                    acc[ST_C20] = vfma(v2, tp0, acc[ST_C20]);
                    acc[ST_C21] = vfma(v2, tp1, acc[ST_C21]);
                    acc[ST_C22] = vfma(v2, tp2, acc[ST_C22]);
                    acc[ST_C30] = vfma(v3, tp0, acc[ST_C30]);
                    acc[ST_C31] = vfma(v3, tp1, acc[ST_C31]);
                    acc[ST_C32] = vfma(v3, tp2, acc[ST_C32]);
                    acc[ST_C33] = vfma(v3, ta[t], acc[ST_C33]);
                    acc[ST_C40] = vfma(v4, tp0, acc[ST_C40]);
                    acc[ST_C41] = vfma(v4, tp1, acc[ST_C41]);
                    acc[ST_C42] = vfma(v4, tp2, acc[ST_C42]);
                    acc[ST_C43] = vfma(v4, ta[t], acc[ST_C43]);
                    acc[ST_C44] = vfma(v4, tb2[t], acc[ST_C44]);
                }
            }
        }
    }
    // H and sumWeights live in lanes 0..3: sum them over the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        accH += __shfl_xor(accH, off);
        accWs += __shfl_xor(accWs, off);
    }
    // fold the workgroup's waves in a fixed order: every wave parks its row in
    // its own LDS slot, one barrier, then each column is summed over the slots
    // in wave order ((a0 + a1) + a2) + a3 -- the order of a wave-by-wave fold,
    // with one barrier instead of WPB (GROUP: the waves' component ranges are
    // disjoint, one slot, each wave writes its own columns)
    const int rowlen = ST_FIELDS * Kp + 2;
    constexpr int NSLOT = GROUP ? 1 : WPB;
    float* mine = red + (GROUP ? 0 : wid * rowlen);
#pragma unroll
    for (int f = 0; f < ST_FIELDS; ++f) {
        mine[ST_FIELDS * kbase + f] = acc[f].x;
        mine[ST_FIELDS * (kbase + 1) + f] = acc[f].y;
    }
    if (lane == 0 && (!GROUP || wid == 0)) {
        mine[ST_FIELDS * Kp] = accH;
        mine[ST_FIELDS * Kp + 1] = accWs;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < rowlen; idx += blockDim.x) {
        float v = red[idx];
#pragma unroll
        for (int w = 1; w < NSLOT; ++w) v += red[w * rowlen + idx];
        prow[idx] = v;
    }
}

// ---------------------------------------------------------------------------
// Deterministic fp64 reduction of the partial rows into the compact stats
// vector [H, wsum, W(K), M(5K), Clow(15K)].  The fixed summation order: the
// rows split into kReduceSlices slices; within slice s four row-interleaved
// fp64 sums (rows r0 + j, r0 + j + 4, ...; j < 4) combined as ((b0 + b1) + b2)
// + b3; the slices summed in order from 0.0.  The batched per-leaf reduction
// (reduce_uncenter_batched_kernel) uses the same order, so a leaf's stats are bitwise those of
// its single-mixture E-step.
constexpr int kReduceSlices = 16;

// Partial-row column of compact index o (component-major rows).
__device__ __forceinline__ int partial_col(int o, int Kp, int K) {
    if (o == 0) return ST_FIELDS * Kp;
    if (o == 1) return ST_FIELDS * Kp + 1;
    const int r = o - 2;
    if (r < K) return ST_FIELDS * r + ST_W;
    if (r < 6 * K) { const int q = r - K; return ST_FIELDS * (q / 5) + ST_M0 + q % 5; }
    const int q = r - 6 * K;
    return ST_FIELDS * (q / 15) + ST_C00 + q % 15;
}
// ... and its inverse: the compact index of partial column c, or -1 (padding)
__device__ __forceinline__ int compact_of(int c, int Kp, int K) {
    if (c == ST_FIELDS * Kp) return 0;
    if (c == ST_FIELDS * Kp + 1) return 1;
    const int k = c / ST_FIELDS, f = c % ST_FIELDS;
    if (k >= K) return -1;
    if (f == ST_W) return 2 + k;
    if (f < ST_C00) return 2 + K + 5 * k + (f - ST_M0);
    return 2 + 6 * K + 15 * k + (f - ST_C00);
}

// The un-centring of one component's spatial statistics (fp64, in place):
//   M_p = M'_p + W mu,  C_pp = C'_pp + M'_p mu^T + mu M'_p^T + W mu mu^T,
//   C_tp = C'_tp + M_t mu^T   (mu = the float mean the E-step subtracted).
__device__ __forceinline__ void uncenter_component(const double mu[3], double w, double M[5], double C[15]) {
    // no FMA contraction: the single-mixture and the batched reduction inline
    // this into different code, and a contraction the backend picks per
    // context would part their bits
#pragma clang fp contract(off)
    // C_pp (entries 0..5: (0,0) (1,0) (1,1) (2,0) (2,1) (2,2))
    int e = 0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j <= i; ++j, ++e)
            C[e] += M[i] * mu[j] + mu[i] * M[j] + w * mu[i] * mu[j];
    // C_tp: rows 3, 4 (entries 6..8 and 10..12)
    for (int j = 0; j < 3; ++j) {
        C[6 + j] += M[3] * mu[j];
        C[10 + j] += M[4] * mu[j];
    }
    for (int i = 0; i < 3; ++i) M[i] = M[i] + w * mu[i];
}

// The whole reduction and the un-centring in ONE launch (round 4: two, a
// (64-column block x slice) pass through an fp64 scratch then a per-component
// slice sum + un-centring; 6.6 + 5.3 us at 512 rows, K = 128, both mostly
// launch and latency): workgroup b owns components kRedCB b .. kRedCB b + 2,
// whose 63 partial columns are contiguous in the component-major rows (one
// lane each; the extra last workgroup owns H and wsum); wave s sums row slice
// s (its four interleaved sums in registers, every load independent), wave 0
// then sums the slices in order and lanes < kRedCB un-centre their component.
// The same operations in the same order as the two-launch form: bitwise equal.
constexpr int kRedCB = 3;
static_assert(ST_FIELDS * kRedCB <= 64, "a workgroup's columns fit one wave");
// Partial column of lane `lane` in component group g (components kRedCB g
// ...; the extra group g == nb holds H and wsum), or -1.
__device__ __forceinline__ int group_col(int lane, int g, int nb, int K, int Kp) {
    if (g == nb) return lane < 2 ? ST_FIELDS * Kp + lane : -1;
    const int k0 = g * kRedCB;
    return (lane < ST_FIELDS * kRedCB && k0 + lane / ST_FIELDS < K) ? ST_FIELDS * k0 + lane : -1;
}

// One slice's sum of a column (rows [r0, r1) of p, stride pstride): four
// row-interleaved fp64 partials, every load of a 16-row batch independent,
// combined as ((b0 + b1) + b2) + b3.
__device__ __forceinline__ double slice_sum(const float* __restrict__ p, int pstride, int r0, int r1) {
    double b[4] = {0.0, 0.0, 0.0, 0.0};
    int r = r0;
    for (; r + 16 <= r1; r += 16) {
        float v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = p[(int64_t)(r + i) * pstride];
#pragma unroll
        for (int i = 0; i < 16; ++i) b[i & 3] += (double)v[i];
    }
    for (; r < r1; ++r) b[(r - r0) & 3] += (double)p[(int64_t)r * pstride];
    return ((b[0] + b[1]) + b[2]) + b[3];
}

// Group g's column totals (lane = column, as group_col) into the compact
// stats: H and wsum, or lanes < kRedCB un-centre their component.  Every lane
// of the wave takes part (the shuffles).
__device__ __forceinline__ void group_store(double v, int lane, int g, int nb, int K, int Kp,
                                            const float* __restrict__ ep, double* __restrict__ stats) {
    if (g == nb) {
        if (lane < 2) stats[lane] = v;
        return;
    }
    // lane l < kRedCB gathers its component's 21 columns from lanes 21 l + f
    const int cl = lane < kRedCB ? ST_FIELDS * lane : 0;
    double c[ST_FIELDS];
#pragma unroll
    for (int f = 0; f < ST_FIELDS; ++f) c[f] = __shfl(v, cl + f);
    const int k = g * kRedCB + lane;
    if (lane < kRedCB && k < K) {
        const double mu[3] = {(double)ep[EP_MU0 * Kp + k], (double)ep[EP_MU1 * Kp + k],
                              (double)ep[EP_MU2 * Kp + k]};
        const double w = c[ST_W];
        double M[5], C[15];
        for (int i = 0; i < 5; ++i) M[i] = c[ST_M0 + i];
        for (int i = 0; i < 15; ++i) C[i] = c[ST_C00 + i];
        uncenter_component(mu, w, M, C);
        stats[2 + k] = w;
        for (int i = 0; i < 5; ++i) stats[2 + K + 5 * k + i] = M[i];
        for (int i = 0; i < 15; ++i) stats[2 + 6 * K + 15 * k + i] = C[i];
    }
}

__global__ void __launch_bounds__(64 * kReduceSlices)
reduce_uncenter_kernel(const float* __restrict__ partials, int rows, int pstride, const float* __restrict__ ep,
                       int Kp, int K, double* __restrict__ stats) {
    __shared__ double sv[kReduceSlices][64];
    const int lane = threadIdx.x & 63;
    const int sl = threadIdx.x >> 6;
    const int nb = (K + kRedCB - 1) / kRedCB;
    const int col = group_col(lane, blockIdx.x, nb, K, Kp);
    const int r0 = (int)((int64_t)rows * sl / kReduceSlices);
    const int r1 = (int)((int64_t)rows * (sl + 1) / kReduceSlices);
    sv[sl][lane] = col >= 0 ? slice_sum(partials + col, pstride, r0, r1) : 0.0;
    __syncthreads();
    if (sl != 0) return;
    double v = 0.0;
#pragma unroll
    for (int s2 = 0; s2 < kReduceSlices; ++s2) v += sv[s2][lane];
    group_store(v, lane, blockIdx.x, nb, K, Kp, ep, stats);
}

// The training pass's batched per-leaf reduction (round 5): ONE wave per
// (leaf, component group), the 16 slices of the leaf's rows summed in order
// by the same wave -- the single-mixture kernel's operations in its order, so
// a batched leaf's stats stay bitwise those of its single-mixture E-step.  A
// training pass's leaves hold a few rows each, so the single-mixture shape
// (16 waves a group, one per slice) would mostly launch idle waves.  Grid
// (leaves, ceil((groups + 1) / 4)), four waves a workgroup.  Round 4 ran one
// workgroup per leaf with a thread per column (~40 columns per thread in
// series at K = 512: 5.4 ms per launch).
__global__ void __launch_bounds__(256)
reduce_uncenter_batched_kernel(const float* __restrict__ partials, int pstride, int Kp, int K,
                               const LeafDesc* __restrict__ leaves) {
    const LeafDesc& L = leaves[blockIdx.x];
    if (L.n <= 0) return;             // uniform over the workgroup
    const int lane = threadIdx.x & 63;
    const int nb = (K + kRedCB - 1) / kRedCB;
    const int g = (int)blockIdx.y * 4 + (int)(threadIdx.x >> 6);
    if (g > nb) return;               // uniform over the wave
    const int col = group_col(lane, g, nb, K, Kp);
    double v = 0.0;
    if (col >= 0) {
        const float* p = partials + (int64_t)L.row0 * pstride + col;
        for (int sl = 0; sl < kReduceSlices; ++sl) {
            const int r0 = (int)((int64_t)L.rows * sl / kReduceSlices);
            const int r1 = (int)((int64_t)L.rows * (sl + 1) / kReduceSlices);
            v += slice_sum(p, pstride, r0, r1);
        }
    }
    group_store(v, lane, g, nb, K, Kp, L.ep, L.stats);
}

hipError_t launch_reduce_finalize_batched(const float* partials, int pstride, int Kp, int K,
                                          const LeafDesc* leaves, int n_leaves, hipStream_t st) {
    if (n_leaves <= 0) return hipSuccess;
    const int nb = (K + kRedCB - 1) / kRedCB;
    hipLaunchKernelGGL(reduce_uncenter_batched_kernel, dim3(n_leaves, (nb + 1 + 3) / 4), dim3(256), 0, st, partials,
                       pstride, Kp, K, leaves);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// host-side launch helpers (called from sdmm_api.cpp)
template <int CPL, int LPS>
static hipError_t launch_resp_t(const float* ep, int Kp, int K, const SamplesDev& s, int64_t n,
                                int64_t chunk, float* resp, hipStream_t st) {
    const int64_t waves = (n + chunk - 1) / chunk;
    const int wpb = 4;
    const int64_t blocks = (waves + wpb - 1) / wpb;
    hipLaunchKernelGGL((estep_resp_kernel<CPL, LPS>), dim3((unsigned)blocks), dim3(64 * wpb), 0, st,
                       ep, Kp, K, s, n, chunk, resp);
    return hipGetLastError();
}

template <int CPL, int LPS>
static hipError_t launch_stats_t(const float* ep, int Kp, int K, const SamplesDev& s, int64_t n,
                                 int64_t chunk, int blocks, int wpb, float* partials, int pstride,
                                 hipStream_t st, const LeafDesc* leaves, const int2* items) {
    const size_t lds = sizeof(float) * (size_t)(ST_FIELDS * Kp + 2);
    hipLaunchKernelGGL((estep_stats_kernel<CPL, LPS>), dim3(blocks), dim3(64 * wpb), lds, st,
                       ep, Kp, K, s, n, chunk, partials, pstride, leaves, items);
    return hipGetLastError();
}

// Layouts (choose_layout in sdmm_api.cpp): CPL = 2 with LPS in {8, 16, 32, 64}
// for K <= 128, then LPS = 64 with CPL in {4, 8}.
#define SDMM_LAYOUTS(X) X(2, 8) X(2, 16) X(2, 32) X(2, 64) X(4, 32) X(4, 64) X(8, 64)

hipError_t launch_estep_resp(int cpl, int lps, const float* ep, int Kp, int K, const SamplesDev& s,
                             int64_t n, int64_t chunk, float* resp, hipStream_t st) {
#define X(C, L) if (cpl == C && lps == L) return launch_resp_t<C, L>(ep, Kp, K, s, n, chunk, resp, st);
    SDMM_LAYOUTS(X)
#undef X
    return hipErrorInvalidValue;
}

// Tiled responsibility kernel (64 < K <= 128, Kp == 128): chunk is a multiple
// of 64 samples per wave.
// Variants (SDMM_RESP_VARIANT): {SB, KT, waves per SIMD}.
#define SDMM_TILE_VARIANTS(X) X(0, 2, 16, 4) X(1, 2, 8, 4) X(2, 2, 16, 3) X(3, 4, 16, 3) X(4, 2, 8, 3)

hipError_t launch_estep_resp_tile(int variant, const float* ep, int Kp, int K, const SamplesDev& s, int64_t n,
                                  int64_t chunk, float* resp, hipStream_t st) {
    if (Kp != 128 || K <= 64 || K > 128) return hipErrorInvalidValue;
    constexpr int wpb = 4;
    const int64_t waves = (n + chunk - 1) / chunk;
    const int64_t blocks = (waves + wpb - 1) / wpb;
#define X(V, SB, KT, OCC)                                                                           \
    if (variant == V) {                                                                            \
        hipLaunchKernelGGL((estep_resp_tile_kernel<wpb, SB, KT, OCC>), dim3((unsigned)blocks), dim3(64 * wpb), 0, \
                           st, ep, Kp, K, s, n, chunk, resp);                                     \
        return hipGetLastError();                                                                  \
    }
    SDMM_TILE_VARIANTS(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t estep_resp_tile_occupancy(int variant, int* blocks_per_cu) {
#define X(V, SB, KT, OCC)                                                                           \
    if (variant == V)                                                                              \
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(                                       \
            blocks_per_cu, reinterpret_cast<const void*>(&estep_resp_tile_kernel<4, SB, KT, OCC>), 256, 0);
    SDMM_TILE_VARIANTS(X)
#undef X
    return hipErrorInvalidValue;
}

const char* estep_resp_tile_name(int variant) {
#define X(V, SB, KT, OCC) \
    if (variant == V) return "estep_resp_tile_kernel<4," #SB "," #KT "," #OCC ">";
    SDMM_TILE_VARIANTS(X)
#undef X
    return "estep_resp_tile_kernel<?>";
}

// Tiled statistics kernel (64 < K <= 128, Kp == 128): `blocks` workgroups of 4
// waves, chunk a multiple of 64 samples per wave; one partial row per block.
hipError_t launch_estep_stats_tile(int variant, const float* ep, int Kp, int K, const SamplesDev& s, int64_t n,
                                   int64_t chunk, int blocks, float* partials, int pstride, hipStream_t st,
                                   const LeafDesc* leaves, const int2* items) {
    // one row slot per wave (GROUP: one shared slot)
    const size_t row = sizeof(float) * (size_t)(ST_FIELDS * Kp + 2);
    const size_t lds = (Kp == 128) ? 4 * row : row;
    if (Kp == 128 && K > 64 && K <= 128) {
        if (variant == 1)
            hipLaunchKernelGGL((estep_stats_tile_kernel<4, 3>), dim3(blocks), dim3(256), lds, st, ep, Kp, K, s, n,
                               chunk, partials, pstride, leaves, items);
        else
            hipLaunchKernelGGL((estep_stats_tile_kernel<4, 2>), dim3(blocks), dim3(256), lds, st, ep, Kp, K, s, n,
                               chunk, partials, pstride, leaves, items);
    } else if (Kp == 256 && K > 128 && K <= 256) {
        hipLaunchKernelGGL((estep_stats_tile_kernel<2, 2, true>), dim3(blocks), dim3(128), lds, st, ep, Kp, K, s, n,
                           chunk, partials, pstride, leaves, items);
    } else if (Kp == 512 && K > 256 && K <= 512) {
        hipLaunchKernelGGL((estep_stats_tile_kernel<4, 2, true>), dim3(blocks), dim3(256), lds, st, ep, Kp, K, s, n,
                           chunk, partials, pstride, leaves, items);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
// resident workgroups per CU; *waves_per_wg: the waves of one (GROUP: one chunk)
hipError_t estep_stats_tile_occupancy(int variant, int Kp, int* blocks_per_cu) {
    const size_t row = sizeof(float) * (size_t)(ST_FIELDS * Kp + 2);
    const size_t lds = (Kp == 128) ? 4 * row : row;
    if (Kp == 256)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(
            blocks_per_cu, reinterpret_cast<const void*>(&estep_stats_tile_kernel<2, 2, true>), 128, lds);
    if (Kp == 512)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(
            blocks_per_cu, reinterpret_cast<const void*>(&estep_stats_tile_kernel<4, 2, true>), 256, lds);
    const void* f = variant == 1 ? reinterpret_cast<const void*>(&estep_stats_tile_kernel<4, 3>)
                                 : reinterpret_cast<const void*>(&estep_stats_tile_kernel<4, 2>);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, f, 256, lds);
}

hipError_t launch_estep_stats(int cpl, int lps, const float* ep, int Kp, int K, const SamplesDev& s,
                              int64_t n, int64_t chunk, int blocks, int wpb, float* partials,
                              int pstride, hipStream_t st, const LeafDesc* leaves, const int2* items) {
#define X(C, L)                                                                                    \
    if (cpl == C && lps == L)                                                                      \
        return launch_stats_t<C, L>(ep, Kp, K, s, n, chunk, blocks, wpb, partials, pstride, st, leaves, items);
    SDMM_LAYOUTS(X)
#undef X
    return hipErrorInvalidValue;
}

// Resident workgroups (of 256 threads) per CU for the layout's kernels: the
// E-step launches exactly one chip-full of waves, each walking a contiguous
// chunk, so the loop's dependent packed-FMA chains are covered by as many
// waves per SIMD as the register budget allows.
hipError_t estep_occupancy(int cpl, int lps, int Kp, int* resp_blocks, int* stats_blocks) {
    const size_t lds = sizeof(float) * (size_t)(ST_FIELDS * Kp + 2);
#define X(C, L)                                                                                    \
    if (cpl == C && lps == L) {                                                                    \
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(                               \
            resp_blocks, reinterpret_cast<const void*>(&estep_resp_kernel<C, L>), 256, 0);         \
        if (e != hipSuccess) return e;                                                             \
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(                                       \
            stats_blocks, reinterpret_cast<const void*>(&estep_stats_kernel<C, L>), 256, lds);     \
    }
    SDMM_LAYOUTS(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t launch_reduce_partials(const float* partials, int rows, int pstride, const float* ep_for_finalize,
                                  int Kp, int K, double* stats, hipStream_t st) {
    const int nb = (K + kRedCB - 1) / kRedCB + 1;
    hipLaunchKernelGGL(reduce_uncenter_kernel, dim3(nb), dim3(64 * kReduceSlices), 0, st, partials, rows, pstride,
                       ep_for_finalize, Kp, K, stats);
    return hipGetLastError();
}

}  // namespace sdmm
