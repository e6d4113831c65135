// estep.hip -- E-step of the stepwise tangent-space EM on gfx950.
//
// Replaces the N x K hot loop of jmm::StepwiseTangentEM::calculateStats
// (mitsuba/src/integrators/dmm/jmm/opt/stepwise_tangent.h:270-353) and
// MixtureModel::posteriorAndLog (mixture_model.h:146-192) with
// MultivariateTangentNormal::pdfAndLog / TangentSpace::log
// (multivariate_tangent_normal.h:146-177, :350-365).
//
// Work mapping (MI355X-first, not the reference's sample-outer loop):
//   * a wave owns ALL K components: lane j of a lane group holds components
//     j*CPL .. j*CPL+CPL-1 with their 28 parameters in VGPRs for the whole
//     kernel (loaded once, coalesced, from the SoA record ep[f*Kp + k]);
//   * the wave walks a contiguous chunk of samples; with LPS == 64 lanes per
//     sample the sample is wave-uniform and is fetched with scalar (SMEM)
//     loads through the constant address space -- no VGPRs, no LDS;
//   * the posterior normaliser sum_k pi_k pdf_k is a DPP + permlane-swap
//     group reduction (group_sum), one per sample;
//   * STATS: each lane accumulates the 21 sufficient statistics of its own
//     components in registers over the whole chunk (no cross-lane traffic in
//     the loop), then the workgroup folds its waves through LDS in a fixed
//     order and writes one fp32 partial row; reduce_partials sums rows in fp64.
//   * RESP: the normalised responsibilities are stored row-major [N][K]; a
//     wave writes one contiguous K*4-byte row per sample (CPL*4 B per lane).
#include "sdmm_device.h"

namespace sdmm {

// log2(NORMALIZATION) of mvtn.h:351-352, NORMALIZATION = (float)pow(0.39894228f, 5)
constexpr float kLog2Norm5 = -6.628740082514092f;

// theta / sin(theta) for cos(theta) = c in [-1, 1], with the reference's quirk
// `(sinAngle < 1e-3) ? 1 : angle / sinAngle` (mvtn.h:163-164).
//
// The reference computes acos and sqrt separately (~40 VALU ops with the
// libm-grade acosf and the IEEE sqrt expansion).  Here, with u = (1-|c|)/2,
//   acos(|c|) = 2 asin(sqrt(u)),  sin(acos|c|) = 2 sqrt(u) sqrt(1-u),
// so theta'/sin(theta') = g(u) / sqrt(1-u) with g(u) = asin(sqrt u)/sqrt u,
// a smooth function on [0, 1/2] fitted by a degree-7 minimax-style polynomial
// (max rel. error 8.8e-8, tools/fit_angle_over_sin.py).  For c < 0,
// theta = pi - theta' gives (pi - theta')/s = pi/s - theta'/s.  Overall
// <= 4e-7 relative (3 ulp) against the exact value; the fp32 acos/sqrt path
// of the reference is itself 1.8e-7 from exact.  ~16 VALU + 2 v_rsq.
__device__ __forceinline__ float angle_over_sin(float c) {
    const float ac = __builtin_fabsf(c);
    const float u = fmaf(-0.5f, ac, 0.5f);
    float g = 0.1111316829919815f;
    g = fmaf(g, u, -0.09260322898626328f);
    g = fmaf(g, u, 0.07724328339099884f);
    g = fmaf(g, u, 0.01616133376955986f);
    g = fmaf(g, u, 0.04657839611172676f);
    g = fmaf(g, u, 0.07487323880195618f);
    g = fmaf(g, u, 0.1666697859764099f);
    g = fmaf(g, u, 1.0f);
    const float fpos = g * __builtin_amdgcn_rsqf(fmaf(0.5f, ac, 0.5f));
    const float s2 = fmaf(-c, c, 1.0f);
    const float fneg = fmaf(3.14159265358979f, __builtin_amdgcn_rsqf(s2), -fpos);
    const float f = (c < 0.0f) ? fneg : fpos;
    return (s2 < 1e-6f) ? 1.0f : f;
}

template <int CPL>
struct Params {
    float v[CPL][EP_FIELDS];
};

// pi_k * pdf_k(x) (unnormalised posterior) and the directional tangent of the
// sample in component k's frame.  p: sample position, d: sample direction.
template <bool WANT_T>
__device__ __forceinline__ float pair_pdf(const float* __restrict__ P, float p0, float p1, float p2,
                                          float d0, float d1, float d2, bool dvalid, float& t0,
                                          float& t1) {
    const float tp0 = p0 - P[EP_MU0], tp1 = p1 - P[EP_MU1], tp2 = p2 - P[EP_MU2];
    const float r0 = fmaf(P[EP_R02], d2, fmaf(P[EP_R01], d1, P[EP_R00] * d0));
    const float r1 = fmaf(P[EP_R12], d2, fmaf(P[EP_R11], d1, P[EP_R10] * d0));
    const float c = fmaf(P[EP_R22], d2, fmaf(P[EP_R21], d1, P[EP_R20] * d0));
    const bool ok = dvalid && (c > -1.0f);   // log map fails for d == 0 or c <= -1 (mvtn.h:152-159)
    const float cc = (c < 1.0f) ? c : 1.0f;
    const float a = angle_over_sin(cc);
    const float ta = r0 * a, tb = r1 * a;
    const float u0 = P[EP_L00] * tp0;
    const float u1 = fmaf(P[EP_L11], tp1, P[EP_L10] * tp0);
    const float u2 = fmaf(P[EP_L22], tp2, fmaf(P[EP_L21], tp1, P[EP_L20] * tp0));
    const float u3 = fmaf(P[EP_L33], ta, fmaf(P[EP_L32], tp2, fmaf(P[EP_L31], tp1, P[EP_L30] * tp0)));
    const float u4 = fmaf(P[EP_L44], tb, fmaf(P[EP_L43], ta,
                     fmaf(P[EP_L42], tp2, fmaf(P[EP_L41], tp1, P[EP_L40] * tp0))));
    const float q = fmaf(u4, u4, fmaf(u3, u3, fmaf(u2, u2, fmaf(u1, u1, u0 * u0))));
    // NORM5 * exp(-q/2) as one v_exp_f32: 2^(q * -log2(e)/2 + log2(NORM5))
    const float e = __builtin_amdgcn_exp2f(fmaf(q, -0.72134752044448170368f, kLog2Norm5));
    const float pdf = e * (P[EP_DI] * a);     // pdf *= m_detInv * jacobian (mvtn.h:361)
    if constexpr (WANT_T) {
        t0 = ok ? ta : 0.0f;
        t1 = ok ? tb : 0.0f;
    }
    return ok ? P[EP_PI] * pdf : 0.0f;        // m_weights[k] * pdf (mixture_model.h:164)
}

struct SampleVals {
    float x0, x1, x2, x3, x4, x5, w, h;
    bool diffuse;
    __device__ bool dvalid() const { return !(x3 == 0.0f && x4 == 0.0f && x5 == 0.0f); }
};

template <int LPS>
__device__ __forceinline__ SampleVals load_sample(const SamplesDev& s, int64_t i) {
    SampleVals v;
    if constexpr (LPS == 64) {
        v.x0 = ((cfloat_p)s.x[0])[i]; v.x1 = ((cfloat_p)s.x[1])[i]; v.x2 = ((cfloat_p)s.x[2])[i];
        v.x3 = ((cfloat_p)s.x[3])[i]; v.x4 = ((cfloat_p)s.x[4])[i]; v.x5 = ((cfloat_p)s.x[5])[i];
        v.w = ((cfloat_p)s.w)[i];
        v.h = s.hpdf ? ((cfloat_p)s.hpdf)[i] : 0.0f;
        // gfx950 SMEM has no byte load: fetch the aligned dword holding byte i
        // as a scalar load and extract it (a plain u8 load would become a
        // per-sample VMEM load + vmcnt(0) stall).
        if (s.isDiffuse) {
            const uintptr_t a = (uintptr_t)(s.isDiffuse + i);
            const unsigned word = *(const __attribute__((address_space(4))) unsigned*)(a & ~(uintptr_t)3);
            v.diffuse = ((word >> ((a & 3) * 8)) & 0xffu) != 0;
        } else {
            v.diffuse = false;
        }
    } else {
        v.x0 = s.x[0][i]; v.x1 = s.x[1][i]; v.x2 = s.x[2][i];
        v.x3 = s.x[3][i]; v.x4 = s.x[4][i]; v.x5 = s.x[5][i];
        v.w = s.w[i];
        v.h = s.hpdf ? s.hpdf[i] : 0.0f;
        v.diffuse = s.isDiffuse ? (s.isDiffuse[i] != 0) : false;
    }
    return v;
}

// ---------------------------------------------------------------------------
// Responsibility E-step: resp[n*K + k] = posterior_k(x_n) exactly as
// posteriorAndLog returns it (zeros when 1/sum is not finite).
template <int CPL, int LPS>
__global__ void __launch_bounds__(256)
estep_resp_kernel(const float* __restrict__ ep, int Kp, int K, SamplesDev s, int64_t n,
                  int64_t chunk, float* __restrict__ resp) {
    constexpr int SPW = 64 / LPS;
    const int lane = threadIdx.x & 63;
    const int g = lane / LPS;
    const int j = lane % LPS;
    // wave-uniform in an SGPR so that sample addresses stay scalar
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
    const int64_t s0 = wave * chunk;
    if (s0 >= n) return;
    const int64_t s1 = (s0 + chunk < n) ? s0 + chunk : n;

    Params<CPL> P;
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int f = 0; f < EP_FIELDS; ++f) P.v[c][f] = ep[f * Kp + j * CPL + c];

    const int kbase = j * CPL;
    const bool full = ((kbase + CPL) <= K) && (K % CPL == 0);  // aligned vector row store
    for (int64_t base = s0; base < s1; base += SPW) {
        const int64_t i = base + g;
        const bool in = i < s1;
        const SampleVals sv = load_sample<LPS>(s, in ? i : s0);
        const bool dv = sv.dvalid();
        float q[CPL];
        float local = 0.0f;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            float t0, t1;
            q[c] = pair_pdf<false>(P.v[c], sv.x0, sv.x1, sv.x2, sv.x3, sv.x4, sv.x5, dv, t0, t1);
            local += q[c];
        }
        const float S = group_sum<LPS>(local);
        const float S2 = sv.diffuse ? ((1.0f - kHeuristicWeight) * S + kHeuristicWeight * sv.h) : S;
        const float inv = 1.0f / S2;
        const float gsc = __builtin_isfinite(inv) ? (sv.diffuse ? inv * (1.0f - kHeuristicWeight) : inv)
                                                  : 0.0f;
        if (!in) continue;
        float* row = resp + i * (int64_t)K + kbase;
        if constexpr (CPL == 4) {
            if (full) {
                typedef float f4 __attribute__((ext_vector_type(4)));
                f4 o = {q[0] * gsc, q[1] * gsc, q[2] * gsc, q[3] * gsc};
                __builtin_nontemporal_store(o, (f4*)row);
                continue;
            }
        } else if constexpr (CPL == 2) {
            if (full) {
                typedef float f2 __attribute__((ext_vector_type(2)));
                f2 o = {q[0] * gsc, q[1] * gsc};
                __builtin_nontemporal_store(o, (f2*)row);
                continue;
            }
        }
#pragma unroll
        for (int c = 0; c < CPL; ++c)
            if (kbase + c < K) __builtin_nontemporal_store(q[c] * gsc, row + c);
    }
}

// ---------------------------------------------------------------------------
// Fused E-step + sufficient statistics (calculateStats + sumWeights).
// partial row layout: [f*Kp + k] for f < ST_FIELDS, then [21Kp] = H, [21Kp+1] = wsum.
template <int CPL, int LPS>
__global__ void __launch_bounds__(256)
estep_stats_kernel(const float* __restrict__ ep, int Kp, int K, SamplesDev s, int64_t n,
                   int64_t chunk, float* __restrict__ partials, int pstride) {
    constexpr int SPW = 64 / LPS;
    extern __shared__ __attribute__((aligned(16))) float red[];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    const int g = lane / LPS;
    const int j = lane % LPS;
    const int64_t wave = (int64_t)blockIdx.x * nw + wid;
    const int64_t s0 = wave * chunk;
    const int64_t s1 = (s0 + chunk < n) ? s0 + chunk : n;  // s1 <= s0: no samples

    Params<CPL> P;
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int f = 0; f < EP_FIELDS; ++f) P.v[c][f] = ep[f * Kp + j * CPL + c];

    float acc[CPL][ST_FIELDS];
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int f = 0; f < ST_FIELDS; ++f) acc[c][f] = 0.0f;
    float accH = 0.0f, accWs = 0.0f;

    for (int64_t base = s0; base < s1; base += SPW) {
        const int64_t i = base + g;
        const bool in = i < s1;
        const SampleVals sv = load_sample<LPS>(s, in ? i : s0);
        const bool finite_w = __builtin_isfinite(sv.w);
        // sumWeights counts every finite weight (stepwise_tangent.h:462-475)
        accWs += (in && finite_w) ? sv.w : 0.0f;
        // calculateStats skips non-finite and zero weights (:288-293)
        const bool use = in && finite_w && (sv.w != 0.0f);
        const bool dv = sv.dvalid();
        float q[CPL], ta[CPL], tb[CPL];
        float local = 0.0f;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            q[c] = pair_pdf<true>(P.v[c], sv.x0, sv.x1, sv.x2, sv.x3, sv.x4, sv.x5, dv, ta[c], tb[c]);
            local += q[c];
        }
        const float S = group_sum<LPS>(local);
        const float S2 = sv.diffuse ? ((1.0f - kHeuristicWeight) * S + kHeuristicWeight * sv.h) : S;
        const float inv = 1.0f / S2;
        const bool fin = __builtin_isfinite(inv);
        const float gsc = fin ? (sv.diffuse ? inv * (1.0f - kHeuristicWeight) : inv) : 0.0f;
        const float w = use ? sv.w : 0.0f;
        const float hpost = (fin && sv.diffuse) ? kHeuristicWeight * sv.h * inv : 0.0f;
        accH = fmaf(w, hpost, accH);
        // Spatial statistics are accumulated centred on the component's mean
        // position (tp = p - mu_k, already formed by pair_pdf) and un-centred in
        // fp64 by finalize_stats_kernel: the M-step's C/W - mu mu^T then does
        // not amplify fp32 accumulation error by |p|^2 / sigma^2.
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const float gam = q[c] * gsc;
            // posterior < 1e-10 is skipped (:312); unused samples have w == 0
            const float v = (gam < 1e-10f || !use) ? 0.0f : w * gam;
            const float tp0 = sv.x0 - P.v[c][EP_MU0];
            const float tp1 = sv.x1 - P.v[c][EP_MU1];
            const float tp2 = sv.x2 - P.v[c][EP_MU2];
            float* A = acc[c];
            A[ST_W] += v;
            const float v0 = v * tp0, v1 = v * tp1, v2 = v * tp2;
            A[ST_M0] += v0;
            A[ST_M1] += v1;
            A[ST_M2] += v2;
            const float v3 = v * ta[c], v4 = v * tb[c];
            A[ST_M3] += v3;
            A[ST_M4] += v4;
            A[ST_C00] = fmaf(v0, tp0, A[ST_C00]);
            A[ST_C10] = fmaf(v1, tp0, A[ST_C10]);
            A[ST_C11] = fmaf(v1, tp1, A[ST_C11]);
            A[ST_C20] = fmaf(v2, tp0, A[ST_C20]);
            A[ST_C21] = fmaf(v2, tp1, A[ST_C21]);
            A[ST_C22] = fmaf(v2, tp2, A[ST_C22]);
            A[ST_C30] = fmaf(v3, tp0, A[ST_C30]);
            A[ST_C31] = fmaf(v3, tp1, A[ST_C31]);
            A[ST_C32] = fmaf(v3, tp2, A[ST_C32]);
            A[ST_C33] = fmaf(v3, ta[c], A[ST_C33]);
            A[ST_C40] = fmaf(v4, tp0, A[ST_C40]);
            A[ST_C41] = fmaf(v4, tp1, A[ST_C41]);
            A[ST_C42] = fmaf(v4, tp2, A[ST_C42]);
            A[ST_C43] = fmaf(v4, ta[c], A[ST_C43]);
            A[ST_C44] = fmaf(v4, tb[c], A[ST_C44]);
        }
    }

    // fold the lane groups of this wave holding the same components
    if constexpr (SPW > 1) {
#pragma unroll
        for (int off = LPS; off < 64; off <<= 1) {
#pragma unroll
            for (int c = 0; c < CPL; ++c)
#pragma unroll
                for (int f = 0; f < ST_FIELDS; ++f) acc[c][f] += __shfl_xor(acc[c][f], off);
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
            for (int c = 0; c < CPL; ++c)
#pragma unroll
                for (int f = 0; f < ST_FIELDS; ++f) {
                    const int idx = f * Kp + j * CPL + c;
                    red[idx] = (w == 0) ? acc[c][f] : red[idx] + acc[c][f];
                }
            if (lane == 0) {
                red[ST_FIELDS * Kp] = (w == 0) ? accH : red[ST_FIELDS * Kp] + accH;
                red[ST_FIELDS * Kp + 1] = (w == 0) ? accWs : red[ST_FIELDS * Kp + 1] + accWs;
            }
        }
        __syncthreads();
    }
    float* out = partials + (int64_t)blockIdx.x * pstride;
    for (int idx = threadIdx.x; idx < rowlen; idx += blockDim.x) out[idx] = red[idx];
}

// ---------------------------------------------------------------------------
// Deterministic fp64 reduction of the partial rows into the compact stats
// vector [H, wsum, W(K), M(5K), Clow(15K)].  One workgroup per 64 output
// columns; its 16 waves split the rows, then combine in a fixed order.
__global__ void __launch_bounds__(1024)
reduce_partials_kernel(const float* __restrict__ partials, int rows, int pstride, int Kp, int K,
                       double* __restrict__ stats) {
    __shared__ double buf[16][64];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int ncols = 2 + ST_FIELDS * K;
    const int o = blockIdx.x * 64 + lane;
    int col = -1;
    if (o < ncols) {
        if (o == 0) col = ST_FIELDS * Kp;
        else if (o == 1) col = ST_FIELDS * Kp + 1;
        else {
            const int r = o - 2;
            if (r < K) col = ST_W * Kp + r;
            else if (r < 6 * K) { const int q = r - K; col = (ST_M0 + q % 5) * Kp + q / 5; }
            else { const int q = r - 6 * K; col = (ST_C00 + q % 15) * Kp + q / 15; }
        }
    }
    double sum = 0.0;
    if (col >= 0) {
        int r = wid;
        for (; r + 48 < rows; r += 64) {
            const float a = partials[(int64_t)r * pstride + col];
            const float b = partials[(int64_t)(r + 16) * pstride + col];
            const float c = partials[(int64_t)(r + 32) * pstride + col];
            const float d = partials[(int64_t)(r + 48) * pstride + col];
            sum += (double)a; sum += (double)b; sum += (double)c; sum += (double)d;
        }
        for (; r < rows; r += 16) sum += (double)partials[(int64_t)r * pstride + col];
    }
    buf[wid][lane] = sum;
    __syncthreads();
    if (wid == 0 && o < ncols) {
        double t = 0.0;
        for (int w = 0; w < 16; ++w) t += buf[w][lane];
        stats[o] = t;
    }
}

// Un-centre the spatial statistics of component k (fp64, in place):
//   M_p = M'_p + W mu,  C_pp = C'_pp + M'_p mu^T + mu M'_p^T + W mu mu^T,
//   C_tp = C'_tp + M_t mu^T   (mu = the float mean the E-step subtracted).
__global__ void finalize_stats_kernel(const float* __restrict__ ep, int Kp, int K,
                                      double* __restrict__ stats) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    double* W = stats + 2 + k;
    double* M = stats + 2 + K + 5 * k;
    double* C = stats + 2 + 6 * K + 15 * k;   // lower triangle, row-major
    const double mu[3] = {(double)ep[EP_MU0 * Kp + k], (double)ep[EP_MU1 * Kp + k],
                          (double)ep[EP_MU2 * Kp + k]};
    const double w = *W;
    const double mp[3] = {M[0], M[1], M[2]};
    // C_pp (entries 0..5: (0,0) (1,0) (1,1) (2,0) (2,1) (2,2))
    int e = 0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j <= i; ++j, ++e)
            C[e] += mp[i] * mu[j] + mu[i] * mp[j] + w * mu[i] * mu[j];
    // C_tp: rows 3, 4 (entries 6..8 and 10..12)
    for (int j = 0; j < 3; ++j) {
        C[6 + j] += M[3] * mu[j];
        C[10 + j] += M[4] * mu[j];
    }
    for (int i = 0; i < 3; ++i) M[i] = mp[i] + w * mu[i];
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
                                 hipStream_t st) {
    const size_t lds = sizeof(float) * (size_t)(ST_FIELDS * Kp + 2);
    hipLaunchKernelGGL((estep_stats_kernel<CPL, LPS>), dim3(blocks), dim3(64 * wpb), lds, st,
                       ep, Kp, K, s, n, chunk, partials, pstride);
    return hipGetLastError();
}

hipError_t launch_estep_resp(int cpl, int lps, const float* ep, int Kp, int K, const SamplesDev& s,
                             int64_t n, int64_t chunk, float* resp, hipStream_t st) {
    if (lps == 64) {
        switch (cpl) {
            case 1: return launch_resp_t<1, 64>(ep, Kp, K, s, n, chunk, resp, st);
            case 2: return launch_resp_t<2, 64>(ep, Kp, K, s, n, chunk, resp, st);
            case 4: return launch_resp_t<4, 64>(ep, Kp, K, s, n, chunk, resp, st);
            case 8: return launch_resp_t<8, 64>(ep, Kp, K, s, n, chunk, resp, st);
        }
    } else if (lps == 32 && cpl == 1) {
        return launch_resp_t<1, 32>(ep, Kp, K, s, n, chunk, resp, st);
    } else if (lps == 16 && cpl == 1) {
        return launch_resp_t<1, 16>(ep, Kp, K, s, n, chunk, resp, st);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_estep_stats(int cpl, int lps, const float* ep, int Kp, int K, const SamplesDev& s,
                              int64_t n, int64_t chunk, int blocks, int wpb, float* partials,
                              int pstride, hipStream_t st) {
    if (lps == 64) {
        switch (cpl) {
            case 1: return launch_stats_t<1, 64>(ep, Kp, K, s, n, chunk, blocks, wpb, partials, pstride, st);
            case 2: return launch_stats_t<2, 64>(ep, Kp, K, s, n, chunk, blocks, wpb, partials, pstride, st);
            case 4: return launch_stats_t<4, 64>(ep, Kp, K, s, n, chunk, blocks, wpb, partials, pstride, st);
            case 8: return launch_stats_t<8, 64>(ep, Kp, K, s, n, chunk, blocks, wpb, partials, pstride, st);
        }
    } else if (lps == 32 && cpl == 1) {
        return launch_stats_t<1, 32>(ep, Kp, K, s, n, chunk, blocks, wpb, partials, pstride, st);
    } else if (lps == 16 && cpl == 1) {
        return launch_stats_t<1, 16>(ep, Kp, K, s, n, chunk, blocks, wpb, partials, pstride, st);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_reduce_partials(const float* partials, int rows, int pstride, const float* ep_for_finalize,
                                  int Kp, int K,
                                  double* stats, hipStream_t st) {
    const int ncols = 2 + ST_FIELDS * K;
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((ncols + 63) / 64), dim3(1024), 0, st,
                       partials, rows, pstride, Kp, K, stats);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(finalize_stats_kernel, dim3((K + 255) / 256), dim3(256), 0, st, ep_for_finalize,
                       Kp, K, stats);
    return hipGetLastError();
}

}  // namespace sdmm
