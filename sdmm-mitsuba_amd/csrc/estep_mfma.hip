// estep_mfma.hip -- responsibility E-step with the linear forms on the matrix
// cores (gfx950 exact-f32 MFMA) and the nonlinear remainder on the VALU.
//
// Replaces the N x K loop of MixtureModel::posteriorAndLog
// (mitsuba/src/integrators/dmm/jmm/mixture_model.h:146-192) over
// MultivariateTangentNormal::pdfAndLog / TangentSpace::log
// (multivariate_tangent_normal.h:146-177, :350-365).
//
// Per (sample n, component k) the pdf needs eight LINEAR forms of the sample:
//   c   = R2_k . d                      (cos of the angle to the mean direction)
//   ad  = (L33 R0)_k . d,  bd = (L43 R0 + L44 R1)_k . d     (folded directional rows)
//   u_m = sum_j L_mj (p_j - mu_kj),  m = 0..4   (u0..u2 and the spatial parts s3, s4)
// and then the nonlinear part: a = theta/sin(theta) of c, u3 = s3 + a ad,
// u4 = s4 + a bd, q = |u|^2, pi pdf = NORM5 exp(-q/2) * detInv pi * a.
//
// The forms are a dense contraction  F[n][(k,f)] = sum_i X[n][i] B[i][(k,f)]
// with four features per sample: (d0, d1, d2, 0) for the directional forms and
// (p0 - o, p1 - o, p2 - o, 1) for the spatial ones, whose constant term
// -sum_j L_mj (mu_j - o) is folded into the coefficient matrix (o = 0.5, the
// centre of the normalised scene box, createCondition sdmm_proc.cpp:263-273).
// v_mfma_f32_16x16x4_f32 computes it exactly as an f32 fma chain: A = 16
// samples x 4 features (one VGPR per lane), B = 4 features x 16 components of
// one form (one VGPR, resident in LDS), D = 16 x 16 (4 VGPRs).  A round of 8
// MFMAs gives every lane all eight forms of ONE component (col = lane & 15) for
// FOUR samples (rows 4 (lane >> 4) .. +3).  The matrix pipe runs beside the
// VALU, which keeps ~25 scalar f32 ops per pair (angle, exp, norm) instead of
// ~45 packed ones.  The pair math is deliberately NOT packed: on gfx950 a
// v_pk_*_f32 issued beside MFMAs costs more than the two plain ops it replaces
// (MI355X_MICROARCH.md, 'price of one filler beside MFMAs'); this file is
// built with -fno-slp-vectorize so the compiler does not re-pack it.
//
// Normalisation: the lanes of one DPP row hold the same four samples, so the
// posterior normaliser is a DPP row sum of the per-lane partials.  Stores:
// lane (row group sg, col) writes component 16 r + col of rows 4 sg + j, i.e.
// every store instruction writes four 64-byte row segments.
#include "sdmm_device.h"

namespace sdmm {

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr float kLog2Norm5M = -6.628740082514092f;   // log2((float)pow(0.39894228f, 5)), mvtn.h:351-352


template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}

// sum over the 16 lanes of a DPP row; every lane of the row gets the sum
__device__ __forceinline__ float row_sum16(float x) {
    x += dppf<0xB1>(x);    // quad_perm [1,0,3,2]
    x += dppf<0x4E>(x);    // quad_perm [2,3,0,1]
    x += dppf<0x141>(x);   // row_half_mirror
    x += dppf<0x140>(x);   // row_mirror
    return x;
}

// theta / sin(theta) for cos(theta) = c, mvtn.h:157-164 (scalar f32: beside
// MFMAs, packed f32 VALU costs more than two plain ops on gfx950).
//   c >= 0:  h(u), u = (1 - c)/2, h a degree-7 fit of asin(sqrt u)/(sqrt u sqrt(1-u))
//            (5.5e-7 relative on [0, 1/2], tools/fit_angle_over_sin.py); for
//            sin < 1e-3 the reference returns exactly 1 where h(u) is within
//            1.7e-7 of it;
//   c <  0:  theta = pi - theta'  ->  pi / sin(theta) - h(u), u = (1 - |c|)/2.
// RARE (wave-uniform): some lane holds c < -0.9999995 (sin < 1e-3 on the far
// side).  The reference then returns a = 1 (the (sinAngle < 1e-3) quirk), and
// the log map fails for c <= -1 (pdf = 0): clamp(2^30 (c + 1)) is 1 above
// -1 + 2^-30 and 0 at or below -1.
__device__ __forceinline__ float angle_over_sin_m(float c, bool rare) {
    const float s2 = fmaf(-c, c, 1.0f);
    const float u = fmaf(-0.5f, fabsf(c), 0.5f);
    float h = fmaf(3.3755881786346436f, u, -3.17423415184021f);
    h = fmaf(h, u, 2.1241207122802734f);
    h = fmaf(h, u, -0.04515757039189339f);
    h = fmaf(h, u, 0.5178175568580627f);
    h = fmaf(h, u, 0.5294308066368103f);
    h = fmaf(h, u, 0.6667603850364685f);
    h = fmaf(h, u, 0.9999996423721313f);
    const float fneg = fmaf(3.14159265358979f, __builtin_amdgcn_rsqf(s2), -h);
    float f = c < 0.0f ? fneg : h;
    if (rare) {
        const float one = __builtin_amdgcn_fmed3f(1073741824.0f * (c + 1.0f), 0.0f, 1.0f);
        f = (c < 0.0f && s2 < 1e-6f) ? one : f;
    }
    return f;
}

// pi_k pdf_k of one (sample, component) pair from its eight forms.
__device__ __forceinline__ float pair_pdf_m(float c, float ad, float bd, float u0, float u1, float u2, float s3,
                                            float s4, float dipi, bool rare) {
    const float a = angle_over_sin_m(c, rare);
    const float u3 = fmaf(a, ad, s3);
    const float u4 = fmaf(a, bd, s4);
    const float q = fmaf(u4, u4, fmaf(u3, u3, fmaf(u2, u2, fmaf(u1, u1, u0 * u0))));
    // NORM5 exp(-q/2) as one v_exp_f32: 2^(q (-log2(e)/2) + log2 NORM5)
    const float e = __builtin_amdgcn_exp2f(fmaf(q, -0.72134752044448170368f, kLog2Norm5M));
    return e * (dipi * a);   // * detInv * pi_k * jacobian (mvtn.h:361, mixture_model.h:164)
}

// row start of L^-1 row m in the packed lower triangle (EP_L00 ...)
__device__ __forceinline__ int lrow(int m) { return EP_L00 + m * (m + 1) / 2; }

}  // namespace

// Coefficient image of one round r (components 16 r .. 16 r + 15) for lane l:
// B[feature l >> 4][component 16 r + (l & 15)] of the eight forms, as two
// float4 (c, ad, bd, u0 | u1, u2, s3, s4).
__device__ __forceinline__ void coef_for(const float* __restrict__ ep, int Kp, int r, int l, f4& b0, f4& b1) {
    const int k = 16 * r + (l & 15);
    const int kk = l >> 4;
    float v[8];
    if (kk < 3) {
        v[0] = ep[(EP_R20 + kk) * Kp + k];
        v[1] = ep[(EP_A0 + kk) * Kp + k];
        v[2] = ep[(EP_B0 + kk) * Kp + k];
        for (int m = 0; m < 5; ++m)
            v[3 + m] = (m <= 2 && kk > m) ? 0.0f : ep[(lrow(m) + kk) * Kp + k];
    } else {
        v[0] = v[1] = v[2] = 0.0f;
        const double mu[3] = {(double)ep[EP_MU0 * Kp + k] - (double)kOrigin,
                              (double)ep[EP_MU1 * Kp + k] - (double)kOrigin,
                              (double)ep[EP_MU2 * Kp + k] - (double)kOrigin};
        for (int m = 0; m < 5; ++m) {
            double acc = 0.0;
            const int jn = m < 3 ? m + 1 : 3;
            for (int j = 0; j < jn; ++j) acc += (double)ep[(lrow(m) + j) * Kp + k] * mu[j];
            v[3 + m] = (float)(-acc);
        }
    }
    b0 = f4{v[0], v[1], v[2], v[3]};
    b1 = f4{v[4], v[5], v[6], v[7]};
}

template <int R, int OCC>
__global__ void __launch_bounds__(256, OCC)
estep_resp_mfma_kernel(const float* __restrict__ ep, int Kp, int K, SamplesDev s, int64_t n, int64_t chunk,
                       float* __restrict__ resp) {
    __shared__ f4 coef[R][2][64];
    __shared__ float dipi_lds[16 * R];
    for (int idx = threadIdx.x; idx < R * 64; idx += blockDim.x) {
        f4 b0, b1;
        coef_for(ep, Kp, idx >> 6, idx & 63, b0, b1);
        coef[idx >> 6][0][idx & 63] = b0;
        coef[idx >> 6][1][idx & 63] = b1;
    }
    for (int k = threadIdx.x; k < 16 * R; k += blockDim.x) dipi_lds[k] = ep[EP_DIPI * Kp + k];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + wid;
    const int64_t s0 = wave * chunk;
    if (s0 >= n) return;
    const int64_t s1 = (s0 + chunk < n) ? s0 + chunk : n;

    const int fi = lane & 15;        // A operand: sample fi of the tile, feature fk
    const int fk = lane >> 4;
    const int sg = lane >> 4;        // D: samples 4 sg .. 4 sg + 3, component 16 r + col
    const int col = lane & 15;
    const float* pp = fk == 0 ? s.x[0] : (fk == 1 ? s.x[1] : s.x[2]);
    const float* pd = fk == 0 ? s.x[3] : (fk == 1 ? s.x[4] : s.x[5]);
    const bool has_h = s.hpdf != nullptr, has_d = s.isDiffuse != nullptr;

    auto load_feat = [&](int64_t t, float& fs, float& fd) {
        int64_t i = t + fi;
        i = (i < s1) ? i : s1 - 1;
        const float xs = __builtin_nontemporal_load(pp + i);
        const float xd = __builtin_nontemporal_load(pd + i);
        fs = (fk < 3) ? xs - kOrigin : 1.0f;
        fd = (fk < 3) ? xd : 0.0f;
    };

    float nfs, nfd;
    load_feat(s0, nfs, nfd);
    for (int64_t t = s0; t < s1; t += 16) {
        const float fs = nfs, fd = nfd;
        load_feat(t + 16, nfs, nfd);     // next tile in flight (clamped past the end)
        // d == 0 fails every log map (mvtn.h:152-154): bit i set when sample i has d == 0
        const uint64_t zb = __builtin_amdgcn_ballot_w64(fk < 3 && fd == 0.0f);
        const uint32_t dz = (uint32_t)(zb & (zb >> 16) & (zb >> 32)) & 0xffffu;

        float pdf[R][4];
        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        // rare-angle detector: c < -0.9999995 <=> its bits, unsigned, exceed
        // those of -0.9999995f (integer max: no NaN canonicalisation)
        uint32_t cbits = 0;
        // one round: the eight forms of component 16 r + col for samples 4 sg .. +3
        auto round = [&](int r, bool rare, float fs, float fd) __attribute__((always_inline)) {
            const f4 b0 = coef[r][0][lane];
            const f4 b1 = coef[r][1][lane];
            const f4 z = f4{0.0f, 0.0f, 0.0f, 0.0f};
            const f4 C = __builtin_amdgcn_mfma_f32_16x16x4f32(fd, b0.x, z, 0, 0, 0);
            const f4 AD = __builtin_amdgcn_mfma_f32_16x16x4f32(fd, b0.y, z, 0, 0, 0);
            const f4 BD = __builtin_amdgcn_mfma_f32_16x16x4f32(fd, b0.z, z, 0, 0, 0);
            const f4 U0 = __builtin_amdgcn_mfma_f32_16x16x4f32(fs, b0.w, z, 0, 0, 0);
            const f4 U1 = __builtin_amdgcn_mfma_f32_16x16x4f32(fs, b1.x, z, 0, 0, 0);
            const f4 U2 = __builtin_amdgcn_mfma_f32_16x16x4f32(fs, b1.y, z, 0, 0, 0);
            const f4 S3 = __builtin_amdgcn_mfma_f32_16x16x4f32(fs, b1.z, z, 0, 0, 0);
            const f4 S4 = __builtin_amdgcn_mfma_f32_16x16x4f32(fs, b1.w, z, 0, 0, 0);
            const float dp = dipi_lds[16 * r + col];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                cbits = __builtin_elementwise_max(cbits, fbits(C[j]));
                pdf[r][j] = pair_pdf_m(C[j], AD[j], BD[j], U0[j], U1[j], U2[j], S3[j], S4[j], dp, rare);
                acc[j] += pdf[r][j];
            }
        };
#pragma unroll
        for (int r = 0; r < R; ++r) {
            round(r, false, fs, fd);
            // one round's MFMA results live at a time (no hoisting across rounds)
            __builtin_amdgcn_sched_barrier(0);
        }
        // rare angle case anywhere in the tile (c < -0.9999995): redo the tile
        // with the reference's quirks (wave-uniform, a few tiles per launch).
        // The test also reads the fast path's sums (a NaN sum -- NaN input --
        // takes the redo too, harmlessly) so that the compiler cannot sink the
        // fast path below the branch and keep every round's MFMA results live.
        const bool odd = cbits > __builtin_bit_cast(uint32_t, -0.9999995f) ||
                         !(acc[0] + acc[1] + acc[2] + acc[3] >= 0.0f);
        if (__builtin_amdgcn_ballot_w64(odd) != 0) {
            // opaque copies: the redo recomputes its MFMAs instead of keeping
            // the fast path's alive
            float fs2 = fs, fd2 = fd;
            asm volatile("" : "+v"(fs2), "+v"(fd2));
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = 0.0f;
#pragma unroll 1
            for (int r = 0; r < R; ++r) round(r, true, fs2, fd2);
        }
        // posterior normalisation of samples 4 sg + j (mixture_model.h:170-191)
        float S[4] = {row_sum16(acc[0]), row_sum16(acc[1]), row_sum16(acc[2]), row_sum16(acc[3])};
        float g[4];
        bool fin_all = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = 4 * sg + j;
            int64_t si = t + i;
            si = (si < s1) ? si : s1 - 1;
            bool dif = false;
            float hp = 0.0f;
            if (has_d) dif = s.isDiffuse[si] != 0;
            if (has_h) hp = s.hpdf[si];
            const float S2 = dif ? fmaf(1.0f - kHeuristicWeight, S[j], kHeuristicWeight * hp) : S[j];
            const float inv = __builtin_amdgcn_rcpf(S2);
            const bool fin = __builtin_isfinite(inv) && !((dz >> i) & 1u);
            g[j] = fin ? (dif ? inv * (1.0f - kHeuristicWeight) : inv) : 0.0f;
            fin_all = fin_all && __builtin_isfinite(S[j]);
        }
        // a non-finite sum means a non-finite pdf (NaN/inf input): zero rows by select
        const bool bad = __builtin_amdgcn_ballot_w64(!fin_all) != 0;
        const bool full = (t + 16 <= s1) && (16 * R == K);
        float* row0 = resp + (t + 4 * sg) * (int64_t)K + col;
        if (full && !bad) {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(pdf[r][j] * g[j], row0 + j * K + 16 * r);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int k = 16 * r + col;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float o = g[j] != 0.0f ? pdf[r][j] * g[j] : 0.0f;
                    if (k < K && t + 4 * sg + j < s1) __builtin_nontemporal_store(o, row0 + j * K + 16 * r);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Rounds R = Kp / 16 and the register budget (waves per SIMD) of each: the
// default budget per R, and variant v (SDMM_RESP_VARIANT) 1..3 = 2, 3, 4 waves.
#define SDMM_MFMA_CONFIGS(X) \
    X(1, 4) X(2, 4) X(4, 4) X(8, 2) X(8, 3) X(8, 4) X(16, 2) X(16, 3) X(32, 2)

static int mfma_occ(int R, int variant) {
    if (variant >= 1 && variant <= 3) {
        const int o = variant + 1;
        if ((R == 8) || (R == 16 && o <= 3)) return o;
    }
    return R <= 4 ? 4 : (R == 8 ? 3 : 2);
}

hipError_t launch_estep_resp_mfma(int variant, const float* ep, int Kp, int K, const SamplesDev& s, int64_t n,
                                  int64_t chunk, float* resp, hipStream_t st) {
    if (Kp % 16 != 0 || K > Kp || chunk % 16 != 0) return hipErrorInvalidValue;
    const int R = Kp / 16;
    const int occ = mfma_occ(R, variant);
    const int64_t waves = (n + chunk - 1) / chunk;
    const int64_t blocks = (waves + 3) / 4;
#define X(RR, OO)                                                                                      \
    if (R == RR && occ == OO) {                                                                        \
        hipLaunchKernelGGL((estep_resp_mfma_kernel<RR, OO>), dim3((unsigned)blocks), dim3(256), 0, st, ep, Kp, K, \
                           s, n, chunk, resp);                                                         \
        return hipGetLastError();                                                                      \
    }
    SDMM_MFMA_CONFIGS(X)
#undef X
    return hipErrorInvalidValue;
}

hipError_t estep_resp_mfma_occupancy(int variant, int Kp, int* blocks_per_cu) {
    const int R = Kp / 16;
    const int occ = mfma_occ(R, variant);
#define X(RR, OO)                                                                                      \
    if (R == RR && occ == OO)                                                                          \
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(                                           \
            blocks_per_cu, reinterpret_cast<const void*>(&estep_resp_mfma_kernel<RR, OO>), 256, 0);
    SDMM_MFMA_CONFIGS(X)
#undef X
    return hipErrorInvalidValue;
}

const char* estep_resp_mfma_name(int variant, int Kp) {
    static thread_local char buf[64];
    snprintf(buf, sizeof buf, "estep_resp_mfma_kernel<%d,%d>", Kp / 16, mfma_occ(Kp / 16, variant));
    return buf;
}

}  // namespace sdmm
