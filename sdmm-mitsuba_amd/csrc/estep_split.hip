// estep_split.hip -- responsibility E-step with the eight linear forms on the
// bf16 matrix cores, exact to fp32 by a three-way bf16 split of both operands.
//
// Replaces the N x K loop of MixtureModel::posteriorAndLog
// (mitsuba/src/integrators/dmm/jmm/mixture_model.h:146-192) over
// MultivariateTangentNormal::pdfAndLog / TangentSpace::log
// (multivariate_tangent_normal.h:146-177, :350-365), like estep_resp_tile_kernel
// (estep.hip) and with the same pair formula; only the linear forms move.
//
// Per (sample n, component k) the pdf needs eight LINEAR forms of the sample
// (estep_mfma.hip header): c = R2.d, ad = (L33 R0).d, bd = (L43 R0 + L44 R1).d,
// and u_m = sum_j L_mj (p_j - o) + NC_m, m = 0..4 (o = kOrigin, NC_m = EP_NC*).
// In the VALU tile kernel they are 21 of the 42 packed FMAs per pair.  Here
// they are v_mfma_f32_16x16x32_bf16 products D[16 samples][16 components] =
// A[16][32] . B[32][16], one MFMA per form and 16 x 16 block:
//
//   * every fp32 operand x is split exactly into three bf16 x = h + m + l
//     (round-to-nearest h, then m of the exact remainder x - h, then l of the
//     exact remainder, which has at most 8 significant bits left);
//   * a product c x is the six largest of the nine split products,
//     hc.h + mc.h + hc.m + lc.h + hc.l + mc.m, each exact in the fp32
//     accumulator; the three dropped ones are below 2^-25 |c x| together (half
//     an fp32 ulp), so every form carries fp32-level error like the FMA chain
//     it replaces (the responsibility bound of tests/test_gpu_parity.py
//     _check_resp holds, as for the f32 MFMA kernel);
//   * the K = 32 reduction of one MFMA holds one feature per 8-lane k group:
//     lane group g = lane >> 4 (g < 3) owns feature g, its eight k entries
//     pair A = [h h m h l m e6 e7] of the sample with B = [hc mc hc lc hc mc
//     X6 X7] of the coefficient; the spatial forms put their constant NC_m in
//     e6/e7 = 1 and X6/X7 = NC's split (group 0: h, m; group 1: l), group 3 is
//     zero.  Building one A fragment is 7 VALU per 16 samples;
//   * the rows of u (spatial forms, ad, bd) carry the factor sqrt(log2(e)/2)
//     (fp64 product rounded to fp32 before the split), so the exponent of
//     NORM5 exp(-q/2) is one FMA chain (pdf_pair).
//
// The B image of the whole mixture (R = Kp/16 blocks x 8 forms x 64 lanes x 16
// B = R x 8 KB, 64 KB at K = 128) is built in LDS by each workgroup from the
// E-step record and read as one ds_read_b128 per fragment, conflict-free.  The
// D layout gives each lane one component (col = lane & 15) of four samples
// (rows 4 (lane >> 4) + j); the nonlinear rest of the pair math (angle, exp,
// pdf) runs packed over sample pairs (j, j+1), the posterior normaliser is a
// DPP row sum, and a store writes four 64-byte row segments.
#include "sdmm_device.h"

namespace sdmm {

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

template <bool B> struct Tag { static constexpr bool value = B; };

constexpr float kLog2Norm5S = -6.628740082514092f;   // log2((float)pow(0.39894228f, 5)), mvtn.h:351-352

__device__ __forceinline__ f2 spl(float x) { return (f2)(x); }
#ifdef SDMM_SPLIT_SCALAR
// A/B build: the pair math as plain VOP3 f32 (no packed f32 beside the MFMAs)
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return f2{fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)}; }
__device__ __forceinline__ f2 pmul(f2 a, f2 b) { return f2{a.x * b.x, a.y * b.y}; }
__device__ __forceinline__ f2 padd(f2 a, f2 b) { return f2{a.x + b.x, a.y + b.y}; }
#else
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 pmul(f2 a, f2 b) { return a * b; }
__device__ __forceinline__ f2 padd(f2 a, f2 b) { return a + b; }
#endif

// two floats -> one dword of two bf16 (round to nearest even): element 0 (lo)
// in bits 0..15, element 1 (hi) in bits 16..31 (v_cvt_pk_bf16_f32)
__device__ __forceinline__ unsigned pk(float lo, float hi) {
    const bf2 v = __builtin_convertvector(f2{lo, hi}, bf2);
    return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ float hi_of(unsigned d) { return __builtin_bit_cast(float, d & 0xFFFF0000u); }
__device__ __forceinline__ float lo_of(unsigned d) { return __builtin_bit_cast(float, d << 16); }

// Split x into (h, m, l) bf16 parts as floats' dwords: see the header.
// Sample fragment of one lane (K layout in the header): lane group g < 3 holds
// the small products of feature g, [h m h l m e5 e6 0]; group 3 holds the
// three large ones and the constant's largest part, [0 0 0 0 x0h x1h x2h e7].
// x: the sample's three features; spatial: the forms with the constant NC.
__device__ __forceinline__ bf8 a_frag(const float (&x)[3], int g, bool spatial) {
    const float xg = g == 0 ? x[0] : (g == 1 ? x[1] : x[2]);   // (g < 3)
    const unsigned t = pk(xg, xg);
    const float r1 = xg - hi_of(t);               // exact
    const unsigned d0 = pk(xg, r1);               // (h, m)
    const float r2 = r1 - hi_of(d0);              // exact, <= 8 significant bits
    const unsigned d1 = pk(xg, r2);               // (h, l)
    const bool cst = spatial && g == 0;
    const unsigned d2 = pk(r1, cst ? 1.0f : 0.0f);   // (m, e5)
    const unsigned d3 = cst ? 0x3F80u : 0u;          // (e6, 0)
    const unsigned q2 = pk(x[0], x[1]);              // (x0h, x1h)
    const unsigned q3 = pk(x[2], spatial ? 1.0f : 0.0f);   // (x2h, e7)
    return __builtin_bit_cast(bf8, g < 3 ? u4{d0, d1, d2, d3} : u4{0u, 0u, q2, q3});
}

// (h, m, l) of an fp32 value as bf16 bit patterns
__device__ __forceinline__ void split3(float c, unsigned& h, unsigned& m, unsigned& l) {
    const unsigned hh = pk(c, c);
    const float r1 = c - hi_of(hh);
    const unsigned mm = pk(r1, r1);
    const float r2 = r1 - lo_of(mm);
    const unsigned ll = pk(r2, r2);
    h = hh & 0xFFFFu;
    m = mm & 0xFFFFu;
    l = ll & 0xFFFFu;
}

// sqrt(log2(e) / 2): the rows of u (spatial forms, ad, bd) are pre-scaled by
// it, so that the exponent 2^(log2 NORM5 - |u'|^2) = NORM5 exp(-q/2) is one
// FMA chain from the constant (no separate q and scaling step)
#ifdef SDMM_SPLIT_NOROWSCALE
constexpr bool kFoldScale = false;
constexpr double kRowScale = 1.0;
#else
constexpr bool kFoldScale = true;
constexpr double kRowScale = 0.84932180028801904272;
#endif

// row start of L^-1 row m in the packed lower triangle (EP_L00 ...)
__device__ __forceinline__ int lrow(int m) { return EP_L00 + m * (m + 1) / 2; }

// Spatial origin of block r (components 16 r .. 16 r + 15): the mean of the
// block's finite component means (kOrigin if none).  The spatial forms are
// u_m = sum_j L_mj (p_j - o_r) + NC_m(o_r); with o_r near the block's
// components the two terms stay small for the samples whose pdfs matter (the
// MFMA accumulation error scales with them; a single scene-centre origin left
// the heuristic row sums at 1.2e-5 of the fp64 evaluation instead of 4e-6).
#ifdef SDMM_SPLIT_BLOCKORIGIN
#ifdef SDMM_SPLIT_PIPE
#error "SDMM_SPLIT_PIPE uses the one scene-centre origin"
#endif
constexpr bool kBlockOrigin = true;
#else
constexpr bool kBlockOrigin = false;
#endif
__device__ __forceinline__ void block_origin(const float* __restrict__ ep, int Kp, int r, float* o) {
    if (!kBlockOrigin) {
        o[0] = o[1] = o[2] = kOrigin;
        return;
    }
    double acc[3] = {0.0, 0.0, 0.0};
    int cnt = 0;
    for (int i = 0; i < 16; ++i) {
        const int k = 16 * r + i;
        const float m0 = ep[EP_MU0 * Kp + k], m1 = ep[EP_MU1 * Kp + k], m2 = ep[EP_MU2 * Kp + k];
        if (!(fabsf(m0) < 1e6f && fabsf(m1) < 1e6f && fabsf(m2) < 1e6f)) continue;
        acc[0] += m0;
        acc[1] += m1;
        acc[2] += m2;
        ++cnt;
    }
    for (int j = 0; j < 3; ++j) o[j] = cnt ? (float)(acc[j] / cnt) : kOrigin;
}

// Coefficient fragment of block r, form f, lane l (the A operand of the
// MFMA; K layout in the header): lane group g < 3 pairs feature g's small
// products, [cm ch cl ch cm X5 X6 0] with X5, X6 = NC's l, m parts in group 0
// of the spatial forms; group 3 holds [0 0 0 0 c0h c1h c2h X7], X7 = NC's h
// part.  Forms: 0 c (R2), 1 ad (A), 2 bd (B), 3 + m the spatial row m
// (L_m0..L_m2 of L^-1, constant NC_m(o) = -sum_j L_mj (mu_j - o) in fp64).
__device__ __forceinline__ u4 coef_frag(const float* __restrict__ ep, int Kp, int r, int f, int l,
                                        const float* __restrict__ o) {
    const int k = 16 * r + (l & 15);
    const int g = l >> 4;
    float c[3];
    unsigned nh = 0u, nm = 0u, nl = 0u;
    if (f < 3) {
        const int base = f == 0 ? EP_R20 : (f == 1 ? EP_A0 : EP_B0);
        for (int j = 0; j < 3; ++j) {
            c[j] = ep[(base + j) * Kp + k];
            if (f > 0) c[j] = (float)((double)c[j] * kRowScale);
        }
    } else {
        const int m = f - 3;
        double acc = 0.0;
        for (int j = 0; j < 3; ++j) {
            const bool z = m <= 2 && j > m;
            c[j] = z ? 0.0f : (float)((double)ep[(lrow(m) + j) * Kp + k] * kRowScale);
            if (!z) acc += (double)ep[(lrow(m) + j) * Kp + k] * ((double)ep[(EP_MU0 + j) * Kp + k] - (double)o[j]);
        }
        split3((float)(-acc * kRowScale), nh, nm, nl);
    }
    if (g < 3) {
        unsigned h, m, lo;
        split3(c[g], h, m, lo);
        const unsigned x5 = g == 0 ? nl : 0u, x6 = g == 0 ? nm : 0u;
        return u4{m | (h << 16), lo | (h << 16), m | (x5 << 16), x6};
    }
    unsigned h0, h1, h2, t1, t2;
    split3(c[0], h0, t1, t2);
    split3(c[1], h1, t1, t2);
    split3(c[2], h2, t1, t2);
    return u4{0u, 0u, h0 | (h1 << 16), h2 | (nh << 16)};
}

// sum over the 16 lanes of a DPP row; every lane of the row gets the sum
template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float x) {
    x += dppf<0xB1>(x);    // quad_perm [1,0,3,2]
    x += dppf<0x4E>(x);    // quad_perm [2,3,0,1]
    x += dppf<0x141>(x);   // row_half_mirror
    x += dppf<0x140>(x);   // row_mirror
    return x;
}

// pi_k pdf_k of the four (sample, component) pairs of one D fragment, as two
// packed pairs (rows j, j+1) advanced in lockstep (two independent chains per
// step: no dependency wait states between the packed FMAs), from the eight
// row-scaled forms u' = sqrt(log2(e)/2) u, so NORM5 exp(-q/2) =
// 2^(log2 NORM5 - |u'|^2) (estep.hip pair_q_tile).  The angle is
// estep.hip angle_over_sin_main's (degree-7 h(u), pi/sqrt(1-c^2) - h(u) for
// c < 0); RARE adds the reference's quirks (mvtn.h:157-164) for the far side:
// a = 1 where sin < 1e-3, a = 0 (failed log map) at c <= -1.
template <bool RARE>
__device__ __forceinline__ void pdf_quad(const f4& C, const f4& AD, const f4& BD, const f4& U0, const f4& U1,
                                         const f4& U2, const f4& S3, const f4& S4, const f4& dipi, f2 (&p)[2]) {
    f2 c[2], s2[2], u[2], h[2], a[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) c[i] = f2{C[2 * i], C[2 * i + 1]};
#pragma unroll
    for (int i = 0; i < 2; ++i) s2[i] = pfma(-c[i], c[i], spl(1.0f));
    // u = (1 - |c|)/2 as VOP3 FMAs with the |.| source modifier (packed FMAs
    // have none; this file is built with -fno-slp-vectorize so the compiler
    // does not re-pack them as v_and + v_pk_fma).  Not inline asm: the
    // compiler's MFMA-result hazard waits do not cover asm operands.
#pragma unroll
    for (int i = 0; i < 2; ++i) u[i] = f2{fmaf(-0.5f, fabsf(c[i].x), 0.5f), fmaf(-0.5f, fabsf(c[i].y), 0.5f)};
    constexpr float kH[8] = {3.3755881786346436f, -3.17423415184021f, 2.1241207122802734f, -0.04515757039189339f,
                             0.5178175568580627f, 0.5294308066368103f, 0.6667603850364685f, 0.9999996423721313f};
#pragma unroll
    for (int i = 0; i < 2; ++i) h[i] = pfma(spl(kH[0]), u[i], spl(kH[1]));
#pragma unroll
    for (int t = 2; t < 8; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i) h[i] = pfma(h[i], u[i], spl(kH[t]));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const f2 r = f2{__builtin_amdgcn_rsqf(s2[i].x), __builtin_amdgcn_rsqf(s2[i].y)};
        const f2 fneg = pfma(spl(3.14159265358979f), r, -h[i]);
        a[i] = f2{c[i].x < 0.0f ? fneg.x : h[i].x, c[i].y < 0.0f ? fneg.y : h[i].y};
        if constexpr (RARE) {
            const float o0 = __builtin_amdgcn_fmed3f(1073741824.0f * (c[i].x + 1.0f), 0.0f, 1.0f);
            const float o1 = __builtin_amdgcn_fmed3f(1073741824.0f * (c[i].y + 1.0f), 0.0f, 1.0f);
            a[i].x = (c[i].x < 0.0f && s2[i].x < 1e-6f) ? o0 : a[i].x;
            a[i].y = (c[i].y < 0.0f && s2[i].y < 1e-6f) ? o1 : a[i].y;
        }
    }
    f2 arg[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const f2 u0 = f2{U0[2 * i], U0[2 * i + 1]};
        arg[i] = kFoldScale ? pfma(-u0, u0, spl(kLog2Norm5S)) : pmul(u0, u0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const f2 u1 = f2{U1[2 * i], U1[2 * i + 1]};
        arg[i] = kFoldScale ? pfma(-u1, u1, arg[i]) : pfma(u1, u1, arg[i]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const f2 u2 = f2{U2[2 * i], U2[2 * i + 1]};
        arg[i] = kFoldScale ? pfma(-u2, u2, arg[i]) : pfma(u2, u2, arg[i]);
    }
    f2 u3[2], u4[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        u3[i] = pfma(a[i], f2{AD[2 * i], AD[2 * i + 1]}, f2{S3[2 * i], S3[2 * i + 1]});
        u4[i] = pfma(a[i], f2{BD[2 * i], BD[2 * i + 1]}, f2{S4[2 * i], S4[2 * i + 1]});
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) arg[i] = kFoldScale ? pfma(-u3[i], u3[i], arg[i]) : pfma(u3[i], u3[i], arg[i]);
#pragma unroll
    for (int i = 0; i < 2; ++i) arg[i] = kFoldScale ? pfma(-u4[i], u4[i], arg[i]) : pfma(u4[i], u4[i], arg[i]);
    if constexpr (!kFoldScale) {
#pragma unroll
        for (int i = 0; i < 2; ++i) arg[i] = pfma(arg[i], spl(-0.72134752044448170368f), spl(kLog2Norm5S));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const f2 e = f2{__builtin_amdgcn_exp2f(arg[i].x), __builtin_amdgcn_exp2f(arg[i].y)};
        p[i] = pmul(e, pmul(f2{dipi[2 * i], dipi[2 * i + 1]}, a[i]));   // * detInv * pi_k * jacobian (mvtn.h:361, mixture_model.h:164)
    }
}

}  // namespace

// LDS rows (K = 128): each block's unnormalised pdfs go to the
// wave's LDS row stage as soon as they are formed (whole rows, 8 KB per wave)
// instead of living in 32 VGPRs until the tile's normaliser is known; the
// flush scales them on the way out.  The freed registers allow 3 waves per
// SIMD (12-wave workgroups: 96 KB of stage + the 64 KB coefficient image fill
// the 160 KB LDS, so detInv pi is then read from the E-step record instead).
// (an option, SDMM_SPLIT_LDSROWS; round 4, four processes each on one box:
// 177.5-180.6 us per launch against 175.7-176.9 us with the pdfs in registers
// until the flush at the same 12-wave / 3-per-SIMD configuration, the default)
#ifdef SDMM_SPLIT_LDSROWS
constexpr bool kLdsRowsOn = true;
#else
constexpr bool kLdsRowsOn = false;
#endif

// the default block loop's scheduling fences (SDMM_SPLIT_NOFENCE, A/B: the
// compiler schedules the MFMAs, the fragment reads and the pair math freely)
#ifdef SDMM_SPLIT_NOFENCE
#define SPLIT_FENCE() ((void)0)
#else
#define SPLIT_FENCE() __builtin_amdgcn_sched_barrier(0)
#endif
template <int R, int WPB, int OCC>
__global__ void __launch_bounds__(64 * WPB, OCC)
estep_resp_split_kernel(const float* __restrict__ ep, int Kp, int K, SamplesDev s, int64_t n, int64_t nwaves,
                        float* __restrict__ resp) {
    constexpr bool LR = kLdsRowsOn && R == 8;
    constexpr bool DIMG = !LR || (WPB * 16 * 32 * 16 + R * 8 * 64 * 16 + R * 4 * 16 <= 163840);
    // coefficient fragments (R blocks x 8 forms x 64 lanes) and detInv pi of
    // components 16 r + 4 g .. +3 (the D rows of lane group g)
    // one LDS block carved into the coefficient image, the per-wave row
    // stages (16 rows x 512 B with LR, else 256-B half rows), detInv pi and
    // the block origins (only the parts the configuration uses)
    constexpr int NC = R * 8 * 64, NS = LR ? 16 * 32 : 16 * 16, ND = DIMG ? R * 4 : 0, NB = kBlockOrigin ? R : 0;
    __shared__ u4 smem[NC + WPB * NS + ND + NB];
    u4* const cimg = smem;
    f4* const stage0 = (f4*)(smem + NC);
    f4* const dimg = (f4*)(smem + NC + WPB * NS);
    float (*const borig)[4] = (float (*)[4])(smem + NC + WPB * NS + ND);
    if (kBlockOrigin && threadIdx.x < R) block_origin(ep, Kp, threadIdx.x, borig[threadIdx.x]);
    __syncthreads();
    // (without per-block origins every block's spatial forms use the one
    // scene-centre origin kOrigin; borig then has no storage)
    const float o_scene[3] = {kOrigin, kOrigin, kOrigin};
#ifdef SDMM_SPLIT_DIAG_NOIMAGE   // (diagnostic: a zero coefficient image -- results are not responsibilities)
    for (int idx = threadIdx.x; idx < NC + WPB * NS + ND; idx += 64 * WPB) smem[idx] = u4{0u, 0u, 0u, 0u};
#else
    for (int idx = threadIdx.x; idx < R * 8 * 64; idx += 64 * WPB)
        cimg[idx] = coef_frag(ep, Kp, idx >> 9, (idx >> 6) & 7, idx & 63, kBlockOrigin ? borig[idx >> 9] : o_scene);
    if constexpr (DIMG)
        for (int i = threadIdx.x; i < R * 4; i += 64 * WPB) {
            const float* d = ep + EP_DIPI * Kp + 4 * i;
            dimg[i] = f4{d[0], d[1], d[2], d[3]};
        }
#endif
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wave = (int64_t)blockIdx.x * WPB + wid;
    // the launch's 16-sample tiles dealt round robin over its waves (one round
    // of resident waves: each workgroup builds the coefficient image once):
    // wave w serves tiles w, w + nwaves, ..., so the waves running at one time
    // write neighbouring 8-KB row blocks.  (A contiguous range per wave put the
    // 2048 waves' concurrent rows 256 KB apart -- the same HBM channel bits --
    // and one configuration ran 170-190 or 340-370 us per launch depending on
    // where the output buffer landed.)
    const int64_t s0 = 16 * wave, step = 16 * nwaves, s1 = n;
    if (wave >= nwaves || s0 >= n) return;

    // MFMA D[component][sample] = A[component][k] . B[k][sample]: A = the
    // coefficient fragment (lane: component 16 r + (lane & 15), k group
    // lane >> 4), B = the sample fragment (lane: feature g of sample col);
    // D gives lane (g, col) components 16 r + 4 g + j (j = 0..3) of sample col
    const int g = lane >> 4;
    const int col = lane & 15;
    const bool has_h = s.hpdf != nullptr, has_d = s.isDiffuse != nullptr;

    // sample col of tile t: position and direction coordinate g (lane group 3
    // loads coordinate 0 and gathers all three from groups 0..2 when the
    // fragments are built) and, when present, the heuristic pdf and the
    // diffuse flag (its dword)
    const int gf = g < 3 ? g : 0;
    struct Feat {
        float p, d, hp;
        int dw;
    };
    auto load_feat = [&](int64_t t) {
        int64_t i = t + col;
        i = (i < s1) ? i : s1 - 1;
        Feat f;
        f.p = __builtin_nontemporal_load(s.x[gf] + i);
        f.d = __builtin_nontemporal_load(s.x[3 + gf] + i);
        // optional planes: loaded only when present (a wave-uniform branch)
        f.hp = 0.0f;
        f.dw = 0;
        if (has_h) f.hp = __builtin_nontemporal_load(s.hpdf + i);
        if (has_d) f.dw = *(const __attribute__((address_space(1))) int*)((uintptr_t)(s.isDiffuse + i) & ~(uintptr_t)3);
        return f;
    };
    // the three coordinates of sample col from lane groups 0..2
    auto gather3 = [&](float v, float (&x)[3]) __attribute__((always_inline)) {
        x[0] = __shfl(v, col);
        x[1] = __shfl(v, 16 + col);
        x[2] = __shfl(v, 32 + col);
    };
    auto pfrag = [&](const float (&p3)[3], const float* o) __attribute__((always_inline)) {
        const float x[3] = {p3[0] - o[0], p3[1] - o[1], p3[2] - o[2]};
        return a_frag(x, g, true);
    };
    // block r's coefficient fragments and detInv pi of the lane's four components
    auto frags = [&](int r, bf8 (&F)[8], f4& dp) __attribute__((always_inline)) {
#pragma unroll
        for (int f = 0; f < 8; ++f) F[f] = __builtin_bit_cast(bf8, cimg[(r * 8 + f) * 64 + lane]);
        if constexpr (DIMG)
            dp = dimg[r * 4 + g];
        else
            dp = *(const f4*)(ep + EP_DIPI * Kp + 16 * r + 4 * g);
    };
    auto forms = [&](const bf8 (&F)[8], bf8 bs, bf8 bd, f4 (&D)[8]) __attribute__((always_inline)) {
        const f4 z = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int f = 0; f < 8; ++f) D[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F[f], f < 3 ? bd : bs, z, 0, 0, 0);
    };

    // The stores of tile t are issued at the top of tile t + 1, BEFORE the
    // loads of tile t + 2: vmcnt counts stores too, and a wait on loads that
    // were issued before pending stores is a wait for those stores (the
    // compiler emits vmcnt(0) on mixed pending events).  In this order the
    // wait for tile t + 1's loads only covers stores issued a tile earlier.
    float pdf[LR ? 1 : R][4];
    f4* const st = stage0 + wid * NS;
    float gsc_p = 0.0f;
    bool full_p = false;
    int64_t tp = -1;
    auto flush = [&]() __attribute__((always_inline)) {
        if (tp < 0) return;
        float* row = resp + (tp + col) * (int64_t)K + 4 * g;
        if constexpr (LR) {
            if (full_p) {
                // whole unnormalised rows in the stage: lane (g, col) scales and
                // stores 16-B chunk 16 h + col of rows g + 4 i (four contiguous
                // 256-B half rows per store instruction)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int rw = g + 4 * i;
                    const float sc = __shfl(gsc_p, rw);   // row rw's normaliser (lane rw holds it)
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int ch = 16 * h + col;
                        const f4 v = st[rw * 32 + (ch ^ rw)];
                        __builtin_nontemporal_store(v * sc, (f4*)(resp + (tp + rw) * (int64_t)K + 4 * ch));
                    }
                }
            } else if (tp + col < s1) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const f4 v = st[col * 32 + ((4 * r + g) ^ col)];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float o = gsc_p != 0.0f ? v[j] * gsc_p : 0.0f;
                        if (16 * r + 4 * g + j < K) __builtin_nontemporal_store(o, row + 16 * r + j);
                    }
                }
            }
            return;
        }
        if (full_p && R != 8) {
            // one 16-B store per block: a sample's 64-B row segment per 4 lanes
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const f2 lo = f2{pdf[r][0], pdf[r][1]} * spl(gsc_p);
                const f2 hi = f2{pdf[r][2], pdf[r][3]} * spl(gsc_p);
                __builtin_nontemporal_store(f4{lo.x, lo.y, hi.x, hi.y}, (f4*)(row + 16 * r));
            }
        } else if (full_p) {
            // R = 8: rows through LDS, half a row (blocks 4h .. 4h+3, 256 B) at a
            // time: the D layout gives each lane 16 B of ONE sample per block,
            // i.e. 64-B row segments per store (measured 230 vs 180 us with
            // whole lines); staged, every store writes four contiguous 256-B
            // half rows.  16-B chunk c of row i sits at chunk c ^ i (conflict-
            // free writes and reads).
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int r = (4 * h + rr) % R;
                    const f2 lo = f2{pdf[r][0], pdf[r][1]} * spl(gsc_p);
                    const f2 hi = f2{pdf[r][2], pdf[r][3]} * spl(gsc_p);
                    st[col * 16 + ((4 * rr + g) ^ col)] = f4{lo.x, lo.y, hi.x, hi.y};
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int rw = g + 4 * i, ch = col;
                    const f4 v = st[rw * 16 + (ch ^ rw)];
                    __builtin_nontemporal_store(v, (f4*)(resp + (tp + rw) * (int64_t)K + 64 * h + 4 * ch));
                }
                __builtin_amdgcn_wave_barrier();
            }
        } else if (tp + col < s1) {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float o = gsc_p != 0.0f ? pdf[r][j] * gsc_p : 0.0f;
                    if (16 * r + 4 * g + j < K) __builtin_nontemporal_store(o, row + 16 * r + j);
                }
        }
    };

    Feat nf = load_feat(s0);
    for (int64_t t = s0; t < s1; t += step) {
        const Feat cf = nf;
        float P3[3], D3[3];
        gather3(cf.p, P3);
        gather3(cf.d, D3);
        // d == 0 fails every log map (mvtn.h:152-154)
        const bool dzero = D3[0] == 0.0f && D3[1] == 0.0f && D3[2] == 0.0f;
        const bool dif = has_d && ((cf.dw >> (8 * (int)((uintptr_t)(s.isDiffuse + ((t + col < s1) ? t + col : s1 - 1)) & 3))) & 0xff) != 0;
        const float hp = has_h ? cf.hp : 0.0f;
        const bf8 Bd = a_frag(D3, g, false);
        const float o0[3] = {kOrigin, kOrigin, kOrigin};
        const bf8 Bs0 = pfrag(P3, o0);   // one origin for every block unless kBlockOrigin
        __builtin_amdgcn_sched_barrier(0);
        flush();                          // tile t - 16's rows
        __builtin_amdgcn_sched_barrier(0);
        nf = load_feat(t + step);         // next tile in flight (clamped past the end)
        __builtin_amdgcn_sched_barrier(0);

        f2 acc = f2{0.0f, 0.0f};
        uint32_t cbits = 0;
        auto pair_math = [&](int r, auto rare, const f4 (&D)[8], const f4& dp) __attribute__((always_inline)) {
            constexpr bool RARE = decltype(rare)::value;
            if constexpr (!RARE)
                cbits = __builtin_elementwise_max(
                    cbits, __builtin_elementwise_max(
                               __builtin_elementwise_max(__builtin_bit_cast(uint32_t, D[0][0]), __builtin_bit_cast(uint32_t, D[0][1])),
                               __builtin_elementwise_max(__builtin_bit_cast(uint32_t, D[0][2]), __builtin_bit_cast(uint32_t, D[0][3]))));
            f2 p[2];
#ifdef SDMM_SPLIT_DIAG_NOMATH
            p[0] = f2{D[0][0] + D[1][0] + D[2][0] + D[3][0], D[4][1] + D[5][1] + D[6][1] + D[7][1]};
            p[1] = f2{D[0][2] + D[1][2] + D[2][2] + D[3][2], D[4][3] + D[5][3] + D[6][3] + D[7][3]};
#else
            pdf_quad<RARE>(D[0], D[1], D[2], D[3], D[4], D[5], D[6], D[7], dp, p);
#endif
            if constexpr (LR) {
                st[col * 32 + ((4 * r + g) ^ col)] = f4{p[0].x, p[0].y, p[1].x, p[1].y};   // row col, chunk 4 r + g
            } else {
                pdf[r][0] = p[0].x;
                pdf[r][1] = p[0].y;
                pdf[r][2] = p[1].x;
                pdf[r][3] = p[1].y;
            }
            acc = padd(acc, padd(p[0], p[1]));
        };
#if defined(SDMM_SPLIT_DIAG_STOREONLY)
        // diagnostic ceiling (tools/build_variant.sh): the same loads, row
        // staging and stores with no matrix or pair math; the rows are not
        // responsibilities
#pragma unroll
        for (int r = 0; r < R; ++r) {
            f4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = P3[j & 1] + D3[j >> 1] + (float)(16 * r + j);
                acc.x += v[j];
            }
            if constexpr (LR)
                st[col * 32 + ((4 * r + g) ^ col)] = v;
            else
#pragma unroll
                for (int j = 0; j < 4; ++j) pdf[r][j] = v[j];
        }
#elif defined(SDMM_SPLIT_PAIR2)
        {
            // two blocks per step: their 16 MFMAs back to back, then both
            // blocks' pair math with no fence between them, so the scheduler
            // interleaves four independent packed chains (the pair math is
            // dependency-bound at two); the next pair's fragments are read
            // from LDS meanwhile
          if constexpr (R % 2 != 0) {
            bf8 F[8];
            f4 dp, D[8];
            frags(0, F, dp);
            forms(F, Bs0, Bd, D);
            pair_math(0, Tag<false>{}, D, dp);
          } else {
            bf8 F[2][8], G[2][8];
            f4 dp[2], dq[2];
            frags(0, F[0], dp[0]);
            frags(1, G[0], dq[0]);
#pragma unroll
            for (int r = 0; r < R; r += 2) {
                const int b = (r >> 1) & 1;
                f4 D0[8], D1[8];
                forms(F[b], Bs0, Bd, D0);
                forms(G[b], Bs0, Bd, D1);
                __builtin_amdgcn_sched_barrier(0);
                if (r + 2 < R) {
                    frags(r + 2, F[b ^ 1], dp[b ^ 1]);
                    frags(r + 3, G[b ^ 1], dq[b ^ 1]);
                }
                __builtin_amdgcn_sched_barrier(0);
                pair_math(r, Tag<false>{}, D0, dp[b]);
                pair_math(r + 1, Tag<false>{}, D1, dq[b]);
                __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
#elif defined(SDMM_SPLIT_PIPE)
        {
            // software-pipelined over the blocks: block r + 1's eight MFMAs are
            // issued before block r's pair math and interleaved with it
            // (sched_group_barrier), block r + 2's fragments are read from LDS
            // meanwhile; the matrix pipe works while the VALU does
            bf8 F[R][8];
            f4 dp[R], D[R][8];
            frags(0, F[0], dp[0]);
            forms(F[0], Bs0, Bd, D[0]);
            if (R > 1) frags(1, F[1], dp[1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (r + 1 < R) forms(F[r + 1], Bs0, Bd, D[r + 1]);
                if (r + 2 < R) frags(r + 2, F[r + 2], dp[r + 2]);
                pair_math(r, Tag<false>{}, D[r], dp[r]);
                if (r + 1 < R) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);              // one MFMA
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);              // one LDS read
                        __builtin_amdgcn_sched_group_barrier(0x002, SDMM_SPLIT_PIPE, 0);  // VALU
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#else
        {
            // pipelined over the blocks: block r + 1's fragments are read from
            // LDS while block r's pair math runs
            bf8 F[2][8], BS[2];
            f4 dp[2];
            frags(0, F[0], dp[0]);
            BS[0] = kBlockOrigin ? pfrag(P3, borig[0]) : Bs0;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                f4 D[8];
                forms(F[r & 1], BS[r & 1], Bd, D);
                SPLIT_FENCE();
#ifndef SDMM_SPLIT_PREFETCH
#define SDMM_SPLIT_PREFETCH 0
#endif
                // SDMM_SPLIT_PREFETCH = n (A/B): block r + 1's first n fragments
                // are read while block r's pair math runs, the rest after it
                // (default 0: 32 VGPRs fewer, 3 waves per SIMD fit, and the
                // other waves cover the reads)
                if (r + 1 < R && SDMM_SPLIT_PREFETCH > 0) {
#pragma unroll
                    for (int f = 0; f < SDMM_SPLIT_PREFETCH; ++f)
                        F[(r + 1) & 1][f] = __builtin_bit_cast(bf8, cimg[((r + 1) * 8 + f) * 64 + lane]);
                }
                SPLIT_FENCE();
                pair_math(r, Tag<false>{}, D, dp[r & 1]);
                if (r + 1 < R) {
#pragma unroll
                    for (int f = SDMM_SPLIT_PREFETCH; f < 8; ++f)
                        F[(r + 1) & 1][f] = __builtin_bit_cast(bf8, cimg[((r + 1) * 8 + f) * 64 + lane]);
                    if constexpr (DIMG)
                        dp[(r + 1) & 1] = dimg[(r + 1) * 4 + g];
                    else
                        dp[(r + 1) & 1] = *(const f4*)(ep + EP_DIPI * Kp + 16 * (r + 1) + 4 * g);
                }
                // the next block's spatial sample fragment, off the MFMA issue path
                if (r + 1 < R) BS[(r + 1) & 1] = kBlockOrigin ? pfrag(P3, borig[r + 1]) : Bs0;
                SPLIT_FENCE();
            }
        }
#endif
        // rare angle case anywhere in the tile (c < -0.9999995; its bits,
        // unsigned, exceed those of -0.9999995f) or a NaN: redo the tile with
        // the reference's quirks (wave-uniform, a few tiles per launch)
        const bool odd = cbits > __builtin_bit_cast(uint32_t, -0.9999995f) || !(acc.x + acc.y >= 0.0f);
#if defined(SDMM_SPLIT_DIAG_NOREDO)
        if (false) {
#elif defined(SDMM_SPLIT_DIAG_ALWAYSREDO)
        if (__builtin_amdgcn_ballot_w64(odd) != 0 || true) {
#else
        if (__builtin_amdgcn_ballot_w64(odd) != 0) {
#endif
            bf8 bd2 = Bd, bs2 = Bs0;
            asm volatile("" : "+v"(bd2), "+v"(bs2));
            acc = f2{0.0f, 0.0f};
#pragma unroll
            for (int r = 0; r < R; ++r) {
                bf8 F[8];
                f4 dp, D[8];
                frags(r, F, dp);
                forms(F, kBlockOrigin ? pfrag(P3, borig[r]) : bs2, bd2, D);
                pair_math(r, Tag<true>{}, D, dp);
            }
        }
        // posterior normalisation of sample col (mixture_model.h:170-191): the
        // lane's 4 R components, then the four lane groups of the sample
        float S = acc.x + acc.y;
        S += __shfl_xor(S, 16);
        S += __shfl_xor(S, 32);
        const float S2 = dif ? fmaf(1.0f - kHeuristicWeight, S, kHeuristicWeight * hp) : S;
        const float inv = __builtin_amdgcn_rcpf(S2);
        const bool fin = __builtin_isfinite(inv) && !dzero;
        gsc_p = fin ? (dif ? inv * (1.0f - kHeuristicWeight) : inv) : 0.0f;
        // a non-finite sum means a non-finite pdf (NaN/inf input): zero rows by select
        const bool bad = __builtin_amdgcn_ballot_w64(!__builtin_isfinite(S)) != 0;
        full_p = (t + 16 <= s1) && (16 * R == K) && !bad;
        tp = t;
    }
    flush();
}

// ---------------------------------------------------------------------------
// Configurations (R = Kp / 16 blocks, waves per workgroup, waves per SIMD).
// The B image takes R x 8 KB of LDS per workgroup.
#define SDMM_SPLIT_CONFIGS(X) X(1, 4, 4) X(2, 4, 4) X(4, 4, 4) X(8, 4, 2) X(8, 8, 2) X(8, 12, 3)

// R = 8 (K = 128): variants 0 and 2 = one 12-wave workgroup per CU at 3 waves
// per SIMD (the 96-KB row stage + the 64-KB coefficient image fill the LDS),
// 1 = two 4-wave workgroups at 2 per SIMD, 3 = one 8-wave workgroup at 2 per
// SIMD (round 3's default)
static void split_cfg(int R, int variant, int* wpb, int* occ) {
    *wpb = 4;
    *occ = 4;
    if (R == 8) {
        // default: 12-wave workgroups at 3 waves per SIMD (round 4: 176 us
        // per launch against 180-188 us for the round-3 configuration,
        // variant 3, which also ran 340-370 us in some processes -- see
        // DESIGN.md section 4)
        *wpb = 12; *occ = 3;
        if (variant == 1) { *wpb = 4; *occ = 2; }
        if (variant == 3) { *wpb = 8; *occ = 2; }
    }
}

bool estep_resp_split_supported(int Kp) { return Kp % 16 == 0 && Kp / 16 <= 8 && (Kp / 16 & (Kp / 16 - 1)) == 0; }

// resident_waves: waves of this kernel the device holds at once (the launch
// is one round of them, fewer when n has fewer tiles)
hipError_t launch_estep_resp_split(int variant, const float* ep, int Kp, int K, const SamplesDev& s, int64_t n,
                                   int64_t resident_waves, float* resp, hipStream_t st) {
    if (!estep_resp_split_supported(Kp) || K > Kp || resident_waves <= 0) return hipErrorInvalidValue;
    const int R = Kp / 16;
    int wpb, occ;
    split_cfg(R, variant, &wpb, &occ);
    const int64_t tiles = (n + 15) / 16;
    const int64_t blocks = ((tiles < resident_waves ? tiles : resident_waves) + wpb - 1) / wpb;
    const int64_t waves = blocks * wpb;
#define X(RR, WW, OO)                                                                                          \
    if (R == RR && wpb == WW && occ == OO) {                                                                   \
        hipLaunchKernelGGL((estep_resp_split_kernel<RR, WW, OO>), dim3((unsigned)blocks), dim3(64 * WW), 0, st, ep, \
                           Kp, K, s, n, waves, resp);                                                          \
        return hipGetLastError();                                                                              \
    }
    SDMM_SPLIT_CONFIGS(X)
#undef X
    return hipErrorInvalidValue;
}

// resident waves per CU of the configuration
hipError_t estep_resp_split_occupancy(int variant, int Kp, int* waves_per_cu) {
    const int R = Kp / 16;
    int wpb, occ;
    split_cfg(R, variant, &wpb, &occ);
    int blocks = 0;
#define X(RR, WW, OO)                                                                                          \
    if (R == RR && wpb == WW && occ == OO) {                                                                   \
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(                                           \
            &blocks, reinterpret_cast<const void*>(&estep_resp_split_kernel<RR, WW, OO>), 64 * WW, 0);         \
        *waves_per_cu = blocks * WW;                                                                           \
        return e;                                                                                              \
    }
    SDMM_SPLIT_CONFIGS(X)
#undef X
    return hipErrorInvalidValue;
}

const char* estep_resp_split_name(int variant, int Kp) {
    static thread_local char buf[64];
    int wpb, occ;
    split_cfg(Kp / 16, variant, &wpb, &occ);
    snprintf(buf, sizeof buf, "estep_resp_split_kernel<%d,%d,%d>", Kp / 16, wpb, occ);
    return buf;
}

}  // namespace sdmm
