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
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 pmul(f2 a, f2 b) { return a * b; }
__device__ __forceinline__ f2 padd(f2 a, f2 b) { return a + b; }

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
constexpr bool kFoldScale = true;
constexpr double kRowScale = 0.84932180028801904272;

// row start of L^-1 row m in the packed lower triangle (EP_L00 ...)
__device__ __forceinline__ int lrow(int m) { return EP_L00 + m * (m + 1) / 2; }

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
        if constexpr (!RARE) {
            // c < 0 ? fneg : h as one median: fneg > h on both sides (pi / s >
            // 2 acos|c| / s), and -2^100 c is +huge for c < 0 and -huge for
            // c > 0, so med3(h, fneg, -2^100 c) picks fneg or h (one packed
            // product + one med3 per pair instead of a compare + a select).
            // Only |c| < 2^-90 lands between (the result then h within
            // ~1e-7: pi / s - 2 h ~ 0 there), NaN pairs go to the RARE redo.
            const f2 t = pmul(c[i], spl(-0x1p100f));
            a[i] = f2{__builtin_amdgcn_fmed3f(h[i].x, fneg.x, t.x), __builtin_amdgcn_fmed3f(h[i].y, fneg.y, t.y)};
        } else {
            a[i] = f2{c[i].x < 0.0f ? fneg.x : h[i].x, c[i].y < 0.0f ? fneg.y : h[i].y};
        }
        if constexpr (RARE) {
            const float o0 = __builtin_amdgcn_fmed3f(1073741824.0f * (c[i].x + 1.0f), 0.0f, 1.0f);
            const float o1 = __builtin_amdgcn_fmed3f(1073741824.0f * (c[i].y + 1.0f), 0.0f, 1.0f);
            a[i].x = (c[i].x < 0.0f && s2[i].x < 1e-6f) ? o0 : a[i].x;
            a[i].y = (c[i].y < 0.0f && s2[i].y < 1e-6f) ? o1 : a[i].y;
        }
    }
    // detInv pi_k * jacobian (mvtn.h:361, mixture_model.h:164) ahead of the
    // exponent chain: the tail after the exp is one product per pair
    f2 da[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) da[i] = pmul(f2{dipi[2 * i], dipi[2 * i + 1]}, a[i]);
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
        p[i] = pmul(e, da[i]);
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// Sample features through LDS by DMA, with counted waits (round 5).
//
// vmcnt counts loads and stores together, in issue order, and the compiler
// waits vmcnt(0) before the first use of a VGPR load whenever stores are
// pending beside it.  With the features loaded into VGPRs every tile, each
// wave therefore waited for ALL of its row stores before it could start the
// next tile: compute and the write stream took turns instead of overlapping
// (store-only shape 135 us against the 88-105 us write stream, the math then
// +45 us on top).  Here the features of tile t + kFeatAhead go by
// global_load_lds_dword (inline asm: the compiler does not track them, so it
// never drains vmcnt for them) into a per-wave LDS ring, and the wave waits
// with an explicit vmcnt(N) that leaves every store younger than that DMA in
// flight: N = 2 kFeatAhead + R k, the two DMA pieces of each tile issued after
// it plus the R row stores of each of the k = min(i, kFeatAhead + 1) flushes
// issued after it (every one of them a full flush of exactly R stores; any
// other flush in that window and the wait is vmcnt(0)).
constexpr int kFeatAhead = 2;
constexpr int kFeatSlots = kFeatAhead + 1;
constexpr int kFeatSlotU4 = 32;   // two 256-B DMA pieces (64 lanes x 4 B)

// vmcnt(N), then this lane's two 16-B feature records from the ring, in ONE
// statement: the compiler sees neither the DMA that wrote the ring nor its
// wait, so a plain read of the ring would be a read of memory it believes
// unwritten (undef: it did fold one of them to an unrelated register).
// lgkmcnt(0) inside: the outputs are complete when the statement ends.
template <int N>
__device__ __forceinline__ void read_feat(unsigned addr, f4& a, f4& b) {
    static_assert(N >= 0 && N <= 63, "gfx950 vmcnt is six bits");
    asm volatile(
        "s_waitcnt vmcnt(%3)\n\t"
        "ds_read_b128 %0, %2\n\t"
        "ds_read_b128 %1, %2 offset:256\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(a), "=&v"(b)
        : "v"(addr), "n"(N)
        : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N <= 63, "gfx950 vmcnt is six bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// (diagnostic SDMM_SPLIT_DIAG_NOSTORE: every row computed, none stored -- the
// compute-only time of the kernel; then only the DMAs are in flight)
#ifdef SDMM_SPLIT_DIAG_NOSTORE
constexpr bool kDiagNoStore = true;
#else
constexpr bool kDiagNoStore = false;
#endif
template <int R>
__device__ __forceinline__ void read_feat_counted(int k, bool window_full, unsigned addr, f4& a, f4& b) {
    if (kDiagNoStore) {
        read_feat<2 * kFeatAhead>(addr, a, b);
        return;
    }
    if (!window_full) {
        read_feat<0>(addr, a, b);
        return;
    }
    switch (k) {   // wave-uniform
        case 0: read_feat<2 * kFeatAhead>(addr, a, b); break;
        case 1: read_feat<2 * kFeatAhead + R>(addr, a, b); break;
        case 2: read_feat<2 * kFeatAhead + 2 * R>(addr, a, b); break;
        default: read_feat<2 * kFeatAhead + 3 * R>(addr, a, b); break;
    }
    static_assert(kFeatAhead == 2, "read_feat_counted enumerates k = 0 .. kFeatAhead + 1");
}

// two LDS-DMA pieces: lane L's dword of a0 to lds[L], of a1 to lds[64 + L]
// (M0 = the wave-uniform LDS byte address of the piece)
__device__ __forceinline__ void dma_pair(uintptr_t a0, uintptr_t a1, unsigned lds0) {
    unsigned keep;   // M0 is reserved by the compiler: saved and restored around the pieces
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %1, off\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %2, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(a0), "v"(a1), "s"(lds0), "s"(lds0 + 256u)
        : "memory");
}

template <int R, int WPB, int OCC>
__global__ void __launch_bounds__(64 * WPB, OCC)
estep_resp_split_kernel(const float* __restrict__ ep, int Kp, int K, SamplesDev s, int64_t n, int64_t nwaves,
                        float* __restrict__ resp) {
    // one LDS block carved into: per wave the feature ring (kFeatSlots x 512 B;
    // first, so every LDS-DMA destination lies below 64 KB), the coefficient
    // image (R blocks x 8 forms x 64 lanes), detInv pi of components 16 r + 4 g
    // .. + 3 (the D rows of lane group g), and per wave the 256-B half-row
    // stage (R = 8: 16 rows)
    constexpr int NC = R * 8 * 64, ND = R * 4, NS = R == 8 ? 16 * 16 : 0, NF = kFeatSlots * kFeatSlotU4;
    constexpr int NTOT = WPB * NF + NC + ND + WPB * NS;
    static_assert(NTOT * 16 <= 163840, "the carved LDS block exceeds the 160 KB of a CU");
    static_assert(WPB * NF * 16 <= 65536, "LDS-DMA destinations stay below 64 KB");
    __shared__ u4 smem[NTOT];
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    u4* const ring = smem + wid * NF;
    u4* const cimg = smem + WPB * NF;
    f4* const dimg = (f4*)(cimg + NC);
    f4* const st = (f4*)(cimg + NC + ND + wid * NS);
    static_assert(WPB * NF + NC + ND + WPB * NS == NTOT && (R != 8 || NS == 256), "LDS carve: every region has storage");

    const float o_scene[3] = {kOrigin, kOrigin, kOrigin};
#ifdef SDMM_SPLIT_DIAG_NOIMAGE   // (diagnostic: a zero coefficient image -- results are not responsibilities)
    for (int idx = threadIdx.x; idx < NC + ND; idx += 64 * WPB) cimg[idx] = u4{0u, 0u, 0u, 0u};
#else
    for (int idx = threadIdx.x; idx < NC; idx += 64 * WPB)
        cimg[idx] = coef_frag(ep, Kp, idx >> 9, (idx >> 6) & 7, idx & 63, o_scene);
    for (int i = threadIdx.x; i < ND; i += 64 * WPB) {
        const float* d = ep + EP_DIPI * Kp + 4 * i;
        dimg[i] = f4{d[0], d[1], d[2], d[3]};
    }
#endif
    __syncthreads();

    const int lane = threadIdx.x & 63;
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

    // DMA sources of this lane: sample sl = lane >> 2 of the tile, plane pl =
    // lane & 3 of piece 0 (x0 x1 x2 x3) and of piece 1 (x4 x5 hpdf isDiffuse;
    // an absent optional plane re-reads x0).  The diffuse flag comes as the
    // dword that holds its byte (the plane's dword-aligned word).
    const int pl = lane & 3, sl = lane >> 2;
    const uintptr_t src0 = (uintptr_t)(pl == 0 ? s.x[0] : pl == 1 ? s.x[1] : pl == 2 ? s.x[2] : s.x[3]);
    const bool byteplane = pl == 3 && has_d;
    const uintptr_t src1 = (uintptr_t)(pl == 0   ? s.x[4]
                                       : pl == 1 ? s.x[5]
                                       : pl == 2 ? (has_h ? s.hpdf : s.x[0])
                                                 : (has_d ? (const float*)s.isDiffuse : s.x[0]));
    const int sh1 = byteplane ? 0 : 2;
    const unsigned ring_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) u4*)ring;
    auto dma = [&](int64_t t, int slot) __attribute__((always_inline)) {
        int64_t i = t + sl;
        i = (i < s1) ? i : s1 - 1;   // past the end: a valid sample, never stored
        const uintptr_t a0 = src0 + ((uintptr_t)i << 2);
        const uintptr_t a1 = (src1 + ((uintptr_t)i << sh1)) & ~(uintptr_t)3;
        dma_pair(a0, a1, ring_lds + (unsigned)slot * (kFeatSlotU4 * 16u));
    };

    auto pfrag = [&](const float (&p3)[3]) __attribute__((always_inline)) {
        const float x[3] = {p3[0] - kOrigin, p3[1] - kOrigin, p3[2] - kOrigin};
        return a_frag(x, g, true);
    };
    // block r's coefficient fragments and detInv pi of the lane's four components
    auto frags = [&](int r, bf8 (&F)[8], f4& dp) __attribute__((always_inline)) {
#pragma unroll
        for (int f = 0; f < 8; ++f) F[f] = __builtin_bit_cast(bf8, cimg[(r * 8 + f) * 64 + lane]);
        dp = dimg[r * 4 + g];
    };
    auto forms = [&](const bf8 (&F)[8], bf8 bs, bf8 bd, f4 (&D)[8]) __attribute__((always_inline)) {
        const f4 z = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int f = 0; f < 8; ++f) D[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F[f], f < 3 ? bd : bs, z, 0, 0, 0);
    };

    // The rows of tile t are stored at the top of the next tile (flush), after
    // the DMA of the features kFeatAhead tiles ahead; a full flush is exactly
    // R store instructions (the count read_feat_counted relies on).
    float pdf[R][4];
    float gsc_p = 0.0f;
    bool full_p = false;
    int64_t tp = -1;
    auto flush = [&]() __attribute__((always_inline)) {
        if (tp < 0) return;
        if (kDiagNoStore && gsc_p != -1.0f) return;   // (never -1: the rows stay live)
        float* row = resp + (tp + col) * (int64_t)K + 4 * g;
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

    // prologue: the first kFeatAhead tiles' features in flight
#pragma unroll
    for (int a = 0; a < kFeatAhead; ++a) dma(s0 + a * step, a);
    unsigned hist = 0;   // bit j: the flush j iterations back was full
    int it = 0;
    for (int64_t t = s0; t < s1; t += step, ++it) {
        const int slot = it % kFeatSlots;
        dma(t + kFeatAhead * step, (it + kFeatAhead) % kFeatSlots);   // clamped past the end
        if (tp >= 0) hist = (hist << 1) | (full_p ? 1u : 0u);
        flush();                                                       // tile t - step's rows
        const int k = it < kFeatAhead + 1 ? it : kFeatAhead + 1;
        const unsigned need = (1u << k) - 1u;
        f4 fa, fb;   // x0 x1 x2 x3 and x4 x5 hpdf flags of sample col
        read_feat_counted<R>(k, (hist & need) == need, ring_lds + (unsigned)slot * (kFeatSlotU4 * 16u) + 16u * col,
                             fa, fb);
        const float P3[3] = {fa.x, fa.y, fa.z};
        const float D3[3] = {fa.w, fb.x, fb.y};
        // d == 0 fails every log map (mvtn.h:152-154)
        const bool dzero = D3[0] == 0.0f && D3[1] == 0.0f && D3[2] == 0.0f;
        const int64_t ic = (t + col < s1) ? t + col : s1 - 1;
        const bool dif = has_d && ((fbits(fb.w) >> (8 * (int)((uintptr_t)(s.isDiffuse + ic) & 3))) & 0xffu) != 0u;
        const float hp = has_h ? fb.z : 0.0f;
        const bf8 Bd = a_frag(D3, g, false);
        const bf8 Bs = pfrag(P3);

        // the normaliser's lane partials: two independent packed chains (rows
        // j, j + 1 and j + 2, j + 3), so no product waits on the previous add
        f2 acc = f2{0.0f, 0.0f}, acc2 = f2{0.0f, 0.0f};
        uint32_t cbits = 0;
        auto pair_math = [&](int r, auto rare, const f4 (&D)[8], const f4& dp) __attribute__((always_inline)) {
            constexpr bool RARE = decltype(rare)::value;
            if constexpr (!RARE)
                cbits = __builtin_elementwise_max(
                    cbits, __builtin_elementwise_max(__builtin_elementwise_max(fbits(D[0][0]), fbits(D[0][1])),
                                                     __builtin_elementwise_max(fbits(D[0][2]), fbits(D[0][3]))));
            f2 p[2];
            pdf_quad<RARE>(D[0], D[1], D[2], D[3], D[4], D[5], D[6], D[7], dp, p);
            pdf[r][0] = p[0].x;
            pdf[r][1] = p[0].y;
            pdf[r][2] = p[1].x;
            pdf[r][3] = p[1].y;
            acc = padd(acc, p[0]);
            acc2 = padd(acc2, p[1]);
        };
#if defined(SDMM_SPLIT_DIAG_STOREONLY)
        // diagnostic ceiling (tools/build_variant.sh "-DSDMM_SPLIT_DIAG_STOREONLY"):
        // the same DMA, row staging and stores with no matrix or pair math; the
        // rows are not responsibilities
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                pdf[r][j] = P3[j & 1] + D3[j >> 1] + (float)(16 * r + j);
                acc.x += pdf[r][j];
            }
#else
        {
            // pipelined over the blocks: block r + 1's fragments are read from
            // LDS while block r's pair math runs
            bf8 F[2][8];
            f4 dp[2];
            frags(0, F[0], dp[0]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                f4 D[8];
                forms(F[r & 1], Bs, Bd, D);
                __builtin_amdgcn_sched_barrier(0);
                pair_math(r, Tag<false>{}, D, dp[r & 1]);
                if (r + 1 < R) frags(r + 1, F[(r + 1) & 1], dp[(r + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#endif
        // rare angle case anywhere in the tile (c < -0.9999995; its bits,
        // unsigned, exceed those of -0.9999995f) or a NaN: redo the tile with
        // the reference's quirks (wave-uniform, a few tiles per launch)
        const bool odd = cbits > __builtin_bit_cast(uint32_t, -0.9999995f) || !((acc.x + acc.y) + (acc2.x + acc2.y) >= 0.0f);
        if (__builtin_amdgcn_ballot_w64(odd) != 0) {
            bf8 bd2 = Bd, bs2 = Bs;
            asm volatile("" : "+v"(bd2), "+v"(bs2));
            acc = f2{0.0f, 0.0f};
            acc2 = f2{0.0f, 0.0f};
#pragma unroll
            for (int r = 0; r < R; ++r) {
                bf8 F[8];
                f4 dp, D[8];
                frags(r, F, dp);
                forms(F, bs2, bd2, D);
                pair_math(r, Tag<true>{}, D, dp);
            }
        }
        // posterior normalisation of sample col (mixture_model.h:170-191): the
        // lane's 4 R components, then the four lane groups of the sample
        float S = (acc.x + acc.y) + (acc2.x + acc2.y);
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
    // the ring's last DMAs (clamped tiles past the end) land before the
    // workgroup's LDS is released
    wait_vm<0>();
}

// ---------------------------------------------------------------------------
// Configurations (R = Kp / 16 blocks, waves per workgroup, waves per SIMD).
// The B image takes R x 8 KB of LDS per workgroup.
#ifndef SDMM_SPLIT_R8_WPB   // (overridable for tools/build_variant.sh A/B builds)
#define SDMM_SPLIT_R8_WPB 12
#define SDMM_SPLIT_R8_OCC 3
#endif
#define SDMM_SPLIT_CONFIGS(X) X(1, 4, 4) X(2, 4, 4) X(4, 4, 4) X(8, SDMM_SPLIT_R8_WPB, SDMM_SPLIT_R8_OCC)

// R = 8 (K = 128): one 12-wave workgroup per CU at 3 waves per SIMD (the
// 64-KB coefficient image, the 48 KB of half-row stages and the 18 KB of
// feature rings share the LDS).  Round 4 measured 4-wave / 2-per-SIMD and
// 8-wave / 2-per-SIMD workgroups slower; the variant
// argument is kept for the ABI's A/B hook and ignored.
static void split_cfg(int R, int /*variant*/, int* wpb, int* occ) {
    *wpb = 4;
    *occ = 4;
    if (R == 8) {
        *wpb = SDMM_SPLIT_R8_WPB;
        *occ = SDMM_SPLIT_R8_OCC;
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
