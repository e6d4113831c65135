// fastexp.h -- NORM * exp(-q/2) rounded to float, bit for bit as the reference.
//
// The reference evaluates every Gaussian weight of the guided conditional as
//     (float)((double)norm * exp(-0.5 * (double)q))
// (MultivariateNormal::pdf, multivariate_normal.h:126; MVTN::pdf,
// multivariate_tangent_normal.h:359, 375; Scalar = float), with the double
// exp of libm.  On gfx950 the double exp is a software routine of ~80
// instructions (range reduction, a degree-11 polynomial, the special cases);
// the guided candidate pass evaluates K of them per query.
//
// Here the double is evaluated to ~2^-44 instead of ~2^-52 with a table-driven
// reduction, and the float rounding is then decided by a Ziv test:
//   x = -q/2, k = rint(64 x / ln 2), r = x - k ln2/64 (|r| <= ln2/128, Cody-Waite
//   with a two-part ln2/64), y = ldexp(norm * (T[k & 63] * p(r)), k >> 6),
//   T[j] = RN64(2^(j/64)), p = the degree-4 Taylor polynomial of e^r.
// Error of y against V = norm e^x: truncation |r|^5/120 e^|r| <= 2^-44.5, plus
// eight double roundings (<= 2^-50) -> |y - V| <= V 2^-44.3.  The reference
// double D = RN64(norm RN64(exp(x))) is within V 2^-51.4 of V (libm exp within
// one ulp, one product rounding).  So |y - D| < y 2^-44 and, when y lies more
// than y 2^-40 (< 2^-16 float ulp) from every float rounding boundary, RN32(D)
// = RN32(y): the fast result is returned.  Otherwise (probability ~2^-15 per
// weight; q negative, NaN or inf; a float result that is a power of two or
// sits at the FLT_MIN flush edge) the reference expression itself is evaluated.  A y below
// FLT_MIN (1 - 2^-20) is 0: D then rounds below FLT_MIN and the plugin's
// FTZ/DAZ (volpath_sdmm.cpp:88-90) flushes it; every caller multiplies the
// weight next, which flushes a denormal input to 0 on both sides anyway.
//
// Shared by the device kernels (table in LDS) and the host test entry
// sdmm_test_norm_exp (tests/test_fastexp.py drives both against libm).
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

namespace sdmm {

// RN64(2^(j/64)), j = 0..63 (Python decimal at 60 digits, correctly rounded)
#define SDMM_EXP2J_TABLE                                                                         \
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0,     \
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0,     \
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0,     \
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0,     \
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0,     \
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0,     \
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0,     \
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0,     \
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0,     \
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0,     \
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0,     \
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0,     \
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0,     \
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0,     \
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0,     \
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0

constexpr double kInvLn2x64 = 0x1.71547652b82fep+6;    // 64 / ln 2
constexpr double kLn2d64Hi = 0x1.62e42fefa39efp-7;     // RN64(ln 2 / 64)
constexpr double kLn2d64Lo = 0x1.abc9e3b39803fp-62;    // RN64(ln 2 / 64 - hi)

// Fast attempt: the float result when decided (*ok = 1), else *ok = 0.
// tbl: the 64 table entries (LDS on the device).
__host__ __device__ __forceinline__ float norm_exp_try(float norm, float q, const double* tbl, int* ok) {
    const double x = -0.5 * (double)q;
    const double kd = rint(x * kInvLn2x64);
    const double r = fma(-kd, kLn2d64Lo, fma(-kd, kLn2d64Hi, x));
    const int k = (int)fmax(fmin(kd, 0.0), -60000.0);   // x <= 0; the clamp keeps NaN / -inf benign
    const double p = fma(fma(fma(fma(r, 1.0 / 24.0, 1.0 / 6.0), r, 0.5), r, 1.0), r, 1.0);
    const double y = ldexp((double)norm * (tbl[k & 63] * p), k >> 6);
    const float f = (float)y;
    uint32_t fb;
    memcpy(&fb, &f, 4);
    const uint32_t e = fb >> 23;   // y >= 0 (norm > 0): the sign bit is 0
    uint64_t ub = (uint64_t)(e + (1023u - 150u)) << 52;   // one float ulp at f, 2^(e - 150)
    double ulp;
    memcpy(&ulp, &ub, 8);
    const bool normal = e - 1u < 254u && (fb & 0x7FFFFFu) != 0u &&
                        fabs(y - (double)f) < ulp * (0.5 - 0x1p-16);
    const bool zero = y < 0x1p-126 * (1.0 - 0x1p-20);   // false for NaN
    *ok = (normal || zero) && q >= 0.0f;   // q is a sum of squares; anything else: the reference
    return normal ? f : 0.0f;
}

// The reference expression (the slow path, and what the fast path reproduces)
__host__ __device__ __forceinline__ float norm_exp_ref(float norm, float q) {
    return (float)((double)norm * exp(-0.5 * (double)q));
}

__host__ __device__ __forceinline__ float norm_exp(float norm, float q, const double* tbl) {
    int ok;
    const float f = norm_exp_try(norm, q, tbl, &ok);
    return ok ? f : norm_exp_ref(norm, q);
}

}  // namespace sdmm
