// learned_bsdf.h -- a glossy material's learned BSDF conditioned per bounce
// (host + device; render.hip's product bounces and the host ABI
// sdmm_learned4_conditional share this code, oracle/sdmm_oracle_li.inc
// restates it in C).
//
// Reference: RoughConductor::getDMM (mitsuba/src/bsdfs/roughconductor.cpp:
// 182-194) conditions the material's learned SDMM4 -- BSDF::SDMM4, a
// spatio-directional mixture over (theta_i, alpha) x direction, tangent
// space (theta, alpha, t1, t2) (include/mitsuba/render/bsdf.h:310-314),
// loaded from an .sdmm file by sdmm::load_json (:230-245) -- on the condition
// (theta_i = acos(min(1, cos theta_i)), alpha) with
// sdmm::create_conditional_pruned(conditioner, condition, dmm, 2), and the
// integrator then rotates the resulting 2-D directional mixture (DMM) about
// the normal onto wi's azimuth (rotate_to_wo, sdmm_proc.cpp:340-355).
//
// sdmm-lib is absent from the snapshot (an empty submodule), so the semantics
// below are this library's reading, stated so that the oracle restates the
// same thing (parity against sdmm-lib itself is unpinned):
//   * component k (weight pi_k, mean (mu_c in R^2, unit direction mu_d),
//     4x4 covariance over (theta, alpha, t1, t2), t = tangent coordinates at
//     mu_d in the Coordinates(mu_d) frame) conditioned on x = (theta, alpha):
//       pi'_k   = pi_k N(x; mu_c, S_cc)
//       shift   = S_dc S_cc^-1 (x - mu_c)            (tangent, at mu_d)
//       S'_dd   = S_dd - S_dc S_cc^-1 S_cd
//       mean'   = exp_{mu_d}(shift) = cos|s| mu_d + sin|s| u, u = (s1 e1 + s2 e2) / |s|
//       S'_dd re-expressed in Coordinates(mean') from the tangent basis e1,
//       e2 of mu_d parallel-transported along that geodesic;
//     a component whose S_cc or S'_dd is not positive definite gets pi' = 0;
//   * pruned(n): the n components of largest pi' (ties: the lower index),
//     renormalised to sum 1; none with pi' > 0 (or a non-finite sum): no
//     valid conditional (getDMM returns false: the plain conditional, h 0.5);
//   * rotate_to_wo(wi): means rotated about the normal by wi's azimuth, each
//     covariance re-expressed in the rotated mean's Coordinates frame (as
//     the round-5 stand-in did).
// Float arithmetic without contraction; exp / sin / cos / acos as the
// correctly rounded (float)f((double)x) of the library's other BSDF code.
#pragma once
#include <hip/hip_runtime.h>

namespace sdmm {

constexpr int kLearnedMaxComp = 8;                                  // components of one SDMM4
constexpr int kLearnedRec = 22;                                     // w, mean (5), cov (16)
constexpr int kLearnedStride = 1 + kLearnedMaxComp * kLearnedRec;   // per BSDF: [M, records]
constexpr int kLearnedKeep = 2;                                     // create_conditional_pruned(..., 2)

__host__ __device__ inline float l4_dot(const float a[3], const float b[3]) {
#pragma clang fp contract(off)
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
// jmm Coordinates (utils.h:32-48), as coordinates_f
__host__ __device__ inline void l4_coords(const float n[3], float to[9]) {
#pragma clang fp contract(off)
    const float sign = copysignf(1.0f, n[2]);
    const float a = -1.0f / (sign + n[2]);
    const float b = n[0] * n[1] * a;
    to[0] = 1.0f + sign * n[0] * n[0] * a; to[1] = sign * b; to[2] = -sign * n[0];
    to[3] = b; to[4] = sign + n[1] * n[1] * a; to[5] = -n[1];
    to[6] = n[0]; to[7] = n[1]; to[8] = n[2];
}
// C = B S B^T for 2x2 B (rows b0 b1) and symmetric S (s00, s01, s11)
__host__ __device__ inline void l4_congruence(float b00, float b01, float b10, float b11, float s00, float s01,
                                              float s11, float c[3]) {
#pragma clang fp contract(off)
    const float t00 = b00 * s00 + b01 * s01, t01 = b00 * s01 + b01 * s11;
    const float t10 = b10 * s00 + b11 * s01, t11 = b10 * s01 + b11 * s11;
    c[0] = t00 * b00 + t01 * b01;
    c[1] = t00 * b10 + t01 * b11;
    c[2] = t10 * b10 + t11 * b11;
}

// The conditional of an M-component SDMM4 (rec: M records of kLearnedRec
// floats) at (theta, alpha), pruned to `keep` lobes and rotated onto the local
// incident direction wl: lobe j's weight w[j], local unit mean mean[3j..],
// 2x2 covariance cov[4j..] in Coordinates(mean) (sdmm_bsdf_table's
// convention).  Returns the number of lobes written (0: no valid conditional).
__host__ __device__ inline int learned4_conditional(const float* rec, int M, float theta, float alpha,
                                                    const float wl[3], int keep, float* w, float* mean, float* cov) {
#pragma clang fp contract(off)
    constexpr float kTwoPi = 6.28318530717958647692f;
    if (M > kLearnedMaxComp) M = kLearnedMaxComp;
    if (keep > kLearnedMaxComp) keep = kLearnedMaxComp;
    float pw[kLearnedMaxComp], sh[kLearnedMaxComp][2], sc[kLearnedMaxComp][3];
    for (int k = 0; k < M; ++k) {
        const float* p = rec + kLearnedRec * k;
        pw[k] = 0.0f;
        sh[k][0] = sh[k][1] = 0.0f;
        sc[k][0] = sc[k][1] = sc[k][2] = 0.0f;
        const float a = p[6], b = p[7], c = p[11];   // S_cc
        if (!(a > 0.0f)) continue;
        const float l00 = sqrtf(a), l10 = b / l00, r = c - l10 * l10;
        if (!(r > 0.0f)) continue;
        const float l11 = sqrtf(r);
        const float z0 = (theta - p[1]) / l00;
        const float z1 = ((alpha - p[2]) - l10 * z0) / l11;
        const float q = z0 * z0 + z1 * z1;
        const float pc = (float)exp((double)(-0.5f * q)) / (kTwoPi * (l00 * l11));
        // S_cc^-1 (x - mu_c) = L^-T z; the tangent shift S_dc of it
        const float y1 = z1 / l11, y0 = (z0 - l10 * y1) / l00;
        sh[k][0] = p[14] * y0 + p[15] * y1;
        sh[k][1] = p[18] * y0 + p[19] * y1;
        // G = L^-1 S_cd (columns t1, t2); S'_dd = S_dd - G^T G
        const float g00 = p[8] / l00, g10 = (p[12] - l10 * g00) / l11;
        const float g01 = p[9] / l00, g11 = (p[13] - l10 * g01) / l11;
        const float s00 = p[16] - (g00 * g00 + g10 * g10);
        const float s01 = p[17] - (g00 * g01 + g10 * g11);
        const float s11 = p[21] - (g01 * g01 + g11 * g11);
        if (!(s00 > 0.0f) || !(s00 * s11 - s01 * s01 > 0.0f)) continue;
        sc[k][0] = s00; sc[k][1] = s01; sc[k][2] = s11;
        pw[k] = p[0] * pc;
    }
    // prune: the `keep` largest weights, ties to the lower index
    int sel[kLearnedMaxComp];
    int n = 0;
    float sum = 0.0f;
    for (int s = 0; s < keep; ++s) {
        int best = -1;
        for (int k = 0; k < M; ++k) {
            bool taken = false;
            for (int t = 0; t < n; ++t) taken = taken || sel[t] == k;
            if (taken || !(pw[k] > 0.0f)) continue;
            if (best < 0 || pw[k] > pw[best]) best = k;
        }
        if (best < 0) break;
        sel[n++] = best;
        sum += pw[best];
    }
    if (n == 0 || !(sum > 0.0f) || !(sum < __builtin_inff())) return 0;
    // rotate_to_wo: R = Rz(phi_i), cos / sin from wi's azimuth (1, 0 at the pole)
    const float sp2 = wl[0] * wl[0] + wl[1] * wl[1];
    float cr = 1.0f, sr = 0.0f;
    if (sp2 > 0.0f) {
        const float rs = 1.0f / sqrtf(sp2);
        cr = wl[0] * rs;
        sr = wl[1] * rs;
    }
    for (int j = 0; j < n; ++j) {
        const int k = sel[j];
        const float* p = rec + kLearnedRec * k;
        const float mu[3] = {p[3], p[4], p[5]};
        float tm[9];
        l4_coords(mu, tm);
        // mean' = exp_{mu}(shift); mu's tangent axes e1, e2 parallel-transported
        // along that geodesic: e_j + (e_j . u) ((cos|s| - 1) u - sin|s| mu),
        // u = the unit shift (e_j . u = s_j / |s|)
        float d[3] = {mu[0], mu[1], mu[2]};
        float e1[3] = {tm[0], tm[1], tm[2]}, e2[3] = {tm[3], tm[4], tm[5]};
        const float s0 = sh[k][0], s1 = sh[k][1];
        const float len2 = s0 * s0 + s1 * s1;
        if (len2 > 0.0f) {
            const float len = sqrtf(len2);
            const float sn = (float)sin((double)len), cs = (float)cos((double)len);
            const float u0 = s0 / len, u1 = s1 / len;
            float u[3];
            for (int i = 0; i < 3; ++i) u[i] = u0 * tm[i] + u1 * tm[3 + i];
            for (int i = 0; i < 3; ++i) d[i] = cs * mu[i] + sn * u[i];
            for (int i = 0; i < 3; ++i) {
                const float g = (cs - 1.0f) * u[i] - sn * mu[i];
                e1[i] = tm[i] + u0 * g;
                e2[i] = tm[3 + i] + u1 * g;
            }
        }
        const float rn = 1.0f / sqrtf(l4_dot(d, d));
        for (int i = 0; i < 3; ++i) d[i] = d[i] * rn;
        // S'_dd in Coordinates(mean'), from the transported axes
        float td[9];
        l4_coords(d, td);
        float c1[3];
        l4_congruence(l4_dot(td, e1), l4_dot(td, e2), l4_dot(td + 3, e1), l4_dot(td + 3, e2), sc[k][0], sc[k][1],
                      sc[k][2], c1);
        // rotate_to_wo: mean R d, the frame's axes R td_0, R td_1 re-expressed
        const float m[3] = {cr * d[0] - sr * d[1], sr * d[0] + cr * d[1], d[2]};
        float tr[9];
        l4_coords(m, tr);
        const float r1[3] = {cr * td[0] - sr * td[1], sr * td[0] + cr * td[1], td[2]};
        const float r2[3] = {cr * td[3] - sr * td[4], sr * td[3] + cr * td[4], td[5]};
        float c2[3];
        l4_congruence(l4_dot(tr, r1), l4_dot(tr, r2), l4_dot(tr + 3, r1), l4_dot(tr + 3, r2), c1[0], c1[1], c1[2],
                      c2);
        w[j] = pw[k] / sum;
        mean[3 * j] = m[0]; mean[3 * j + 1] = m[1]; mean[3 * j + 2] = m[2];
        cov[4 * j] = c2[0]; cov[4 * j + 1] = c2[1]; cov[4 * j + 2] = c2[1]; cov[4 * j + 3] = c2[2];
    }
    return n;
}

}  // namespace sdmm
