// render.hip -- the guided path tracer's device side: SDMMRenderer::Li
// (sdmm_proc.cpp:592-968) as a wavefront over an analytic quad scene, and the
// training-data producer of its tail (push_back_data + jittered neighbour
// routing, :876-965).
//
// One path per thread, path state in SoA planes in HBM.  A bounce is three
// launches on one stream:
//   li_query_kernel   the loop head for every live path (:649-691): depth cap,
//                     condition c = (p - scene_min) / spatial_norm
//                     (createCondition :263-273), the BSDF direction and the
//                     plugin's BSDF/guide choice (h = 0.5, :383-392);
//   the guided wavefront (guide.hip, sdmm_guide_pdf_wavefront): the leaf's
//                     conditional built once per query, then a GMM sample or
//                     the gmmPdf of the BSDF direction (:368-421, :510-590);
//   li_shade_kernel   the rest of sampleSurface (:392-507) and of the loop
//                     body (:759-871): BSDF weight / mixture pdf, throughput,
//                     the next ray, the emitter it hits, recordRadiance and the
//                     saved vertex (:815-846), Russian roulette.
// The camera kernel starts the paths (first hit, its emission: :641-677); the
// film kernel averages each pixel's samples in sample order (box filter).
//
// Scene: parallelograms (Mitsuba rectangles; a cube is six), diffuse BSDFs
// (diffuse.cpp: cosine-hemisphere sampling, f = rho / pi) and smooth plastic
// (plastic.cpp: a delta specular lobe with the dielectric Fresnel reflectance
// over a diffuse base, the lobe chosen by Fresnel-weighted probability), one-
// sided area emitters (area.cpp: Le = radiance on the normal side).  No NEE (the plugin's
// NEE block is compiled out, :700-734; emitterPdf = 0, MIS weight 1, :811-816).
//
// Random numbers: counter-based (rng_uniform below), one fixed slot per
// (path, stream, dimension) -- a path's outcome does not depend on which other
// paths run, nor on the order the reference's sampler would consume numbers;
// the reference's Mitsuba sampler itself is not reproducible here.
#include "sdmm_device.h"
#include "render_device.h"
#include "learned_bsdf.h"

#include <hipcub/hipcub.hpp>

#pragma clang fp contract(off)

namespace sdmm {

// RNG, scene / path / query records: render_device.h
constexpr float kEpsilon = 1e-4f;          // Mitsuba single-precision Epsilon (ray mint)
constexpr float kInvPi = 0.31830988618379067154f;

__device__ __forceinline__ float dot3(const float a[3], const float b[3]) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

// closest hit with t in (mint, maxt); -1: none
__device__ __forceinline__ int intersect(const SceneDev& S, const float o[3], const float d[3], float mint,
                                         float maxt, float& t_hit) {
    int best = -1;
    float tb = maxt;
    for (int q = 0; q < S.n_quads; ++q) {
        const QuadDev& Q = S.quads[q];
        const float denom = dot3(d, Q.n);
        if (denom == 0.0f) continue;
        const float r0[3] = {Q.p0[0] - o[0], Q.p0[1] - o[1], Q.p0[2] - o[2]};
        const float t = dot3(r0, Q.n) / denom;
        if (!(t > mint && t < tb)) continue;
        const float r[3] = {o[0] + t * d[0] - Q.p0[0], o[1] + t * d[1] - Q.p0[1], o[2] + t * d[2] - Q.p0[2]};
        const float a = dot3(r, Q.g1), b = dot3(r, Q.g2);
        if (a < 0.0f || a > 1.0f || b < 0.0f || b > 1.0f) continue;
        tb = t;
        best = q;
    }
    t_hit = tb;
    return best;
}

// Frame(n): Mitsuba coordinateSystem (s, t, n)
__device__ __forceinline__ void frame_of(const float n[3], float s[3], float t[3]) {
    if (fabsf(n[0]) > fabsf(n[1])) {
        const float inv = 1.0f / sqrtf(n[0] * n[0] + n[2] * n[2]);
        t[0] = n[2] * inv; t[1] = 0.0f; t[2] = -n[0] * inv;
    } else {
        const float inv = 1.0f / sqrtf(n[1] * n[1] + n[2] * n[2]);
        t[0] = 0.0f; t[1] = n[2] * inv; t[2] = -n[1] * inv;
    }
    s[0] = t[1] * n[2] - t[2] * n[1];
    s[1] = t[2] * n[0] - t[0] * n[2];
    s[2] = t[0] * n[1] - t[1] * n[0];
}

// warp::squareToCosineHemisphere (concentric disk, z guarded to 1e-10)
__device__ __forceinline__ void cosine_hemisphere(float u0, float u1, float w[3]) {
    const float r1 = 2.0f * u0 - 1.0f, r2 = 2.0f * u1 - 1.0f;
    float r, phi;
    if (r1 == 0.0f && r2 == 0.0f) {
        r = 0.0f; phi = 0.0f;
    } else if (r1 * r1 > r2 * r2) {
        r = r1; phi = (float)(kPi / 4.0) * (r2 / r1);
    } else {
        r = r2; phi = (float)(kPi / 2.0) - (r1 / r2) * (float)(kPi / 4.0);
    }
    // sin / cos in double, rounded: the float values the CPU restatement
    // (oracle/sdmm_oracle_li.inc) forms with the C library
    double sd, cd;
    sincos((double)phi, &sd, &cd);
    const float sp = (float)sd, cp = (float)cd;
    w[0] = r * cp;
    w[1] = r * sp;
    float z = sqrtf(fmaxf(0.0f, 1.0f - w[0] * w[0] - w[1] * w[1]));
    if (z == 0.0f) z = 1e-10f;
    w[2] = z;
}

// fresnelDielectricExt (libcore/util.cpp:651-681): the unpolarised
// reflectance at cos(theta_i) for the relative index eta
__device__ __forceinline__ float fresnel_dielectric(float cos_i, float eta) {
    if (eta == 1.0f) return 0.0f;
    const float scale = cos_i > 0.0f ? 1.0f / eta : eta;
    const float ct2 = 1.0f - (1.0f - cos_i * cos_i) * (scale * scale);
    if (ct2 <= 0.0f) return 1.0f;
    const float ci = fabsf(cos_i), ct = sqrtf(ct2);
    const float rs = (ci - eta * ct) / (ci + eta * ct);
    const float rp = (eta * ci - ct) / (eta * ci + ct);
    return 0.5f * (rs * rs + rp * rp);
}

// SmoothPlastic's specular sampling probability (plastic.cpp:339-342)
__device__ __forceinline__ float plastic_prob_specular(float Fi, float ssw) {
    // 0 / 0 (no specular weight at a total reflection, or weight 1 with Fi =
    // 0) is 0 here, NaN in plastic.cpp:339-342: both lobes then carry no
    // energy along that direction, and a NaN would only poison the sample
    const float num = Fi * ssw, den = num + (1.0f - Fi) * (1.0f - ssw);
    return den == 0.0f ? 0.0f : num / den;
}

// ---------------------------------------------------------------------------
// Rough conductor (bsdfs/roughconductor.cpp:296-470 over microfacet.h): the
// Beckmann distribution with isotropic alpha, sampleVisible = false (sampleAll
// / pdfAll, microfacet.h:287-407 -- a documented choice of the plugin), a gray
// conductor (eta, k equal over the channels; fresnelConductorExact's Spectrum
// form, libcore/util.cpp:739-761) times the specular reflectance.  exp / log /
// sin / cos as (float)f((double)x): math::fastexp / fastlog on Linux x86_64
// (math.h:185-197) and the library's sincos convention.
constexpr float kPiF = 3.14159265358979323846f;

__device__ __forceinline__ float fresnel_conductor(float ci, float eta, float k) {
    const float ci2 = ci * ci, si2 = 1.0f - ci2, si4 = si2 * si2;
    const float t1 = eta * eta - k * k - si2;
    const float a2pb2 = sqrtf(fmaxf(0.0f, t1 * t1 + k * k * eta * eta * 4.0f));
    const float a = sqrtf(fmaxf(0.0f, (a2pb2 + t1) * 0.5f));
    const float term1 = a2pb2 + ci2, term2 = a * (2.0f * ci);
    const float rs2 = (term1 - term2) / (term1 + term2);
    const float term3 = a2pb2 * ci2 + si4, term4 = term2 * si2;
    const float rp2 = rs2 * (term3 - term4) / (term3 + term4);
    return 0.5f * (rp2 + rs2);
}

// MicrofacetDistribution::eval (microfacet.h:191-233), Beckmann
__device__ __forceinline__ float beckmann_d(const float m[3], float alpha) {
    if (m[2] <= 0.0f) return 0.0f;
    const float ct2 = m[2] * m[2];
    const float ex = ((m[0] * m[0]) / (alpha * alpha) + (m[1] * m[1]) / (alpha * alpha)) / ct2;
    float r = (float)exp((double)-ex) / (kPiF * alpha * alpha * ct2 * ct2);
    if (r * m[2] < 1e-20f) r = 0.0f;
    return r;
}

// smithG1 (microfacet.h:477-518), Beckmann's rational approximation
__device__ __forceinline__ float beckmann_g1(const float v[3], const float m[3], float alpha) {
    if (dot3(v, m) * v[2] <= 0.0f) return 0.0f;
    const float tmp = 1.0f - v[2] * v[2];
    const float tan_t = tmp <= 0.0f ? 0.0f : fabsf(sqrtf(tmp) / v[2]);
    if (tan_t == 0.0f) return 1.0f;
    const float a = 1.0f / (alpha * tan_t);
    if (a >= 1.6f) return 1.0f;
    const float a2 = a * a;
    return (3.535f * a + 2.181f * a2) / (1.0f + 2.276f * a + 2.577f * a2);
}

// Vector3 normalize (v * (1 / |v|), vector.h:625-627)
__device__ __forceinline__ void normalize3(const float v[3], float r[3]) {
    const float rc = 1.0f / sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    r[0] = v[0] * rc; r[1] = v[1] * rc; r[2] = v[2] * rc;
}

// RoughConductor::sample(bRec, pdf, sample) (roughconductor.cpp:414-462) in the
// local frame, wi.z > 0: wo, the weight F * (D G (wi.m) / (pdf cos)) and the
// solid-angle pdf; false: the sample is void (weight 0)
__device__ __forceinline__ bool conductor_sample(const float wi[3], const float* bp, float u0, float u1,
                                                 float wo[3], float bw[3], float* pdf) {
    const float alpha = bp[6];
    // sampleAll (microfacet.h:287-395), isotropic Beckmann
    const float phi = (2.0f * kPiF) * u1;
    double sd, cd;
    sincos((double)phi, &sd, &cd);
    const float sp = (float)sd, cp = (float)cd;
    const float a2 = alpha * alpha;
    const float tan2 = a2 * -(float)log((double)(1.0f - u0));
    const float ct = 1.0f / sqrtf(1.0f + tan2);
    float mpdf = (1.0f - u0) / (kPiF * alpha * alpha * ct * ct * ct);
    if (mpdf < 1e-20f) mpdf = 0.0f;
    const float st = sqrtf(fmaxf(0.0f, 1.0f - ct * ct));
    const float m[3] = {st * cp, st * sp, ct};
    *pdf = 0.0f;
    bw[0] = bw[1] = bw[2] = 0.0f;
    wo[0] = 0.0f; wo[1] = 0.0f; wo[2] = 1.0f;
    if (mpdf == 0.0f) return false;
    const float dm = dot3(wi, m);
    for (int a = 0; a < 3; ++a) wo[a] = 2.0f * dm * m[a] - wi[a];   // reflect
    if (wo[2] <= 0.0f) return false;
    const float fr = fresnel_conductor(dm, bp[4], bp[5]);
    const float g = beckmann_g1(wi, m, alpha) * beckmann_g1(wo, m, alpha);
    const float weight = beckmann_d(m, alpha) * g * dm / (mpdf * wi[2]);
    for (int ch = 0; ch < 3; ++ch) bw[ch] = fr * bp[1 + ch] * weight;
    *pdf = mpdf / (4.0f * dot3(wo, m));
    return true;
}

// RoughConductor::eval (ESolidAngle, :302-339) and pdf (:341-366) in the local
// frame
__device__ __forceinline__ float conductor_eval_pdf(const float wi[3], const float wo[3], const float* bp,
                                                    float f[3]) {
    f[0] = f[1] = f[2] = 0.0f;
    if (wi[2] <= 0.0f || wo[2] <= 0.0f) return 0.0f;
    const float alpha = bp[6];
    const float hs[3] = {wo[0] + wi[0], wo[1] + wi[1], wo[2] + wi[2]};
    float H[3];
    normalize3(hs, H);
    const float D = beckmann_d(H, alpha);
    if (D != 0.0f) {
        const float fr = fresnel_conductor(dot3(wi, H), bp[4], bp[5]);
        const float G = beckmann_g1(wi, H, alpha) * beckmann_g1(wo, H, alpha);
        const float model = D * G / (4.0f * wi[2]);
        for (int ch = 0; ch < 3; ++ch) f[ch] = fr * bp[1 + ch] * model;
    }
    return D * H[2] / (4.0f * fabsf(dot3(wo, H)));
}

__device__ __forceinline__ float& vrec(const PathsDev& P, int f, int v, int64_t p) {
    return P.rec[((int64_t)f * P.V + v) * P.P + p];
}

// recordRadiance (:628-637): every saved vertex's weight gets the radiance
// divided by its throughput and sampling pdf (Vertex::record, :615-621)
__device__ __forceinline__ void record_radiance(const PathsDev& P, int64_t p, int nv, const float rad[3]) {
    for (int v = 0; v < nv; ++v) {
        const float pdf = vrec(P, 6, v, p);
        for (int ch = 0; ch < 3; ++ch) {
            const float thr = vrec(P, 3 + ch, v, p);
            if (thr > kEpsilon) vrec(P, ch, v, p) += rad[ch] / (thr * pdf);
        }
    }
}

// ---------------------------------------------------------------------------
// camera rays: pixel = path / spp (box filter, uniform jitter), Mitsuba's
// perspective mapping (fov along x): local d = ((1 - 2 sx) tan, (1 - 2 sy) tan / aspect, 1)
__global__ void __launch_bounds__(256)
li_camera_kernel(SceneDev S, PathsDev P, int64_t path0, int spp, uint64_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.P) return;
    const int64_t gp = path0 + i;
    const int64_t pix = gp / spp;
    const int px = (int)(pix % S.width), py = (int)(pix / S.width);
    const float sx = ((float)px + rng_uniform(seed, (uint64_t)gp, 0, 0)) / (float)S.width;
    const float sy = ((float)py + rng_uniform(seed, (uint64_t)gp, 0, 1)) / (float)S.height;
    float l[3] = {(1.0f - 2.0f * sx) * S.tanx, (1.0f - 2.0f * sy) * S.tanx / S.aspect, 1.0f};
    const float inv = 1.0f / sqrtf(dot3(l, l));
    for (int a = 0; a < 3; ++a) l[a] *= inv;
    float d[3], o[3];
    for (int r = 0; r < 3; ++r) {
        d[r] = S.cam[4 * r] * l[0] + S.cam[4 * r + 1] * l[1] + S.cam[4 * r + 2] * l[2];
        o[r] = S.cam[4 * r + 3];
    }
    const float dn = 1.0f / sqrtf(dot3(d, d));
    for (int a = 0; a < 3; ++a) d[a] *= dn;
    float t;
    const int q = intersect(S, o, d, S.near_clip / l[2], INFINITY, t);
    P.tr[i] = 1.0f; P.tg[i] = 1.0f; P.tb[i] = 1.0f;
    P.nv[i] = 0;
    P.nray[i] = 0;
    P.dx[i] = d[0]; P.dy[i] = d[1]; P.dz[i] = d[2];
    float L[3] = {0.0f, 0.0f, 0.0f};
    if (q >= 0) {
        const QuadDev& Q = S.quads[q];
        P.px[i] = o[0] + t * d[0]; P.py[i] = o[1] + t * d[1]; P.pz[i] = o[2] + t * d[2];
        // emission seen directly (:674-677), before any vertex exists
        if (Q.emitter >= 0 && -dot3(d, Q.n) > 0.0f)
            for (int ch = 0; ch < 3; ++ch) L[ch] = S.rad[3 * Q.emitter + ch];
    }
    P.lr[i] = L[0]; P.lg[i] = L[1]; P.lb[i] = L[2];
    P.quad[i] = q;
    P.depth[i] = q >= 0 ? 1 : -1;   // no hit: no environment emitter, the path ends
}

// ---------------------------------------------------------------------------
// Loop head of bounce b for every live path.  guided: the tree holds trained
// leaves (m_iteration != 0, :311-316); otherwise every query is BSDF only.
__global__ void __launch_bounds__(256)
li_query_kernel(SceneDev S, PathsDev P, QueryDev Q, int64_t path0, int bounce, int max_depth, int guided,
                float h, uint64_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.P) return;
    int depth = P.depth[i];
    bool live = depth >= 0;
    if (live && max_depth >= 0 && depth >= max_depth) live = false;   // :684-685
    int q = live ? P.quad[i] : -1;
    float n[3] = {0, 0, 0}, wi[3] = {0, 0, 0};
    if (live) {
        const QuadDev& QD = S.quads[q];
        n[0] = QD.n[0]; n[1] = QD.n[1]; n[2] = QD.n[2];
        wi[0] = -P.dx[i]; wi[1] = -P.dy[i]; wi[2] = -P.dz[i];
        const float* rho = S.refl + 3 * QD.bsdf;
        const float* bp = S.bpar ? S.bpar + kBsdfParams * QD.bsdf : nullptr;
        const int kind = bp ? (int)bp[0] : kBsdfDiffuse;
        const bool zero_spec = kind == kBsdfDiffuse || (bp[1] == 0.0f && bp[2] == 0.0f && bp[3] == 0.0f);
        const bool zero_diff = kind == kBsdfConductor || (rho[0] == 0.0f && rho[1] == 0.0f && rho[2] == 0.0f);
        // no reflection from the back side or with zero reflectances (the
        // light's BSDF): sample and eval are 0, the path ends (:772-774)
        if (!(dot3(wi, n) > 0.0f) || (zero_diff && zero_spec)) live = false;
    }
    Q.live[i] = (uint8_t)((live && guided) ? 1 : 0);
    Q.slot[i] = -1;
    if (!live) {
        P.depth[i] = -1;
        return;
    }
    const uint64_t gp = (uint64_t)(path0 + i);
    const uint32_t stream = 1u + (uint32_t)bounce;
    const float p[3] = {P.px[i], P.py[i], P.pz[i]};
    Q.c0[i] = (p[0] - S.smin[0]) / S.snorm;
    Q.c1[i] = (p[1] - S.smin[1]) / S.snorm;
    Q.c2[i] = (p[2] - S.smin[2]) / S.snorm;
    float s[3], t[3], w[3];
    frame_of(n, s, t);
    const float* bp = S.bpar ? S.bpar + kBsdfParams * S.quads[q].bsdf : nullptr;
    uint8_t delta = 0;
    if (bp && bp[0] == (float)kBsdfPlastic) {
        // SmoothPlastic::sample(bRec, pdf, sample) (plastic.cpp:378-420): the
        // delta mirror lobe with probability probSpecular, else the cosine
        // hemisphere on the rescaled first coordinate; weight and pdf for the
        // shade kernel (a mixture bounce keeps the sampled lobe, :392-407)
        const float* rho = S.refl + 3 * S.quads[q].bsdf;
        const float wl[3] = {dot3(wi, s), dot3(wi, t), dot3(wi, n)};   // Frame::toLocal
        const float Fi = fresnel_dielectric(wl[2], bp[4]);
        const float ps = plastic_prob_specular(Fi, bp[7]);
        const float u0 = rng_uniform(seed, gp, stream, 0), u1 = rng_uniform(seed, gp, stream, 1);
        if (u0 < ps) {
            delta = 1;
            w[0] = -wl[0]; w[1] = -wl[1]; w[2] = wl[2];
            // Spectrum * Fi / probSpecular (TSpectrum::operator/: times the reciprocal)
            const float rs = 1.0f / ps;
            Q.bw0[i] = bp[1] * Fi * rs; Q.bw1[i] = bp[2] * Fi * rs; Q.bw2[i] = bp[3] * Fi * rs;
            Q.bpdf[i] = ps;
        } else {
            cosine_hemisphere((u0 - ps) / (1.0f - ps), u1, w);
            const float Fo = fresnel_dielectric(w[2], bp[4]);
            // diff /= 1 - fdrInt; diff * (invEta2 (1 - Fi) (1 - Fo) / (1 - probSpecular))
            const float rd = 1.0f / (1.0f - bp[6]);
            const float k = bp[5] * (1.0f - Fi) * (1.0f - Fo) / (1.0f - ps);
            Q.bw0[i] = rho[0] * rd * k;
            Q.bw1[i] = rho[1] * rd * k;
            Q.bw2[i] = rho[2] * rd * k;
            Q.bpdf[i] = (1.0f - ps) * (kInvPi * w[2]);
        }
    } else if (bp && bp[0] == (float)kBsdfConductor) {
        // RoughConductor::sample (roughconductor.cpp:414-462); a void sample
        // has weight 0 (the path ends if the BSDF direction is taken)
        const float wl[3] = {dot3(wi, s), dot3(wi, t), dot3(wi, n)};
        float bw[3], bpdf;
        conductor_sample(wl, bp, rng_uniform(seed, gp, stream, 0), rng_uniform(seed, gp, stream, 1), w, bw, &bpdf);
        Q.bw0[i] = bw[0]; Q.bw1[i] = bw[1]; Q.bw2[i] = bw[2];
        Q.bpdf[i] = bpdf;
    } else {
        cosine_hemisphere(rng_uniform(seed, gp, stream, 0), rng_uniform(seed, gp, stream, 1), w);
    }
    Q.bdelta[i] = delta;
    Q.b0[i] = s[0] * w[0] + t[0] * w[1] + n[0] * w[2];
    Q.b1[i] = s[1] * w[0] + t[1] * w[1] + n[1] * w[2];
    Q.b2[i] = s[2] * w[0] + t[2] * w[1] + n[2] * w[2];
    Q.u0[i] = rng_uniform(seed, gp, stream, 3);
    Q.u1[i] = rng_uniform(seed, gp, stream, 4);
    Q.u2[i] = rng_uniform(seed, gp, stream, 5);
    const float choice = rng_uniform(seed, gp, stream, 2);
    Q.ch[i] = choice;
    Q.mode[i] = (!guided || choice <= h) ? 1 : 0;
}

// the live guided queries, compacted: query j serves path idx[j].  With
// product sampling also the query's shading frame F = [s t n] (Frame(n) of
// the hit quad), its material (the quad's BSDF: its learned-BSDF table row;
// diffuse here, so getDMM succeeds for every live path, cosTheta(wi) > 0,
// bsdfs/diffuse.cpp:86-92) and the BSDF/guide draw.
__global__ void __launch_bounds__(256)
li_compact_kernel(SceneDev S, PathsDev P, QueryDev Q, const int32_t* __restrict__ count, int product) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= *count) return;
    const int i = Q.idx[j];
    Q.k_c0[j] = Q.c0[i]; Q.k_c1[j] = Q.c1[i]; Q.k_c2[j] = Q.c2[i];
    Q.k_u0[j] = Q.u0[i]; Q.k_u1[j] = Q.u1[i]; Q.k_u2[j] = Q.u2[i];
    Q.k_b0[j] = Q.b0[i]; Q.k_b1[j] = Q.b1[i]; Q.k_b2[j] = Q.b2[i];
    Q.k_mode[j] = Q.mode[i];
    Q.slot[i] = j;
    if (product) {
        const QuadDev& QD = S.quads[P.quad[i]];
        float s[3], t[3];
        frame_of(QD.n, s, t);
        for (int r = 0; r < 3; ++r) {
            Q.k_F[3 * r][j] = s[r];
            Q.k_F[3 * r + 1][j] = t[r];
            Q.k_F[3 * r + 2][j] = QD.n[r];
        }
        Q.k_mat[j] = QD.bsdf;
        Q.k_ch[j] = Q.ch[i];
        const float* bp = S.bpar ? S.bpar + kBsdfParams * QD.bsdf : nullptr;
        if (Q.lw && bp && bp[0] == (float)kBsdfConductor) {
            // getDMM (roughconductor.cpp:182-194: the material's SDMM4
            // conditioned on (theta_i, alpha), pruned to 2) + rotate_to_wo
            // (sdmm_proc.cpp:340-355): the query's own lobes, local frame, in
            // its row of the extended table; no model or no valid conditional:
            // no learned BSDF (the plain conditional, h 0.5)
            const float wi[3] = {-P.dx[i], -P.dy[i], -P.dz[i]};
            const float wl[3] = {dot3(wi, s), dot3(wi, t), dot3(wi, QD.n)};
            const int64_t row = (int64_t)Q.lrow0 + j;
            const float* lm = S.lmodel ? S.lmodel + (size_t)kLearnedStride * QD.bsdf : nullptr;
            const int M = lm ? (int)lm[0] : 0;
            int kept = 0;
            if (M > 0) {
                const float theta = (float)acos((double)fminf(1.0f, wl[2]));
                kept = learned4_conditional(lm + 1, M, theta, bp[6], wl, kLearnedKeep, Q.lw + row * Q.lM,
                                            Q.lm + row * Q.lM * 3, Q.lc + row * Q.lM * 4);
            }
            for (int l = kept; l < Q.lM; ++l) Q.lw[row * Q.lM + l] = 0.0f;   // (skipped lobes)
            Q.k_mat[j] = kept > 0 ? (int32_t)row : -1;
        }
    }
}

// ---------------------------------------------------------------------------
// The rest of the bounce (:392-507, :759-871).
// product: the query's own heuristicConditionalWeight (0.3 with a usable
// product, 0.5 for the plain conditional, sdmm_proc.cpp:383-392) replaces h.
// The wavefront marks a query whose BSDF sample was chosen comp == -2 (valid
// conditional) -- the plain bounce's pdf_mode and the product bounce's
// choice <= h alike.
__global__ void __launch_bounds__(256)
li_shade_kernel(SceneDev S, PathsDev P, QueryDev Q, int64_t path0, int bounce, int rr_depth, float h,
                uint64_t seed, int product) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.P) return;
    int depth = P.depth[i];
    if (depth < 0) return;
    const QuadDev& QD = S.quads[P.quad[i]];
    const float n[3] = {QD.n[0], QD.n[1], QD.n[2]};
    const float* rho = S.refl + 3 * QD.bsdf;
    const float c[3] = {Q.c0[i], Q.c1[i], Q.c2[i]};
    const int j = Q.slot[i];            // the path's guided query (-1: none, BSDF only)
    const int comp = j >= 0 ? Q.comp[j] : -1;
    const bool valid = comp != -1;      // validConditional (:368)
    if (product && valid) h = Q.hq[j];
    float wo[3], weight[3], mis_pdf;
    const float* bp = S.bpar ? S.bpar + kBsdfParams * QD.bsdf : nullptr;
    bool cacheable = true;
    if (bp && bp[0] == (float)kBsdfPlastic) {
        // smooth plastic (plastic.cpp): the loop head's sample (weight, pdf,
        // lobe) or the guide's direction under eval / pdf, the smooth part only
        const float wi[3] = {-P.dx[i], -P.dy[i], -P.dz[i]};
        const float Fi = fresnel_dielectric(dot3(wi, n), bp[4]);
        const float ps = plastic_prob_specular(Fi, bp[7]);
        const bool delta = Q.bdelta[i] != 0;
        const float bw[3] = {Q.bw0[i], Q.bw1[i], Q.bw2[i]};
        if (!valid || comp == -2) {
            wo[0] = Q.b0[i]; wo[1] = Q.b1[i]; wo[2] = Q.b2[i];
            cacheable = !delta;                 // :764
            if (!valid) {
                // BSDF only, h = 1 (:316-323, :392-405)
                mis_pdf = Q.bpdf[i];
                for (int ch = 0; ch < 3; ++ch) weight[ch] = bw[ch];
            } else if (delta) {
                // a delta lobe of the chosen BSDF sample: gmmPdf = 0, pdf *= h,
                // weight / h (:401-405)
                mis_pdf = Q.bpdf[i] * h;
                const float rh = 1.0f / h;
                for (int ch = 0; ch < 3; ++ch) weight[ch] = bw[ch] * rh;
            } else {
                // (bsdfWeight * bsdfPdf) / pdfSurface (:407, :531-534, :587-589)
                const float bsdf_pdf = Q.bpdf[i];
                mis_pdf = bsdf_pdf > 0.0f ? h * bsdf_pdf + (1.0f - h) * Q.pdf[j] : 0.0f;
                for (int ch = 0; ch < 3; ++ch) weight[ch] = mis_pdf == 0.0f ? 0.0f : (bw[ch] * bsdf_pdf) * (1.0f / mis_pdf);
            }
        } else {
            // the guide's direction: bsdf->eval (smooth lobe, ESolidAngle) / pdfSurface (:456-507)
            wo[0] = Q.d0[j]; wo[1] = Q.d1[j]; wo[2] = Q.d2[j];
            const float cos_o = dot3(wo, n);
            const bool zero = (wo[0] == 0.0f && wo[1] == 0.0f && wo[2] == 0.0f) || !__builtin_isfinite(cos_o);
            const bool up = !zero && cos_o > 0.0f;
            const float cpdf = kInvPi * cos_o;   // warp::squareToCosineHemispherePdf
            const float bsdf_pdf = up ? cpdf * (1.0f - ps) : 0.0f;
            mis_pdf = bsdf_pdf > 0.0f ? h * bsdf_pdf + (1.0f - h) * Q.pdf[j] : 0.0f;
            const float Fo = up ? fresnel_dielectric(cos_o, bp[4]) : 0.0f;
            const float rd = 1.0f / (1.0f - bp[6]);
            const float k = cpdf * bp[5] * (1.0f - Fi) * (1.0f - Fo);
            for (int ch = 0; ch < 3; ++ch) {
                const float f = up ? S.refl[3 * QD.bsdf + ch] * rd * k : 0.0f;
                weight[ch] = mis_pdf == 0.0f ? 0.0f : f * (1.0f / mis_pdf);
            }
        }
    } else if (bp && bp[0] == (float)kBsdfConductor) {
        // rough conductor: the loop head's sample (weight, pdf) or the guide's
        // direction under eval / pdf (:392-407, :456-507)
        const float bw[3] = {Q.bw0[i], Q.bw1[i], Q.bw2[i]};
        if (!valid || comp == -2) {
            wo[0] = Q.b0[i]; wo[1] = Q.b1[i]; wo[2] = Q.b2[i];
            const float bsdf_pdf = Q.bpdf[i];
            if (!valid) {
                mis_pdf = bsdf_pdf;
                for (int ch = 0; ch < 3; ++ch) weight[ch] = bw[ch];
            } else {
                mis_pdf = bsdf_pdf > 0.0f ? h * bsdf_pdf + (1.0f - h) * Q.pdf[j] : 0.0f;
                for (int ch = 0; ch < 3; ++ch) weight[ch] = mis_pdf == 0.0f ? 0.0f : (bw[ch] * bsdf_pdf) * (1.0f / mis_pdf);
            }
        } else {
            wo[0] = Q.d0[j]; wo[1] = Q.d1[j]; wo[2] = Q.d2[j];
            float s[3], t[3];
            frame_of(n, s, t);
            const float wi[3] = {-P.dx[i], -P.dy[i], -P.dz[i]};
            const float wil[3] = {dot3(wi, s), dot3(wi, t), dot3(wi, n)};
            const float wol[3] = {dot3(wo, s), dot3(wo, t), dot3(wo, n)};
            const bool zero = (wo[0] == 0.0f && wo[1] == 0.0f && wo[2] == 0.0f) || !__builtin_isfinite(wol[2]);
            float f[3] = {0.0f, 0.0f, 0.0f};
            const float bsdf_pdf = zero ? 0.0f : conductor_eval_pdf(wil, wol, bp, f);
            mis_pdf = bsdf_pdf > 0.0f ? h * bsdf_pdf + (1.0f - h) * Q.pdf[j] : 0.0f;
            for (int ch = 0; ch < 3; ++ch) weight[ch] = mis_pdf == 0.0f ? 0.0f : f[ch] * (1.0f / mis_pdf);
        }
    } else if (!valid) {
        // BSDF only, h = 1 (:316-323, :392-405): weight = rho, pdf = bsdfPdf
        wo[0] = Q.b0[i]; wo[1] = Q.b1[i]; wo[2] = Q.b2[i];
        const float cos_o = dot3(wo, n);
        mis_pdf = kInvPi * cos_o;
        for (int ch = 0; ch < 3; ++ch) weight[ch] = rho[ch];
    } else if (comp == -2) {
        // BSDF chosen: (bsdf weight * bsdfPdf) / (h bsdfPdf + (1 - h) gmmPdf) (:393-407, :587-589)
        wo[0] = Q.b0[i]; wo[1] = Q.b1[i]; wo[2] = Q.b2[i];
        const float bsdf_pdf = kInvPi * dot3(wo, n);
        mis_pdf = bsdf_pdf > 0.0f ? h * bsdf_pdf + (1.0f - h) * Q.pdf[j] : 0.0f;   // pdfSurface (:531-534)
        for (int ch = 0; ch < 3; ++ch) weight[ch] = mis_pdf == 0.0f ? 0.0f : (rho[ch] * bsdf_pdf) * (1.0f / mis_pdf);
    } else {
        // guide sample: bsdf->eval / pdf (:456-463, :504-507)
        wo[0] = Q.d0[j]; wo[1] = Q.d1[j]; wo[2] = Q.d2[j];
        const float cos_o = dot3(wo, n);
        const bool zero = (wo[0] == 0.0f && wo[1] == 0.0f && wo[2] == 0.0f) || !__builtin_isfinite(cos_o);
        const float bsdf_pdf = (!zero && cos_o > 0.0f) ? kInvPi * cos_o : 0.0f;
        mis_pdf = bsdf_pdf > 0.0f ? h * bsdf_pdf + (1.0f - h) * Q.pdf[j] : 0.0f;   // pdfSurface (:531-534)
        for (int ch = 0; ch < 3; ++ch) weight[ch] = mis_pdf == 0.0f ? 0.0f : (rho[ch] * (kInvPi * cos_o)) * (1.0f / mis_pdf);
    }
    const float cos_o = dot3(wo, n);
    // zero weight, or strict normals (wo . n_geo * cos(wo) <= 0, :777-780): the path ends
    if ((weight[0] == 0.0f && weight[1] == 0.0f && weight[2] == 0.0f) || !(cos_o * cos_o > 0.0f) ||
        !__builtin_isfinite(weight[0] + weight[1] + weight[2])) {
        P.depth[i] = -1;
        return;
    }
    float thr[3] = {P.tr[i] * weight[0], P.tg[i] * weight[1], P.tb[i] * weight[2]};
    // trace and look for an emitter (rayIntersectAndLookForEmitter)
    const float o[3] = {P.px[i], P.py[i], P.pz[i]};
    float t;
    const int q = intersect(S, o, wo, kEpsilon, INFINITY, t);
    float value[3] = {0.0f, 0.0f, 0.0f};
    if (q >= 0) {
        const QuadDev& H = S.quads[q];
        if (H.emitter >= 0 && -dot3(wo, H.n) > 0.0f)
            for (int ch = 0; ch < 3; ++ch) value[ch] = S.rad[3 * H.emitter + ch];
    }
    int nv = P.nv[i];
    if (value[0] != 0.0f || value[1] != 0.0f || value[2] != 0.0f) {
        const float rad[3] = {thr[0] * value[0], thr[1] * value[1], thr[2] * value[2]};
        P.lr[i] += rad[0]; P.lg[i] += rad[1]; P.lb[i] += rad[2];
        record_radiance(P, i, nv, rad);
    }
    P.nray[i] += 1;
    // the saved vertex (cacheable: not a delta lobe, :764, :821-845)
    if (cacheable && nv < P.V) {
        const float clamped = fmaxf(mis_pdf, 0.1f);
        const float inv_pdf = 1.0f / clamped;
        for (int ch = 0; ch < 3; ++ch) {
            vrec(P, ch, nv, i) = value[ch] * inv_pdf;
            vrec(P, 3 + ch, nv, i) = thr[ch];
        }
        vrec(P, 6, nv, i) = clamped;
        for (int a = 0; a < 3; ++a) {
            vrec(P, 7 + a, nv, i) = c[a];
            vrec(P, 10 + a, nv, i) = wo[a];
            vrec(P, 13 + a, nv, i) = n[a];
        }
        P.nv[i] = nv + 1;
    }
    // Russian roulette (:858-868)
    bool live = q >= 0;
    if (depth >= rr_depth && live) {
        const float qq = fminf(fmaxf(thr[0], fmaxf(thr[1], thr[2])), 0.95f);
        if (rng_uniform(seed, (uint64_t)(path0 + i), 1u + (uint32_t)bounce, 6) >= qq) live = false;
        else for (int ch = 0; ch < 3; ++ch) thr[ch] /= qq;
    }
    P.tr[i] = thr[0]; P.tg[i] = thr[1]; P.tb[i] = thr[2];
    P.dx[i] = wo[0]; P.dy[i] = wo[1]; P.dz[i] = wo[2];
    if (live) {
        P.px[i] = o[0] + t * wo[0]; P.py[i] = o[1] + t * wo[1]; P.pz[i] = o[2] + t * wo[2];
        P.quad[i] = q;
    }
    P.depth[i] = live ? depth + 1 : -1;
}

// pixel mean over its spp samples, in sample order; image planes [3][W*H];
// image_sqr (nullable): the mean of the squared samples (the reference's
// m_blockSqr, sdmm_wr.cpp:144-145)
__global__ void __launch_bounds__(256)
li_film_kernel(PathsDev P, int64_t pix0, int64_t npix, int spp, int64_t plane, float* __restrict__ image,
               float* __restrict__ image_sqr) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= npix) return;
    float acc[3] = {0.0f, 0.0f, 0.0f}, sq[3] = {0.0f, 0.0f, 0.0f};
    for (int s = 0; s < spp; ++s) {
        const int64_t i = j * spp + s;
        const float l[3] = {P.lr[i], P.lg[i], P.lb[i]};
        for (int ch = 0; ch < 3; ++ch) {
            acc[ch] += l[ch];
            sq[ch] += l[ch] * l[ch];
        }
    }
    const float inv = 1.0f / (float)spp;
    for (int ch = 0; ch < 3; ++ch) image[ch * plane + pix0 + j] = acc[ch] * inv;
    if (image_sqr)
        for (int ch = 0; ch < 3; ++ch) image_sqr[ch * plane + pix0 + j] = sq[ch] * inv;
}

// ---------------------------------------------------------------------------
// Training-data producer (:876-965).  Per path, vertices d = nv-1 .. firstSaved:
// find its leaf (with the leaf's box), push (point, normal, average weight)
// there with a stats entry when the weight is finite (jmm isValidSample); then
// nJitters = (d == nv-1) + (average > 1000) pushes to the leaf at position +
// (u - 1/2) * leaf diagonal, a draw that lands outside the tree or in the same
// leaf (equal box min) retried while fewer than 8 draws failed.  Pass 0 counts
// a path's records, pass 1 writes (leaf, code) at its offset; code =
// ((path * V + d) << 1) | stats.  Records keep (path, push) order.
// a record staged in path order (48 B, one or two cache lines) for the
// leaf-order gather: point + wo, normal, average weight, code
struct alignas(16) ProducedRec {
    float x[6];
    float n[3];
    float w;
    int64_t code;
};
static_assert(sizeof(ProducedRec) == 48, "ProducedRec layout");

template <bool WRITE>
__device__ __forceinline__ int produce_path(const STNodeDev* __restrict__ nodes, const PathsDev& P, int64_t p,
                                            int64_t path0, int saved, uint64_t seed, uint32_t* keys,
                                            int64_t* codes, ProducedRec* recs, int64_t off, int* lost) {
    const int nv = P.nv[p];
    const int first = nv - saved > 0 ? nv - saved : 0;
    int cnt = 0;
    for (int d = nv - 1; d >= first; --d) {
        const float pos[3] = {vrec(P, 7, d, p), vrec(P, 8, d, p), vrec(P, 9, d, p)};
        const int leaf = stree_find_point(nodes, pos[0], pos[1], pos[2]);
        if (leaf < 0) {   // the reference throws (:924-930)
            if (WRITE) atomicAdd(lost, 1);
            continue;
        }
        const STNodeDev box = nodes[leaf];
        const float avg = (vrec(P, 0, d, p) + vrec(P, 1, d, p) + vrec(P, 2, d, p)) * (1.0f / 3.0f);
        const bool ok = __builtin_isfinite(avg);
        const int64_t code = ((int64_t)p * P.V + d) << 1;
        ProducedRec r{};
        if (WRITE && ok) {
            for (int a = 0; a < 3; ++a) {
                r.x[a] = pos[a];
                r.x[3 + a] = vrec(P, 10 + a, d, p);
                r.n[a] = vrec(P, 13 + a, d, p);
            }
            r.w = avg;
        }
        auto put = [&](uint32_t key, int64_t c) {
            const int64_t at = off + cnt;
            keys[at] = key;
            codes[at] = at;   // the sort's payload: the staged record's slot
            r.code = c;
            recs[at] = r;
        };
        if (ok) {
            if (WRITE) put((uint32_t)leaf, code | 1);
            ++cnt;
        }
        int jitters = (d >= nv - 1 ? 1 : 0) + (avg > 1000.0f ? 1 : 0);
        int attempts = 0, draw = 0;
        const float diag[3] = {box.mx[0] - box.mn[0], box.mx[1] - box.mn[1], box.mx[2] - box.mn[2]};
        for (int j = 0; j < jitters; ++j) {
            const uint64_t gp = (uint64_t)(path0 + p);
            float jp[3];
            for (int a = 0; a < 3; ++a)
                jp[a] = pos[a] + (rng_uniform(seed, gp, kJitterStream + (uint32_t)d, 3 * draw + a) - 0.5f) * diag[a];
            ++draw;
            const int nb = stree_find_point(nodes, jp[0], jp[1], jp[2]);
            bool same = nb < 0;
            if (!same) {
                const STNodeDev b = nodes[nb];
                same = b.mn[0] == box.mn[0] && b.mn[1] == box.mn[1] && b.mn[2] == box.mn[2];
            }
            if (same) {
                ++attempts;
                if (attempts < 8) --j;
                continue;
            }
            if (ok) {
                if (WRITE) put((uint32_t)nb, code);
                ++cnt;
            }
        }
    }
    return cnt;
}

__global__ void __launch_bounds__(256)
produce_count_kernel(const STNodeDev* __restrict__ nodes, PathsDev P, int64_t path0, int saved, uint64_t seed,
                     int64_t* __restrict__ count) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P.P) return;
    count[p] = produce_path<false>(nodes, P, p, path0, saved, seed, nullptr, nullptr, nullptr, 0, nullptr);
}

__global__ void __launch_bounds__(256)
produce_write_kernel(const STNodeDev* __restrict__ nodes, PathsDev P, int64_t path0, int saved, uint64_t seed,
                     const int64_t* __restrict__ offset, uint32_t* __restrict__ keys, int64_t* __restrict__ codes,
                     ProducedRec* __restrict__ recs, int* __restrict__ lost) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P.P) return;
    (void)produce_path<true>(nodes, P, p, path0, saved, seed, keys, codes, recs, offset[p], lost);
}

// leaf-contiguous records -> training planes (slot: the staged record of
// sorted position j)
__global__ void __launch_bounds__(256)
produce_gather_kernel(const ProducedRec* __restrict__ recs, const int64_t* __restrict__ slot, int64_t n, float* x0,
                      float* x1, float* x2, float* x3, float* x4, float* x5, float* n0, float* n1, float* n2,
                      float* w, uint8_t* stats, const uint32_t* __restrict__ keys, int32_t* node, int64_t* source) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const ProducedRec r = recs[slot[j]];
    x0[j] = r.x[0]; x1[j] = r.x[1]; x2[j] = r.x[2];
    x3[j] = r.x[3]; x4[j] = r.x[4]; x5[j] = r.x[5];
    if (n0) { n0[j] = r.n[0]; n1[j] = r.n[1]; n2[j] = r.n[2]; }
    w[j] = r.w;
    if (stats) stats[j] = (uint8_t)(r.code & 1);
    if (node) node[j] = (int32_t)keys[j];
    if (source) source[j] = r.code >> 1;   // p * V + d
}

// seg[v] = first sorted position with key >= v, v = 0..num_nodes
__global__ void produce_seg_kernel(const uint32_t* __restrict__ keys, int64_t n, int num_nodes,
                                   int64_t* __restrict__ seg) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v > num_nodes) return;
    int64_t lo = 0, count = n;
    while (count > 0) {
        const int64_t step = count / 2, it = lo + step;
        if (keys[it] < (uint32_t)v) { lo = it + 1; count -= step + 1; }
        else count = step;
    }
    seg[v] = lo;
}

// ---------------------------------------------------------------------------
// host launchers
static inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

hipError_t launch_li_camera(const SceneDev& S, const PathsDev& P, int64_t path0, int spp, uint64_t seed,
                            hipStream_t st) {
    hipLaunchKernelGGL(li_camera_kernel, grid_for(P.P), dim3(256), 0, st, S, P, path0, spp, seed);
    return hipGetLastError();
}
hipError_t launch_li_query(const SceneDev& S, const PathsDev& P, const QueryDev& Q, int64_t path0, int bounce,
                           int max_depth, int guided, float h, uint64_t seed, hipStream_t st) {
    hipLaunchKernelGGL(li_query_kernel, grid_for(P.P), dim3(256), 0, st, S, P, Q, path0, bounce, max_depth, guided,
                       h, seed);
    return hipGetLastError();
}
size_t li_select_temp_bytes(int64_t n) {
    size_t b = 0;
    (void)hipcub::DeviceSelect::Flagged(nullptr, b, hipcub::CountingInputIterator<int32_t>(0), (const uint8_t*)nullptr,
                                        (int32_t*)nullptr, (int32_t*)nullptr, (int)n);
    return b;
}
// live guided queries -> compact planes; *count_dev = their number
hipError_t launch_li_compact(const SceneDev& S, const PathsDev& P, const QueryDev& Q, int64_t n, int32_t* count_dev,
                             void* temp, size_t temp_bytes, int product, hipStream_t st) {
    hipError_t e = hipcub::DeviceSelect::Flagged(temp, temp_bytes, hipcub::CountingInputIterator<int32_t>(0), Q.live,
                                                 Q.idx, count_dev, (int)n, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(li_compact_kernel, grid_for(n), dim3(256), 0, st, S, P, Q, (const int32_t*)count_dev,
                       product);
    return hipGetLastError();
}

hipError_t launch_li_shade(const SceneDev& S, const PathsDev& P, const QueryDev& Q, int64_t path0, int bounce,
                           int rr_depth, float h, uint64_t seed, int product, hipStream_t st) {
    hipLaunchKernelGGL(li_shade_kernel, grid_for(P.P), dim3(256), 0, st, S, P, Q, path0, bounce, rr_depth, h, seed,
                       product);
    return hipGetLastError();
}
// getDMM + rotate_to_wo for a batch of local incident directions against one
// learned model (sdmm_learned4_conditional_device): query q's lobes at
// w[q * keep ..], mean[(q * keep + j) * 3 ..], cov[(q * keep + j) * 4 ..],
// its lobe count n[q] (0: no valid conditional, or cos theta_i <= 0)
struct Learned4Rec {
    float r[kLearnedMaxComp * kLearnedRec];
};
__global__ void __launch_bounds__(256)
learned4_kernel(Learned4Rec model, int M, float alpha, int64_t nq, const float* __restrict__ w0,
                const float* __restrict__ w1, const float* __restrict__ w2, int keep, float* __restrict__ w,
                float* __restrict__ mean, float* __restrict__ cov, int32_t* __restrict__ n) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const float wl[3] = {w0[q], w1[q], w2[q]};
    int kept = 0;
    if (wl[2] > 0.0f) {
        const float theta = (float)acos((double)fminf(1.0f, wl[2]));
        float lw[kLearnedMaxComp], lm[3 * kLearnedMaxComp], lc[4 * kLearnedMaxComp];
        kept = learned4_conditional(model.r, M, theta, alpha, wl, keep, lw, lm, lc);
        for (int j = 0; j < kept; ++j) {
            w[q * keep + j] = lw[j];
            for (int i = 0; i < 3; ++i) mean[(q * keep + j) * 3 + i] = lm[3 * j + i];
            for (int i = 0; i < 4; ++i) cov[(q * keep + j) * 4 + i] = lc[4 * j + i];
        }
    }
    for (int j = kept; j < keep; ++j) w[q * keep + j] = 0.0f;
    n[q] = kept;
}
hipError_t launch_learned4(const float* rec, int M, float alpha, int64_t nq, const float* const wl[3], int keep,
                           float* w, float* mean, float* cov, int32_t* n, hipStream_t st) {
    if (M < 0 || M > kLearnedMaxComp || keep < 1 || keep > kLearnedMaxComp) return hipErrorInvalidValue;
    if (nq <= 0) return hipSuccess;
    Learned4Rec m{};
    for (int i = 0; i < M * kLearnedRec; ++i) m.r[i] = rec[i];
    hipLaunchKernelGGL(learned4_kernel, grid_for(nq), dim3(256), 0, st, m, M, alpha, nq, wl[0], wl[1], wl[2], keep, w,
                       mean, cov, n);
    return hipGetLastError();
}

hipError_t launch_li_film(const PathsDev& P, int64_t pix0, int64_t npix, int spp, int64_t plane, float* image,
                          float* image_sqr, hipStream_t st) {
    hipLaunchKernelGGL(li_film_kernel, grid_for(npix), dim3(256), 0, st, P, pix0, npix, spp, plane, image, image_sqr);
    return hipGetLastError();
}

size_t produce_temp_bytes(int64_t n_paths, int64_t n_records, int key_bits) {
    size_t a = 0, b = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const int64_t*)nullptr, (int64_t*)nullptr, (int)n_paths);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int64_t*)nullptr, (int64_t*)nullptr, (int)n_records, 0,
                                             key_bits);
    return a > b ? a : b;
}

// count + scan: offsets[p] (n_paths + 1 entries; offsets[n_paths] = total)
hipError_t launch_produce_count(const void* nodes, const PathsDev& P, int64_t path0, int saved, uint64_t seed,
                                int64_t* count, int64_t* offsets, void* temp, size_t temp_bytes, hipStream_t st) {
    hipLaunchKernelGGL(produce_count_kernel, grid_for(P.P), dim3(256), 0, st, (const STNodeDev*)nodes, P, path0,
                       saved, seed, count);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, count, offsets, (int)P.P + 1, st);
}

hipError_t launch_produce_records(const void* nodes, int num_nodes, int key_bits, const PathsDev& P, int64_t path0,
                                  int saved, uint64_t seed, const int64_t* offsets, int64_t n_rec, uint32_t* keys0,
                                  uint32_t* keys1, int64_t* codes0, int64_t* codes1, void* recs, void* temp,
                                  size_t temp_bytes, int64_t* seg_dev, int* lost, float* const x[6],
                                  float* const nrm[3], float* w, uint8_t* stats, int32_t* node, int64_t* source,
                                  hipStream_t st) {
    hipLaunchKernelGGL(produce_write_kernel, grid_for(P.P), dim3(256), 0, st, (const STNodeDev*)nodes, P, path0,
                       saved, seed, offsets, keys0, codes0, (ProducedRec*)recs, lost);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || n_rec == 0) return e;
    // stable: a leaf's records stay in (path, push) order
    e = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys0, keys1, codes0, codes1, (int)n_rec, 0, key_bits,
                                           st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(produce_seg_kernel, grid_for(num_nodes + 1), dim3(256), 0, st, keys1, n_rec, num_nodes,
                       seg_dev);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(produce_gather_kernel, grid_for(n_rec), dim3(256), 0, st, (const ProducedRec*)recs, codes1,
                       n_rec, x[0], x[1], x[2],
                       x[3], x[4], x[5], nrm ? nrm[0] : nullptr, nrm ? nrm[1] : nullptr, nrm ? nrm[2] : nullptr, w,
                       stats, keys1, node, source);
    return hipGetLastError();
}

}  // namespace sdmm
