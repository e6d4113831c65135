// render_api.cpp -- host side of the device Li (render.hip) behind
// include/sdmm_gpu.h: the analytic scene, the per-bounce launch sequence
// (camera -> [query -> guided wavefront -> shade] x bounces -> film) and the
// path / query / vertex buffers, grown on demand and reused across renders.
#include <hip/hip_runtime.h>
#include <xmmintrin.h>

#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/sdmm_gpu.h"
#include "render_device.h"
#include "learned_bsdf.h"

// the scene's derived quad data in plain IEEE float (no FMA contraction), as
// the CPU restatement of Li forms it (oracle/sdmm_oracle_li.inc)
#pragma clang fp contract(off)

namespace sdmm {
hipError_t launch_li_camera(const SceneDev& S, const PathsDev& P, int64_t path0, int spp, uint64_t seed,
                            hipStream_t st);
hipError_t launch_li_query(const SceneDev& S, const PathsDev& P, const QueryDev& Q, int64_t path0, int bounce,
                           int max_depth, int guided, float h, uint64_t seed, hipStream_t st);
hipError_t launch_li_shade(const SceneDev& S, const PathsDev& P, const QueryDev& Q, int64_t path0, int bounce,
                           int rr_depth, float h, uint64_t seed, int product, hipStream_t st);
size_t li_select_temp_bytes(int64_t n);
hipError_t launch_li_compact(const SceneDev& S, const PathsDev& P, const QueryDev& Q, int64_t n, int32_t* count_dev,
                             void* temp, size_t temp_bytes, int product, hipStream_t st);
hipError_t launch_li_film(const PathsDev& P, int64_t pix0, int64_t npix, int spp, int64_t plane, float* image,
                          float* image_sqr, hipStream_t st);
hipError_t launch_learned4(const float* rec, int M, float alpha, int64_t nq, const float* const wl[3], int keep,
                           float* w, float* mean, float* cov, int32_t* n, hipStream_t st);
}  // namespace sdmm

namespace sdmm_detail {
int set_error(int code, const char* msg);
int tree_stream(sdmm_stree* t, hipStream_t* st);   // sdmm_api.cpp: device nodes uploaded, the tree's stream
const int* tree_fallback_count(const sdmm_stree* t);   // sdmm_api.cpp
}  // namespace sdmm_detail

using namespace sdmm;

struct sdmm_scene {
    int device = 0;
    SceneDev S{};
    QuadDev* dquads = nullptr;
    float* drefl = nullptr;
    float* dbpar = nullptr;
    float* dlmod = nullptr;   // kLearnedStride per BSDF (learned_models), null: none
    float* drad = nullptr;
    float smin[3] = {0, 0, 0}, snorm = 1.0f, tmin[3] = {0, 0, 0}, tmax[3] = {0, 0, 0};
    // per-render buffers (grown)
    void* buf = nullptr;
    size_t buf_bytes = 0;
    int64_t cap_paths = 0;
    int cap_v = 0;
    PathsDev P{};
    QueryDev Q{};
    int64_t* dsum = nullptr;
    int32_t* dcount = nullptr;   // live guided queries of the current bounce
    int32_t* hcount = nullptr;   // (pinned host copy)
    int32_t* hfb = nullptr;      // per bounce: fallback queries of its wavefront (pinned)
    int hfb_cap = 0;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    // rough conductors with product sampling: the extended learned-BSDF
    // table -- the caller's B rows re-strided to lM >= kLearnedKeep lobes, then
    // one row per compact query for the conductor's per-bounce lobes
    bool has_conductor = false;
    void* lt = nullptr;
    size_t lt_bytes = 0;
};

namespace {

int fail(int code, const std::string& m) { return sdmm_detail::set_error(code, m.c_str()); }

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(SDMM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

void cross3(const float a[3], const float b[3], float c[3]) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
float dot3h(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// path + query + vertex planes for P paths with V vertex slots
int grow(sdmm_scene* s, int64_t P, int V, hipStream_t st) {
    if (P <= s->cap_paths && V <= s->cap_v && s->buf) return SDMM_OK;
    const int64_t cap = std::max<int64_t>(P, s->cap_paths);
    const int cv = std::max(V, s->cap_v);
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t f = al(sizeof(float) * (size_t)cap), i4 = al(sizeof(int32_t) * (size_t)cap), u1 = al((size_t)cap);
    const size_t recb = al(sizeof(float) * (size_t)kVertexFields * (size_t)cv * (size_t)cap);
    size_t tb = 0;
    (void)hipcub::DeviceReduce::Sum(nullptr, tb, (const int32_t*)nullptr, (int64_t*)nullptr, (int)cap);
    tb = std::max(tb, li_select_temp_bytes(cap));
    const size_t need = 12 * f + 4 * i4 + recb + 13 * f + u1 + i4 + 256 + al(tb) + 9 * f + 2 * u1 + 3 * i4 +
                        (1 + 1 + 9 + 1) * f + i4 + u1 + 4 * f;
    HIP_TRY(hipStreamSynchronize(st));
    if (s->buf) HIP_TRY(hipFree(s->buf));
    s->buf = nullptr;
    HIP_TRY(hipMalloc(&s->buf, need));
    s->buf_bytes = need;
    s->cap_paths = cap;
    s->cap_v = cv;
    char* b = (char*)s->buf;
    auto take = [&](size_t n) { char* r = b; b += n; return r; };
    float** pf[12] = {&s->P.px, &s->P.py, &s->P.pz, &s->P.dx, &s->P.dy, &s->P.dz,
                      &s->P.tr, &s->P.tg, &s->P.tb, &s->P.lr, &s->P.lg, &s->P.lb};
    for (float** q : pf) *q = (float*)take(f);
    s->P.depth = (int*)take(i4);
    s->P.quad = (int*)take(i4);
    s->P.nv = (int*)take(i4);
    s->P.nray = (int*)take(i4);
    s->P.rec = (float*)take(recb);
    float** qf[13] = {&s->Q.c0, &s->Q.c1, &s->Q.c2, &s->Q.u0, &s->Q.u1, &s->Q.u2, &s->Q.b0,
                      &s->Q.b1, &s->Q.b2, &s->Q.d0, &s->Q.d1, &s->Q.d2, &s->Q.pdf};
    for (float** q : qf) *q = (float*)take(f);
    s->Q.mode = (uint8_t*)take(u1);
    s->Q.comp = (int32_t*)take(i4);
    s->dsum = (int64_t*)take(256);
    s->temp = take(al(tb));
    s->temp_bytes = al(tb);
    float** kf[9] = {&s->Q.k_c0, &s->Q.k_c1, &s->Q.k_c2, &s->Q.k_u0, &s->Q.k_u1, &s->Q.k_u2,
                     &s->Q.k_b0, &s->Q.k_b1, &s->Q.k_b2};
    for (float** q : kf) *q = (float*)take(f);
    s->Q.k_mode = (uint8_t*)take(u1);
    s->Q.live = (uint8_t*)take(u1);
    s->Q.idx = (int32_t*)take(i4);
    s->Q.slot = (int32_t*)take(i4);
    s->dcount = (int32_t*)take(i4);
    s->Q.ch = (float*)take(f);
    s->Q.k_ch = (float*)take(f);
    for (int i = 0; i < 9; ++i) s->Q.k_F[i] = (float*)take(f);
    s->Q.hq = (float*)take(f);
    s->Q.k_mat = (int32_t*)take(i4);
    s->Q.bdelta = (uint8_t*)take(u1);
    float** bf[4] = {&s->Q.bw0, &s->Q.bw1, &s->Q.bw2, &s->Q.bpdf};
    for (float** q : bf) *q = (float*)take(f);
    return SDMM_OK;
}

// The extended learned-BSDF table of a render with rough conductors: rows
// 0 .. B-1 the caller's (device arrays, re-strided to lM = max(M,
// kLearnedKeep) lobes, the extra lobes weight 0 -- skipped by the product),
// rows B .. B + cap - 1 the compact queries' own conductor lobes (written by
// li_compact_kernel).  *tab describes it; s->Q points at the query rows.
int extend_learned(sdmm_scene* s, const sdmm_bsdf_table& user, int64_t cap, hipStream_t st, sdmm_bsdf_table* tab) {
    const int M = user.M, lM = std::max(M, kLearnedKeep), B = user.B;
    const int64_t rows = (int64_t)B + cap;
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t wb = al(sizeof(float) * (size_t)rows * lM), mb = 3 * wb, cb = 4 * wb, db = al((size_t)rows);
    const size_t need = wb + mb + cb + db;
    if (need > s->lt_bytes) {
        HIP_TRY(hipStreamSynchronize(st));
        if (s->lt) HIP_TRY(hipFree(s->lt));
        s->lt = nullptr;
        s->lt_bytes = 0;
        HIP_TRY(hipMalloc(&s->lt, need));
        s->lt_bytes = need;
    }
    char* b = (char*)s->lt;
    float* w = (float*)b;
    float* m = (float*)(b + wb);
    float* c = (float*)(b + wb + mb);
    uint8_t* dflag = (uint8_t*)(b + wb + mb + cb);
    HIP_TRY(hipMemsetAsync(w, 0, sizeof(float) * (size_t)B * lM, st));
    HIP_TRY(hipMemcpy2DAsync(w, sizeof(float) * lM, user.weights, sizeof(float) * M, sizeof(float) * M, B,
                             hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemsetAsync(m, 0, sizeof(float) * 3 * (size_t)B * lM, st));
    HIP_TRY(hipMemcpy2DAsync(m, sizeof(float) * 3 * lM, user.means, sizeof(float) * 3 * M, sizeof(float) * 3 * M, B,
                             hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemsetAsync(c, 0, sizeof(float) * 4 * (size_t)B * lM, st));
    HIP_TRY(hipMemcpy2DAsync(c, sizeof(float) * 4 * lM, user.covs, sizeof(float) * 4 * M, sizeof(float) * 4 * M, B,
                             hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipMemsetAsync(dflag, 0, (size_t)rows, st));
    if (user.diffuse) HIP_TRY(hipMemcpyAsync(dflag, user.diffuse, (size_t)B, hipMemcpyDeviceToDevice, st));
    *tab = sdmm_bsdf_table{w, m, c, (int)std::min<int64_t>(rows, INT32_MAX), lM, dflag};
    s->Q.lw = w;
    s->Q.lm = m;
    s->Q.lc = c;
    s->Q.lrow0 = B;
    s->Q.lM = lM;
    return SDMM_OK;
}

}  // namespace

extern "C" {

int sdmm_scene_create(const sdmm_scene_desc* d, int device, sdmm_scene** out) {
    if (!out || !d || d->n_quads < 1 || !d->quads || !d->bsdf || d->n_bsdfs < 1 || !d->reflectance ||
        d->width < 1 || d->height < 1 || !(d->fov_x_deg > 0.0f && d->fov_x_deg < 180.0f))
        return fail(SDMM_E_INVALID, "sdmm_scene_create: invalid description");
    if (d->emitter && (d->n_emitters < 1 || !d->radiance))
        return fail(SDMM_E_INVALID, "sdmm_scene_create: emitters without radiance");
    if (d->bsdf_params)
        for (int b = 0; b < d->n_bsdfs; ++b) {
            const float* bp = d->bsdf_params + kBsdfParams * b;
            const bool ok = bp[0] == (float)kBsdfDiffuse ||
                            (bp[0] == (float)kBsdfPlastic && bp[4] > 0.0f && bp[5] > 0.0f && bp[6] < 1.0f &&
                             bp[7] >= 0.0f && bp[7] <= 1.0f) ||
                            (bp[0] == (float)kBsdfConductor && bp[1] >= 0.0f && bp[2] >= 0.0f && bp[3] >= 0.0f &&
                             std::isfinite(bp[1] + bp[2] + bp[3]) && bp[4] > 0.0f && std::isfinite(bp[4]) &&
                             bp[5] >= 0.0f && std::isfinite(bp[5]) && bp[6] > 0.0f && bp[6] <= 2.0f);
            if (!ok) return fail(SDMM_E_INVALID, "sdmm_scene_create: invalid bsdf_params");
        }
    // learned models: at most kLearnedMaxComp components, finite, unit directions
    std::vector<float> lmod;
    if (d->learned_models) {
        lmod.assign((size_t)kLearnedStride * (size_t)d->n_bsdfs, 0.0f);
        for (int b = 0; b < d->n_bsdfs; ++b) {
            const sdmm_learned_bsdf4& L = d->learned_models[b];
            if (L.M == 0) continue;
            if (L.M < 0 || L.M > kLearnedMaxComp || !L.weights || !L.means || !L.covs)
                return fail(SDMM_E_INVALID, "sdmm_scene_create: invalid learned model (1 <= M <= 8, arrays)");
            float* o = lmod.data() + (size_t)kLearnedStride * b;
            o[0] = (float)L.M;
            for (int k = 0; k < L.M; ++k) {
                float* r = o + 1 + kLearnedRec * k;
                r[0] = L.weights[k];
                for (int i = 0; i < 5; ++i) r[1 + i] = L.means[5 * k + i];
                for (int i = 0; i < 16; ++i) r[6 + i] = L.covs[16 * k + i];
                bool ok = r[0] >= 0.0f;
                for (int i = 0; i < kLearnedRec; ++i) ok = ok && std::isfinite(r[i]);
                const double n2 = (double)r[3] * r[3] + (double)r[4] * r[4] + (double)r[5] * r[5];
                if (!ok || std::fabs(n2 - 1.0) > 1e-5)
                    return fail(SDMM_E_INVALID, "sdmm_scene_create: learned model with a non-finite value, a "
                                                "negative weight or a non-unit direction");
            }
        }
    }
    *out = nullptr;
    std::vector<QuadDev> qs((size_t)d->n_quads);
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int q = 0; q < d->n_quads; ++q) {
        QuadDev& Q = qs[(size_t)q];
        const float* v = d->quads + 9 * q;
        for (int a = 0; a < 3; ++a) { Q.p0[a] = v[a]; Q.e1[a] = v[3 + a]; Q.e2[a] = v[6 + a]; }
        float n[3];
        cross3(Q.e1, Q.e2, n);
        const float len = std::sqrt(dot3h(n, n));
        if (!(len > 0.0f)) return fail(SDMM_E_INVALID, "sdmm_scene_create: degenerate quad");
        const float sg = (d->flip_normals && d->flip_normals[q]) ? -1.0f : 1.0f;
        for (int a = 0; a < 3; ++a) Q.n[a] = sg * n[a] / len;
        // duals: g1 . e1 = 1, g1 . e2 = 0 (g1 ~ e2 x n), likewise g2
        float a1[3], a2[3];
        cross3(Q.e2, n, a1);
        cross3(n, Q.e1, a2);
        const float s1 = dot3h(Q.e1, a1), s2 = dot3h(Q.e2, a2);
        for (int a = 0; a < 3; ++a) { Q.g1[a] = a1[a] / s1; Q.g2[a] = a2[a] / s2; }
        Q.bsdf = d->bsdf[q];
        Q.emitter = d->emitter ? d->emitter[q] : -1;
        if (Q.bsdf < 0 || Q.bsdf >= d->n_bsdfs || Q.emitter < -1 || (Q.emitter >= 0 && Q.emitter >= d->n_emitters))
            return fail(SDMM_E_INVALID, "sdmm_scene_create: material index out of range");
        // scene AABB without the camera: the four corners
        for (int c = 0; c < 4; ++c)
            for (int a = 0; a < 3; ++a) {
                const float x = Q.p0[a] + ((c & 1) ? Q.e1[a] : 0.0f) + ((c & 2) ? Q.e2[a] : 0.0f);
                mn[a] = std::min(mn[a], x);
                mx[a] = std::max(mx[a], x);
            }
    }
    sdmm_scene* s = new (std::nothrow) sdmm_scene();
    if (!s) return fail(SDMM_E_NOMEM, "out of host memory");
    s->device = device;
    // (a conductor some quad uses: the CPU restatement's rule)
    if (d->bsdf_params)
        for (int q = 0; q < d->n_quads; ++q)
            if (d->bsdf_params[kBsdfParams * d->bsdf[q]] == (float)kBsdfConductor) s->has_conductor = true;
    // render() (volpath_sdmm.cpp:375-393): spatialNormalization = the largest
    // extent; the tree box getAABB (:314-332)
    float ext[3], norm = 0.0f;
    for (int a = 0; a < 3; ++a) { ext[a] = mx[a] - mn[a]; norm = std::max(norm, ext[a]); }
    for (int a = 0; a < 3; ++a) {
        s->smin[a] = mn[a];
        s->tmin[a] = 0.0f - 1e-5f;
        s->tmax[a] = ext[a] / norm + 1e-5f;
    }
    s->snorm = norm;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipMalloc(&s->dquads, sizeof(QuadDev) * qs.size());
    if (e == hipSuccess) e = hipMalloc(&s->drefl, sizeof(float) * 3 * (size_t)d->n_bsdfs);
    if (e == hipSuccess && d->emitter) e = hipMalloc(&s->drad, sizeof(float) * 3 * (size_t)d->n_emitters);
    if (e == hipSuccess && d->bsdf_params)
        e = hipMalloc(&s->dbpar, sizeof(float) * kBsdfParams * (size_t)d->n_bsdfs);
    if (e == hipSuccess && d->bsdf_params)
        e = hipMemcpy(s->dbpar, d->bsdf_params, sizeof(float) * kBsdfParams * (size_t)d->n_bsdfs,
                      hipMemcpyHostToDevice);
    if (e == hipSuccess && !lmod.empty()) e = hipMalloc(&s->dlmod, sizeof(float) * lmod.size());
    if (e == hipSuccess && !lmod.empty())
        e = hipMemcpy(s->dlmod, lmod.data(), sizeof(float) * lmod.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(s->dquads, qs.data(), sizeof(QuadDev) * qs.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(s->drefl, d->reflectance, sizeof(float) * 3 * (size_t)d->n_bsdfs, hipMemcpyHostToDevice);
    if (e == hipSuccess && d->emitter)
        e = hipMemcpy(s->drad, d->radiance, sizeof(float) * 3 * (size_t)d->n_emitters, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        sdmm_scene_destroy(s);
        return fail(SDMM_E_HIP, std::string("sdmm_scene_create: ") + hipGetErrorString(e));
    }
    SceneDev& S = s->S;
    S.quads = s->dquads;
    S.n_quads = d->n_quads;
    S.refl = s->drefl;
    S.bpar = s->dbpar;
    S.lmodel = s->dlmod;
    S.rad = s->drad;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) S.cam[4 * r + c] = d->camera_to_world[4 * r + c];
    S.tanx = (float)std::tan(0.5 * (double)d->fov_x_deg * 3.14159265358979323846 / 180.0);
    S.aspect = (float)d->width / (float)d->height;
    S.near_clip = d->near_clip > 0.0f ? d->near_clip : 1e-2f;
    S.width = d->width;
    S.height = d->height;
    for (int a = 0; a < 3; ++a) S.smin[a] = s->smin[a];
    S.snorm = s->snorm;
    *out = s;
    return SDMM_OK;
}

int sdmm_learned4_conditional(const sdmm_learned_bsdf4* m, float alpha, const float wi_local[3], int keep,
                              int* n_out, float* weights, float* means, float* covs) {
    if (!m || !wi_local || !n_out || keep < 1 || m->M < 0 || m->M > kLearnedMaxComp ||
        (m->M > 0 && (!m->weights || !m->means || !m->covs)) || !weights || !means || !covs)
        return fail(SDMM_E_INVALID, "sdmm_learned4_conditional: invalid argument");
    *n_out = 0;
    if (m->M == 0 || !(wi_local[2] > 0.0f)) return SDMM_OK;   // getDMM: no model, or cosTheta(wi) <= 0
    float rec[kLearnedMaxComp * kLearnedRec];
    for (int k = 0; k < m->M; ++k) {
        float* r = rec + kLearnedRec * k;
        r[0] = m->weights[k];
        for (int i = 0; i < 5; ++i) r[1 + i] = m->means[5 * k + i];
        for (int i = 0; i < 16; ++i) r[6 + i] = m->covs[16 * k + i];
    }
    // the device's float environment: denormals flushed (-fgpu-flush-denormals-to-zero)
    const unsigned csr = _mm_getcsr();
    _mm_setcsr(csr | 0x8040u);
    const float theta = (float)std::acos((double)std::fmin(1.0f, wi_local[2]));
    float w[kLearnedMaxComp], mm[3 * kLearnedMaxComp], cc[4 * kLearnedMaxComp];
    const int n = learned4_conditional(rec, m->M, theta, alpha, wi_local, keep, w, mm, cc);
    _mm_setcsr(csr);
    for (int j = 0; j < n; ++j) {
        weights[j] = w[j];
        for (int i = 0; i < 3; ++i) means[3 * j + i] = mm[3 * j + i];
        for (int i = 0; i < 4; ++i) covs[4 * j + i] = cc[4 * j + i];
    }
    *n_out = n;
    return SDMM_OK;
}

int sdmm_learned4_conditional_device(const sdmm_learned_bsdf4* m, float alpha, int64_t nq, const float* const wi_local[3],
                                     int keep, float* weights, float* means, float* covs, int32_t* n_out,
                                     void* hip_stream) {
    if (!m || nq < 0 || keep < 1 || keep > kLearnedMaxComp || m->M < 0 || m->M > kLearnedMaxComp ||
        (m->M > 0 && (!m->weights || !m->means || !m->covs)))
        return fail(SDMM_E_INVALID, "sdmm_learned4_conditional_device: invalid argument");
    if (nq == 0) return SDMM_OK;
    if (!wi_local || !wi_local[0] || !wi_local[1] || !wi_local[2] || !weights || !means || !covs || !n_out)
        return fail(SDMM_E_INVALID, "sdmm_learned4_conditional_device: invalid argument");
    float rec[kLearnedMaxComp * kLearnedRec];
    for (int k = 0; k < m->M; ++k) {
        float* r = rec + kLearnedRec * k;
        r[0] = m->weights[k];
        for (int i = 0; i < 5; ++i) r[1 + i] = m->means[5 * k + i];
        for (int i = 0; i < 16; ++i) r[6 + i] = m->covs[16 * k + i];
    }
    HIP_TRY(launch_learned4(rec, m->M, alpha, nq, wi_local, keep, weights, means, covs, n_out,
                            (hipStream_t)hip_stream));
    return SDMM_OK;
}

void sdmm_scene_destroy(sdmm_scene* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    (void)hipDeviceSynchronize();
    if (s->dquads) (void)hipFree(s->dquads);
    if (s->drefl) (void)hipFree(s->drefl);
    if (s->dbpar) (void)hipFree(s->dbpar);
    if (s->dlmod) (void)hipFree(s->dlmod);
    if (s->drad) (void)hipFree(s->drad);
    if (s->buf) (void)hipFree(s->buf);
    if (s->lt) (void)hipFree(s->lt);
    if (s->hcount) (void)hipHostFree(s->hcount);
    if (s->hfb) (void)hipHostFree(s->hfb);
    delete s;
}

int sdmm_scene_normalization(const sdmm_scene* s, float scene_min[3], float* spatial_norm, float tree_min[3],
                             float tree_max[3]) {
    if (!s) return fail(SDMM_E_INVALID, "null scene");
    for (int a = 0; a < 3; ++a) {
        if (scene_min) scene_min[a] = s->smin[a];
        if (tree_min) tree_min[a] = s->tmin[a];
        if (tree_max) tree_max[a] = s->tmax[a];
    }
    if (spatial_norm) *spatial_norm = s->snorm;
    return SDMM_OK;
}

int sdmm_li_render(sdmm_scene* s, sdmm_stree* t, const sdmm_mix* const* node_mix, const sdmm_li_params* p,
                   float* image, float* image_sqr, sdmm_path_vertices* vout, sdmm_li_stats* stats) {
    if (!s || !t || !p || !image) return fail(SDMM_E_INVALID, "invalid argument");
    const int64_t npix_all = (int64_t)s->S.width * s->S.height;
    if (p->spp < 1 || p->pixel_begin < 0 || p->pixel_end > npix_all || p->pixel_end <= p->pixel_begin ||
        p->rr_depth < 1 || p->max_depth == 0 || p->max_depth < -1 || p->saved_vertices < 1)
        return fail(SDMM_E_INVALID, "sdmm_li_render: invalid parameters");
    if (p->max_depth > 0 && p->saved_vertices < p->max_depth - 1)
        return fail(SDMM_E_INVALID, "sdmm_li_render: saved_vertices < max_depth - 1");
    if (p->guided && !(p->bsdf_fraction >= 0.0f && p->bsdf_fraction <= 1.0f))
        return fail(SDMM_E_INVALID, "sdmm_li_render: bsdf_fraction outside [0, 1]");
    const int product = p->sample_product ? 1 : 0;
    if (product) {
        const sdmm_bsdf_table& lb = p->learned_bsdf;
        if (lb.M < 1 || lb.M > 64 || lb.B < 1 || !lb.weights || !lb.means || !lb.covs)
            return fail(SDMM_E_INVALID, "sdmm_li_render: sample_product needs a learned-BSDF table (B >= 1, 1 <= M <= 64)");
    }
    const int64_t npix = p->pixel_end - p->pixel_begin;
    const int64_t P = npix * p->spp;
    if (P > INT32_MAX) return fail(SDMM_E_INVALID, "sdmm_li_render: at most 2^31 - 1 paths per call");
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = nullptr;
    int r = sdmm_detail::tree_stream(t, &st);
    if (r) return r;
    const int V = p->saved_vertices;
    r = grow(s, P, V, st);
    if (r) return r;
    s->P.V = V;
    s->P.P = P;
    sdmm_bsdf_table ltab{};
    s->Q.lw = s->Q.lm = s->Q.lc = nullptr;
    if (product && p->guided && s->has_conductor) {
        r = extend_learned(s, p->learned_bsdf, s->cap_paths, st, &ltab);
        if (r) return r;
    }
    const int64_t path0 = p->pixel_begin * p->spp;
    HIP_TRY(launch_li_camera(s->S, s->P, path0, p->spp, p->seed, st));
    // bounces: rRec.depth 1 .. maxDepth - 1 scatter (:649, :684); unbounded
    // paths stop at the vertex slots
    const int bounces = p->max_depth > 0 ? p->max_depth - 1 : V;
    int64_t guided_queries = 0;
    if (!s->hcount) HIP_TRY(hipHostMalloc((void**)&s->hcount, sizeof(int32_t), hipHostMallocDefault));
    if (stats && p->guided && s->hfb_cap < bounces) {
        if (s->hfb) HIP_TRY(hipHostFree(s->hfb));
        s->hfb = nullptr;
        s->hfb_cap = 0;
        HIP_TRY(hipHostMalloc((void**)&s->hfb, sizeof(int32_t) * (size_t)bounces, hipHostMallocDefault));
        s->hfb_cap = bounces;
    }
    if (stats && p->guided)
        for (int b = 0; b < bounces; ++b) s->hfb[b] = 0;
    const float h = p->bsdf_fraction;
    for (int b = 0; b < bounces; ++b) {
        HIP_TRY(launch_li_query(s->S, s->P, s->Q, path0, b, p->max_depth > 0 ? p->max_depth : INT32_MAX, p->guided,
                                h, p->seed, st));
        if (p->guided) {
            // only the live paths query the guide: compact them (the order of
            // the compact queries does not change any query's outputs)
            HIP_TRY(launch_li_compact(s->S, s->P, s->Q, P, s->dcount, s->temp, s->temp_bytes, product, st));
            HIP_TRY(hipMemcpyAsync(s->hcount, s->dcount, sizeof(int32_t), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            const int64_t nlive = *s->hcount;
            const float* c[3] = {s->Q.k_c0, s->Q.k_c1, s->Q.k_c2};
            const float* u[3] = {s->Q.k_u0, s->Q.k_u1, s->Q.k_u2};
            const float* bd[3] = {s->Q.k_b0, s->Q.k_b1, s->Q.k_b2};
            float* d[3] = {s->Q.d0, s->Q.d1, s->Q.d2};
            if (nlive > 0) {
                if (product) {
                    // sampleSurface with sampleProduct (:327-392): the product
                    // of the leaf's conditional and the material's learned
                    // BSDF, h = 0.3 (0.5 without a usable product), the BSDF /
                    // guide choice taken against the query's own h
                    const float* F[9];
                    for (int i = 0; i < 9; ++i) F[i] = s->Q.k_F[i];
                    r = sdmm_guide_product_wavefront(t, node_mix, nlive, c, u, s->Q.k_ch, bd,
                                                     s->Q.lw ? &ltab : &p->learned_bsdf, s->Q.k_mat, F, d,
                                                     s->Q.pdf, s->Q.comp, s->Q.hq, nullptr);
                } else {
                    r = sdmm_guide_pdf_wavefront(t, node_mix, nlive, c, u, bd, s->Q.k_mode, d, s->Q.pdf,
                                                 s->Q.comp, nullptr);
                }
                if (r) return r;
                // (stream-ordered copy, read after the final synchronisation)
                const int* fb = sdmm_detail::tree_fallback_count(t);
                if (stats && fb)
                    HIP_TRY(hipMemcpyAsync(s->hfb + b, fb, sizeof(int32_t), hipMemcpyDeviceToHost, st));
            }
            guided_queries += nlive;
        }
        HIP_TRY(launch_li_shade(s->S, s->P, s->Q, path0, b, p->rr_depth, h, p->seed, product && p->guided, st));
    }
    HIP_TRY(launch_li_film(s->P, p->pixel_begin, npix, p->spp, npix_all, image, image_sqr, st));
    if (vout) {
        vout->n_paths = P;
        vout->max_vertices = V;
        vout->path0 = path0;
        vout->rec = s->P.rec;
        vout->nv = s->P.nv;
    }
    if (stats) {
        // traced bounce rays (a delta lobe's ray saves no vertex)
        size_t tb = s->temp_bytes;
        HIP_TRY(hipcub::DeviceReduce::Sum(s->temp, tb, (const int32_t*)s->P.nray, s->dsum, (int)P, st));
        int64_t seg = 0;
        HIP_TRY(hipMemcpyAsync(&seg, s->dsum, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        stats->paths = P;
        stats->segments = seg;
        stats->guided_queries = guided_queries;
        stats->fallback_queries = 0;
        if (p->guided)
            for (int b = 0; b < bounces; ++b) stats->fallback_queries += s->hfb[b];
    }
    return SDMM_OK;
}

}  // extern "C"
