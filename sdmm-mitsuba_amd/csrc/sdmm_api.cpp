// sdmm_api.cpp -- host runtime behind include/sdmm_gpu.h.
//
// Owns one mixture + its stepwise EM state on one GPU and sequences the
// kernels of estep.hip / mstep.hip / guide.hip on the handle's HIP stream.
// The reference counterpart is the per-leaf SDMMContext of the sdmm plugin
// (sdmm_proc.h:92-93) driving sdmm-lib's em_step / create_conditional.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>
#include <algorithm>
#include <atomic>
#include <future>
#include <thread>
#include <mutex>

#include "../../include/sdmm_gpu.h"
#include "sdmm_device.h"
#include "render_device.h"
#include "host_xfer.h"

#pragma clang fp contract(off)

namespace sdmm {
hipError_t launch_estep_resp(int cpl, int lps, const float* ep, int Kp, int K, const SamplesDev& s,
                             int64_t n, int64_t chunk, float* resp, hipStream_t st);
hipError_t launch_estep_stats(int cpl, int lps, const float* ep, int Kp, int K, const SamplesDev& s,
                              int64_t n, int64_t chunk, int blocks, int wpb, float* partials,
                              int pstride, hipStream_t st, const LeafDesc* leaves = nullptr,
                              const int2* items = nullptr);
hipError_t launch_reduce_finalize_batched(const float* partials, int pstride, int Kp, int K,
                                          const LeafDesc* leaves, int n_leaves, hipStream_t st);
hipError_t launch_mstep_batched(int K, int Kp, const MixDesc* mixes, int n_mix, float norm5, hipStream_t st);
hipError_t launch_set_f64(double* p, double v, hipStream_t st);
hipError_t estep_occupancy(int cpl, int lps, int Kp, int* resp_blocks, int* stats_blocks);
hipError_t launch_estep_resp_tile(int variant, const float* ep, int Kp, int K, const SamplesDev& s, int64_t n,
                                  int64_t chunk, float* resp, hipStream_t st);
hipError_t estep_resp_tile_occupancy(int variant, int* blocks_per_cu);
const char* estep_resp_tile_name(int variant);
hipError_t launch_estep_resp_mfma(int variant, const float* ep, int Kp, int K, const SamplesDev& s, int64_t n,
                                  int64_t chunk, float* resp, hipStream_t st);
hipError_t estep_resp_mfma_occupancy(int variant, int Kp, int* blocks_per_cu);
const char* estep_resp_mfma_name(int variant, int Kp);
bool estep_resp_split_supported(int Kp);
hipError_t launch_estep_resp_split(int variant, const float* ep, int Kp, int K, const SamplesDev& s, int64_t n,
                                   int64_t resident_waves, float* resp, hipStream_t st);
hipError_t estep_resp_split_occupancy(int variant, int Kp, int* waves_per_cu);
const char* estep_resp_split_name(int variant, int Kp);
hipError_t launch_estep_stats_tile(int variant, const float* ep, int Kp, int K, const SamplesDev& s, int64_t n,
                                   int64_t chunk, int blocks, float* partials, int pstride, hipStream_t st,
                                   const LeafDesc* leaves = nullptr, const int2* items = nullptr);
hipError_t estep_stats_tile_occupancy(int variant, int Kp, int* blocks_per_cu);
hipError_t launch_reduce_partials(const float* partials, int rows, int pstride, const float* ep_for_finalize,
                                  int Kp, int K, double* stats, hipStream_t st);
hipError_t launch_set_all(int K, int Kp, const double* mean, const double* cov, const CanonDev& C,
                          float* ep, float* gp, float norm5, hipStream_t st);
hipError_t launch_pack_all(int K, int Kp, const CanonDev& C, float* ep, float* gp, float norm5,
                           hipStream_t st);
hipError_t launch_init_state(int K, const double* scal, const float* bprior, float eps, double* sc, float* bp,
                             float* bd, hipStream_t st);
hipError_t launch_hemi_gen_batched(int n, int K, const float* pos, const float* nrm, const float* dist,
                                   const uint64_t* seed, int skip, float depth_prior, void* staging, size_t per,
                                   hipStream_t st);
hipError_t launch_set_all_batched(int n, int K, int Kp, const void* tab, const void* staging, size_t per, float norm5,
                                  hipStream_t st);
hipError_t launch_copy_many(int n, const void* src_tab, const void* dst_tab, size_t bytes, hipStream_t st);
hipError_t launch_gather_f64(const void* src_tab, int n, double* out, hipStream_t st);
struct InitDescHost {
    CanonDev C;
    float *ep, *gp, *bp, *bd;
    double *tmean, *tcov;
};
hipError_t launch_init_pack_many(int n, int K, int Kp, const double* scal, const float* bprior, float eps,
                                 double* sc, float* bp, float* bd, const CanonDev& C, float* ep, float* gp,
                                 float norm5, size_t stride, hipStream_t st);
hipError_t launch_mstep(int K, int Kp, const double* stats, int64_t nSamples, const CanonDev& C,
                        const EmStateDev& S, float* ep, float* gp, float norm5, double* newW, unsigned* count,
                        hipStream_t st);
size_t guide_sort_temp_bytes(int n);
hipError_t launch_stree_find(const void* nodes, int64_t n, const float* p0, const float* p1, const float* p2,
                             int32_t* out, hipStream_t st);
size_t stree_route_temp_bytes(int n, int key_bits);
hipError_t launch_stree_route(const void* nodes, int num_nodes, int key_bits, const SamplesDev& in, int n,
                              uint32_t* keys0, uint32_t* keys1, int32_t* idx0, int32_t* idx1, void* temp,
                              size_t temp_bytes, int64_t* seg_dev, float* const out_x[6], float* out_w,
                              float* out_h, uint8_t* out_d, hipStream_t st);
hipError_t launch_guide(const float* gp, int Kp, int K, int64_t nq, const float* const c[3],
                        const float* const u[3], const float* const dgiven[3], float* const d[3], float* pdf,
                        int32_t* comp, float norm2, float norm3, int cap, int* fb_count, int32_t* fb_list,
                        int cus, hipStream_t st, const GuideSortScratch* sort, int* fb2 = nullptr);
hipError_t launch_guide_tree(const void* nodes, const void* tab, int kmax, int64_t nq, const float* const c[3],
                             const float* const u[3], const float* const dgiven[3], float* const d[3],
                             float* pdf, int32_t* comp, int32_t* node_out, float norm2, float norm3, int cap,
                             int* fb_count, int32_t* fb_list, int cus, hipStream_t st,
                             const GuideSortScratch* sort, const uint8_t* pmode = nullptr, int* fb2 = nullptr,
                             int nn = 0);
hipError_t launch_guide_product(const float* gp, int Kp, int K, const float* condCov, int64_t nq,
                                const float* const c[3], const float* const u[3], const float* const dgiven[3],
                                float* const d[3], float* pdf, int32_t* comp, const int32_t* material,
                                const float* const frame[9], float* h, const float* bw, const float* bmean,
                                const float* bcov, const uint8_t* diffuse, int B, int M, float norm2, float norm3,
                                int cap, int* fb_count, int32_t* fb_list, int cus, hipStream_t st,
                                const GuideSortScratch* sort, ProductScratch* scratch);
hipError_t launch_guide_product_tree(const void* nodes, const void* tab, const void* cctab, int kmax, int64_t nq,
                                     const float* const c[3], const float* const u[3], const float* choice,
                                     const float* const dgiven[3], float* const d[3], float* pdf, int32_t* comp,
                                     int32_t* node_out, const int32_t* material, const float* const frame[9],
                                     float* h, const float* bw, const float* bmean, const float* bcov,
                                     const uint8_t* diffuse, int B, int M, float norm2, float norm3, int cap,
                                     int* fb_count, int32_t* fb_list, int cus, hipStream_t st,
                                     const GuideSortScratch* sort, ProductScratch* scratch, int nn = 0);
#ifndef SDMM_GUIDE_CAP_MAX
#define SDMM_GUIDE_CAP_MAX 64
#endif
constexpr int kGuideCapMax = SDMM_GUIDE_CAP_MAX;
// default capacity: 40 (round 4 A/B, Cornell K=128 tree wavefront: 12.3 ms per
// guided pass at 40 against 13.3 ms at 64 -- a third of the fallback queries
// but 2 instead of 3 waves per SIMD; K=512 product 92.2 vs 91.4 ms; the single
// K=128 mixture 613 vs 816 us)
#ifndef SDMM_GUIDE_CAP_DEFAULT
#define SDMM_GUIDE_CAP_DEFAULT 40
#endif
constexpr int kGuideCapDefault = SDMM_GUIDE_CAP_DEFAULT;
hipError_t launch_split_load(const float* const p[3], const int64_t* src_start, const int64_t* dst_start, int n_items,
                             int64_t total, float* ox, float* oy, float* oz, int32_t* oitem, hipStream_t st);
hipError_t launch_split_sums(const float* x, const float* y, const float* z, const void* chunks, int n_chunks,
                             double* partial, hipStream_t st);
hipError_t launch_split_flags(const float* x, const float* y, const float* z, const int32_t* item, int64_t n,
                              const void* cand, int n_items, int32_t* flags, int64_t* rank, void* temp,
                              size_t temp_bytes, long long* counts, hipStream_t st);
hipError_t launch_split_scatter(const float* x, const float* y, const float* z, const int32_t* item, int64_t n,
                                const void* cand, const int32_t* flags, const int64_t* rank, float* ox, float* oy,
                                float* oz, int32_t* oitem, hipStream_t st);
hipError_t launch_split_decide(const void* items, int n_items, const double* partial, int threshold, void* cand,
                               void* dec, hipStream_t st);
size_t split_scan_temp_bytes(int64_t n);
int split_chunk_samples();
hipError_t launch_sample_cdf(const float* cdf, int n, const float* u, int64_t nq, int32_t* out,
                             hipStream_t st);
hipError_t launch_produce_count(const void* nodes, const PathsDev& P, int64_t path0, int saved, uint64_t seed,
                                int64_t* count, int64_t* offsets, void* temp, size_t temp_bytes, hipStream_t st);
hipError_t launch_produce_records(const void* nodes, int num_nodes, int key_bits, const PathsDev& P, int64_t path0,
                                  int saved, uint64_t seed, const int64_t* offsets, int64_t n_rec, uint32_t* keys0,
                                  uint32_t* keys1, int64_t* codes0, int64_t* codes1, void* recs, void* temp,
                                  size_t temp_bytes, int64_t* seg_dev, int* lost, float* const x[6],
                                  float* const nrm[3], float* w, uint8_t* stats, int32_t* node, int64_t* source,
                                  hipStream_t st);
size_t produce_temp_bytes(int64_t n_paths, int64_t n_records, int key_bits);
}  // namespace sdmm

using namespace sdmm;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

}  // namespace

// the error slot for the library's other host translation units (checkpoint.cpp)
namespace sdmm_detail {
int set_error(int code, const char* msg) { return fail(code, msg); }
void destroy_impl(sdmm_mix* m, bool sync);
void destroy_many(sdmm_mix* const* ms, int n);
}  // namespace sdmm_detail

namespace {

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(SDMM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

// release a scratch buffer before regrowing it: the pointer is cleared first,
// so an error return can never leave it dangling for a second free (the free
// itself is not checked, as in destroy)
template <class T>
void release_dev(T*& p) {
    void* q = (void*)p;
    p = nullptr;
    if (q) (void)hipFree(q);
}
template <class T>
void release_host(T*& p) {
    void* q = (void*)p;
    p = nullptr;
    if (q) (void)hipHostFree(q);
}

}  // namespace

// ==========================================================================
// Host transfer and scratch rules for entry points that host threads call at
// once (round 6; DESIGN.md section 2 "Concurrency"):
//   * no DMA from or to caller (pageable) memory: caller data is copied on the
//     host into the calling thread's pinned bounce buffer and moves by one
//     pinned copy (the runtime's pageable path pins user pages on the fly;
//     two threads' buffers can share a page, and one thread's unpin under the
//     other's transfer is a fault the GPU reports, or a transfer that never
//     completes);
//   * per-call device scratch comes from a pool keyed by (device, stream),
//     held until the call has synchronised that stream: threads on distinct
//     streams never wait for each other, and nothing is freed under a kernel;
//   * a buffer is only ever freed or regrown after the stream that used it
//     has been synchronised.
namespace sdmm_detail {

namespace {
struct PinnedBounce {
    char* p = nullptr;
    size_t cap = 0;
    ~PinnedBounce() {
        if (p) (void)hipHostFree(p);
    }
};
thread_local PinnedBounce t_bounce;

struct ScratchEntry {
    int device = -1;
    hipStream_t st = nullptr;
    std::mutex mu;
    StreamScratch s;
};
std::mutex g_scratch_mu;
std::vector<ScratchEntry*> g_scratch;
}  // namespace

hipError_t bounce_buf(size_t bytes, char** out) {
    if (bytes > t_bounce.cap) {
        if (t_bounce.p) (void)hipHostFree(t_bounce.p);   // idle: its last user synchronised
        t_bounce.p = nullptr;
        t_bounce.cap = 0;
        const size_t cap = std::max<size_t>(bytes + bytes / 4, (size_t)64 << 10);
        const hipError_t e = hipHostMalloc((void**)&t_bounce.p, cap, hipHostMallocDefault);
        if (e != hipSuccess) {
            t_bounce.p = nullptr;
            return e;
        }
        t_bounce.cap = cap;
    }
    *out = t_bounce.p;
    return hipSuccess;
}

std::unique_lock<std::mutex> stream_scratch(int device, hipStream_t st, StreamScratch** out) {
    ScratchEntry* e = nullptr;
    {
        std::lock_guard<std::mutex> g(g_scratch_mu);
        for (ScratchEntry* x : g_scratch)
            if (x->device == device && x->st == st) { e = x; break; }
        if (!e) {
            e = new ScratchEntry();
            e->device = device;
            e->st = st;
            g_scratch.push_back(e);
        }
    }
    *out = &e->s;
    return std::unique_lock<std::mutex>(e->mu);
}

hipError_t scratch_reserve(StreamScratch& s, size_t bytes) {
    if (bytes <= s.cap) return hipSuccess;
    if (s.p) (void)hipFree(s.p);   // idle: every holder synchronised its stream before unlocking
    s.p = nullptr;
    s.cap = 0;
    const size_t cap = std::max<size_t>(bytes + bytes / 2, (size_t)64 << 10);
    const hipError_t e = hipMalloc((void**)&s.p, cap);
    if (e == hipSuccess) s.cap = cap;
    else s.p = nullptr;
    return e;
}

void release_stream_scratch() {
    std::lock_guard<std::mutex> g(g_scratch_mu);
    for (ScratchEntry* x : g_scratch) {
        {
            std::lock_guard<std::mutex> h(x->mu);
            if (x->s.p) {
                (void)hipSetDevice(x->device);
                (void)hipFree(x->s.p);
            }
        }
        delete x;
    }
    g_scratch.clear();
}

}  // namespace sdmm_detail

using sdmm_detail::bounce_buf;
using sdmm_detail::scratch_reserve;
using sdmm_detail::stream_scratch;
using sdmm_detail::StreamScratch;

namespace {

// Copies between caller host memory and device memory as pinned DMAs through
// the thread's bounce buffer, synchronised on st before return.  Items with a
// NULL host pointer are skipped.
struct XferItem {
    void* host;
    void* dev;
    size_t bytes;
};
int xfer(const XferItem* items, int n, bool to_device, hipStream_t st) {
    size_t total = 0;
    for (int i = 0; i < n; ++i)
        if (items[i].host) total += (items[i].bytes + 15) / 16 * 16;
    if (total == 0) return SDMM_OK;
    char* pin = nullptr;
    HIP_TRY(bounce_buf(total, &pin));
    size_t off = 0;
    hipError_t e = hipSuccess;
    for (int i = 0; i < n && e == hipSuccess; ++i) {
        const XferItem& it = items[i];
        if (!it.host) continue;
        if (to_device) {
            std::memcpy(pin + off, it.host, it.bytes);
            e = hipMemcpyAsync(it.dev, pin + off, it.bytes, hipMemcpyHostToDevice, st);
        } else {
            e = hipMemcpyAsync(pin + off, it.dev, it.bytes, hipMemcpyDeviceToHost, st);
        }
        off += (it.bytes + 15) / 16 * 16;
    }
    const hipError_t es = hipStreamSynchronize(st);   // always: the bounce buffer is reused
    if (e == hipSuccess) e = es;
    if (e != hipSuccess) return fail(SDMM_E_HIP, std::string("host transfer: ") + hipGetErrorString(e));
    if (!to_device) {
        off = 0;
        for (int i = 0; i < n; ++i) {
            const XferItem& it = items[i];
            if (!it.host) continue;
            std::memcpy(it.host, pin + off, it.bytes);
            off += (it.bytes + 15) / 16 * 16;
        }
    }
    return SDMM_OK;
}

// (float) pow((double)(float)INV_SQRT_TWO_PI, d) -- mvtn.h:351-352
float norm_const(int d) {
    return (float)std::pow((double)(float)0.39894228040143267793994605993438186847585863116492, (double)d);
}

// --------------------------------------------------------------------------
// PCG32 + uniformHemisphereInit on the host (O(K), runs once per mixture).
struct Pcg32 {
    uint64_t state, inc;
    void seed(uint64_t initstate, uint64_t initseq) {
        state = 0u;
        inc = (initseq << 1u) | 1u;
        next_uint();
        state += initstate;
        next_uint();
    }
    uint32_t next_uint() {
        uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((~rot + 1u) & 31));
    }
    float next_float() {
        union { uint32_t u; float f; } x;
        x.u = (next_uint() >> 9) | 0x3f800000u;
        return x.f - 1.0f;
    }
};

void coordinates_f(const float n[3], float to[9]) {
    float sign = std::copysign(1.0f, n[2]);
    const float a = -1.0f / (sign + n[2]);
    const float b = n[0] * n[1] * a;
    to[0] = 1.0f + sign * n[0] * n[0] * a; to[1] = sign * b; to[2] = -sign * n[0];
    to[3] = b; to[4] = sign + n[1] * n[1] * a; to[5] = -n[1];
    to[6] = n[0]; to[7] = n[1]; to[8] = n[2];
}

float fl_cos(float x) { return (float)std::cos((double)x); }
float fl_sin(float x) { return (float)std::sin((double)x); }

// mixture_model_init.h:79-242 (kMeansPlusPlus == false branch).
// skip: draws already taken from the stream (kMeansPlusPlus: one per position
// for the k-means++ choice, :130-138, before the direction jitter)
void hemisphere_init(const float* positions, const float* normals, int nPositions, float depthPrior,
                     float minDist, uint64_t seed, float* weights, float* means, float* covs,
                     float* bpriors, float* bdepth, int skip = 0) {
    const double PI = 3.14159265358979323846;
    Pcg32 rng;
    rng.seed(seed, 0xda3e39cb94b95bdbULL);
    for (int i = 0; i < skip; ++i) (void)rng.next_uint();
    const float maxRadiusSqr = (float)10.644640675668422;  // chi2(6).quantile(0.9)
    const float widthVarSqr = (float)(0.5 * (double)minDist * (double)minDist / (double)maxRadiusSqr);
    const float depthVarSqr = depthPrior * depthPrior / maxRadiusSqr;
    const float nThetas = 2.0f, nPhis = 4.0f;
    const float directionalInit = 1.0f / (nThetas * nPhis);
    const int K = nPositions * 8;
    int k = 0;
    for (int pi = 0; pi < nPositions; ++pi) {
        const float* p = positions + 3 * pi;
        const float* n = normals + 3 * pi;
        float to[9];
        coordinates_f(n, to);
        const float* s = to;
        const float* t = to + 3;
        float cov[25] = {0};
        for (int i = 0; i < 5; ++i) cov[6 * i] = 1.0f;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                cov[5 * i + j] = (s[i] * s[j] * widthVarSqr + t[i] * t[j] * widthVarSqr) +
                                 n[i] * n[j] * depthVarSqr;
        const float dcov = (float)(2.0 * PI * (double)directionalInit);
        cov[18] = dcov; cov[24] = dcov; cov[19] = 0.0f; cov[23] = 0.0f;
        float bPrior[25] = {0};
        for (int i = 0; i < 5; ++i) bPrior[6 * i] = 1.0f;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                bPrior[5 * i + j] = s[i] * s[j] * 1e-4f + t[i] * t[j] * 1e-4f + n[i] * n[j] * 1e-4f;
        bPrior[18] = 1e-5f; bPrior[24] = 1e-5f;
        float theta = 0.0f;
        for (int ti = 0; ti < (int)nThetas; ++ti) {
            float rn = (float)(((double)rng.next_float() - 0.5) * 2e-1);
            theta = (float)((double)theta + (0.5 * PI / (double)(nThetas + 1.0f) + (double)rn));
            const float cosTheta = fl_cos(theta);
            const float sinTheta = std::sqrt(1.0f - cosTheta * cosTheta);
            float phi = 0.0f;
            for (int fi = 0; fi < (int)nPhis; ++fi) {
                rn = (float)(((double)rng.next_float() - 0.5) * 1e-1);
                phi = (float)((double)phi + (2.0 * PI / (double)nPhis + (double)rn));
                const float sinPhi = fl_sin(phi), cosPhi = fl_cos(phi);
                const float dl0 = sinTheta * cosPhi, dl1 = sinTheta * sinPhi, dl2 = cosTheta;
                float* mean = means + 6 * k;
                for (int i = 0; i < 3; ++i) mean[i] = p[i];
                for (int i = 0; i < 3; ++i) mean[3 + i] = (s[i] * dl0 + t[i] * dl1) + n[i] * dl2;
                std::memcpy(covs + 25 * k, cov, sizeof(cov));
                weights[k] = 1.0f / (float)K;
                std::memcpy(bpriors + 25 * k, bPrior, sizeof(bPrior));
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j) bdepth[9 * k + 3 * i + j] = n[i] * n[j] * 1e-6f;
                ++k;
            }
        }
    }
}

}  // namespace

// ==========================================================================
// one stream-ordered allocation holding the blocks of many mixtures; freed
// with its last mixture
struct Slab {
    void* p = nullptr;
    std::atomic<int> refs{0};   // members may be destroyed from different host threads
    hipStream_t st = nullptr;
};

struct sdmm_mix {
    int K = 0, Kp = 0, cpl = 1, lps = 64;   // statistics E-step layout
    int rcpl = 2, rlps = 64;                 // responsibility E-step layout (same Kp)
    int rtile = 0;                           // 1: estep_resp_tile_kernel (64 < K <= 128)
                                             // 2: estep_resp_mfma_kernel (every K)
                                             // 3: estep_resp_split_kernel (bf16x3 MFMA forms, Kp <= 128)
    int rvariant = 4;                        // tile / mfma kernel variant: KT=8, 3 waves/SIMD
    int stile = 0;                           // 1: estep_stats_tile_kernel (64 < K <= 128)
                                             // 2: its GROUP form (128 < K <= 512: Kp / 128 waves per chunk)
    int svariant = 0;                        // its occupancy variant
    int device = 0;
    int cus = 256;
    int resp_blocks = 2, stats_blocks = 2;   // resident 256-thread WGs per CU
    // guided-query scratch: fallback counter + list of fallback query indices
    int guide_cap = kGuideCapDefault;   // candidate-list capacity (sdmm_set_guide_capacity)
    mutable int* guide_fb = nullptr;
    mutable int64_t guide_fb_cap = 0;
    mutable GuideSortScratch guide_sort{};
    mutable ProductScratch product_scratch{};   // grow-only (guide.hip product_scratch)
    int guide_order = 1;            // 1: serve large batches in Morton order of c (sdmm_set_guide_order)
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    sdmm_em_params params{};
    float norm2 = 0, norm3 = 0, norm5 = 0;
    bool initialised = false;

    // device memory
    void* block = nullptr;       // canonical + state + packed records
    struct Slab* slab = nullptr; // block carved from a shared slab (sdmm_create_many_on_stream)
    CanonDev C{};
    EmStateDev S{};
    float* ep = nullptr;
    float* gp = nullptr;
    double* stats = nullptr;     // compact stats (2 + 21K)
    double* tmp_mean = nullptr;  // K*6 (set_params / init)
    double* tmp_cov = nullptr;   // K*25
    unsigned* mcount = nullptr;  // the spread M-step's two counters (zero between launches)
    float* partials = nullptr;
    int partial_rows = 0;
    int pstride = 0;
    // staging for host-resident samples
    void* staging = nullptr;
    size_t staging_bytes = 0;
    // batched per-leaf EM tables (this handle as mixes[0]): device + pinned host
    void* batch_dev = nullptr;
    void* batch_host = nullptr;
    // sdmm_iterations_run's gather scratch (this handle as mixes[0]): the
    // pointer table + the counters, device and pinned host, grown on demand
    mutable void* it_dev = nullptr;
    mutable void* it_host = nullptr;
    mutable size_t it_cap = 0;
    size_t batch_bytes = 0;
    hipEvent_t batch_copied = nullptr;   // the last table upload has completed
    hipEvent_t batch_done = nullptr;     // the last batch's kernels have completed
    // sample-sharded batched EM: the leaves' stats + counts, all-reduced as one buffer
    double* shard_stats = nullptr;
    size_t shard_bytes = 0;
};

// ==========================================================================
// Multi-GPU transport (include/sdmm_gpu.h, sdmm_comm_*).  The reference has no
// collective; the library's exchange steps are (a) the SUM of
// the fp64 sufficient statistics before each M-step of a sample-sharded EM and
// (b) broadcasts of leaf mixtures from their owner rank (leaf-sharded EM).
// Transports: RCCL (one rank per GPU, over xGMI) or host callbacks (the caller's
// own collective on host buffers -- MPI, gloo -- staged through pinned memory).
struct sdmm_comm {
    int rank = 0, nranks = 1, device = 0;
    ncclComm_t nccl = nullptr;
    sdmm_host_allreduce_f64 h_allreduce = nullptr;
    sdmm_host_broadcast h_broadcast = nullptr;
    void* user = nullptr;
    void* pinned = nullptr;   // host transport staging
    size_t pinned_bytes = 0;
};

namespace {

int nccl_fail(ncclResult_t r, const char* what) {
    return fail(SDMM_E_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

int comm_pinned(sdmm_comm* c, size_t bytes) {
    if (bytes <= c->pinned_bytes) return SDMM_OK;
    release_host(c->pinned);
    c->pinned = nullptr;
    c->pinned_bytes = 0;
    HIP_TRY(hipHostMalloc(&c->pinned, bytes, hipHostMallocDefault));
    c->pinned_bytes = bytes;
    return SDMM_OK;
}

// SUM over ranks of count doubles in device memory, in place, ordered on st.
int comm_allreduce(sdmm_comm* c, double* dbuf, size_t count, hipStream_t st) {
    if (c->nranks == 1 && !c->nccl) return SDMM_OK;
    if (c->nccl) {
        const ncclResult_t r = ncclAllReduce(dbuf, dbuf, count, ncclFloat64, ncclSum, c->nccl, st);
        return r == ncclSuccess ? SDMM_OK : nccl_fail(r, "ncclAllReduce");
    }
    int r = comm_pinned(c, sizeof(double) * count);
    if (r) return r;
    HIP_TRY(hipMemcpyAsync(c->pinned, dbuf, sizeof(double) * count, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (c->h_allreduce((double*)c->pinned, count, c->user) != 0)
        return fail(SDMM_E_STATE, "host all-reduce callback failed");
    HIP_TRY(hipMemcpyAsync(dbuf, c->pinned, sizeof(double) * count, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    return SDMM_OK;
}

// bytes of device memory broadcast from rank root, in place, ordered on st
// (RCCL: call between ncclGroupStart/End to fuse several).
int comm_broadcast(sdmm_comm* c, void* dbuf, size_t bytes, int root, hipStream_t st) {
    if (c->nranks == 1 && !c->nccl) return SDMM_OK;
    if (c->nccl) {
        const ncclResult_t r = ncclBroadcast(dbuf, dbuf, bytes, ncclUint8, root, c->nccl, st);
        return r == ncclSuccess ? SDMM_OK : nccl_fail(r, "ncclBroadcast");
    }
    int r = comm_pinned(c, bytes);
    if (r) return r;
    HIP_TRY(hipMemcpyAsync(c->pinned, dbuf, bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (c->h_broadcast(c->pinned, bytes, root, c->user) != 0)
        return fail(SDMM_E_STATE, "host broadcast callback failed");
    HIP_TRY(hipMemcpyAsync(dbuf, c->pinned, bytes, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    return SDMM_OK;
}

}  // namespace

namespace {

int choose_layout(int K, int& cpl, int& lps) {
    // components are evaluated in packed pairs: CPL is always even
    if (K <= 16) { lps = 8; cpl = 2; }
    else if (K <= 32) { lps = 16; cpl = 2; }
    else if (K <= 64) { lps = 32; cpl = 2; }
    else if (K <= 128) { lps = 64; cpl = 2; }
    else if (K <= 256) { lps = 64; cpl = 4; }
    else if (K <= 512) { lps = 64; cpl = 8; }
    else return -1;
    return 0;
}

// Work split of an E-step launch: contiguous chunk of samples per wave.
struct Split {
    int64_t chunk;
    int blocks;
    int wpb;
};

Split split_for(const sdmm_mix* m, int64_t n, int lps, int blocks_per_cu) {
    const int spw = 64 / lps;
    const int64_t target_waves = (int64_t)m->cus * 4 * (blocks_per_cu > 0 ? blocks_per_cu : 2);
    int64_t chunk = (n + target_waves - 1) / target_waves;
    if (chunk < 4 * spw) chunk = 4 * spw;
    chunk = ((chunk + spw - 1) / spw) * spw;
    const int wpb = 4;
    int64_t waves = (n + chunk - 1) / chunk;
    int64_t blocks = (waves + wpb - 1) / wpb;
    if (blocks < 1) blocks = 1;
    return Split{chunk, (int)blocks, wpb};
}

SamplesDev to_dev(const sdmm_samples* s) {
    SamplesDev d;
    for (int i = 0; i < 6; ++i) d.x[i] = s->x[i];
    d.w = s->w;
    d.hpdf = s->hpdf;
    d.isDiffuse = s->is_diffuse;
    return d;
}

int check_samples(const sdmm_samples* s) {
    if (!s) return fail(SDMM_E_INVALID, "samples is NULL");
    if (s->n < 0) return fail(SDMM_E_INVALID, "negative sample count");
    if (s->n == 0) return SDMM_OK;
    for (int i = 0; i < 6; ++i)
        if (!s->x[i]) return fail(SDMM_E_INVALID, "sample plane x[i] is NULL");
    if (!s->w) return fail(SDMM_E_INVALID, "weight plane is NULL");
    return SDMM_OK;
}

int ensure_partials(sdmm_mix* m, int rows) {
    if (rows <= m->partial_rows) return SDMM_OK;
    // the handle's earlier launches may still read or write the old rows
    if (m->partials) HIP_TRY(hipStreamSynchronize(m->stream));
    release_dev(m->partials);
    m->partials = nullptr;
    int cap = rows < 1024 ? 1024 : rows;
    HIP_TRY(hipMalloc(&m->partials, sizeof(float) * (size_t)cap * m->pstride));
    m->partial_rows = cap;
    return SDMM_OK;
}

// Guided-batch scratch, one allocation grown on demand: [count, fallback
// list...] (cap + 1 ints), then the coherent-order buffers (2 x cap keys,
// 2 x cap indices, the radix sort's temporary storage).  The previous buffer
// is only released after a stream sync.
int grow_guide_scratch(int*& fb, int64_t& fb_cap, GuideSortScratch& sort, hipStream_t st, int64_t nq) {
    if (nq + 1 <= fb_cap) return SDMM_OK;
    if (fb) {
        HIP_TRY(hipStreamSynchronize(st));
        release_dev(fb);
        fb = nullptr;
        fb_cap = 0;
    }
    const int64_t cap = (nq + 1 < (1 << 20)) ? (1 << 20) : nq + 1;
    const size_t a = ((sizeof(int) * (size_t)cap + 255) / 256) * 256;
    const size_t kb = ((sizeof(uint32_t) * (size_t)cap + 255) / 256) * 256;
    const size_t tb = guide_sort_temp_bytes((int)(cap > INT32_MAX ? INT32_MAX : cap));
    char* base = nullptr;
    HIP_TRY(hipMalloc((void**)&base, a + 4 * kb + tb + 256));
    fb = (int*)base;
    sort.keys[0] = (uint32_t*)(base + a);
    sort.keys[1] = (uint32_t*)(base + a + kb);
    sort.idx[0] = (int32_t*)(base + a + 2 * kb);
    sort.idx[1] = (int32_t*)(base + a + 3 * kb);
    sort.temp = base + a + 4 * kb;
    sort.temp_bytes = tb;
    fb_cap = cap;
    return SDMM_OK;
}
int ensure_guide_scratch(const sdmm_mix* m, int64_t nq) {
    return grow_guide_scratch(m->guide_fb, m->guide_fb_cap, m->guide_sort, m->stream, nq);
}

// coherent order for batches large enough to fill the chip several times
const GuideSortScratch* guide_order(const sdmm_mix* m, int64_t nq) {
    return (m->guide_order && nq >= (1 << 14)) ? &m->guide_sort : nullptr;
}

// Work split of m's statistics E-step over n samples (the same for a
// single-mixture call and for that mixture as a leaf of a batched call).
struct StatsPlan {
    int64_t chunk;
    int blocks;
};
StatsPlan stats_plan(const sdmm_mix* m, int64_t n) {
    if (m->stile == 2) {
        // GROUP form: a workgroup (Kp / 128 waves) per chunk; one round of
        // resident workgroups, chunks of whole 64-sample blocks
        const int64_t resident = (int64_t)m->cus * (m->stats_blocks > 0 ? m->stats_blocks : 1);
        int64_t chunk = (n + resident - 1) / resident;
        chunk = ((chunk + 63) / 64) * 64;
        if (chunk < 64) chunk = 64;
        const int64_t blocks = (n + chunk - 1) / chunk;
        return StatsPlan{chunk, (int)(blocks > 0 ? blocks : 1)};
    }
    if (m->stile) {
        // one round of resident waves, each a whole number of 64-sample blocks
        const int64_t resident = (int64_t)m->cus * 4 * (m->stats_blocks > 0 ? m->stats_blocks : 1);
        int64_t chunk = (n + resident - 1) / resident;
        chunk = ((chunk + 63) / 64) * 64;
        if (chunk < 64) chunk = 64;
        const int64_t waves = (n + chunk - 1) / chunk;
        return StatsPlan{chunk, (int)((waves + 3) / 4 > 0 ? (waves + 3) / 4 : 1)};
    }
    const Split sp = split_for(m, n, m->lps, m->stats_blocks);
    return StatsPlan{sp.chunk, sp.blocks};
}

hipError_t launch_stats_kernel(const sdmm_mix* m, const SamplesDev& d, int64_t n, const StatsPlan& p, int blocks,
                               float* partials, hipStream_t st, const LeafDesc* leaves, const int2* items) {
    if (m->stile)
        return launch_estep_stats_tile(m->svariant, m->ep, m->Kp, m->K, d, n, p.chunk, blocks, partials, m->pstride,
                                       st, leaves, items);
    return launch_estep_stats(m->cpl, m->lps, m->ep, m->Kp, m->K, d, n, p.chunk, blocks, 4, partials, m->pstride,
                              st, leaves, items);
}

int run_estep_stats(sdmm_mix* m, const sdmm_samples* s, double* stats_out) {
    SamplesDev d = to_dev(s);
    const StatsPlan p = stats_plan(m, s->n);
    int r = ensure_partials(m, p.blocks);
    if (r) return r;
    HIP_TRY(launch_stats_kernel(m, d, s->n, p, p.blocks, m->partials, m->stream, nullptr, nullptr));
    HIP_TRY(launch_reduce_partials(m->partials, p.blocks, m->pstride, m->ep, m->Kp, m->K, stats_out, m->stream));
    return SDMM_OK;
}

}  // namespace

// ==========================================================================
extern "C" {

const char* sdmm_last_error(void) { return g_err.c_str(); }

int sdmm_release_cached_scratch(void) {
    sdmm_detail::release_stream_scratch();
    return SDMM_OK;
}
int sdmm_abi_version(void) { return SDMM_ABI_VERSION; }

void sdmm_em_params_default(sdmm_em_params* p) {
    if (!p) return;
    p->alpha = 0.9f;
    for (int i = 0; i < 5; ++i) p->bprior[i] = 1e-5f;
    p->ni_prior_minus_one = 6e-5f;
    p->epsilon = 1e-100;
    p->decrease_prior = 1;
}

size_t sdmm_stats_len(int K) { return 2 + (size_t)ST_FIELDS * (size_t)K; }

namespace {
int create_impl(int K, const sdmm_em_params* params, int device, hipStream_t ordered, bool on_stream,
                sdmm_mix** out, void* ext_block = nullptr);
}  // namespace

int sdmm_create(int K, const sdmm_em_params* params, int device, sdmm_mix** out) {
    return create_impl(K, params, device, nullptr, false, out);
}

int sdmm_create_on_stream(int K, const sdmm_em_params* params, int device, void* hip_stream, sdmm_mix** out) {
    return create_impl(K, params, device, (hipStream_t)hip_stream, true, out);
}

}  // extern "C"

namespace {

// The handle's fixed-size device arrays, all 16-byte aligned, carved from one
// block at base (base NULL: only the size); returns the block size.  The
// parameters, derived arrays, packed records and stepwise state come first:
// everything before `stats` is the mixture (copied by sdmm_clone, broadcast by
// sdmm_mix_broadcast).
size_t layout_block(sdmm_mix* m, char* base) {
    const size_t Kc = (size_t)m->K;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* p = base ? base + off : nullptr;
        off += (bytes + 15) / 16 * 16;
        return p;
    };
    float* w = (float*)take(4 * Kc);
    float* cdf = (float*)take(4 * Kc);
    float* mean = (float*)take(24 * Kc);
    float* cov = (float*)take(100 * Kc);
    float* to = (float*)take(36 * Kc);
    float* cl = (float*)take(100 * Kc);
    float* cli = (float*)take(100 * Kc);
    float* di = (float*)take(4 * Kc);
    float* mp = (float*)take(24 * Kc);
    float* cc = (float*)take(16 * Kc);
    float* ml = (float*)take(36 * Kc);
    float* mdi = (float*)take(4 * Kc);
    float* cdl = (float*)take(16 * Kc);
    float* cdli = (float*)take(16 * Kc);
    float* cdi = (float*)take(4 * Kc);
    int* valid = (int*)take(4 * Kc);
    double* sc = (double*)take(8 * SC_COUNT);
    double* T = (double*)take(8 * Kc);
    double* sgW = (double*)take(8 * Kc);
    double* sgM = (double*)take(40 * Kc);
    double* sgC = (double*)take(200 * Kc);
    float* bp = (float*)take(100 * Kc);
    float* bd = (float*)take(36 * Kc);
    float* ep = (float*)take(4 * (size_t)EP_FIELDS * m->Kp);
    float* gp = (float*)take(4 * (size_t)GP_STRIDE * m->Kp);
    double* stats = (double*)take(8 * (sdmm_stats_len(m->K) + 1));   // + the sample count of a sharded step
    double* tmean = (double*)take(48 * Kc);
    double* tcov = (double*)take(200 * Kc);
    unsigned* mcount = (unsigned*)take(8);
    if (base) {
        m->C = CanonDev{w, cdf, mean, cov, to, cl, cli, di, mp, cc, ml, mdi, cdl, cdli, cdi, valid};
        m->S = EmStateDev{sc, T, sgW, sgM, sgC, bp, bd};
        m->ep = ep;
        m->gp = gp;
        m->stats = stats;
        m->tmp_mean = tmean;
        m->tmp_cov = tcov;
        m->mcount = mcount;
    }
    return (off + 255) / 256 * 256;
}

void constructor_scalars(const sdmm_mix* m, double* scal) {
    for (int i = 0; i < SC_COUNT; ++i) scal[i] = 0.0;
    scal[SC_NORM] = 1.0;
    scal[SC_ALPHA] = (double)m->params.alpha;
    scal[SC_NI] = (double)m->params.ni_prior_minus_one;
    scal[SC_DECP] = m->params.decrease_prior ? 1.0 : 0.0;
    scal[SC_CUT] = 32.0;
}

// E-step occupancy per K and kernel choice (the layout depends on K and the
// process's environment only): queried once per combination
struct OccCache {
    int K = -1, kern = -1, resp = 0, stats = 0;
};

int create_impl(int K, const sdmm_em_params* params, int device, hipStream_t ordered, bool on_stream,
                sdmm_mix** out, void* ext_block) {
    if (!out) return fail(SDMM_E_INVALID, "out is NULL");
    *out = nullptr;
    int cpl, lps;
    if (K < 1 || choose_layout(K, cpl, lps)) return fail(SDMM_E_INVALID, "K must be in [1, 512]");
    sdmm_mix* m = new (std::nothrow) sdmm_mix();
    if (!m) return fail(SDMM_E_NOMEM, "out of host memory");
    m->K = K;
    m->cpl = cpl;
    m->lps = lps;
    m->Kp = cpl * lps;
    m->device = device;
    if (params) m->params = *params; else sdmm_em_params_default(&m->params);
    m->norm2 = norm_const(2);
    m->norm3 = norm_const(3);
    m->norm5 = norm_const(5);
    m->pstride = ((ST_FIELDS * m->Kp + 2 + 3) / 4) * 4;

    auto cleanup = [&](int code) { sdmm_destroy(m); return code; };
    if (hipSetDevice(device) != hipSuccess) return cleanup(fail(SDMM_E_HIP, "hipSetDevice failed"));
    (void)hipDeviceGetAttribute(&m->cus, hipDeviceAttributeMultiprocessorCount, device);
    if (m->cus <= 0) m->cus = 256;
    // responsibilities: for 64 < K <= 128, 4 components per lane and 2 samples
    // per wave halve the per-sample reduction/normalisation overhead per pair
    // and give each lane two independent packed chains (same Kp = 128)
    m->rcpl = cpl;
    m->rlps = lps;
    if (K > 64 && K <= 128) { m->rcpl = 4; m->rlps = 32; }
    // 64 < K <= 128 (Kp = 128): the bf16x3 split-MFMA kernel (estep_split.hip:
    // the eight linear forms on the matrix cores, the rest packed f32; 186 vs
    // 204 us per 2^20 samples).  SDMM_RESP_KERNEL selects
    // the others for A/B measurements: tile (estep_resp_tile_kernel, the VALU
    // form), mfma (f32 matrix cores, estep_mfma.hip), legacy
    // (estep_resp_kernel<4,32>); split also for other K with Kp / 16 in {1, 2, 4}.
    {
        const char* ev = std::getenv("SDMM_RESP_KERNEL");
        const bool legacy = ev && std::strcmp(ev, "legacy") == 0;
        const bool mfma = ev && std::strcmp(ev, "mfma") == 0;
        const bool tile = ev && std::strcmp(ev, "tile") == 0;
        const bool split = ev && std::strcmp(ev, "split") == 0;
        if (K > 64 && K <= 128 && !legacy && !mfma) {
            m->rtile = 1;
            m->rcpl = 2;
            m->rlps = 64;
            if (!tile && estep_resp_split_supported(m->Kp)) m->rtile = 3;
        }
        if (mfma) m->rtile = 2;
        if (split && estep_resp_split_supported(m->Kp)) m->rtile = 3;
        // statistics: the tile kernel for 64 < K <= 128, its GROUP form for
        // 128 < K <= 512 (estep.hip), estep_stats_kernel otherwise
        if (K > 64 && K <= 128) m->stile = 1;
        if (K > 128 && K <= 512) m->stile = 2;
    }
    static thread_local OccCache occ[8];
    OccCache& oc = occ[(K * 7 + device) & 7];
    const int kern = ((m->rtile * 16 + m->rvariant) * 16 + m->stile) * 16 + m->svariant;
    if (oc.K == K * 64 + device && oc.kern == kern) {
        m->resp_blocks = oc.resp;
        m->stats_blocks = oc.stats;
    } else {
        int unused = 0;
        if (estep_occupancy(m->rcpl, m->rlps, m->Kp, &m->resp_blocks, &unused) != hipSuccess ||
            estep_occupancy(m->cpl, m->lps, m->Kp, &unused, &m->stats_blocks) != hipSuccess)
            return cleanup(fail(SDMM_E_HIP, "E-step occupancy query failed"));
        if (m->rtile == 2 && estep_resp_mfma_occupancy(m->rvariant, m->Kp, &m->resp_blocks) != hipSuccess)
            return cleanup(fail(SDMM_E_HIP, "E-step occupancy query failed"));
        if (m->rtile == 3) {
            int wpc = 0;
            if (estep_resp_split_occupancy(m->rvariant, m->Kp, &wpc) != hipSuccess)
                return cleanup(fail(SDMM_E_HIP, "E-step occupancy query failed"));
            m->resp_blocks = wpc;   // resident waves per CU (split kernel)
        }
        if (m->rtile == 1 && estep_resp_tile_occupancy(m->rvariant, &m->resp_blocks) != hipSuccess)
            return cleanup(fail(SDMM_E_HIP, "E-step occupancy query failed"));
        if (m->stile && estep_stats_tile_occupancy(m->svariant, m->Kp, &m->stats_blocks) != hipSuccess)
            return cleanup(fail(SDMM_E_HIP, "E-step occupancy query failed"));
        oc.K = K * 64 + device;
        oc.kern = kern;
        oc.resp = m->resp_blocks;
        oc.stats = m->stats_blocks;
    }
    if (on_stream) {
        m->stream = ordered;
    } else {
        if (hipStreamCreateWithFlags(&m->own_stream, hipStreamNonBlocking) != hipSuccess)
            return cleanup(fail(SDMM_E_HIP, "hipStreamCreate failed"));
        m->stream = m->own_stream;
    }

    if (ext_block) {   // a slab member: carve only (the caller initialises)
        layout_block(m, (char*)ext_block);
        *out = m;
        return SDMM_OK;
    }
    // one allocation for every fixed-size array (all 16-byte aligned)
    const size_t total = layout_block(m, nullptr);
    // hipMalloc also for a handle created on a caller's stream (sdmm_clone,
    // sdmm_create_on_stream): no stream-ordered pool allocation on an entry
    // point host threads may call at once (host transfer rules above).  The
    // memset goes on the handle's stream, ordered before the init kernels
    // below (a plain hipMemset runs on the null stream, which a non-blocking
    // stream does not wait for -- it could land after them and zero the state).
    if (hipMalloc(&m->block, total) != hipSuccess) return cleanup(fail(SDMM_E_HIP, "hipMalloc failed"));
    if (hipMemsetAsync(m->block, 0, total, m->stream) != hipSuccess)
        return cleanup(fail(SDMM_E_HIP, "hipMemsetAsync failed"));
    layout_block(m, (char*)m->block);
    const size_t Kc = (size_t)K;
    double* sc = m->S.scalars;
    float* bp = m->S.bPriors;
    float* bd = m->S.bDepth;
    // StepwiseTangentEM constructor state (stepwise_tangent.h:221-252)
    double scal[SC_COUNT];
    constructor_scalars(m, scal);
    (void)Kc;
    const float eps = (float)m->params.epsilon;
    // the constructor state by a kernel, ordered on the handle's stream
    if (launch_init_state(K, scal, m->params.bprior, eps, sc, bp, bd, m->stream) != hipSuccess)
        return cleanup(fail(SDMM_E_HIP, "state init kernel launch failed"));
    // packed records: every component dead until init/set_params
    if (launch_pack_all(K, m->Kp, m->C, m->ep, m->gp, m->norm5, m->stream) != hipSuccess)
        return cleanup(fail(SDMM_E_HIP, "pack kernel launch failed"));
    if (!on_stream && hipStreamSynchronize(m->stream) != hipSuccess)
        return cleanup(fail(SDMM_E_HIP, "hipStreamSynchronize failed"));
    *out = m;
    return SDMM_OK;
}

// n handles whose blocks are carved from ONE stream-ordered slab: one
// allocation, one memset, one init + one pack launch for the whole set
int create_many(int K, const sdmm_em_params* params, int device, hipStream_t st, int n, sdmm_mix** out) {
    if (n < 0 || (n > 0 && !out)) return fail(SDMM_E_INVALID, "invalid argument");
    for (int i = 0; i < n; ++i) out[i] = nullptr;
    if (n == 0) return SDMM_OK;
    if (hipSetDevice(device) != hipSuccess) return fail(SDMM_E_HIP, "hipSetDevice failed");
    Slab* slab = new (std::nothrow) Slab();
    if (!slab) return fail(SDMM_E_NOMEM, "out of host memory");
    slab->st = st;
    sdmm_mix probe;
    probe.K = K;
    {
        int cpl, lps;
        if (K < 1 || choose_layout(K, cpl, lps)) { delete slab; return fail(SDMM_E_INVALID, "K must be in [1, 512]"); }
        probe.Kp = cpl * lps;
    }
    const size_t stride = layout_block(&probe, nullptr);
    if (hipMallocAsync(&slab->p, stride * (size_t)n, st) != hipSuccess) {
        delete slab;
        return fail(SDMM_E_HIP, "hipMallocAsync failed");
    }
    int r = SDMM_OK;
    // fault injection for the cleanup path's test (tests/test_gpu_batched.py),
    // behind the explicit debug switch SDMM_DEBUG_FAULT_INJECTION=1 (README):
    // member SDMM_TEST_FAIL_MEMBER then fails as if its creation had
    int fail_at = -1;
    if (const char* dbg = std::getenv("SDMM_DEBUG_FAULT_INJECTION"); dbg && std::strcmp(dbg, "1") == 0) {
        const char* inject = std::getenv("SDMM_TEST_FAIL_MEMBER");
        fail_at = inject ? std::atoi(inject) : -1;
        if (fail_at >= 0) std::fprintf(stderr, "sdmm: debug fault injection at create_many member %d\n", fail_at);
    }
    for (int i = 0; i < n && !r; ++i) {
        if (i == fail_at) { r = fail(SDMM_E_HIP, "create_many: injected failure"); break; }
        r = create_impl(K, params, device, st, true, &out[i], (char*)slab->p + stride * (size_t)i);
        if (!r) { out[i]->slab = slab; ++slab->refs; }
    }
    hipError_t e = r ? hipSuccess : hipMemsetAsync(slab->p, 0, stride * (size_t)n, st);
    if (!r && e == hipSuccess) {
        sdmm_mix* m0 = out[0];
        double scal[SC_COUNT];
        constructor_scalars(m0, scal);
        e = launch_init_pack_many(n, K, m0->Kp, scal, m0->params.bprior, (float)m0->params.epsilon, m0->S.scalars,
                                  m0->S.bPriors, m0->S.bDepth, m0->C, m0->ep, m0->gp, m0->norm5, stride, st);
    }
    if (r || e != hipSuccess) {
        // hold the slab across the members' destruction: the last member's
        // sdmm_destroy must not free it under us (it is freed once, below)
        ++slab->refs;
        for (int i = 0; i < n; ++i) { sdmm_destroy(out[i]); out[i] = nullptr; }
        if (--slab->refs == 0) { (void)hipFreeAsync(slab->p, st); delete slab; }
        return r ? r : fail(SDMM_E_HIP, std::string("create_many: ") + hipGetErrorString(e));
    }
    return SDMM_OK;
}

}  // namespace

extern "C" {

void sdmm_destroy(sdmm_mix* m) { sdmm_detail::destroy_impl(m, true); }

}  // extern "C"

// synced: the caller has synchronised the handle's streams (destroy_many)
void sdmm_detail::destroy_impl(sdmm_mix* m, bool sync) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    if (sync && m->own_stream) (void)hipStreamSynchronize(m->own_stream);
    if (sync && m->stream && m->stream != m->own_stream) (void)hipStreamSynchronize(m->stream);
    if (m->slab) {
        if (--m->slab->refs == 0) {
            // on the destroying handle's current stream (synchronised above):
            // the slab's creation stream may be gone by now, or no longer be
            // any member's stream after sdmm_set_stream
            (void)hipFreeAsync(m->slab->p, m->stream);
            delete m->slab;
        }
    } else if (m->block) {
        (void)hipFree(m->block);
    }
    if (m->partials) (void)hipFree(m->partials);
    if (m->guide_fb) (void)hipFree(m->guide_fb);
    // after the handle's last product launch (streams are synchronised above
    // or by destroy_many)
    if (m->product_scratch.base) (void)hipFree(m->product_scratch.base);
    if (m->staging) (void)hipFree(m->staging);
    if (m->batch_dev) (void)hipFree(m->batch_dev);
    if (m->batch_host) (void)hipHostFree(m->batch_host);
    if (m->it_dev) (void)hipFree(m->it_dev);
    if (m->it_host) (void)hipHostFree(m->it_host);
    if (m->shard_stats) (void)hipFree(m->shard_stats);
    if (m->batch_copied) (void)hipEventDestroy(m->batch_copied);
    if (m->batch_done) (void)hipEventDestroy(m->batch_done);
    if (m->own_stream) (void)hipStreamDestroy(m->own_stream);
    delete m;
}

// many handles: each distinct stream synchronised once (a training pass
// destroys the mixtures of every split leaf: ~1 us of synchronisation each)
void sdmm_detail::destroy_many(sdmm_mix* const* ms, int n) {
    std::vector<hipStream_t> seen;
    for (int i = 0; i < n; ++i) {
        const sdmm_mix* m = ms[i];
        if (!m) continue;
        for (hipStream_t st : {m->own_stream, m->stream})
            if (st && std::find(seen.begin(), seen.end(), st) == seen.end()) {
                (void)hipSetDevice(m->device);
                (void)hipStreamSynchronize(st);
                seen.push_back(st);
            }
    }
    for (int i = 0; i < n; ++i) destroy_impl(ms[i], false);
}

extern "C" {

int sdmm_create_many_on_stream(int K, const sdmm_em_params* params, int device, void* hip_stream, int n,
                               sdmm_mix** out) {
    return create_many(K, params, device, (hipStream_t)hip_stream, n, out);
}

}  // extern "C"

namespace {

// dst[i]'s mixture (the block prefix before the stats: parameters, derived
// arrays, packed records, stepwise state) = src[i]'s, one kernel on `st`
// after the sources' pending work
int copy_prefix_many(const sdmm_mix* const* src, sdmm_mix* const* dst, int n, hipStream_t st) {
    for (int i = 0; i < n; ++i)
        if (src[i]->stream != st) HIP_TRY(hipStreamSynchronize(src[i]->stream));
    const size_t bytes = (size_t)((char*)src[0]->stats - (char*)src[0]->C.weights);   // 16-aligned pieces
    // the pointer table: built in the thread's pinned bounce buffer, uploaded
    // into the (device, stream) scratch entry held until the sync below (host
    // transfer rules at the top of this file)
    const size_t tb = sizeof(void*) * 2 * (size_t)n;
    char* pin = nullptr;
    HIP_TRY(bounce_buf(tb, &pin));
    void** ptrs = (void**)pin;
    for (int i = 0; i < n; ++i) {
        dst[i]->params = src[i]->params;
        dst[i]->guide_cap = src[i]->guide_cap;
        dst[i]->guide_order = src[i]->guide_order;
        dst[i]->initialised = src[i]->initialised;
        ptrs[(size_t)i] = src[i]->C.weights;
        ptrs[(size_t)n + i] = dst[i]->C.weights;
    }
    StreamScratch* ss = nullptr;
    std::unique_lock<std::mutex> hold = stream_scratch(src[0]->device, st, &ss);
    hipError_t e = scratch_reserve(*ss, tb);
    void* dtab = ss->p;
    if (e == hipSuccess) e = hipMemcpyAsync(dtab, ptrs, tb, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = launch_copy_many(n, dtab, (void**)dtab + n, bytes, st);
    {   // always: the bounce buffer and the table go to the next user
        const hipError_t es = hipStreamSynchronize(st);
        if (e == hipSuccess) e = es;
    }
    if (e != hipSuccess) return fail(SDMM_E_HIP, std::string("mixture copy: ") + hipGetErrorString(e));
    return SDMM_OK;
}

int check_same_kind(const sdmm_mix* const* a, int n) {
    for (int i = 0; i < n; ++i) {
        if (!a[i]) return fail(SDMM_E_INVALID, "NULL handle");
        if (a[i]->K != a[0]->K || a[i]->device != a[0]->device)
            return fail(SDMM_E_INVALID, "handles must share K and device");
    }
    return SDMM_OK;
}

}  // namespace

extern "C" {

int sdmm_clone_many_on_stream(const sdmm_mix* const* src, int n, void* hip_stream, sdmm_mix** out) {
    if (n < 0 || (n > 0 && (!src || !out))) return fail(SDMM_E_INVALID, "invalid argument");
    if (n == 0) return SDMM_OK;
    int r = check_same_kind(src, n);
    if (r) return r;
    HIP_TRY(hipSetDevice(src[0]->device));
    const hipStream_t st = (hipStream_t)hip_stream;
    r = create_many(src[0]->K, &src[0]->params, src[0]->device, st, n, out);
    if (r) return r;
    r = copy_prefix_many(src, out, n, st);
    if (r)
        for (int j = 0; j < n; ++j) { sdmm_destroy(out[j]); out[j] = nullptr; }
    return r;
}

int sdmm_clone_many(const sdmm_mix* const* src, int n, sdmm_mix** out) {
    if (n < 0 || (n > 0 && (!src || !out))) return fail(SDMM_E_INVALID, "invalid argument");
    if (n == 0) return SDMM_OK;
    if (!src[0]) return fail(SDMM_E_INVALID, "NULL handle in src");
    return sdmm_clone_many_on_stream(src, n, (void*)src[0]->stream, out);
}

int sdmm_copy_many(const sdmm_mix* const* src, sdmm_mix* const* dst, int n) {
    if (n < 0 || (n > 0 && (!src || !dst))) return fail(SDMM_E_INVALID, "invalid argument");
    if (n == 0) return SDMM_OK;
    int r = check_same_kind(src, n);
    if (!r) r = check_same_kind(dst, n);
    if (r) return r;
    if (src[0]->K != dst[0]->K || src[0]->device != dst[0]->device)
        return fail(SDMM_E_INVALID, "sources and destinations must share K and device");
    HIP_TRY(hipSetDevice(dst[0]->device));
    const hipStream_t st = dst[0]->stream;
    for (int i = 1; i < n; ++i)
        if (dst[i]->stream != st) HIP_TRY(hipStreamSynchronize(dst[i]->stream));
    return copy_prefix_many(src, dst, n, st);
}

int sdmm_num_components(const sdmm_mix* m) { return m ? m->K : 0; }

int sdmm_set_guide_order(sdmm_mix* m, int coherent) {
    if (!m) return fail(SDMM_E_INVALID, "null handle");
    m->guide_order = coherent ? 1 : 0;
    return SDMM_OK;
}

int sdmm_set_guide_capacity(sdmm_mix* m, int cap) {
    if (!m) return fail(SDMM_E_INVALID, "null handle");
    if (cap < 0 || cap > kGuideCapMax) return fail(SDMM_E_INVALID, "guide capacity must be in [0, 64]");
    m->guide_cap = cap;
    return SDMM_OK;
}

int sdmm_guide_fallback_count(const sdmm_mix* m, int* count) {
    if (!m || !count) return fail(SDMM_E_INVALID, "invalid argument");
    *count = 0;
    if (!m->guide_fb) return SDMM_OK;
    HIP_TRY(hipSetDevice(m->device));
    HIP_TRY(hipMemcpyAsync(count, m->guide_fb, sizeof(int), hipMemcpyDeviceToHost, m->stream));
    HIP_TRY(hipStreamSynchronize(m->stream));
    return SDMM_OK;
}

int sdmm_layout(const sdmm_mix* m, int* resp_cpl, int* resp_lps, int* stats_cpl, int* stats_lps) {
    if (!m) return fail(SDMM_E_INVALID, "null handle");
    if (resp_cpl) *resp_cpl = m->rcpl;
    if (resp_lps) *resp_lps = m->rlps;
    if (stats_cpl) *stats_cpl = m->cpl;
    if (stats_lps) *stats_lps = m->lps;
    return SDMM_OK;
}

const char* sdmm_kernel_name(const sdmm_mix* m, int which) {
    if (!m) return "";
    static thread_local char buf[64];
    if (which == 0) {
        if (m->rtile == 3) {
            std::snprintf(buf, sizeof buf, "%s", estep_resp_split_name(m->rvariant, m->Kp));
            return buf;
        } else if (m->rtile == 2) {
            std::snprintf(buf, sizeof buf, "%s", estep_resp_mfma_name(m->rvariant, m->Kp));
            return buf;
        } else if (m->rtile) {
            std::snprintf(buf, sizeof buf, "%s", estep_resp_tile_name(m->rvariant));
            return buf;
        }
        std::snprintf(buf, sizeof buf, "estep_resp_kernel<%d,%d>", m->rcpl, m->rlps);
        return buf;
    }
    if (m->stile == 2)
        std::snprintf(buf, sizeof buf, "estep_stats_tile_kernel<%d,2,true>", m->Kp / 128);
    else if (m->stile)
        std::snprintf(buf, sizeof buf, "estep_stats_tile_kernel<4,%d>", m->svariant == 1 ? 3 : 2);
    else
        std::snprintf(buf, sizeof buf, "estep_stats_kernel<%d,%d>", m->cpl, m->lps);
    return buf;
}

int sdmm_set_stream(sdmm_mix* m, void* hip_stream) {
    if (!m) return fail(SDMM_E_INVALID, "handle is NULL");
    HIP_TRY(hipSetDevice(m->device));
    // the handle's scratch (partial rows, staging, guide lists) may still be in
    // use by work on the old stream
    if ((hipStream_t)hip_stream != m->stream) HIP_TRY(hipStreamSynchronize(m->stream));
    m->stream = (hipStream_t)hip_stream;  // taken literally: NULL is the HIP null stream
    return SDMM_OK;
}

void* sdmm_get_stream(const sdmm_mix* m) { return m ? (void*)m->stream : nullptr; }

int sdmm_synchronize(sdmm_mix* m) {
    if (!m) return fail(SDMM_E_INVALID, "handle is NULL");
    HIP_TRY(hipSetDevice(m->device));
    HIP_TRY(hipStreamSynchronize(m->stream));
    return SDMM_OK;
}

int sdmm_hemisphere_init_host(const float* positions, const float* normals, int n_pos, float depth_prior,
                              float min_spatial_distance, uint64_t seed, float* weights, float* means,
                              float* covs, float* bpriors, float* bdepth) {
    if (!positions || !normals || n_pos <= 0 || !weights || !means || !covs || !bpriors || !bdepth)
        return fail(SDMM_E_INVALID, "invalid argument to sdmm_hemisphere_init_host");
    hemisphere_init(positions, normals, n_pos, depth_prior, min_spatial_distance, seed, weights, means,
                    covs, bpriors, bdepth);
    return SDMM_OK;
}

static int upload_and_set(sdmm_mix* m, const float* weights, const float* means, const float* covs) {
    const size_t K = (size_t)m->K;
    // fp64-widened means and covariances, then the weights, in the thread's
    // pinned bounce buffer (no pageable DMA)
    char* pin = nullptr;
    HIP_TRY(bounce_buf(8 * 31 * K + 4 * K, &pin));
    double* md = (double*)pin;
    double* cd = md + 6 * K;
    for (size_t i = 0; i < 6 * K; ++i) md[i] = (double)means[i];
    for (size_t i = 0; i < 25 * K; ++i) cd[i] = (double)covs[i];
    std::memcpy(cd + 25 * K, weights, 4 * K);
    HIP_TRY(hipMemcpyAsync(m->tmp_mean, md, 8 * 6 * K, hipMemcpyHostToDevice, m->stream));
    HIP_TRY(hipMemcpyAsync(m->tmp_cov, cd, 8 * 25 * K, hipMemcpyHostToDevice, m->stream));
    HIP_TRY(hipMemcpyAsync(m->C.weights, cd + 25 * K, 4 * K, hipMemcpyHostToDevice, m->stream));
    HIP_TRY(launch_set_all(m->K, m->Kp, m->tmp_mean, m->tmp_cov, m->C, m->ep, m->gp, m->norm5, m->stream));
    HIP_TRY(hipStreamSynchronize(m->stream));  // the bounce buffer is reused by the thread's next call
    m->initialised = true;
    return SDMM_OK;
}

static int init_hemisphere_batched_impl(sdmm_mix* const* mixes, int n, const float* positions,
                                        const float* normals, float depth_prior, const float* min_spatial_distance,
                                        const uint64_t* seeds, int skip);

int sdmm_init_hemisphere(sdmm_mix* m, const float* positions, const float* normals, int n_pos,
                         float depth_prior, float min_spatial_distance, uint64_t seed) {
    if (!m) return fail(SDMM_E_INVALID, "handle is NULL");
    HIP_TRY(hipSetDevice(m->device));
    if (n_pos * 8 != m->K) return fail(SDMM_E_INVALID, "K must equal 8 * n_pos");
    if (!positions || !normals) return fail(SDMM_E_INVALID, "invalid argument to sdmm_init_hemisphere");
    // the batched path with one mixture: the same device generator
    return init_hemisphere_batched_impl(&m, 1, positions, normals, depth_prior, &min_spatial_distance, &seed, 0);
}


int sdmm_init_hemisphere_batched(sdmm_mix* const* mixes, int n, const float* positions, const float* normals,
                                 float depth_prior, const float* min_spatial_distance, const uint64_t* seeds) {
    return init_hemisphere_batched_impl(mixes, n, positions, normals, depth_prior, min_spatial_distance, seeds, 0);
}

int sdmm_init_hemisphere_kmeanspp_batched(sdmm_mix* const* mixes, int n, const sdmm_samples* s,
                                          const float* const normals[3], const int64_t* seg, float depth_prior,
                                          const float* min_spatial_distance, const uint64_t* seeds) {
    if (n < 0 || (n > 0 && (!mixes || !s || !normals || !seg || !min_spatial_distance || !seeds)))
        return fail(SDMM_E_INVALID, "invalid argument");
    if (n == 0) return SDMM_OK;
    if (!mixes[0]) return fail(SDMM_E_INVALID, "NULL handle in mixes");
    const int K = mixes[0]->K;
    if (K % 8) return fail(SDMM_E_INVALID, "K must be a multiple of 8");
    const int npos = K / 8;
    // one PCG32 stream per mixture: npos draws for the k-means++ choice, then
    // the direction jitter (uniformHemisphereInit's rng, :130-138, :199-232)
    std::vector<float> u((size_t)n * npos);
    for (int i = 0; i < n; ++i) {
        Pcg32 rng;
        rng.seed(seeds[i], 0xda3e39cb94b95bdbULL);
        for (int j = 0; j < npos; ++j) u[(size_t)i * npos + j] = rng.next_float();
    }
    std::vector<int64_t> idx((size_t)n * npos);
    std::vector<float> pos((size_t)n * npos * 3), nrm((size_t)n * npos * 3);
    int r = sdmm_kmeanspp_select(s, normals, seg, n, npos, u.data(), mixes[0]->device, (void*)mixes[0]->stream,
                                 idx.data(), pos.data(), nrm.data());
    if (r) return r;
    return init_hemisphere_batched_impl(mixes, n, pos.data(), nrm.data(), depth_prior, min_spatial_distance, seeds,
                                        npos);
}

static int init_hemisphere_batched_impl(sdmm_mix* const* mixes, int n, const float* positions,
                                        const float* normals, float depth_prior, const float* min_spatial_distance,
                                        const uint64_t* seeds, int skip) {
    if (n < 0 || (n > 0 && (!mixes || !positions || !normals || !min_spatial_distance || !seeds)))
        return fail(SDMM_E_INVALID, "invalid argument");
    if (n == 0) return SDMM_OK;
    const int K = mixes[0]->K;
    for (int i = 0; i < n; ++i) {
        if (!mixes[i] || mixes[i]->K != K) return fail(SDMM_E_INVALID, "mixtures must share K");
        if (mixes[i]->device != mixes[0]->device) return fail(SDMM_E_INVALID, "mixtures on different devices");
    }
    if (K % 8) return fail(SDMM_E_INVALID, "K must be a multiple of 8");
    const int npos = K / 8;
    HIP_TRY(hipSetDevice(mixes[0]->device));
    const hipStream_t st = mixes[0]->stream;
    for (int i = 1; i < n; ++i)
        if (mixes[i]->stream != st) HIP_TRY(hipStreamSynchronize(mixes[i]->stream));
    // per mixture: weights K, means 6K, covs 25K, bPriors 25K, bDepth 9K, all
    // f32 (the initial means and covariances are float values: the kernel
    // widens them to the fp64 MVTN::set takes)
    const size_t Kz = (size_t)K;
    const size_t per = 4 * Kz + 4 * 6 * Kz + 4 * 25 * Kz + 4 * 25 * Kz + 4 * 9 * Kz;
    // pinned staging: the calling thread's bounce buffer; the device block of
    // the call: the (device, stream) scratch pool entry, held until the
    // stream sync below (host transfer rules at the top of this file)
    StreamScratch* ss = nullptr;
    std::unique_lock<std::mutex> hold = stream_scratch(mixes[0]->device, st, &ss);
    // the staging block is generated on the device (hemi_gen_batched_kernel):
    // only the inputs and the pointer table travel.  SDMM_HEMI_HOST=1 runs the
    // host generator into pinned memory and uploads the whole block instead.
    static const bool host_gen = [] {
        const char* e = std::getenv("SDMM_HEMI_HOST");
        return e && std::atoi(e) != 0;
    }();
    const size_t stage_bytes = (per * (size_t)n + 255) / 256 * 256;
    const size_t tab_bytes = (sizeof(InitDescHost) * (size_t)n + 255) / 256 * 256;
    const size_t pn_bytes = sizeof(float) * 3 * (size_t)npos * (size_t)n;   // positions, then normals
    const size_t in_bytes = host_gen ? 0 : 2 * pn_bytes + sizeof(float) * (size_t)n + sizeof(uint64_t) * (size_t)n + 16;
    const size_t up_off = host_gen ? 0 : stage_bytes;   // device offset of what is uploaded
    const size_t want = (host_gen ? stage_bytes : 0) + tab_bytes + in_bytes;
    char* pin = nullptr;   // pinned image of device bytes [up_off, stage_bytes + tab_bytes + in_bytes)
    HIP_TRY(bounce_buf(want, &pin));
    int r = SDMM_OK;
    if (host_gen) {
        // the host fp64 initialisations, in parallel over the mixtures (each is
        // independent and writes its own staging slice: bitwise as sequential)
        auto init_range = [&](int i0, int i1) {
            for (int i = i0; i < i1; ++i) {
                char* b = pin + per * (size_t)i;
                float* pw = (float*)b;
                float* pm = (float*)(b + 4 * Kz);
                float* pc = (float*)(b + 28 * Kz);
                float* pb = (float*)(b + 128 * Kz);
                float* pd = (float*)(b + 228 * Kz);
                hemisphere_init(positions + 3 * (size_t)npos * i, normals + 3 * (size_t)npos * i, npos, depth_prior,
                                min_spatial_distance[i], seeds[i], pw, pm, pc, pb, pd, skip);
            }
        };
        const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
        const int nt = std::max(1, std::min({16, hw, n / 64}));
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) {
            const int a = (int)((int64_t)n * t / nt), b = (int)((int64_t)n * (t + 1) / nt);
            // a thread that cannot be started (std::system_error must not leave
            // this extern "C" call): its range runs here instead
            try {
                th.emplace_back(init_range, a, b);
            } catch (...) {
                init_range(a, b);
            }
        }
        init_range(0, (int)((int64_t)n / nt));
        for (auto& x : th) x.join();
    }
    InitDescHost* tab = (InitDescHost*)(pin + stage_bytes - up_off);
    for (int i = 0; i < n; ++i) {
        sdmm_mix* m = mixes[i];
        tab[i] = InitDescHost{m->C, m->ep, m->gp, m->S.bPriors, m->S.bDepth, m->tmp_mean, m->tmp_cov};
    }
    const size_t in_off = stage_bytes + tab_bytes;   // device offsets of the inputs
    const size_t dist_off = in_off + 2 * pn_bytes;
    const size_t seed_off = (dist_off + sizeof(float) * (size_t)n + 7) / 8 * 8;
    if (!host_gen) {
        std::memcpy(pin + in_off - up_off, positions, pn_bytes);
        std::memcpy(pin + in_off - up_off + pn_bytes, normals, pn_bytes);
        std::memcpy(pin + dist_off - up_off, min_spatial_distance, sizeof(float) * (size_t)n);
        std::memcpy(pin + seed_off - up_off, seeds, sizeof(uint64_t) * (size_t)n);
    }
    // one upload, then (device generation) one kernel filling the staging
    // block and one kernel (a workgroup per mixture: copy in, MVTN::set, CDF,
    // pack)
    const size_t total = stage_bytes + tab_bytes + in_bytes;
    hipError_t e0 = r ? hipSuccess : scratch_reserve(*ss, total);
    char* d = ss->p;
    if (!r && e0 == hipSuccess) e0 = hipMemcpyAsync(d + up_off, pin, total - up_off, hipMemcpyHostToDevice, st);
    if (!r && e0 == hipSuccess && !host_gen)
        e0 = launch_hemi_gen_batched(n, K, (const float*)(d + in_off), (const float*)(d + in_off + pn_bytes),
                                     (const float*)(d + dist_off), (const uint64_t*)(d + seed_off), skip, depth_prior,
                                     d, per, st);
    if (!r && e0 == hipSuccess)
        e0 = launch_set_all_batched(n, K, mixes[0]->Kp, d + stage_bytes, d, per, mixes[0]->norm5, st);
    if (!r && e0 != hipSuccess) r = fail(SDMM_E_HIP, std::string("init_hemisphere_batched: ") + hipGetErrorString(e0));
    const hipError_t e = hipStreamSynchronize(st);   // the pinned staging is reused by the next call
    if (r) return r;
    if (e != hipSuccess) return fail(SDMM_E_HIP, std::string("init_hemisphere_batched: ") + hipGetErrorString(e));
    for (int i = 0; i < n; ++i) mixes[i]->initialised = true;
    return SDMM_OK;
}

int sdmm_iterations_run(const sdmm_mix* const* mixes, int n, int* out) {
    if (n < 0 || (n > 0 && (!mixes || !out))) return fail(SDMM_E_INVALID, "invalid argument");
    if (n == 0) return SDMM_OK;
    for (int i = 0; i < n; ++i)
        if (!mixes[i]) return fail(SDMM_E_INVALID, "NULL handle in mixes");
    const sdmm_mix* m0 = mixes[0];
    HIP_TRY(hipSetDevice(m0->device));
    // every mixture's pending work first (its own stream), then ONE gather of
    // the n counters and one copy back on mixes[0]'s stream (a copy per leaf
    // cost ~3 us of launch each: ~10 ms per training pass of a few thousand
    // leaves).  The scratch is mixes[0]'s own, device + pinned, allocated
    // once and reused: no stream-ordered allocation and no pageable copy in
    // the call.  (Round 2's version took hipMallocAsync / hipFreeAsync from the
    // device's default pool and pageable hipMemcpyAsync both ways; called from
    // the plugin's per-leaf worker threads at once it hung -- the one place
    // where pool allocations on many streams (release threshold 0: the pool
    // trims at each synchronisation) met other threads' hipMalloc / hipFree
    // (device-wide synchronisations) and staged pageable copies.  Calls on one
    // handle are serialised by the caller (the ABI's rule), so mixes[0]'s
    // scratch needs no lock.)
    std::vector<hipStream_t> seen;
    for (int i = 0; i < n; ++i)
        if (std::find(seen.begin(), seen.end(), mixes[i]->stream) == seen.end()) {
            seen.push_back(mixes[i]->stream);
            HIP_TRY(hipStreamSynchronize(mixes[i]->stream));
        }
    const hipStream_t st = m0->stream;
    const size_t tab_bytes = ((sizeof(void*) * (size_t)n + 255) / 256) * 256;
    const size_t need = tab_bytes + sizeof(double) * (size_t)n;
    if (need > m0->it_cap) {
        // pointers cleared before any error can return (destroy must not free
        // them twice); free errors are ignored as in destroy
        void* od = m0->it_dev;
        void* oh = m0->it_host;
        m0->it_dev = m0->it_host = nullptr;
        m0->it_cap = 0;
        if (od) (void)hipFree(od);
        if (oh) (void)hipHostFree(oh);
        const size_t cap = std::max<size_t>(need, 4096);
        HIP_TRY(hipMalloc(&m0->it_dev, cap));
        HIP_TRY(hipHostMalloc(&m0->it_host, cap, hipHostMallocDefault));
        m0->it_cap = cap;
    }
    const double** src = (const double**)m0->it_host;
    for (int i = 0; i < n; ++i) src[i] = mixes[i]->S.scalars + SC_IT;
    char* db = (char*)m0->it_dev;
    double* vals = (double*)((char*)m0->it_host + tab_bytes);
    HIP_TRY(hipMemcpyAsync(db, src, sizeof(void*) * (size_t)n, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_gather_f64(db, n, (double*)(db + tab_bytes), st));
    HIP_TRY(hipMemcpyAsync(vals, db + tab_bytes, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (int i = 0; i < n; ++i) out[i] = (int)vals[i];
    return SDMM_OK;
}

int sdmm_set_params(sdmm_mix* m, const float* weights, const float* means, const float* covs) {
    if (!m || !weights || !means || !covs) return fail(SDMM_E_INVALID, "invalid argument");
    HIP_TRY(hipSetDevice(m->device));
    return upload_and_set(m, weights, means, covs);
}

int sdmm_estep_stats(sdmm_mix* m, const sdmm_samples* s, double* stats) {
    if (!m || !stats) return fail(SDMM_E_INVALID, "invalid argument");
    if (!m->initialised) return fail(SDMM_E_STATE, "mixture not initialised");
    HIP_TRY(hipSetDevice(m->device));
    int r = check_samples(s);
    if (r) return r;
    if (s->n == 0) {
        HIP_TRY(hipMemsetAsync(stats, 0, 8 * sdmm_stats_len(m->K), m->stream));
        return SDMM_OK;
    }
    return run_estep_stats(m, s, stats);
}

int sdmm_mstep(sdmm_mix* m, const double* stats, int64_t n_total) {
    if (!m || !stats) return fail(SDMM_E_INVALID, "invalid argument");
    if (!m->initialised) return fail(SDMM_E_STATE, "mixture not initialised");
    HIP_TRY(hipSetDevice(m->device));
    HIP_TRY(launch_mstep(m->K, m->Kp, stats, n_total, m->C, m->S, m->ep, m->gp, m->norm5, m->tmp_mean,
                         m->mcount, m->stream));
    return SDMM_OK;
}

// ---- multi-GPU -------------------------------------------------------------
int sdmm_comm_unique_id(void* id) {
    if (!id) return fail(SDMM_E_INVALID, "id is NULL");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof(u));
    return SDMM_OK;
}

int sdmm_comm_init_rccl(const void* id, int nranks, int rank, int device, sdmm_comm** out) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(SDMM_E_INVALID, "invalid argument");
    *out = nullptr;
    HIP_TRY(hipSetDevice(device));
    sdmm_comm* c = new (std::nothrow) sdmm_comm();
    if (!c) return fail(SDMM_E_NOMEM, "out of host memory");
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    const ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return nccl_fail(r, "ncclCommInitRank");
    }
    *out = c;
    return SDMM_OK;
}

int sdmm_comm_init_host(int nranks, int rank, int device, sdmm_host_allreduce_f64 allreduce,
                        sdmm_host_broadcast broadcast, void* user, sdmm_comm** out) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && (!allreduce || !broadcast)))
        return fail(SDMM_E_INVALID, "invalid argument");
    sdmm_comm* c = new (std::nothrow) sdmm_comm();
    if (!c) return fail(SDMM_E_NOMEM, "out of host memory");
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    c->h_allreduce = allreduce;
    c->h_broadcast = broadcast;
    c->user = user;
    *out = c;
    return SDMM_OK;
}

void sdmm_comm_destroy(sdmm_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    if (c->pinned) (void)hipHostFree(c->pinned);
    delete c;
}

int sdmm_comm_rank(const sdmm_comm* c) { return c ? c->rank : -1; }
int sdmm_comm_size(const sdmm_comm* c) { return c ? c->nranks : 0; }

int sdmm_comm_allreduce_f64(sdmm_comm* c, double* buf, size_t count, void* hip_stream) {
    if (!c || (count > 0 && !buf)) return fail(SDMM_E_INVALID, "invalid argument");
    if (count == 0) return SDMM_OK;
    HIP_TRY(hipSetDevice(c->device));
    return comm_allreduce(c, buf, count, (hipStream_t)hip_stream);
}

int sdmm_em_step_sharded(sdmm_mix* m, sdmm_comm* c, const sdmm_samples* shard, int iterations) {
    if (!m || !c) return fail(SDMM_E_INVALID, "invalid argument");
    if (!m->initialised) return fail(SDMM_E_STATE, "mixture not initialised");
    if (c->device != m->device) return fail(SDMM_E_INVALID, "communicator on another device");
    int r = check_samples(shard);
    if (r) return r;
    HIP_TRY(hipSetDevice(m->device));
    const size_t len = sdmm_stats_len(m->K);
    for (int it = 0; it < iterations; ++it) {
        // this shard's statistics (zero for an empty shard) and its sample count
        if (shard->n == 0) {
            HIP_TRY(hipMemsetAsync(m->stats, 0, 8 * len, m->stream));
        } else if ((r = run_estep_stats(m, shard, m->stats))) {
            return r;
        }
        HIP_TRY(launch_set_f64(m->stats + len, (double)shard->n, m->stream));
        // SUM over ranks, then the same M-step everywhere (n from the summed count)
        if ((r = comm_allreduce(c, m->stats, len + 1, m->stream))) return r;
        HIP_TRY(launch_mstep(m->K, m->Kp, m->stats, -1, m->C, m->S, m->ep, m->gp, m->norm5, m->tmp_mean,
                             m->mcount, m->stream));
    }
    return SDMM_OK;
}

int sdmm_mix_broadcast(sdmm_mix* const* mixes, int n_mix, const int32_t* owner, sdmm_comm* c) {
    if (n_mix < 0 || !c || (n_mix > 0 && (!mixes || !owner))) return fail(SDMM_E_INVALID, "invalid argument");
    if (n_mix == 0) return SDMM_OK;
    for (int i = 0; i < n_mix; ++i) {
        if (!mixes[i]) return fail(SDMM_E_INVALID, "NULL handle in mixes");
        if (owner[i] < 0 || owner[i] >= c->nranks) return fail(SDMM_E_INVALID, "owner rank out of range");
        if (mixes[i]->device != c->device) return fail(SDMM_E_INVALID, "mixture on another device");
        if (mixes[i]->K != mixes[0]->K) return fail(SDMM_E_INVALID, "mixtures must share K");
    }
    HIP_TRY(hipSetDevice(c->device));
    const hipStream_t st = mixes[0]->stream;
    for (int i = 1; i < n_mix; ++i)
        if (mixes[i]->stream != st) HIP_TRY(hipStreamSynchronize(mixes[i]->stream));
    // a mixture's parameters, derived arrays, packed records and stepwise state
    // are one contiguous prefix of its device block (everything before the stats)
    const size_t bytes = (size_t)((char*)mixes[0]->stats - (char*)mixes[0]->C.weights);
    if (c->nccl) {
        ncclResult_t g = ncclGroupStart();
        if (g != ncclSuccess) return nccl_fail(g, "ncclGroupStart");
        for (int i = 0; i < n_mix; ++i) {
            const int r = comm_broadcast(c, mixes[i]->C.weights, bytes, owner[i], st);
            if (r) { (void)ncclGroupEnd(); return r; }
        }
        g = ncclGroupEnd();
        if (g != ncclSuccess) return nccl_fail(g, "ncclGroupEnd");
    } else {
        for (int i = 0; i < n_mix; ++i) {
            const int r = comm_broadcast(c, mixes[i]->C.weights, bytes, owner[i], st);
            if (r) return r;
        }
    }
    for (int i = 0; i < n_mix; ++i) mixes[i]->initialised = true;
    HIP_TRY(hipStreamSynchronize(st));
    return SDMM_OK;
}

int sdmm_clone(const sdmm_mix* src, sdmm_mix** out) {
    if (!src || !out) return fail(SDMM_E_INVALID, "invalid argument");
    *out = nullptr;
    sdmm_mix* m = nullptr;
    // stream-ordered on the source's stream: after its pending work
    int r = sdmm_create_on_stream(src->K, &src->params, src->device, (void*)src->stream, &m);
    if (r) return r;
    m->guide_cap = src->guide_cap;
    m->guide_order = src->guide_order;
    // parameters, derived arrays, packed records and stepwise state: the block
    // prefix before the stats (as sdmm_mix_broadcast)
    const size_t bytes = (size_t)((char*)src->stats - (char*)src->C.weights);
    hipError_t e = hipSetDevice(src->device);
    if (e == hipSuccess) e = hipMemcpyAsync(m->C.weights, src->C.weights, bytes, hipMemcpyDeviceToDevice, m->stream);
    if (e != hipSuccess) {
        sdmm_destroy(m);
        return fail(SDMM_E_HIP, std::string("sdmm_clone: ") + hipGetErrorString(e));
    }
    m->initialised = src->initialised;
    *out = m;
    return SDMM_OK;
}

int sdmm_em_step(sdmm_mix* m, const sdmm_samples* s, int iterations) {
    if (!m) return fail(SDMM_E_INVALID, "handle is NULL");
    if (!m->initialised) return fail(SDMM_E_STATE, "mixture not initialised");
    HIP_TRY(hipSetDevice(m->device));
    int r = check_samples(s);
    if (r) return r;
    if (s->n == 0) return SDMM_OK;  // weightSum == 0: optimize() returns early
    for (int it = 0; it < iterations; ++it) {
        r = run_estep_stats(m, s, m->stats);
        if (r) return r;
        HIP_TRY(launch_mstep(m->K, m->Kp, m->stats, s->n, m->C, m->S, m->ep, m->gp, m->norm5, m->tmp_mean,
                             m->mcount, m->stream));
    }
    return SDMM_OK;
}

}  // extern "C"

namespace {

// Validation shared by the batched entry points: handles present, initialised,
// distinct, one K and one device; offsets/counts inside the batch.
int check_batch(sdmm_mix* const* mixes, int n_mix, const sdmm_samples* s, const int64_t* s0, const int64_t* cnt) {
    std::vector<const sdmm_mix*> seen;
    seen.reserve((size_t)n_mix);
    const sdmm_mix* m0 = mixes[0];
    for (int i = 0; i < n_mix; ++i) {
        const sdmm_mix* m = mixes[i];
        if (!m) return fail(SDMM_E_INVALID, "NULL handle in mixes");
        if (!m->initialised) return fail(SDMM_E_STATE, "mixture not initialised");
        if (m->K != m0->K || m->device != m0->device)
            return fail(SDMM_E_INVALID, "batched mixtures must share K and the device");
        if (cnt[i] < 0 || s0[i] < 0 || s0[i] + cnt[i] > s->n)
            return fail(SDMM_E_INVALID, "segment offsets outside the sample batch");
        seen.push_back(m);
    }
    std::sort(seen.begin(), seen.end());
    if (std::adjacent_find(seen.begin(), seen.end()) != seen.end())
        return fail(SDMM_E_INVALID, "a handle appears twice in mixes");
    return SDMM_OK;
}

// ONE stepwise EM iteration of every listed leaf: mixes[i] over samples
// [s0[i], s0[i] + cnt[i]) of the device planes s, on mixes[0]'s stream.
// comm == nullptr: a leaf with no samples is left unchanged.  comm != null
// (sample-sharded over ranks): each rank's statistics of every leaf -- and the
// leaves' sample counts -- go to one contiguous fp64 buffer, ONE all-reduce
// sums them, and every rank runs the same M-steps on the global statistics.
int batched_iteration(sdmm_mix* const* mixes, int n_mix, const sdmm_samples* s, const int64_t* s0,
                      const int64_t* cnt, sdmm_comm* comm);

}  // namespace

extern "C" {

int sdmm_em_step_batched(sdmm_mix* const* mixes, int n_mix, const sdmm_samples* s, const int64_t* seg,
                         int iterations) {
    if (n_mix < 0 || (n_mix > 0 && (!mixes || !seg))) return fail(SDMM_E_INVALID, "invalid argument");
    if (n_mix == 0) return SDMM_OK;
    std::vector<int> it((size_t)n_mix, iterations > 0 ? iterations : 0);
    return sdmm_em_step_batched_iters(mixes, n_mix, s, seg, it.data());
}

int sdmm_em_step_batched_iters(sdmm_mix* const* mixes, int n_mix, const sdmm_samples* s, const int64_t* seg,
                               const int* iterations) {
    return sdmm_em_step_batched_sharded(mixes, n_mix, nullptr, s, seg, iterations);
}

int sdmm_em_step_batched_sharded(sdmm_mix* const* mixes, int n_mix, sdmm_comm* comm, const sdmm_samples* s,
                                 const int64_t* seg, const int* iterations) {
    if (n_mix < 0 || (n_mix > 0 && (!mixes || !seg || !iterations))) return fail(SDMM_E_INVALID, "invalid argument");
    if (n_mix == 0) return SDMM_OK;
    int r = check_samples(s);
    if (r) return r;
    if (!mixes[0]) return fail(SDMM_E_INVALID, "mixes[0] is NULL");
    for (int i = 0; i < n_mix; ++i)
        if (seg[i + 1] < seg[i]) return fail(SDMM_E_INVALID, "segment offsets must be non-decreasing");
    std::vector<int64_t> s0((size_t)n_mix), cnt((size_t)n_mix);
    int max_it = 0;
    for (int i = 0; i < n_mix; ++i) {
        s0[(size_t)i] = seg[i];
        cnt[(size_t)i] = seg[i + 1] - seg[i];
        max_it = std::max(max_it, iterations[i]);
    }
    if ((r = check_batch(mixes, n_mix, s, s0.data(), cnt.data()))) return r;
    if (comm && comm->device != mixes[0]->device) return fail(SDMM_E_INVALID, "communicator on another device");
    // iteration t steps the leaves that asked for more than t iterations (the
    // plugin: 2 while a leaf's em.iterations_run < 4, else 1, volpath_sdmm.cpp:299-305)
    std::vector<sdmm_mix*> am;
    std::vector<int64_t> as0, acnt;
    for (int t = 0; t < max_it; ++t) {
        am.clear(); as0.clear(); acnt.clear();
        for (int i = 0; i < n_mix; ++i)
            if (iterations[i] > t) {
                am.push_back(mixes[i]);
                as0.push_back(s0[(size_t)i]);
                acnt.push_back(cnt[(size_t)i]);
            }
        if (am.empty()) break;
        // leaves stepped in this round run on the first one's stream: make the
        // caller's mixes[0] stream the one, so the ordering is the caller's
        if (am[0] != mixes[0]) {
            am.insert(am.begin(), mixes[0]);
            as0.insert(as0.begin(), 0);
            acnt.insert(acnt.begin(), -1);   // placeholder: not stepped (see below)
        }
        r = batched_iteration(am.data(), (int)am.size(), s, as0.data(), acnt.data(), comm);
        if (r) return r;
    }
    return SDMM_OK;
}

}  // extern "C"

namespace {

int batched_iteration(sdmm_mix* const* mixes, int n_mix, const sdmm_samples* s, const int64_t* s0,
                      const int64_t* cnt, sdmm_comm* comm) {
    sdmm_mix* m0 = mixes[0];
    HIP_TRY(hipSetDevice(m0->device));
    const hipStream_t st = m0->stream;
    for (int i = 1; i < n_mix; ++i)
        if (mixes[i]->stream != st) HIP_TRY(hipStreamSynchronize(mixes[i]->stream));
    // a leaf with cnt < 0 only carries mixes[0]'s stream: no work, no M-step
    std::vector<StatsPlan> plans((size_t)n_mix);
    int64_t rows = 0, any = 0;
    for (int i = 0; i < n_mix; ++i) {
        const int64_t n = cnt[i];
        plans[(size_t)i] = n > 0 ? stats_plan(mixes[i], n) : StatsPlan{0, 0};
        rows += plans[(size_t)i].blocks;
        any += n > 0 ? n : 0;
    }
    if (!comm && any == 0) return SDMM_OK;   // nothing to step
    if (rows > (int64_t)1 << 30) return fail(SDMM_E_INVALID, "batch too large");
    const size_t len = sdmm_stats_len(m0->K);
    const size_t off_mix = ((sizeof(LeafDesc) * (size_t)n_mix + 255) / 256) * 256;
    const size_t off_items = off_mix + ((sizeof(MixDesc) * (size_t)n_mix + 255) / 256) * 256;
    const size_t off_cnt = off_items + ((sizeof(int2) * (size_t)rows + 255) / 256) * 256;
    const size_t need = off_cnt + sizeof(double) * (size_t)n_mix;
    if (!m0->batch_copied) {
        HIP_TRY(hipEventCreateWithFlags(&m0->batch_copied, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&m0->batch_done, hipEventDisableTiming));
    }
    HIP_TRY(hipEventSynchronize(m0->batch_copied));   // the pinned tables are free again
    if (need > m0->batch_bytes) {
        HIP_TRY(hipStreamSynchronize(st));
        release_dev(m0->batch_dev);
        release_host(m0->batch_host);
        m0->batch_dev = m0->batch_host = nullptr;
        m0->batch_bytes = 0;
        const size_t cap = need < (1u << 16) ? (1u << 16) : need + need / 2;
        HIP_TRY(hipMalloc(&m0->batch_dev, cap));
        HIP_TRY(hipHostMalloc(&m0->batch_host, cap, hipHostMallocDefault));
        m0->batch_bytes = cap;
    }
    // sharded: the leaves' statistics + counts, contiguous (one all-reduce)
    double* sh = nullptr;
    if (comm) {
        const size_t sbytes = sizeof(double) * (len + 1) * (size_t)n_mix;
        if (sbytes > m0->shard_bytes) {
            HIP_TRY(hipStreamSynchronize(st));
            release_dev(m0->shard_stats);
            m0->shard_stats = nullptr;
            m0->shard_bytes = 0;
            HIP_TRY(hipMalloc((void**)&m0->shard_stats, sbytes));
            m0->shard_bytes = sbytes;
        }
        sh = m0->shard_stats;
        HIP_TRY(hipMemsetAsync(sh, 0, sizeof(double) * len * (size_t)n_mix, st));
    }
    int r = ensure_partials(m0, (int)(rows > 0 ? rows : 1));
    if (r) return r;
    char* hb = (char*)m0->batch_host;
    char* db = (char*)m0->batch_dev;
    LeafDesc* leaves = (LeafDesc*)hb;
    MixDesc* mixd = (MixDesc*)(hb + off_mix);
    int2* items = (int2*)(hb + off_items);
    double* counts = (double*)(hb + off_cnt);
    const double* dcounts = (const double*)(db + off_cnt);
    int row = 0;
    for (int i = 0; i < n_mix; ++i) {
        sdmm_mix* m = mixes[i];
        const int64_t n = cnt[i] > 0 ? cnt[i] : 0;
        double* lstats = comm ? sh + len * (size_t)i : m->stats;
        leaves[i] = LeafDesc{m->ep, lstats, s0[i], n, plans[(size_t)i].chunk, row, plans[(size_t)i].blocks};
        mixd[i] = MixDesc{m->C, m->S, m->ep, m->gp, lstats, m->tmp_mean, m->tmp_cov, cnt[i] < 0 ? 0 : n,
                          (comm && cnt[i] >= 0) ? sh + len * (size_t)n_mix + i : nullptr};
        counts[i] = (double)n;
        for (int b = 0; b < plans[(size_t)i].blocks; ++b) items[row + b] = int2{i, b};
        row += plans[(size_t)i].blocks;
    }
    HIP_TRY(hipMemcpyAsync(db, hb, need, hipMemcpyHostToDevice, st));
    HIP_TRY(hipEventRecord(m0->batch_copied, st));
    const LeafDesc* dleaves = (const LeafDesc*)db;
    const MixDesc* dmix = (const MixDesc*)(db + off_mix);
    const int2* ditems = (const int2*)(db + off_items);
    const SamplesDev d = to_dev(s);
    if (rows > 0)
        HIP_TRY(launch_stats_kernel(m0, d, 0, StatsPlan{0, 0}, (int)rows, m0->partials, st, dleaves, ditems));
    HIP_TRY(launch_reduce_finalize_batched(m0->partials, m0->pstride, m0->Kp, m0->K, dleaves, n_mix, st));
    if (comm) {
        HIP_TRY(hipMemcpyAsync(sh + len * (size_t)n_mix, dcounts, sizeof(double) * (size_t)n_mix,
                               hipMemcpyDeviceToDevice, st));
        r = comm_allreduce(comm, sh, (len + 1) * (size_t)n_mix, st);
        if (r) return r;
    }
    HIP_TRY(launch_mstep_batched(m0->K, m0->Kp, dmix, n_mix, m0->norm5, st));
    HIP_TRY(hipEventRecord(m0->batch_done, st));
    for (int i = 1; i < n_mix; ++i)
        if (mixes[i]->stream != st) HIP_TRY(hipStreamWaitEvent(mixes[i]->stream, m0->batch_done, 0));
    return SDMM_OK;
}

}  // namespace

extern "C" {

// Stage host sample planes into m's staging buffer (device SoA view in *d):
// the planes are gathered on the host into the thread's pinned bounce buffer
// and move as ONE pinned copy (no pageable DMA; host transfer rules at the top
// of this file).  The caller synchronises m's stream before it returns.
static int stage_host_samples(sdmm_mix* m, const sdmm_samples* s, sdmm_samples* d) {
    const size_t n = (size_t)s->n;
    const size_t planes = 7 + (s->hpdf ? 1 : 0);
    const size_t bytes = 4 * n * planes + (s->is_diffuse ? n : 0);
    const size_t need = n * (7 * 4 + 4 + 1) + 64;
    if (need > m->staging_bytes) {
        HIP_TRY(hipStreamSynchronize(m->stream));   // the old block may still be read
        release_dev(m->staging);
        m->staging_bytes = 0;
        HIP_TRY(hipMalloc(&m->staging, need));
        m->staging_bytes = need;
    }
    char* pin = nullptr;
    HIP_TRY(bounce_buf(bytes, &pin));
    float* hp = (float*)pin;
    float* f = (float*)m->staging;
    *d = sdmm_samples{};
    for (int i = 0; i < 6; ++i) {
        std::memcpy(hp + i * n, s->x[i], 4 * n);
        d->x[i] = f + i * n;
    }
    std::memcpy(hp + 6 * n, s->w, 4 * n);
    d->w = f + 6 * n;
    if (s->hpdf) {
        std::memcpy(hp + 7 * n, s->hpdf, 4 * n);
        d->hpdf = f + 7 * n;
    }
    HIP_TRY(hipMemcpyAsync(f, hp, 4 * n * planes, hipMemcpyHostToDevice, m->stream));
    if (s->is_diffuse) {
        std::memcpy(pin + 4 * n * planes, s->is_diffuse, n);
        HIP_TRY(hipMemcpyAsync(f + 8 * n, pin + 4 * n * planes, n, hipMemcpyHostToDevice, m->stream));
        d->is_diffuse = (const uint8_t*)(f + 8 * n);
    }
    d->n = s->n;
    return SDMM_OK;
}

int sdmm_em_step_batched_host(sdmm_mix* const* mixes, int n_mix, const sdmm_samples* s, const int64_t* seg,
                              int iterations) {
    if (n_mix < 0 || (n_mix > 0 && (!mixes || !mixes[0]))) return fail(SDMM_E_INVALID, "invalid argument");
    if (n_mix == 0) return SDMM_OK;
    int r = check_samples(s);
    if (r) return r;
    if (s->n == 0) return sdmm_em_step_batched(mixes, n_mix, s, seg, iterations);
    sdmm_mix* m0 = mixes[0];
    HIP_TRY(hipSetDevice(m0->device));
    sdmm_samples d;
    r = stage_host_samples(m0, s, &d);
    if (r) return r;
    r = sdmm_em_step_batched(mixes, n_mix, &d, seg, iterations);
    // always: the bounce buffer is reused by the thread's next call
    const hipError_t e = hipStreamSynchronize(m0->stream);
    if (r) return r;
    if (e != hipSuccess) return fail(SDMM_E_HIP, std::string("sdmm_em_step_batched_host: ") + hipGetErrorString(e));
    return SDMM_OK;
}

int sdmm_em_step_batched_host_iters(sdmm_mix* const* mixes, int n_mix, const sdmm_samples* s, const int64_t* seg,
                                    const int* iterations) {
    if (n_mix < 0 || (n_mix > 0 && (!mixes || !mixes[0] || !iterations))) return fail(SDMM_E_INVALID, "invalid argument");
    if (n_mix == 0) return SDMM_OK;
    int r = check_samples(s);
    if (r) return r;
    if (s->n == 0) return sdmm_em_step_batched_iters(mixes, n_mix, s, seg, iterations);
    sdmm_mix* m0 = mixes[0];
    HIP_TRY(hipSetDevice(m0->device));
    sdmm_samples d;
    r = stage_host_samples(m0, s, &d);
    if (r) return r;
    r = sdmm_em_step_batched_iters(mixes, n_mix, &d, seg, iterations);
    // always: the bounce buffer is reused by the thread's next call
    const hipError_t e = hipStreamSynchronize(m0->stream);
    if (r) return r;
    if (e != hipSuccess) return fail(SDMM_E_HIP, std::string("sdmm_em_step_batched_host: ") + hipGetErrorString(e));
    return SDMM_OK;
}

int sdmm_em_step_host(sdmm_mix* m, const sdmm_samples* s, int iterations) {
    if (!m) return fail(SDMM_E_INVALID, "handle is NULL");
    HIP_TRY(hipSetDevice(m->device));
    int r = check_samples(s);
    if (r) return r;
    if (s->n == 0) return SDMM_OK;
    if (!m->initialised) return fail(SDMM_E_STATE, "mixture not initialised");
    sdmm_samples d;
    r = stage_host_samples(m, s, &d);
    if (r) return r;
    r = sdmm_em_step(m, &d, iterations);
    // always: the bounce buffer is reused by the thread's next call
    const hipError_t e = hipStreamSynchronize(m->stream);
    if (r) return r;
    if (e != hipSuccess) return fail(SDMM_E_HIP, std::string("sdmm_em_step_host: ") + hipGetErrorString(e));
    return SDMM_OK;
}

int sdmm_responsibilities(sdmm_mix* m, const sdmm_samples* s, float* resp) {
    if (!m || !resp) return fail(SDMM_E_INVALID, "invalid argument");
    if (!m->initialised) return fail(SDMM_E_STATE, "mixture not initialised");
    HIP_TRY(hipSetDevice(m->device));
    int r = check_samples(s);
    if (r) return r;
    if (s->n == 0) return SDMM_OK;
    if (m->rtile == 3) {
        const int64_t resident = (int64_t)m->cus * (m->resp_blocks > 0 ? m->resp_blocks : 1);
        HIP_TRY(launch_estep_resp_split(m->rvariant, m->ep, m->Kp, m->K, to_dev(s), s->n, resident, resp, m->stream));
        return SDMM_OK;
    }
    if (m->rtile == 2) {
        // chunks of whole 16-sample tiles, ~3 rounds of resident waves
        const int64_t resident = (int64_t)m->cus * 4 * (m->resp_blocks > 0 ? m->resp_blocks : 1);
        int64_t chunk = (s->n + 3 * resident - 1) / (3 * resident);
        chunk = ((chunk + 15) / 16) * 16;
        if (chunk < 64) chunk = 64;
        HIP_TRY(launch_estep_resp_mfma(m->rvariant, m->ep, m->Kp, m->K, to_dev(s), s->n, chunk, resp, m->stream));
        return SDMM_OK;
    }
    if (m->rtile) {
        // chunks of whole 64-sample blocks; ~3 rounds of resident waves so the
        // tail of the launch stays short
        const int64_t resident = (int64_t)m->cus * 4 * (m->resp_blocks > 0 ? m->resp_blocks : 1);
        int64_t chunk = (s->n + 3 * resident - 1) / (3 * resident);
        chunk = ((chunk + 63) / 64) * 64;
        if (chunk < 64) chunk = 64;   // one staged 64-sample block: small (per-rank) batches still fill the chip
        HIP_TRY(launch_estep_resp_tile(m->rvariant, m->ep, m->Kp, m->K, to_dev(s), s->n, chunk, resp, m->stream));
        return SDMM_OK;
    }
    const Split sp = split_for(m, s->n, m->rlps, m->resp_blocks);
    HIP_TRY(launch_estep_resp(m->rcpl, m->rlps, m->ep, m->Kp, m->K, to_dev(s), s->n, sp.chunk, resp,
                              m->stream));
    return SDMM_OK;
}

int sdmm_guide_batch(const sdmm_mix* m, int64_t nq, const float* const c[3], const float* const u[3],
                     float* const d[3], float* pdf, int32_t* comp) {
    if (!m || !c || !u || !d || !pdf || !comp) return fail(SDMM_E_INVALID, "invalid argument");
    if (!m->initialised) return fail(SDMM_E_STATE, "mixture not initialised");
    HIP_TRY(hipSetDevice(m->device));
    if (nq <= 0) return SDMM_OK;
    int r = ensure_guide_scratch(m, nq);
    if (r) return r;
    HIP_TRY(launch_guide(m->gp, m->Kp, m->K, nq, c, u, nullptr, d, pdf, comp, m->norm2, m->norm3,
                         m->guide_cap, m->guide_fb, m->guide_fb + 1, m->cus, m->stream, guide_order(m, nq),
                         (int*)m->guide_sort.keys[0]));
    return SDMM_OK;
}

int sdmm_pdf_batch(const sdmm_mix* m, int64_t nq, const float* const c[3], const float* const d[3],
                   float* pdf) {
    if (!m || !c || !d || !pdf) return fail(SDMM_E_INVALID, "invalid argument");
    if (!m->initialised) return fail(SDMM_E_STATE, "mixture not initialised");
    HIP_TRY(hipSetDevice(m->device));
    if (nq <= 0) return SDMM_OK;
    int r = ensure_guide_scratch(m, nq);
    if (r) return r;
    HIP_TRY(launch_guide(m->gp, m->Kp, m->K, nq, c, nullptr, d, nullptr, pdf, nullptr, m->norm2, m->norm3,
                         m->guide_cap, m->guide_fb, m->guide_fb + 1, m->cus, m->stream, guide_order(m, nq),
                         (int*)m->guide_sort.keys[0]));
    return SDMM_OK;
}

static int check_bsdf(const sdmm_bsdf_table* b, const int32_t* material, const float* const frame[9]) {
    if (!b || !material || !frame) return fail(SDMM_E_INVALID, "product: bsdf table, material and frame required");
    if (b->B < 0 || b->M < 0 || b->M > 64) return fail(SDMM_E_INVALID, "product: need B >= 0, 0 <= M <= 64");
    if (b->B > 0 && b->M > 0 && (!b->weights || !b->means || !b->covs))
        return fail(SDMM_E_INVALID, "product: bsdf table arrays missing");
    for (int i = 0; i < 9; ++i)
        if (!frame[i]) return fail(SDMM_E_INVALID, "product: frame plane missing");
    return SDMM_OK;
}

int sdmm_guide_product_batch(const sdmm_mix* m, int64_t nq, const float* const c[3], const float* const u[3],
                             const sdmm_bsdf_table* bsdf, const int32_t* material, const float* const frame[9],
                             float* const d[3], float* pdf, int32_t* comp, float* heuristic) {
    if (!m || !c || !u || !d || !pdf || !comp) return fail(SDMM_E_INVALID, "invalid argument");
    if (!m->initialised) return fail(SDMM_E_STATE, "mixture not initialised");
    HIP_TRY(hipSetDevice(m->device));
    if (nq <= 0) return SDMM_OK;
    int r = check_bsdf(bsdf, material, frame);
    if (r) return r;
    if ((r = ensure_guide_scratch(m, nq))) return r;
    HIP_TRY(launch_guide_product(m->gp, m->Kp, m->K, m->C.condCov, nq, c, u, nullptr, d, pdf, comp, material,
                                 frame, heuristic, bsdf->weights, bsdf->means, bsdf->covs, bsdf->diffuse, bsdf->B,
                                 bsdf->M,
                                 m->norm2, m->norm3, m->guide_cap, m->guide_fb, m->guide_fb + 1, m->cus, m->stream,
                                 guide_order(m, nq), &m->product_scratch));
    return SDMM_OK;
}

int sdmm_pdf_product_batch(const sdmm_mix* m, int64_t nq, const float* const c[3], const float* const d[3],
                           const sdmm_bsdf_table* bsdf, const int32_t* material, const float* const frame[9],
                           float* pdf, float* heuristic) {
    if (!m || !c || !d || !pdf) return fail(SDMM_E_INVALID, "invalid argument");
    if (!m->initialised) return fail(SDMM_E_STATE, "mixture not initialised");
    HIP_TRY(hipSetDevice(m->device));
    if (nq <= 0) return SDMM_OK;
    int r = check_bsdf(bsdf, material, frame);
    if (r) return r;
    if ((r = ensure_guide_scratch(m, nq))) return r;
    HIP_TRY(launch_guide_product(m->gp, m->Kp, m->K, m->C.condCov, nq, c, nullptr, d, nullptr, pdf, nullptr,
                                 material, frame, heuristic, bsdf->weights, bsdf->means, bsdf->covs, bsdf->diffuse,
                                 bsdf->B, bsdf->M, m->norm2, m->norm3, m->guide_cap, m->guide_fb, m->guide_fb + 1, m->cus,
                                 m->stream, guide_order(m, nq), &m->product_scratch));
    return SDMM_OK;
}

int sdmm_sample_discrete_cdf(const sdmm_mix* m, const float* cdf, int n, const float* u, int64_t nq,
                             int32_t* out) {
    if (!m || !cdf || n <= 0 || !u || !out) return fail(SDMM_E_INVALID, "invalid argument");
    HIP_TRY(hipSetDevice(m->device));
    HIP_TRY(launch_sample_cdf(cdf, n, u, nq, out, m->stream));
    return SDMM_OK;
}

int sdmm_get_params(const sdmm_mix* m, const sdmm_params_out* o) {
    if (!m || !o) return fail(SDMM_E_INVALID, "invalid argument");
    HIP_TRY(hipSetDevice(m->device));
    const size_t K = (size_t)m->K;
    double sc[SC_COUNT];
    const XferItem items[] = {
        {o->weights, m->C.weights, 4 * K}, {o->cdf, m->C.cdf, 4 * K}, {o->mean, m->C.mean, 24 * K},
        {o->cov, m->C.cov, 100 * K}, {o->to, m->C.to, 36 * K}, {o->cholL, m->C.cholL, 100 * K},
        {o->cholLInv, m->C.cholLInv, 100 * K}, {o->detInv, m->C.detInv, 4 * K},
        {o->muPremult, m->C.muPremult, 24 * K}, {o->condCov, m->C.condCov, 16 * K},
        {o->margL, m->C.margL, 36 * K}, {o->margDetInv, m->C.margDetInv, 4 * K},
        {o->condL, m->C.condL, 16 * K}, {o->condLInv, m->C.condLInv, 16 * K},
        {o->condDetInv, m->C.condDetInv, 4 * K}, {o->valid, m->C.valid, 4 * K},
        {sc, m->S.scalars, sizeof(sc)},
    };
    const int r = xfer(items, (int)(sizeof(items) / sizeof(items[0])), false, m->stream);
    if (r) return r;
    if (o->normalization) *o->normalization = (float)sc[SC_NORM];
    return SDMM_OK;
}

int sdmm_get_state(const sdmm_mix* m, double* scalars, double* T, double* sgW, double* sgM, double* sgC,
                   float* bpriors, float* bdepth) {
    if (!m) return fail(SDMM_E_INVALID, "handle is NULL");
    HIP_TRY(hipSetDevice(m->device));
    const size_t K = (size_t)m->K;
    const XferItem items[] = {
        {scalars, m->S.scalars, 8 * SC_COUNT}, {T, m->S.T, 8 * K}, {sgW, m->S.sgW, 8 * K},
        {sgM, m->S.sgM, 40 * K}, {sgC, m->S.sgC, 200 * K}, {bpriors, m->S.bPriors, 100 * K},
        {bdepth, m->S.bDepth, 36 * K},
    };
    const int r = xfer(items, (int)(sizeof(items) / sizeof(items[0])), false, m->stream);
    if (r) return r;
    return SDMM_OK;
}

int sdmm_set_state(sdmm_mix* m, const double* scalars, const double* T, const double* sgW, const double* sgM,
                   const double* sgC, const float* bpriors, const float* bdepth) {
    if (!m) return fail(SDMM_E_INVALID, "handle is NULL");
    HIP_TRY(hipSetDevice(m->device));
    const size_t K = (size_t)m->K;
    const XferItem items[] = {
        {(void*)scalars, m->S.scalars, 8 * SC_COUNT}, {(void*)T, m->S.T, 8 * K}, {(void*)sgW, m->S.sgW, 8 * K},
        {(void*)sgM, m->S.sgM, 40 * K}, {(void*)sgC, m->S.sgC, 200 * K}, {(void*)bpriors, m->S.bPriors, 100 * K},
        {(void*)bdepth, m->S.bDepth, 36 * K},
    };
    const int r = xfer(items, (int)(sizeof(items) / sizeof(items[0])), true, m->stream);
    if (r) return r;
    return SDMM_OK;
}

int sdmm_get_em_params(const sdmm_mix* m, sdmm_em_params* p) {
    if (!m || !p) return fail(SDMM_E_INVALID, "invalid argument");
    *p = m->params;
    return SDMM_OK;
}

// Checkpoint restore: the exact inverse of sdmm_get_params (every canonical and
// derived array, so a restored mixture is bitwise the saved one -- no MVTN::set
// re-derivation), then the kernels' packed records from them.
int sdmm_restore_params(sdmm_mix* m, const sdmm_params_out* in) {
    if (!m || !in) return fail(SDMM_E_INVALID, "invalid argument");
    const size_t K = (size_t)m->K;
    hipStream_t st = m->stream;
    const XferItem items[] = {
        {in->weights, m->C.weights, 4 * K}, {in->cdf, m->C.cdf, 4 * K}, {in->mean, m->C.mean, 24 * K},
        {in->cov, m->C.cov, 100 * K}, {in->to, m->C.to, 36 * K}, {in->cholL, m->C.cholL, 100 * K},
        {in->cholLInv, m->C.cholLInv, 100 * K}, {in->detInv, m->C.detInv, 4 * K},
        {in->muPremult, m->C.muPremult, 24 * K}, {in->condCov, m->C.condCov, 16 * K},
        {in->margL, m->C.margL, 36 * K}, {in->margDetInv, m->C.margDetInv, 4 * K},
        {in->condL, m->C.condL, 16 * K}, {in->condLInv, m->C.condLInv, 16 * K},
        {in->condDetInv, m->C.condDetInv, 4 * K}, {(void*)in->valid, m->C.valid, 4 * K},
    };
    for (const XferItem& it : items)
        if (!it.host) return fail(SDMM_E_INVALID, "sdmm_restore_params: every array is required");
    HIP_TRY(hipSetDevice(m->device));
    const int r = xfer(items, (int)(sizeof(items) / sizeof(items[0])), true, st);
    if (r) return r;
    HIP_TRY(launch_pack_all(m->K, m->Kp, m->C, m->ep, m->gp, m->norm5, st));
    HIP_TRY(hipStreamSynchronize(st));
    m->initialised = true;
    return SDMM_OK;
}

}  // extern "C"

// ==========================================================================
// Spatial tree: jmm SNTree (mitsuba/src/integrators/dmm/jmm/sntree.h:93-299),
// spatial part.  The plugin's accelerator is sdmm-lib's DMMSTree
// (sdmm_proc.h:91), absent from the snapshot; SNTree is its readable
// counterpart.  Construction runs on the host, as in the reference (it is a
// once-per-iteration, data-dependent recursion); find() and the routing of a
// sample batch into leaf-contiguous order run on the device.
//
// Restated behaviour (file:line of sntree.h):
//   * the root box is the given AABB enlarged to a cube (:101-106);
//   * split_to_depth(d) (:195-233): midpoint splits along the node's axis,
//     children take axis (a + 1) % 3, "depth" advances after the z split;
//   * split(threshold) (:235-283): a leaf holding more than `threshold`
//     samples splits at the sample mean along its max-variance axis
//     (getSplitLocation :141-170, strict > so ties keep the lower axis);
//     each child receives the parent's samples its box contains (inclusive
//     on both sides: a sample on the plane goes to both, :174-192), and the
//     children are split recursively, child 0 first;
//   * child 0 is the UPPER part (min[axis] += s * diag), child 1 the lower
//     (max[axis] -= (1 - s) * diag) (createChildNode :172-186);
//   * nodes are appended in creation order, so node ids are the reference's
//     m_nodes indices.
// Deviations (documented): the mean/variance are summed in double
// (jmm: float Eigen sums, order unspecified); a split that would not separate
// the samples (zero variance: the reference recurses forever) is skipped;
// the per-normal NGridNode cells are not modelled (one value per leaf).
struct STNodeHost {
    float mn[3], mx[3];
    int axis = 0;
    int child[2] = {-1, -1};
};

// host image of guide.hip's GuideMix (one per tree node)
struct GuideMixHost {
    const float* gp;
    int Kp, K;
    bool operator!=(const GuideMixHost& o) const { return gp != o.gp || Kp != o.Kp || K != o.K; }
};
static_assert(sizeof(GuideMixHost) == 16, "GuideMix");

struct sdmm_stree {
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<STNodeHost> nodes;
    void* dnodes = nullptr;
    size_t dnodes_cap = 0;
    bool dirty = true;
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    bool own_stream = true;
    // guided wavefront: per-node mixture table (device + the host copy it
    // was uploaded from) and the guided-batch scratch
    std::vector<GuideMixHost> tab_host;
    std::vector<const float*> cc_host;   // per node: the mixture's condCov (product wavefront)
    void* dtab = nullptr;                // [nn] GuideMix, then [nn] condCov pointers (dcctab)
    void* dcctab = nullptr;
    size_t dtab_cap = 0;
    int tab_kmax = 0;
    int tab_cap = kGuideCapDefault; // candidate capacity: the smallest of the bound mixtures' (sdmm_set_guide_capacity)
    bool tab_valid = false;     // bound table matches the current nodes
    int* guide_fb = nullptr;
    int64_t guide_fb_cap = 0;
    GuideSortScratch guide_sort{};
    ProductScratch product_scratch{};
    bool stream_set = false;    // sdmm_stree_set_stream called (NULL then means the null stream)
    // the bound mixtures' streams other than the tree's: a wavefront waits for
    // their pending work (EM steps) through one event per stream
    std::vector<hipStream_t> mix_streams;
    std::vector<hipEvent_t> mix_events;
    // device split scratch (level buffers, flags / ranks, scan temp; per-level
    // tables), kept across calls
    void* split_mem = nullptr;
    int64_t split_cap = 0;
    void* split_small = nullptr;
    size_t split_small_cap = 0;
    // sdmm_stree_publish: nodes, mixture table and the bound mixtures' pending
    // work complete; guide contexts may read them from any thread until the
    // next change (an upload of either clears it)
    bool published = false;
};

namespace {

bool st_contains(const STNodeHost& n, const float p[3]) {
    return n.mn[0] <= p[0] && p[0] <= n.mx[0] && n.mn[1] <= p[1] && p[1] <= n.mx[1] && n.mn[2] <= p[2] &&
           p[2] <= n.mx[2];
}

STNodeHost st_child(const STNodeHost& parent, int child_i, float split) {
    STNodeHost c;
    const int axis = parent.axis;
    c.axis = (axis + 1) % 3;
    for (int i = 0; i < 3; ++i) { c.mn[i] = parent.mn[i]; c.mx[i] = parent.mx[i]; }
    const float diag = parent.mx[axis] - parent.mn[axis];
    if (child_i == 0) {
        const float d = split * diag;
        c.mn[axis] = parent.mn[axis] + d;
    } else {
        const float d = (1.0f - split) * diag;
        c.mx[axis] = parent.mx[axis] - d;
    }
    return c;
}

void st_split_depth(sdmm_stree* t, int node, int depth, int max_depth) {
    const int next = (t->nodes[node].axis == 2) ? depth + 1 : depth;
    if (t->nodes[node].child[0] >= 0) {
        for (int c = 0; c < 2; ++c) st_split_depth(t, t->nodes[node].child[c], next, max_depth);
        return;
    }
    if (depth < max_depth) {
        for (int c = 0; c < 2; ++c) {
            STNodeHost ch = st_child(t->nodes[node], c, 0.5f);
            t->nodes[node].child[c] = (int)t->nodes.size();
            t->nodes.push_back(ch);
        }
        for (int c = 0; c < 2; ++c) st_split_depth(t, t->nodes[node].child[c], next, max_depth);
    }
}

// split_recurse (sntree.h:235-283) of leaf `node` of the node list L (children
// appended to L, depth first); samples: indices into the position planes
// px/py/pz owned by node.  Works on a LOCAL list so that independent leaves
// can split in parallel; st_merge_local then appends the new nodes to the
// tree in the order a sequential split would have created them.
// The split's fp64 sums over a node's samples (sum p, then sum p^2, per axis)
// in ONE fixed order, the order the device reduction forms them
// (stree.hip split_sums_kernel): chunks of split_chunk_samples() consecutive
// samples; within a chunk lane t of 256 sums samples t, t + 256, ... in order,
// products separately rounded; the 256 lane sums fold pairwise (stride 128,
// 64, .., 1); the chunk sums are added in chunk order to 0.  (jmm sums in
// float in an unspecified order; oracle/sdmm_oracle_stree.c mirrors this.)
void split_sums_host(const std::vector<int64_t>& idx, const float* px, const float* py, const float* pz,
                     double out[6]) {
#pragma clang fp contract(off)
    const int64_t n = (int64_t)idx.size(), C = split_chunk_samples();
    for (int k = 0; k < 6; ++k) out[k] = 0.0;
    std::vector<double> lane(256 * 6);
    for (int64_t c0 = 0; c0 < n; c0 += C) {
        const int64_t len = std::min(C, n - c0);
        std::fill(lane.begin(), lane.end(), 0.0);
        for (int64_t j = 0; j < len; ++j) {
            double* a = &lane[(size_t)(j % 256) * 6];
            const int64_t i = idx[(size_t)(c0 + j)];
            const double p[3] = {px[i], py[i], pz[i]};
            for (int k = 0; k < 3; ++k) {
                a[k] = a[k] + p[k];
                const double sq = p[k] * p[k];
                a[3 + k] = a[3 + k] + sq;
            }
        }
        for (int st = 128; st > 0; st >>= 1)
            for (int t = 0; t < st; ++t)
                for (int k = 0; k < 6; ++k) lane[(size_t)t * 6 + k] = lane[(size_t)t * 6 + k] + lane[(size_t)(t + st) * 6 + k];
        for (int k = 0; k < 6; ++k) out[k] = out[k] + lane[k];
    }
}

// sntree.h:235-283's choice from the sums: the mean along the axis of largest
// variance (the first of equals); false when the split position is not
// strictly inside the node (zero variance / outside: the reference would
// recurse forever)
bool split_decide(const STNodeHost& nd, const double sums[6], int64_t n, int& ax, float& split) {
    float m[3], var[3];
    for (int a = 0; a < 3; ++a) {
        const double mu = sums[a] / (double)n;
        m[a] = (float)mu;
        var[a] = (float)(sums[3 + a] / (double)n - mu * mu);
    }
    ax = 0;
    for (int a = 0; a < 3; ++a)
        if (var[a] > var[ax]) ax = a;
    split = (m[ax] - nd.mn[ax]) / (nd.mx[ax] - nd.mn[ax]);
    return split > 0.0f && split < 1.0f;
}

void st_split_local(std::vector<STNodeHost>& L, int node, std::vector<int64_t>& idx, const float* px,
                    const float* py, const float* pz, int threshold) {
    if (L[(size_t)node].child[0] >= 0) return;   // (inner nodes are routed by the caller)
    const int64_t n = (int64_t)idx.size();
    if (n <= threshold) return;
    double sums[6];
    split_sums_host(idx, px, py, pz, sums);
    int ax = 0;
    float split = 0.0f;
    if (!split_decide(L[(size_t)node], sums, n, ax, split)) return;   // degenerate (zero variance / outside)
    const STNodeHost& nd = L[(size_t)node];
    STNodeHost parent = nd;
    parent.axis = ax;
    STNodeHost ch[2] = {st_child(parent, 0, split), st_child(parent, 1, split)};
    // both children's members in one pass (a sample on the split plane goes to both)
    std::vector<int64_t> sub[2];
    sub[0].reserve((size_t)n / 2 + 16);
    sub[1].reserve((size_t)n / 2 + 16);
    for (int64_t i : idx) {
        const float p[3] = {px[i], py[i], pz[i]};
        if (st_contains(ch[0], p)) sub[0].push_back(i);
        if (st_contains(ch[1], p)) sub[1].push_back(i);
    }
    for (int c = 0; c < 2; ++c)
        if ((int64_t)sub[c].size() == n) return;   // would not separate the samples
    L[(size_t)node].axis = ax;
    for (int c = 0; c < 2; ++c) {
        L[(size_t)node].child[c] = (int)L.size();
        L.push_back(ch[c]);
    }
    idx.clear();
    idx.shrink_to_fit();
    const int c0 = L[(size_t)node].child[0], c1 = L[(size_t)node].child[1];
    // Two large children: child 1's subtree on a thread of its own, built as a
    // local node list and appended after child 0's -- the creation (DFS)
    // order, hence every node id, is that of the sequential recursion.
    constexpr int64_t kParallelSplit = 1 << 15;
    if ((int64_t)sub[0].size() > kParallelSplit && (int64_t)sub[1].size() > kParallelSplit) {
        std::vector<STNodeHost> L1{L[(size_t)c1]};
        std::future<void> f1;
        try {
            f1 = std::async(std::launch::async, [&] { st_split_local(L1, 0, sub[1], px, py, pz, threshold); });
        } catch (...) {
            f1 = std::future<void>();
        }
        st_split_local(L, c0, sub[0], px, py, pz, threshold);
        if (f1.valid())
            f1.get();
        else
            st_split_local(L1, 0, sub[1], px, py, pz, threshold);
        const int base = (int)L.size() - 1;
        auto remap = [&](STNodeHost x) {
            if (x.child[0] >= 0) { x.child[0] = base + x.child[0]; x.child[1] = base + x.child[1]; }
            return x;
        };
        L[(size_t)c1] = remap(L1[0]);
        for (size_t i = 1; i < L1.size(); ++i) L.push_back(remap(L1[i]));
        return;
    }
    st_split_local(L, c0, sub[0], px, py, pz, threshold);
    st_split_local(L, c1, sub[1], px, py, pz, threshold);
}

// L[0] is tree node v after st_split_local; its new nodes get the next ids
void st_merge_local(sdmm_stree* t, int v, const std::vector<STNodeHost>& L) {
    const int base = (int)t->nodes.size() - 1;
    auto gid = [&](int i) { return i == 0 ? v : base + i; };
    auto remap = [&](STNodeHost n) {
        if (n.child[0] >= 0) { n.child[0] = gid(n.child[0]); n.child[1] = gid(n.child[1]); }
        return n;
    };
    t->nodes[(size_t)v] = remap(L[0]);
    for (size_t i = 1; i < L.size(); ++i) t->nodes.push_back(remap(L[i]));
}

// split_leaf_recurse of leaves[i] with its own positions, independent leaves
// on parallel host threads, merged in the given order
void st_split_many(sdmm_stree* t, int n, const int* leaves, std::vector<int64_t>* idx, const float* const* p,
                   int threshold) {
    std::vector<std::vector<STNodeHost>> L((size_t)n);
    for (int i = 0; i < n; ++i) L[(size_t)i].push_back(t->nodes[(size_t)leaves[i]]);
    unsigned nt = std::thread::hardware_concurrency();
    nt = std::max(1u, std::min(nt, 32u));
    if ((int)nt > n) nt = (unsigned)std::max(n, 1);
    std::atomic<int> next{0};
    auto work = [&]() {
        for (int i = next++; i < n; i = next++)
            st_split_local(L[(size_t)i], 0, idx[i], p[3 * i], p[3 * i + 1], p[3 * i + 2], threshold);
    };
    if (nt <= 1) {
        work();
    } else {
        std::vector<std::thread> th;
        try {
            for (unsigned k = 0; k < nt; ++k) th.emplace_back(work);
        } catch (...) {
            work();   // the shared counter hands this thread what is left
        }
        for (auto& x : th) x.join();
    }
    for (int i = 0; i < n; ++i) st_merge_local(t, leaves[i], L[(size_t)i]);
}

// SNTreeNode::find (jmm/sntree.h:62-83): depth first, child 0 first, with
// backtracking out of subtrees that hold no leaf box with the point.
int st_find_host(const sdmm_stree* t, const float p[3]) {
    if (!st_contains(t->nodes[0], p)) return -1;
    // pending siblings: at most one per level (a few dozen levels at most)
    int stack[256];
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const int i = stack[--sp];
        const STNodeHost& n = t->nodes[(size_t)i];
        if (n.child[0] < 0) return i;
        if (sp + 2 > 256) return -1;
        if (st_contains(t->nodes[(size_t)n.child[1]], p)) stack[sp++] = n.child[1];
        if (st_contains(t->nodes[(size_t)n.child[0]], p)) stack[sp++] = n.child[0];
    }
    return -1;
}

int st_upload(sdmm_stree* t) {
    if (!t->stream && !t->stream_set) HIP_TRY(hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking));
    if (!t->dirty) return SDMM_OK;
    t->published = false;
    const size_t bytes = 32 * t->nodes.size();
    if (bytes > t->dnodes_cap) {
        HIP_TRY(hipStreamSynchronize(t->stream));
        release_dev(t->dnodes);
        t->dnodes = nullptr;
        const size_t cap = bytes * 2 > 4096 ? bytes * 2 : 4096;
        HIP_TRY(hipMalloc(&t->dnodes, cap));
        t->dnodes_cap = cap;
    }
    std::vector<float> rec(8 * t->nodes.size());
    for (size_t i = 0; i < t->nodes.size(); ++i) {
        const STNodeHost& n = t->nodes[i];
        for (int a = 0; a < 3; ++a) { rec[8 * i + a] = n.mn[a]; rec[8 * i + 3 + a] = n.mx[a]; }
        int c0 = n.child[0], c1 = n.child[1];
        std::memcpy(&rec[8 * i + 6], &c0, 4);
        std::memcpy(&rec[8 * i + 7], &c1, 4);
    }
    HIP_TRY(hipMemcpyAsync(t->dnodes, rec.data(), bytes, hipMemcpyHostToDevice, t->stream));
    HIP_TRY(hipStreamSynchronize(t->stream));   // rec is a host temporary
    t->dirty = false;
    return SDMM_OK;
}

}  // namespace

extern "C" {

int sdmm_stree_create(const float aabb_min[3], const float aabb_max[3], int device, sdmm_stree** out) {
    if (!out || !aabb_min || !aabb_max) return fail(SDMM_E_INVALID, "invalid argument");
    *out = nullptr;
    float size = 0.0f;
    for (int a = 0; a < 3; ++a) {
        if (!(aabb_max[a] >= aabb_min[a])) return fail(SDMM_E_INVALID, "empty AABB");
        size = std::max(size, aabb_max[a] - aabb_min[a]);
    }
    sdmm_stree* t = new (std::nothrow) sdmm_stree();
    if (!t) return fail(SDMM_E_NOMEM, "out of host memory");
    t->device = device;
    STNodeHost root;
    for (int a = 0; a < 3; ++a) { root.mn[a] = aabb_min[a]; root.mx[a] = aabb_min[a] + size; }   // cube (:101-106)
    t->nodes.push_back(root);
    *out = t;   // (the device stream is created on first device use: building needs no GPU)
    return SDMM_OK;
}

void sdmm_stree_destroy(sdmm_stree* t) {
    if (!t) return;
    (void)hipSetDevice(t->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    if (t->dnodes) (void)hipFree(t->dnodes);
    if (t->scratch) (void)hipFree(t->scratch);
    if (t->dtab) (void)hipFree(t->dtab);
    if (t->split_mem) (void)hipFree(t->split_mem);
    if (t->split_small) (void)hipFree(t->split_small);
    if (t->guide_fb) (void)hipFree(t->guide_fb);
    if (t->product_scratch.base) (void)hipFree(t->product_scratch.base);   // stream synced above
    for (hipEvent_t e : t->mix_events) (void)hipEventDestroy(e);
    if (t->stream && t->own_stream) (void)hipStreamDestroy(t->stream);
    delete t;
}

int sdmm_stree_split_to_depth(sdmm_stree* t, int max_depth) {
    if (!t || max_depth < 0 || max_depth > 8) return fail(SDMM_E_INVALID, "max_depth must be in [0, 8]");
    st_split_depth(t, 0, 0, max_depth);
    t->dirty = true;
    t->tab_valid = false;
    return SDMM_OK;
}

int sdmm_stree_split(sdmm_stree* t, const float* const p[3], int64_t n, int threshold) {
    if (!t || (n > 0 && (!p || !p[0] || !p[1] || !p[2])) || n < 0 || threshold < 1)
        return fail(SDMM_E_INVALID, "invalid argument");
    // leaf assignment of the given samples (find), then the recursive split
    std::vector<std::vector<int64_t>> per(t->nodes.size());
    for (int64_t i = 0; i < n; ++i) {
        const float q[3] = {p[0][i], p[1][i], p[2][i]};
        const int id = st_find_host(t, q);
        if (id >= 0) per[(size_t)id].push_back(i);
    }
    std::vector<int> leaves;
    std::vector<std::vector<int64_t>> idx;
    std::vector<const float*> planes;
    for (size_t id = 0; id < t->nodes.size(); ++id)
        if (t->nodes[id].child[0] < 0 && (int64_t)per[id].size() > threshold) {
            leaves.push_back((int)id);
            idx.push_back(std::move(per[id]));
            planes.insert(planes.end(), {p[0], p[1], p[2]});
        }
    st_split_many(t, (int)leaves.size(), leaves.data(), idx.data(), planes.data(), threshold);
    t->dirty = true;
    t->tab_valid = false;
    return SDMM_OK;
}

int sdmm_stree_num_nodes(const sdmm_stree* t) { return t ? (int)t->nodes.size() : 0; }

int sdmm_stree_leaf_nodes(const sdmm_stree* t) {
    if (!t) return 0;
    int n = 0;
    for (const STNodeHost& nd : t->nodes) n += nd.child[0] < 0 ? 1 : 0;
    return n;
}

int sdmm_stree_split_leaf_recurse(sdmm_stree* t, int node, const float* const p[3], int64_t n, int threshold) {
    if (!t || node < 0 || node >= (int)t->nodes.size() || n < 0 || threshold < 1 ||
        (n > 0 && (!p || !p[0] || !p[1] || !p[2])))
        return fail(SDMM_E_INVALID, "invalid argument");
    if (t->nodes[(size_t)node].child[0] >= 0) return SDMM_OK;   // an inner node: nothing to split
    std::vector<int64_t> idx((size_t)n);
    for (int64_t i = 0; i < n; ++i) idx[(size_t)i] = i;
    const float* planes[3] = {p[0], p[1], p[2]};
    st_split_many(t, 1, &node, &idx, planes, threshold);
    t->dirty = true;
    t->tab_valid = false;
    return SDMM_OK;
}

}  // extern "C"

namespace {

// split_leaf_recurse of many leaves on device-resident positions: the
// recursion level by level (every item = a node being split + its samples,
// contiguous in a level buffer in the parent's order); per level ONE sums
// launch (canonical fp64 order, split_sums_host), the decisions on the host
// (split_decide), one count launch (a split that would not separate its
// samples is dropped, as in st_split_local), one stable partition into the
// next level.  Each leaf's new nodes are collected breadth first and
// renumbered to the sequential recursion's creation order (depth first,
// both children at a split, child 0's subtree first) before merging.
struct DevSplitBuf {
    float* x = nullptr;
    float* y = nullptr;
    float* z = nullptr;
    int32_t* item = nullptr;
};

// the split scratch of t for levels of up to `need` samples (contents kept
// only by the caller's own copies: grown before a level is loaded / written)
struct DevSplitScratch {
    DevSplitBuf buf[2];
    int32_t* flags = nullptr;
    int64_t* rank = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0;
};

DevSplitScratch split_layout(void* mem, int64_t nc) {
    const size_t plane = ((sizeof(float) * (size_t)nc + 255) / 256) * 256;
    const size_t fl = ((sizeof(int32_t) * (2 * (size_t)nc + 1) + 255) / 256) * 256;
    const size_t rk = ((sizeof(int64_t) * (2 * (size_t)nc + 1) + 255) / 256) * 256;
    DevSplitScratch S;
    char* b = (char*)mem;
    for (int k = 0; k < 2; ++k) {
        S.buf[k].x = (float*)b; b += plane;
        S.buf[k].y = (float*)b; b += plane;
        S.buf[k].z = (float*)b; b += plane;
        S.buf[k].item = (int32_t*)b; b += plane;
    }
    S.flags = (int32_t*)b; b += fl;
    S.rank = (int64_t*)b; b += rk;
    S.temp = b;
    S.temp_bytes = ((split_scan_temp_bytes(2 * nc + 1) + 255) / 256) * 256;
    return S;
}
size_t split_mem_bytes(int64_t nc) {
    const size_t plane = ((sizeof(float) * (size_t)nc + 255) / 256) * 256;
    const size_t fl = ((sizeof(int32_t) * (2 * (size_t)nc + 1) + 255) / 256) * 256;
    const size_t rk = ((sizeof(int64_t) * (2 * (size_t)nc + 1) + 255) / 256) * 256;
    return 8 * plane + fl + rk + ((split_scan_temp_bytes(2 * nc + 1) + 255) / 256) * 256;
}

// the flag scan covers 2 n + 1 entries of a level as an int item count
constexpr int64_t kSplitLevelMax = (INT32_MAX - 1) / 2;

// grow t's split scratch to `need` samples per level; keep >= 0: the buffer
// set whose first `live` entries are copied over
int split_grow(sdmm_stree* t, int64_t need, int keep, int64_t live, hipStream_t st, DevSplitScratch& S) {
    if (need <= t->split_cap && t->split_mem) {
        S = split_layout(t->split_mem, t->split_cap);
        return SDMM_OK;
    }
    // SDMM_SPLIT_TIGHT=1 (a test knob): no headroom, so that duplicates on
    // split planes take the regrowth path below (tests/test_stree.py)
    const char* tight = std::getenv("SDMM_SPLIT_TIGHT");
    const int64_t nc = (tight && std::strcmp(tight, "1") == 0) ? need : need + need / 4 + 4096;
    if (nc > kSplitLevelMax) return fail(SDMM_E_INVALID, "device split: a level exceeds 2^30 samples");
    void* nm = nullptr;
    HIP_TRY(hipMalloc(&nm, split_mem_bytes(nc)));
    DevSplitScratch N = split_layout(nm, nc);
    if (keep >= 0 && t->split_mem && live > 0) {
        const DevSplitScratch O = split_layout(t->split_mem, t->split_cap);
        HIP_TRY(hipMemcpyAsync(N.buf[keep].x, O.buf[keep].x, sizeof(float) * (size_t)live, hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipMemcpyAsync(N.buf[keep].y, O.buf[keep].y, sizeof(float) * (size_t)live, hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipMemcpyAsync(N.buf[keep].z, O.buf[keep].z, sizeof(float) * (size_t)live, hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipMemcpyAsync(N.buf[keep].item, O.buf[keep].item, sizeof(int32_t) * (size_t)live,
                               hipMemcpyDeviceToDevice, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    release_dev(t->split_mem);
    t->split_mem = nm;
    t->split_cap = nc;
    S = N;
    return SDMM_OK;
}

int split_small(sdmm_stree* t, size_t need) {
    if (need <= t->split_small_cap && t->split_small) return SDMM_OK;
    release_dev(t->split_small);
    t->split_small = nullptr;
    t->split_small_cap = 0;
    const size_t cap = need + need / 2 + 4096;
    HIP_TRY(hipMalloc(&t->split_small, cap));
    t->split_small_cap = cap;
    return SDMM_OK;
}

int st_split_device(sdmm_stree* t, const std::vector<int>& leaves, const float* const p[3],
                    const std::vector<int64_t>& src_start, const std::vector<int64_t>& counts, int threshold,
                    hipStream_t st) {
    const int nl = (int)leaves.size();
    std::vector<std::vector<STNodeHost>> L((size_t)nl);   // per leaf, breadth first: [0] = the leaf
    for (int i = 0; i < nl; ++i) L[(size_t)i].push_back(t->nodes[(size_t)leaves[(size_t)i]]);
    struct Item { int leaf, local; int64_t start, n; };
    std::vector<Item> items;
    std::vector<int64_t> tabs;   // src starts, then dst starts
    int64_t total = 0;
    for (int i = 0; i < nl; ++i) {
        items.push_back({i, 0, total, counts[(size_t)i]});
        total += counts[(size_t)i];
    }
    for (int i = 0; i < nl; ++i) tabs.push_back(src_start[(size_t)i]);
    for (int i = 0; i < nl; ++i) tabs.push_back(items[(size_t)i].start);
    DevSplitScratch S;
    int r = split_grow(t, total, -1, 0, st, S);
    if (r) return r;
    const int C = split_chunk_samples();
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    // level 0: gather the leaves' positions
    {
        r = split_small(t, al(sizeof(int64_t) * tabs.size()));
        if (r) return r;
        int64_t* dt = (int64_t*)t->split_small;
        HIP_TRY(hipMemcpyAsync(dt, tabs.data(), sizeof(int64_t) * tabs.size(), hipMemcpyHostToDevice, st));
        HIP_TRY(launch_split_load(p, dt, dt + nl, nl, total, S.buf[0].x, S.buf[0].y, S.buf[0].z, S.buf[0].item, st));
    }
    int cur = 0;
    while (!items.empty()) {
        const int ni = (int)items.size();
        const int64_t lvl_n = items.back().start + items.back().n;
        // (1) fp64 sums of the items above the threshold, by chunks; (2) the
        // decisions (split_decide) and the children's counts, on the device:
        // one round trip per level
        std::vector<SplitChunkDev> chunks;
        std::vector<SplitItemDev> idesc((size_t)ni);
        for (int i = 0; i < ni; ++i) {
            const Item& it = items[(size_t)i];
            const STNodeHost& nd = L[(size_t)it.leaf][(size_t)it.local];
            SplitItemDev& d = idesc[(size_t)i];
            for (int a = 0; a < 3; ++a) { d.mn[a] = nd.mn[a]; d.mx[a] = nd.mx[a]; }
            d.start = it.start;
            d.n = it.n;
            d.c0 = d.c1 = (int32_t)chunks.size();
            if (it.n <= threshold) continue;
            for (int64_t c0 = 0; c0 < it.n; c0 += C) {
                SplitChunkDev c{};
                c.start = it.start + c0;
                c.len = (int32_t)std::min<int64_t>(C, it.n - c0);
                chunks.push_back(c);
            }
            d.c1 = (int32_t)chunks.size();
        }
        if (chunks.empty()) break;
        const size_t nch = chunks.size();
        r = split_small(t, al(sizeof(SplitChunkDev) * nch) + al(sizeof(double) * 6 * nch) +
                               al(sizeof(SplitCandDev) * (size_t)ni) + al(sizeof(long long) * 2 * (size_t)ni) +
                               al(sizeof(SplitItemDev) * (size_t)ni) + al(sizeof(SplitDecisionDev) * (size_t)ni));
        if (r) return r;
        char* sb = (char*)t->split_small;
        SplitChunkDev* dch = (SplitChunkDev*)sb; sb += al(sizeof(SplitChunkDev) * nch);
        double* dpart = (double*)sb; sb += al(sizeof(double) * 6 * nch);
        SplitCandDev* dcand = (SplitCandDev*)sb; sb += al(sizeof(SplitCandDev) * (size_t)ni);
        long long* dcnt = (long long*)sb; sb += al(sizeof(long long) * 2 * (size_t)ni);
        SplitItemDev* ditem = (SplitItemDev*)sb; sb += al(sizeof(SplitItemDev) * (size_t)ni);
        SplitDecisionDev* ddec = (SplitDecisionDev*)sb;
        const DevSplitBuf I = S.buf[cur];
        HIP_TRY(hipMemcpyAsync(dch, chunks.data(), sizeof(SplitChunkDev) * nch, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(ditem, idesc.data(), sizeof(SplitItemDev) * (size_t)ni, hipMemcpyHostToDevice, st));
        HIP_TRY(launch_split_sums(I.x, I.y, I.z, dch, (int)nch, dpart, st));
        HIP_TRY(launch_split_decide(ditem, ni, dpart, threshold, dcand, ddec, st));
        HIP_TRY(launch_split_flags(I.x, I.y, I.z, I.item, lvl_n, dcand, ni, S.flags, S.rank, S.temp, S.temp_bytes,
                                   dcnt, st));
        std::vector<long long> cnt(2 * (size_t)ni);
        std::vector<SplitDecisionDev> dec((size_t)ni);
        HIP_TRY(hipMemcpyAsync(cnt.data(), dcnt, sizeof(long long) * 2 * (size_t)ni, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(dec.data(), ddec, sizeof(SplitDecisionDev) * (size_t)ni, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        // the candidates as the device formed them (st_child of its decision)
        std::vector<SplitCandDev> cand((size_t)ni);
        std::vector<int> axes((size_t)ni, 0);
        std::vector<STNodeHost> kids(2 * (size_t)ni);
        int n_active = 0;
        for (int i = 0; i < ni; ++i) {
            SplitCandDev& c = cand[(size_t)i];
            std::memset(&c, 0, sizeof(c));
            const Item& it = items[(size_t)i];
            c.start = it.start;
            c.n = it.n;
            if (!dec[(size_t)i].active) continue;
            STNodeHost parent = L[(size_t)it.leaf][(size_t)it.local];
            parent.axis = dec[(size_t)i].axis;
            for (int k = 0; k < 2; ++k) kids[2 * (size_t)i + (size_t)k] = st_child(parent, k, dec[(size_t)i].split);
            for (int a = 0; a < 3; ++a) {
                c.mn0[a] = kids[2 * (size_t)i].mn[a]; c.mx0[a] = kids[2 * (size_t)i].mx[a];
                c.mn1[a] = kids[2 * (size_t)i + 1].mn[a]; c.mx1[a] = kids[2 * (size_t)i + 1].mx[a];
            }
            c.active = 1;
            axes[(size_t)i] = dec[(size_t)i].axis;
            ++n_active;
        }
        if (n_active == 0) break;
        // (3) accept the splits that separate their samples (st_split_local)
        std::vector<Item> next;
        int64_t ntotal = 0;
        for (int i = 0; i < ni; ++i) {
            SplitCandDev& c = cand[(size_t)i];
            if (!c.active) continue;
            const Item& it = items[(size_t)i];
            if (cnt[2 * (size_t)i] == it.n || cnt[2 * (size_t)i + 1] == it.n) {
                c.active = 0;
                continue;
            }
            auto& ln = L[(size_t)it.leaf];
            ln[(size_t)it.local].axis = axes[(size_t)i];
            for (int k = 0; k < 2; ++k) {
                ln[(size_t)it.local].child[k] = (int)ln.size();
                ln.push_back(kids[2 * (size_t)i + (size_t)k]);
                c.child_item[k] = (int32_t)next.size();
                c.out[k] = ntotal;
                next.push_back({it.leaf, (int)ln.size() - 1, ntotal, (int64_t)cnt[2 * (size_t)i + (size_t)k]});
                ntotal += (int64_t)cnt[2 * (size_t)i + (size_t)k];
            }
        }
        if (next.empty()) break;
        if (ntotal > t->split_cap) {
            // rare (many samples on split planes): the current level and its
            // flags / ranks move to a larger scratch, recomputed there
            r = split_grow(t, ntotal, cur, lvl_n, st, S);
            if (r) return r;
            HIP_TRY(hipMemcpyAsync(dcand, cand.data(), sizeof(SplitCandDev) * (size_t)ni, hipMemcpyHostToDevice,
                                   st));
            HIP_TRY(launch_split_flags(S.buf[cur].x, S.buf[cur].y, S.buf[cur].z, S.buf[cur].item, lvl_n, dcand, ni,
                                       S.flags, S.rank, S.temp, S.temp_bytes, dcnt, st));
        }
        // (4) the stable partition into the next level (rejected items: inactive)
        HIP_TRY(hipMemcpyAsync(dcand, cand.data(), sizeof(SplitCandDev) * (size_t)ni, hipMemcpyHostToDevice, st));
        const DevSplitBuf In = S.buf[cur], O = S.buf[1 - cur];
        HIP_TRY(launch_split_scatter(In.x, In.y, In.z, In.item, lvl_n, dcand, S.flags, S.rank, O.x, O.y, O.z,
                                     O.item, st));
        items.swap(next);
        cur = 1 - cur;
    }
    HIP_TRY(hipStreamSynchronize(st));
    // renumber each leaf's breadth-first nodes to the creation (depth-first) order
    for (int i = 0; i < nl; ++i) {
        const auto& Bn = L[(size_t)i];
        std::vector<STNodeHost> D;
        D.push_back(Bn[0]);
        D[0].child[0] = D[0].child[1] = -1;
        // pre-order: a node's two children are numbered when it is visited,
        // child 0's subtree before child 1's
        std::vector<std::pair<int, int>> stack{{0, 0}};   // (BFS index, D index)
        while (!stack.empty()) {
            const auto [b, d] = stack.back();
            stack.pop_back();
            if (Bn[(size_t)b].child[0] < 0) continue;
            D[(size_t)d].axis = Bn[(size_t)b].axis;
            int ids[2];
            for (int k = 0; k < 2; ++k) {
                STNodeHost c = Bn[(size_t)Bn[(size_t)b].child[k]];
                c.child[0] = c.child[1] = -1;
                ids[k] = (int)D.size();
                D.push_back(c);
                D[(size_t)d].child[k] = ids[k];
            }
            stack.push_back({Bn[(size_t)b].child[1], ids[1]});
            stack.push_back({Bn[(size_t)b].child[0], ids[0]});
        }
        st_merge_local(t, leaves[(size_t)i], D);
    }
    t->dirty = true;
    t->tab_valid = false;
    return SDMM_OK;
}

}  // namespace

extern "C" {

int sdmm_stree_split_leaf_recurse_device(sdmm_stree* t, int n, const int32_t* nodes, const float* const p[3],
                                         const int64_t* starts, const int64_t* counts, int threshold) {
    if (!t || n < 0 || threshold < 1 || (n > 0 && (!nodes || !p || !p[0] || !p[1] || !p[2] || !starts || !counts)))
        return fail(SDMM_E_INVALID, "invalid argument");
    std::vector<int> leaves;
    std::vector<int64_t> st0, cn;
    for (int i = 0; i < n; ++i) {
        const int v = nodes[i];
        if (v < 0 || v >= (int)t->nodes.size() || counts[i] < 0 || starts[i] < 0)
            return fail(SDMM_E_INVALID, "invalid argument");
        if (i > 0 && v <= nodes[i - 1]) return fail(SDMM_E_INVALID, "nodes must be increasing");
        if (t->nodes[(size_t)v].child[0] >= 0 || counts[i] <= threshold) continue;
        leaves.push_back(v);
        st0.push_back(starts[i]);
        cn.push_back(counts[i]);
    }
    if (leaves.empty()) return SDMM_OK;
    HIP_TRY(hipSetDevice(t->device));
    int r = st_upload(t);
    if (r) return r;
    return st_split_device(t, leaves, p, st0, cn, threshold, t->stream);
}

int sdmm_stree_split_leaf_recurse_many(sdmm_stree* t, int n, const int32_t* nodes, const float* const* p,
                                       const int64_t* counts, int threshold) {
    if (!t || n < 0 || threshold < 1 || (n > 0 && (!nodes || !p || !counts)))
        return fail(SDMM_E_INVALID, "invalid argument");
    std::vector<int> leaves;
    std::vector<std::vector<int64_t>> idx;
    std::vector<const float*> planes;
    for (int i = 0; i < n; ++i) {
        const int v = nodes[i];
        if (v < 0 || v >= (int)t->nodes.size() || counts[i] < 0 || (counts[i] > 0 && (!p[3 * i] || !p[3 * i + 1] ||
                                                                                        !p[3 * i + 2])))
            return fail(SDMM_E_INVALID, "invalid argument");
        if (i > 0 && v <= nodes[i - 1]) return fail(SDMM_E_INVALID, "nodes must be increasing");
        if (t->nodes[(size_t)v].child[0] >= 0 || counts[i] <= threshold) continue;
        leaves.push_back(v);
        std::vector<int64_t> ix((size_t)counts[i]);
        for (int64_t k = 0; k < counts[i]; ++k) ix[(size_t)k] = k;
        idx.push_back(std::move(ix));
        planes.insert(planes.end(), {p[3 * i], p[3 * i + 1], p[3 * i + 2]});
    }
    if (leaves.empty()) return SDMM_OK;
    st_split_many(t, (int)leaves.size(), leaves.data(), idx.data(), planes.data(), threshold);
    t->dirty = true;
    t->tab_valid = false;
    return SDMM_OK;
}

int sdmm_stree_split_leaves(sdmm_stree* t, const float* const p[3], int64_t n, int threshold, int max_leaf_nodes) {
    if (!t) return fail(SDMM_E_INVALID, "invalid argument");
    if (max_leaf_nodes >= 0 && sdmm_stree_leaf_nodes(t) > max_leaf_nodes) return SDMM_OK;
    return sdmm_stree_split(t, p, n, threshold);
}

int sdmm_stree_set_nodes(sdmm_stree* t, int n, const float* aabb, const int32_t* child, const int32_t* axis) {
    if (!t || n < 1 || !aabb || !child || !axis) return fail(SDMM_E_INVALID, "invalid argument");
    std::vector<STNodeHost> nodes((size_t)n);
    for (int i = 0; i < n; ++i) {
        STNodeHost& d = nodes[(size_t)i];
        for (int a = 0; a < 3; ++a) { d.mn[a] = aabb[6 * i + a]; d.mx[a] = aabb[6 * i + 3 + a]; }
        d.axis = axis[i];
        d.child[0] = child[2 * i];
        d.child[1] = child[2 * i + 1];
        const bool leaf = d.child[0] < 0 && d.child[1] < 0;
        // children come after their parent (the builder appends them), so a
        // valid table is acyclic and find() terminates
        const bool inner = d.child[0] > i && d.child[0] < n && d.child[1] > i && d.child[1] < n;
        if ((!leaf && !inner) || d.axis < 0 || d.axis > 2)
            return fail(SDMM_E_INVALID, "sdmm_stree_set_nodes: malformed node table");
    }
    t->nodes.swap(nodes);
    t->dirty = true;
    t->tab_valid = false;
    return SDMM_OK;
}

int sdmm_stree_get_nodes(const sdmm_stree* t, float* aabb, int32_t* child, int32_t* axis) {
    if (!t) return fail(SDMM_E_INVALID, "null tree");
    for (size_t i = 0; i < t->nodes.size(); ++i) {
        const STNodeHost& n = t->nodes[i];
        if (aabb)
            for (int a = 0; a < 3; ++a) { aabb[6 * i + a] = n.mn[a]; aabb[6 * i + 3 + a] = n.mx[a]; }
        if (child) { child[2 * i] = n.child[0]; child[2 * i + 1] = n.child[1]; }
        if (axis) axis[i] = n.axis;
    }
    return SDMM_OK;
}

int sdmm_stree_find(sdmm_stree* t, int64_t n, const float* const p[3], int32_t* node_out) {
    if (!t || n < 0 || (n > 0 && (!p || !node_out))) return fail(SDMM_E_INVALID, "invalid argument");
    if (n == 0) return SDMM_OK;
    HIP_TRY(hipSetDevice(t->device));
    int r = st_upload(t);
    if (r) return r;
    HIP_TRY(launch_stree_find(t->dnodes, n, p[0], p[1], p[2], node_out, t->stream));
    return SDMM_OK;
}

int sdmm_stree_route(sdmm_stree* t, const sdmm_samples* in, const sdmm_samples* out, int64_t* seg) {
    if (!t || !in || !out || !seg) return fail(SDMM_E_INVALID, "invalid argument");
    int r = check_samples(in);
    if (r) return r;
    const int64_t n = in->n;
    const int nn = (int)t->nodes.size();
    if (n > INT32_MAX) return fail(SDMM_E_INVALID, "route: at most 2^31 - 1 samples");
    for (int i = 0; i < 6; ++i)
        if (n > 0 && !out->x[i]) return fail(SDMM_E_INVALID, "route: output plane missing");
    if (n > 0 && !out->w) return fail(SDMM_E_INVALID, "route: output weight plane missing");
    if ((in->hpdf != nullptr) != (out->hpdf != nullptr) ||
        (in->is_diffuse != nullptr) != (out->is_diffuse != nullptr))
        return fail(SDMM_E_INVALID, "route: optional planes must match");
    if (n == 0) {
        for (int v = 0; v <= nn; ++v) seg[v] = 0;
        return SDMM_OK;
    }
    HIP_TRY(hipSetDevice(t->device));
    r = st_upload(t);
    if (r) return r;
    int key_bits = 1;
    while ((1 << key_bits) <= nn) ++key_bits;             // keys 0..nn
    const size_t kb = ((sizeof(uint32_t) * (size_t)n + 255) / 256) * 256;
    const size_t sb = ((sizeof(int64_t) * (size_t)(nn + 2) + 255) / 256) * 256;
    const size_t tb = stree_route_temp_bytes((int)n, key_bits);
    const size_t need = 4 * kb + sb + tb + 256;
    if (need > t->scratch_bytes) {
        HIP_TRY(hipStreamSynchronize(t->stream));
        release_dev(t->scratch);
        t->scratch = nullptr;
        HIP_TRY(hipMalloc(&t->scratch, need));
        t->scratch_bytes = need;
    }
    char* b = (char*)t->scratch;
    uint32_t* k0 = (uint32_t*)b;
    uint32_t* k1 = (uint32_t*)(b + kb);
    int32_t* i0 = (int32_t*)(b + 2 * kb);
    int32_t* i1 = (int32_t*)(b + 3 * kb);
    int64_t* sdev = (int64_t*)(b + 4 * kb);
    void* temp = b + 4 * kb + sb;
    float* ox[6];
    for (int i = 0; i < 6; ++i) ox[i] = const_cast<float*>(out->x[i]);
    HIP_TRY(launch_stree_route(t->dnodes, nn, key_bits, to_dev(in), (int)n, k0, k1, i0, i1, temp, tb, sdev, ox,
                               const_cast<float*>(out->w), const_cast<float*>(out->hpdf),
                               const_cast<uint8_t*>(out->is_diffuse), t->stream));
    HIP_TRY(hipMemcpyAsync(seg, sdev, sizeof(int64_t) * (size_t)(nn + 1), hipMemcpyDeviceToHost, t->stream));
    HIP_TRY(hipStreamSynchronize(t->stream));
    return SDMM_OK;
}


int sdmm_stree_set_stream(sdmm_stree* t, void* hip_stream) {
    if (!t) return fail(SDMM_E_INVALID, "invalid argument");
    HIP_TRY(hipSetDevice(t->device));
    if (t->stream || t->stream_set) {
        HIP_TRY(hipStreamSynchronize(t->stream));   // scratch in use by the old stream
        if (t->own_stream && t->stream) HIP_TRY(hipStreamDestroy(t->stream));
    }
    t->stream = (hipStream_t)hip_stream;   // taken literally: NULL is the HIP null stream
    t->own_stream = false;
    t->stream_set = true;
    return SDMM_OK;
}

void* sdmm_stree_get_stream(const sdmm_stree* t) { return t ? (void*)t->stream : nullptr; }

}  // extern "C"

namespace {

// Per-node mixture table for the wavefront; re-uploaded only when it changes
// (the host copy stays alive as the source of the async copy until then).
int st_upload_table(sdmm_stree* t, const sdmm_mix* const* node_mix) {
    const size_t nn = t->nodes.size();
    std::vector<GuideMixHost> tab(nn);
    std::vector<const float*> cc(nn, nullptr);
    int kmax = 0, cap = kGuideCapMax;   // (lowered to the bound mixtures' capacities)
    t->mix_streams.clear();
    for (size_t i = 0; i < nn; ++i) {
        const sdmm_mix* m = node_mix[i];
        tab[i] = GuideMixHost{nullptr, 0, 0};
        if (!m || !m->initialised) continue;
        if (m->device != t->device) return fail(SDMM_E_INVALID, "wavefront: mixture on another device");
        tab[i] = GuideMixHost{m->gp, m->Kp, m->K};
        cc[i] = m->C.condCov;
        kmax = std::max(kmax, m->K);
        cap = std::min(cap, m->guide_cap);
        if (m->stream != t->stream &&
            std::find(t->mix_streams.begin(), t->mix_streams.end(), m->stream) == t->mix_streams.end())
            t->mix_streams.push_back(m->stream);
    }
    while (t->mix_events.size() < t->mix_streams.size()) {
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        t->mix_events.push_back(e);
    }
    bool same = tab.size() == t->tab_host.size() && cc == t->cc_host;
    for (size_t i = 0; same && i < nn; ++i) same = !(tab[i] != t->tab_host[i]);
    t->tab_kmax = kmax;
    t->tab_cap = cap;
    t->tab_valid = true;
    if (same && t->dtab) return SDMM_OK;
    t->published = false;
    HIP_TRY(hipStreamSynchronize(t->stream));   // the previous copy may still read tab_host
    const size_t nb = nn ? nn : 1;
    const size_t bytes = (sizeof(GuideMixHost) + sizeof(const float*)) * nb;
    if (bytes > t->dtab_cap) {
        release_dev(t->dtab);
        t->dtab = nullptr;
        HIP_TRY(hipMalloc(&t->dtab, bytes));
        t->dtab_cap = bytes;
    }
    t->dcctab = (char*)t->dtab + sizeof(GuideMixHost) * nb;
    t->tab_host.swap(tab);
    t->cc_host.swap(cc);
    HIP_TRY(hipMemcpyAsync(t->dtab, t->tab_host.data(), sizeof(GuideMixHost) * nn, hipMemcpyHostToDevice,
                           t->stream));
    HIP_TRY(hipMemcpyAsync(t->dcctab, t->cc_host.data(), sizeof(const float*) * nn, hipMemcpyHostToDevice,
                           t->stream));
    return SDMM_OK;
}

// The wavefronts' common prologue: device nodes and mixture table current,
// scratch for nq queries, the tree's stream ordered after the mixtures'
// pending work on their own streams.  *cus: the device's CUs.
int st_prepare(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, int* cus) {
    HIP_TRY(hipSetDevice(t->device));
    int r = st_upload(t);
    if (r) return r;
    if (node_mix) {
        r = st_upload_table(t, node_mix);
        if (r) return r;
    } else if (!t->tab_valid) {
        return fail(SDMM_E_STATE, "wavefront: no mixtures bound to the current tree (sdmm_stree_bind_mixtures)");
    }
    r = grow_guide_scratch(t->guide_fb, t->guide_fb_cap, t->guide_sort, t->stream, nq);
    if (r) return r;
    for (size_t i = 0; i < t->mix_streams.size(); ++i) {
        HIP_TRY(hipEventRecord(t->mix_events[i], t->mix_streams[i]));
        HIP_TRY(hipStreamWaitEvent(t->stream, t->mix_events[i], 0));
    }
    *cus = 256;
    (void)hipDeviceGetAttribute(cus, hipDeviceAttributeMultiprocessorCount, t->device);
    if (*cus <= 0) *cus = 256;
    return SDMM_OK;
}

// smallest tree wavefront served in coherent order: below it the batch is
// served as given -- the sort's ~10 launches cost more than the coherence
// they buy on a small batch (round 4: a minimum of 64 K / 256 K or no sort at
// all measured 11.9 / 13.6 / 20.5 ms per Cornell K = 128 guided pass against
// 11.4 ms at 16 K)
constexpr int64_t kTreeOrderMin = 1 << 14;

int st_guide(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
             const float* const u[3], const float* const dgiven[3], float* const d[3], float* pdf, int32_t* comp,
             int32_t* node_out, const uint8_t* pmode = nullptr) {
    int cus = 256;
    const int r = st_prepare(t, node_mix, nq, &cus);
    if (r) return r;
    const GuideSortScratch* sort = (nq >= kTreeOrderMin) ? &t->guide_sort : nullptr;
    HIP_TRY(launch_guide_tree(t->dnodes, t->dtab, t->tab_kmax, nq, c, u, dgiven, d, pdf, comp, node_out,
                              norm_const(2), norm_const(3), t->tab_cap, t->guide_fb, t->guide_fb + 1,
                              cus, t->stream, sort, pmode,
                              // the NaN hand-off list of the group fallback: the
                              // Morton keys' input buffer, free once the order is built
                              (int*)t->guide_sort.keys[0], (int)t->nodes.size()));
    return SDMM_OK;
}

int st_guide_product(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
                     const float* const u[3], const float* choice, const float* const dgiven[3],
                     const sdmm_bsdf_table* bsdf, const int32_t* material, const float* const frame[9],
                     float* const d[3], float* pdf, int32_t* comp, float* heuristic, int32_t* node_out) {
    int cus = 256;
    const int r = st_prepare(t, node_mix, nq, &cus);
    if (r) return r;
    const GuideSortScratch* sort = (nq >= kTreeOrderMin) ? &t->guide_sort : nullptr;
    HIP_TRY(launch_guide_product_tree(t->dnodes, t->dtab, t->dcctab, t->tab_kmax, nq, c, u, choice, dgiven, d, pdf,
                                      comp, node_out, material, frame, heuristic, bsdf->weights, bsdf->means,
                                      bsdf->covs, bsdf->diffuse, bsdf->B, bsdf->M, norm_const(2), norm_const(3),
                                      t->tab_cap, t->guide_fb, t->guide_fb + 1, cus, t->stream, sort,
                                      &t->product_scratch, (int)t->nodes.size()));
    return SDMM_OK;
}

// ---------------------------------------------------------------------------
// Guide contexts (round 6): the reference's render workers
// call create_conditional / sample / pdf concurrently, each with thread_local
// scratch (sdmm_proc.cpp:1086-1106).  A context is one worker's: its own
// stream and guided-batch / product scratch.  Its wavefront calls read the
// tree's device nodes and bound mixture table -- immutable once the tree is
// published -- and write only the context's scratch and the caller's planes,
// so contexts run at once from different host threads without a lock.
}  // namespace

struct sdmm_guide_ctx {
    sdmm_stree* t = nullptr;
    int device = 0;
    int cus = 256;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int* guide_fb = nullptr;
    int64_t guide_fb_cap = 0;
    GuideSortScratch guide_sort{};
    ProductScratch product_scratch{};
    int64_t order_min = 0;   // smallest call served in leaf-major order
    char* hbuf = nullptr;    // host-batch planes on the device (sdmm_ctx_guide_pdf_host_batch)
    int64_t hbuf_cap = 0;    // queries it holds
};

namespace {

int ctx_prepare(sdmm_guide_ctx* g, int64_t nq) {
    const sdmm_stree* t = g->t;
    if (!t->published || t->dirty || !t->tab_valid)
        return fail(SDMM_E_STATE, "guide context: the tree changed since sdmm_stree_publish (publish it again)");
    HIP_TRY(hipSetDevice(g->device));
    return grow_guide_scratch(g->guide_fb, g->guide_fb_cap, g->guide_sort, g->stream, nq);
}

}  // namespace

extern "C" {

int sdmm_stree_bind_mixtures(sdmm_stree* t, const sdmm_mix* const* node_mix) {
    if (!t || !node_mix) return fail(SDMM_E_INVALID, "invalid argument");
    HIP_TRY(hipSetDevice(t->device));
    int r = st_upload(t);
    if (r) return r;
    return st_upload_table(t, node_mix);
}

int sdmm_stree_publish(sdmm_stree* t, const sdmm_mix* const* node_mix) {
    if (!t) return fail(SDMM_E_INVALID, "invalid argument");
    HIP_TRY(hipSetDevice(t->device));
    int r = st_upload(t);
    if (r) return r;
    if (node_mix) {
        r = st_upload_table(t, node_mix);
        if (r) return r;
    } else if (!t->tab_valid) {
        return fail(SDMM_E_STATE, "sdmm_stree_publish: no mixtures bound to the current tree");
    }
    // the bound mixtures' pending work (EM steps, copies) and the uploads
    for (hipStream_t st : t->mix_streams) HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipStreamSynchronize(t->stream));
    t->published = true;
    return SDMM_OK;
}

int sdmm_guide_ctx_create(sdmm_stree* t, void* hip_stream, sdmm_guide_ctx** out) {
    if (!t || !out) return fail(SDMM_E_INVALID, "invalid argument");
    *out = nullptr;
    HIP_TRY(hipSetDevice(t->device));
    sdmm_guide_ctx* g = new (std::nothrow) sdmm_guide_ctx();
    if (!g) return fail(SDMM_E_NOMEM, "out of host memory");
    g->t = t;
    g->device = t->device;
    g->order_min = kTreeOrderMin;
    if (const char* e = std::getenv("SDMM_CTX_ORDER_MIN")) g->order_min = std::atoll(e);   // (A/B switch)
    (void)hipDeviceGetAttribute(&g->cus, hipDeviceAttributeMultiprocessorCount, t->device);
    if (g->cus <= 0) g->cus = 256;
    if (hip_stream) {
        g->stream = (hipStream_t)hip_stream;
    } else {
        const hipError_t e = hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete g;
            return fail(SDMM_E_HIP, std::string("sdmm_guide_ctx_create: ") + hipGetErrorString(e));
        }
        g->own_stream = true;
    }
    *out = g;
    return SDMM_OK;
}

void sdmm_guide_ctx_destroy(sdmm_guide_ctx* g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    (void)hipStreamSynchronize(g->stream);
    if (g->guide_fb) (void)hipFree(g->guide_fb);
    if (g->product_scratch.base) (void)hipFree(g->product_scratch.base);
    if (g->hbuf) (void)hipFree(g->hbuf);
    if (g->own_stream) (void)hipStreamDestroy(g->stream);
    delete g;
}

void* sdmm_guide_ctx_stream(const sdmm_guide_ctx* g) { return g ? (void*)g->stream : nullptr; }

int sdmm_ctx_guide_pdf_wavefront(sdmm_guide_ctx* g, int64_t nq, const float* const c[3], const float* const u[3],
                                 const float* const dgiven[3], const uint8_t* pdf_mode, float* const d[3], float* pdf,
                                 int32_t* comp, int32_t* node_out) {
    if (!g || nq < 0) return fail(SDMM_E_INVALID, "invalid argument");
    if (nq == 0) return SDMM_OK;
    if (!c || !u || !dgiven || !pdf_mode || !d || !pdf || !comp) return fail(SDMM_E_INVALID, "invalid argument");
    const int r = ctx_prepare(g, nq);
    if (r) return r;
    const sdmm_stree* t = g->t;
    const GuideSortScratch* sort = (nq >= g->order_min) ? &g->guide_sort : nullptr;
    HIP_TRY(launch_guide_tree(t->dnodes, t->dtab, t->tab_kmax, nq, c, u, dgiven, d, pdf, comp, node_out,
                              norm_const(2), norm_const(3), t->tab_cap, g->guide_fb, g->guide_fb + 1, g->cus,
                              g->stream, sort, pdf_mode, (int*)g->guide_sort.keys[0], (int)t->nodes.size()));
    return SDMM_OK;
}

int sdmm_pinned_alloc(size_t bytes, void** out) {
    if (!out) return fail(SDMM_E_INVALID, "invalid argument");
    *out = nullptr;
    if (bytes == 0) return SDMM_OK;
    HIP_TRY(hipHostMalloc(out, bytes, hipHostMallocDefault));
    return SDMM_OK;
}
void sdmm_pinned_free(void* p) {
    if (p) (void)hipHostFree(p);
}

// The requests' planes stacked on the device (plane p of the batch at
// din + p * N, request r's queries at offset off_r), one wavefront, outputs
// copied back per request; 2-D copies carry a request's planes in one call.
int sdmm_ctx_guide_pdf_host_batch(sdmm_guide_ctx* g, int nreq, const sdmm_guide_host_req* reqs) {
    if (!g || nreq < 0 || (nreq > 0 && !reqs)) return fail(SDMM_E_INVALID, "invalid argument");
    int64_t N = 0;
    auto pinned = [](const void* p) {
        hipPointerAttribute_t a{};
        return hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost;
    };
    for (int i = 0; i < nreq; ++i) {
        const sdmm_guide_host_req& q = reqs[i];
        if (q.n < 0) return fail(SDMM_E_INVALID, "sdmm_ctx_guide_pdf_host_batch: negative request size");
        if (q.n == 0) continue;
        if (!q.in || !q.mode || !q.out || !q.comp || q.in_stride < q.n || q.out_stride < q.n)
            return fail(SDMM_E_INVALID, "sdmm_ctx_guide_pdf_host_batch: invalid request");
        if (!pinned(q.in) || !pinned(q.mode) || !pinned(q.out) || !pinned(q.comp)) {
            (void)hipGetLastError();   // (the query's own error on pageable memory)
            return fail(SDMM_E_INVALID, "sdmm_ctx_guide_pdf_host_batch: host buffers must be pinned");
        }
        N += q.n;
    }
    if (N == 0) return SDMM_OK;
    int r = ctx_prepare(g, N);
    if (r) return r;
    // planes: in 9 + out 4 floats, comp int32, mode u8 per query
    const size_t per = 13 * sizeof(float) + sizeof(int32_t) + 1;
    if (N > g->hbuf_cap) {
        if (g->hbuf) {
            HIP_TRY(hipStreamSynchronize(g->stream));
            (void)hipFree(g->hbuf);
            g->hbuf = nullptr;
            g->hbuf_cap = 0;
        }
        const int64_t cap = N + N / 4;
        HIP_TRY(hipMalloc((void**)&g->hbuf, per * (size_t)cap + 256));
        g->hbuf_cap = cap;
    }
    float* din = (float*)g->hbuf;
    float* dout = din + 9 * N;
    int32_t* dcomp = (int32_t*)(dout + 4 * N);
    uint8_t* dmode = (uint8_t*)(dcomp + N);
    const size_t dp = sizeof(float) * (size_t)N;
    int64_t off = 0;
    for (int i = 0; i < nreq; ++i) {
        const sdmm_guide_host_req& q = reqs[i];
        if (q.n == 0) continue;
        HIP_TRY(hipMemcpy2DAsync(din + off, dp, q.in, sizeof(float) * (size_t)q.in_stride, sizeof(float) * (size_t)q.n,
                                 9, hipMemcpyHostToDevice, g->stream));
        HIP_TRY(hipMemcpyAsync(dmode + off, q.mode, (size_t)q.n, hipMemcpyHostToDevice, g->stream));
        off += q.n;
    }
    const float* c[3] = {din, din + N, din + 2 * N};
    const float* u[3] = {din + 3 * N, din + 4 * N, din + 5 * N};
    const float* dg[3] = {din + 6 * N, din + 7 * N, din + 8 * N};
    float* d[3] = {dout, dout + N, dout + 2 * N};
    r = sdmm_ctx_guide_pdf_wavefront(g, N, c, u, dg, dmode, d, dout + 3 * N, dcomp, nullptr);
    if (r) return r;
    off = 0;
    for (int i = 0; i < nreq; ++i) {
        const sdmm_guide_host_req& q = reqs[i];
        if (q.n == 0) continue;
        HIP_TRY(hipMemcpy2DAsync(q.out, sizeof(float) * (size_t)q.out_stride, dout + off, dp,
                                 sizeof(float) * (size_t)q.n, 4, hipMemcpyDeviceToHost, g->stream));
        HIP_TRY(hipMemcpyAsync(q.comp, dcomp + off, sizeof(int32_t) * (size_t)q.n, hipMemcpyDeviceToHost, g->stream));
        off += q.n;
    }
    HIP_TRY(hipStreamSynchronize(g->stream));
    return SDMM_OK;
}

int sdmm_ctx_guide_product_wavefront(sdmm_guide_ctx* g, int64_t nq, const float* const c[3], const float* const u[3],
                                     const float* choice, const float* const dgiven[3], const sdmm_bsdf_table* bsdf,
                                     const int32_t* material, const float* const frame[9], float* const d[3],
                                     float* pdf, int32_t* comp, float* heuristic, int32_t* node_out) {
    if (!g || nq < 0) return fail(SDMM_E_INVALID, "invalid argument");
    if (nq == 0) return SDMM_OK;
    if (!c || !u || !d || !pdf || !comp || (choice && !dgiven)) return fail(SDMM_E_INVALID, "invalid argument");
    int r = check_bsdf(bsdf, material, frame);
    if (r) return r;
    r = ctx_prepare(g, nq);
    if (r) return r;
    const sdmm_stree* t = g->t;
    const GuideSortScratch* sort = (nq >= g->order_min) ? &g->guide_sort : nullptr;
    HIP_TRY(launch_guide_product_tree(t->dnodes, t->dtab, t->dcctab, t->tab_kmax, nq, c, u, choice,
                                      choice ? dgiven : nullptr, d, pdf, comp, node_out, material, frame, heuristic,
                                      bsdf->weights, bsdf->means, bsdf->covs, bsdf->diffuse, bsdf->B, bsdf->M,
                                      norm_const(2), norm_const(3), t->tab_cap, g->guide_fb, g->guide_fb + 1, g->cus,
                                      g->stream, sort, &g->product_scratch, (int)t->nodes.size()));
    return SDMM_OK;
}

int sdmm_guide_wavefront(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
                         const float* const u[3], float* const d[3], float* pdf, int32_t* comp,
                         int32_t* node_out) {
    if (!t || nq < 0) return fail(SDMM_E_INVALID, "invalid argument");
    if (nq == 0) return SDMM_OK;
    if (!c || !u || !d || !pdf || !comp) return fail(SDMM_E_INVALID, "invalid argument");
    return st_guide(t, node_mix, nq, c, u, nullptr, d, pdf, comp, node_out);
}

int sdmm_guide_pdf_wavefront(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
                             const float* const u[3], const float* const dgiven[3], const uint8_t* pdf_mode,
                             float* const d[3], float* pdf, int32_t* comp, int32_t* node_out) {
    if (!t || nq < 0) return fail(SDMM_E_INVALID, "invalid argument");
    if (nq == 0) return SDMM_OK;
    if (!c || !u || !dgiven || !pdf_mode || !d || !pdf || !comp) return fail(SDMM_E_INVALID, "invalid argument");
    return st_guide(t, node_mix, nq, c, u, dgiven, d, pdf, comp, node_out, pdf_mode);
}

int sdmm_pdf_wavefront(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
                       const float* const d[3], float* pdf) {
    if (!t || nq < 0) return fail(SDMM_E_INVALID, "invalid argument");
    if (nq == 0) return SDMM_OK;
    if (!c || !d || !pdf) return fail(SDMM_E_INVALID, "invalid argument");
    return st_guide(t, node_mix, nq, c, nullptr, d, nullptr, pdf, nullptr, nullptr);
}

int sdmm_guide_product_wavefront(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
                                 const float* const u[3], const float* choice, const float* const dgiven[3],
                                 const sdmm_bsdf_table* bsdf, const int32_t* material, const float* const frame[9],
                                 float* const d[3], float* pdf, int32_t* comp, float* heuristic, int32_t* node_out) {
    if (!t || nq < 0) return fail(SDMM_E_INVALID, "invalid argument");
    if (nq == 0) return SDMM_OK;
    if (!c || !u || !d || !pdf || !comp || (choice && !dgiven)) return fail(SDMM_E_INVALID, "invalid argument");
    const int r = check_bsdf(bsdf, material, frame);
    if (r) return r;
    return st_guide_product(t, node_mix, nq, c, u, choice, choice ? dgiven : nullptr, bsdf, material, frame, d, pdf,
                            comp, heuristic, node_out);
}

int sdmm_pdf_product_wavefront(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
                               const float* const d[3], const sdmm_bsdf_table* bsdf, const int32_t* material,
                               const float* const frame[9], float* pdf, float* heuristic) {
    if (!t || nq < 0) return fail(SDMM_E_INVALID, "invalid argument");
    if (nq == 0) return SDMM_OK;
    if (!c || !d || !pdf) return fail(SDMM_E_INVALID, "invalid argument");
    const int r = check_bsdf(bsdf, material, frame);
    if (r) return r;
    return st_guide_product(t, node_mix, nq, c, nullptr, nullptr, d, bsdf, material, frame, nullptr, pdf, nullptr,
                            heuristic, nullptr);
}

}  // extern "C"


// ---------------------------------------------------------------------------
// the device Li (render_api.cpp) runs on the tree's stream
namespace sdmm_detail {
int tree_stream(sdmm_stree* t, hipStream_t* st) {
    HIP_TRY(hipSetDevice(t->device));
    const int r = st_upload(t);
    if (r) return r;
    *st = t->stream;
    return SDMM_OK;
}
// the device count of full-K (fallback) queries of the tree's last guided call
const int* tree_fallback_count(const sdmm_stree* t) { return t->guide_fb; }
}  // namespace sdmm_detail

extern "C" {

}  // extern "C"

namespace sdmm_detail {
// sdmm_push_training with reuse_counts: the call directly follows a count-only
// call with the same tree, paths, saved_per_path and seed, so the per-path
// record offsets still in the tree's scratch are reused (no second producer
// count pass, no second synchronisation).  Without seg and lost nothing is read
// back: the call returns with the writes in flight on the tree's stream.
int push_training_ex(sdmm_stree* t, const sdmm_path_vertices* v, int saved_per_path, uint64_t seed,
                     const sdmm_training_out* out, int64_t* n_out, int64_t* seg, int64_t* lost, bool reuse_counts,
                     int64_t known_count);
}  // namespace sdmm_detail

extern "C" {

int sdmm_push_training(sdmm_stree* t, const sdmm_path_vertices* v, int saved_per_path, uint64_t seed,
                       const sdmm_training_out* out, int64_t* n_out, int64_t* seg, int64_t* lost) {
    int64_t hl = 0;
    const int r = sdmm_detail::push_training_ex(t, v, saved_per_path, seed, out, n_out, seg, &hl, false, -1);
    if (lost) *lost = hl;
    return r;
}

}  // extern "C"

int sdmm_detail::push_training_ex(sdmm_stree* t, const sdmm_path_vertices* v, int saved_per_path, uint64_t seed,
                                  const sdmm_training_out* out, int64_t* n_out, int64_t* seg, int64_t* lost,
                                  bool reuse_counts, int64_t known_count) {
    if (!t || !v || !n_out || saved_per_path < 1 || v->n_paths < 0 || v->max_vertices < 1 ||
        (v->n_paths > 0 && (!v->rec || !v->nv)))
        return fail(SDMM_E_INVALID, "invalid argument");
    const int64_t P = v->n_paths;
    const int nn = (int)t->nodes.size();
    *n_out = 0;
    if (lost) *lost = 0;
    if (P == 0) {
        if (seg) for (int i = 0; i <= nn; ++i) seg[i] = 0;
        return SDMM_OK;
    }
    if (P > INT32_MAX - 1) return fail(SDMM_E_INVALID, "push_training: at most 2^31 - 2 paths");
    HIP_TRY(hipSetDevice(t->device));
    int r = st_upload(t);
    if (r) return r;
    int key_bits = 1;
    while ((1 << key_bits) <= nn) ++key_bits;
    const int64_t max_rec = P * 3 * (int64_t)std::min(saved_per_path, v->max_vertices);
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t tb = al(produce_temp_bytes(P + 1, max_rec, key_bits));
    const size_t cb = al(sizeof(int64_t) * (size_t)(P + 1));
    // the records' count first: the sorted arrays are sized by it
    const size_t need0 = 2 * cb + tb + al(sizeof(int64_t) * (size_t)(nn + 2)) + 256;
    if (need0 > t->scratch_bytes) {
        HIP_TRY(hipStreamSynchronize(t->stream));
        release_dev(t->scratch);
        t->scratch = nullptr;
        HIP_TRY(hipMalloc(&t->scratch, need0));
        t->scratch_bytes = need0;
    }
    PathsDev PD{};
    PD.rec = const_cast<float*>(v->rec);
    PD.nv = const_cast<int*>(v->nv);
    PD.V = v->max_vertices;
    PD.P = P;
    char* b = (char*)t->scratch;
    int64_t* count = (int64_t*)b;
    int64_t* offs = (int64_t*)(b + cb);
    void* temp = b + 2 * cb;
    int64_t n_rec = known_count;
    if (!reuse_counts || known_count < 0) {
        HIP_TRY(hipMemsetAsync(count + P, 0, sizeof(int64_t), t->stream));
        HIP_TRY(launch_produce_count(t->dnodes, PD, v->path0, saved_per_path, seed, count, offs, temp, tb,
                                     t->stream));
        HIP_TRY(hipMemcpyAsync(&n_rec, offs + P, sizeof(int64_t), hipMemcpyDeviceToHost, t->stream));
        HIP_TRY(hipStreamSynchronize(t->stream));
    }
    *n_out = n_rec;
    if (!out) return SDMM_OK;   // count only
    if (n_rec > out->capacity) return fail(SDMM_E_INVALID, "push_training: output capacity too small");
    if (n_rec > 0) {
        for (int i = 0; i < 6; ++i)
            if (!out->x[i]) return fail(SDMM_E_INVALID, "push_training: output plane missing");
        if (!out->w) return fail(SDMM_E_INVALID, "push_training: output weight plane missing");
    }
    const size_t kb = al(sizeof(uint32_t) * (size_t)std::max<int64_t>(n_rec, 1));
    const size_t qb = al(sizeof(int64_t) * (size_t)std::max<int64_t>(n_rec, 1));
    const size_t sb = al(sizeof(int64_t) * (size_t)(nn + 2));
    const size_t rb = al((size_t)48 * (size_t)std::max<int64_t>(n_rec, 1));   // staged records (render.hip)
    const size_t need = 2 * cb + tb + 2 * kb + 2 * qb + sb + 256 + rb;
    if (need > t->scratch_bytes) {
        // keep the offsets: copy them out through a fresh buffer
        void* nb = nullptr;
        HIP_TRY(hipMalloc(&nb, need));
        HIP_TRY(hipMemcpyAsync(nb, t->scratch, 2 * cb, hipMemcpyDeviceToDevice, t->stream));
        HIP_TRY(hipStreamSynchronize(t->stream));
        release_dev(t->scratch);
        t->scratch = nb;
        t->scratch_bytes = need;
    }
    b = (char*)t->scratch;
    offs = (int64_t*)(b + cb);
    temp = b + 2 * cb;
    uint32_t* k0 = (uint32_t*)(b + 2 * cb + tb);
    uint32_t* k1 = (uint32_t*)(b + 2 * cb + tb + kb);
    int64_t* q0 = (int64_t*)(b + 2 * cb + tb + 2 * kb);
    int64_t* q1 = (int64_t*)(b + 2 * cb + tb + 2 * kb + qb);
    int64_t* sdev = (int64_t*)(b + 2 * cb + tb + 2 * kb + 2 * qb);
    int* dlost = (int*)(b + 2 * cb + tb + 2 * kb + 2 * qb + sb);
    void* recs = b + 2 * cb + tb + 2 * kb + 2 * qb + sb + 256;
    HIP_TRY(hipMemsetAsync(dlost, 0, sizeof(int), t->stream));
    if (n_rec == 0) HIP_TRY(hipMemsetAsync(sdev, 0, sizeof(int64_t) * (size_t)(nn + 1), t->stream));
    float* ox[6];
    for (int i = 0; i < 6; ++i) ox[i] = out->x[i];
    float* on[3] = {out->normal[0], out->normal[1], out->normal[2]};
    HIP_TRY(launch_produce_records(t->dnodes, nn, key_bits, PD, v->path0, saved_per_path, seed, offs, n_rec, k0, k1,
                                   q0, q1, recs, temp, tb, sdev, dlost, ox, out->normal[0] ? on : nullptr, out->w,
                                   out->stats, out->node, out->source, t->stream));
    if (!seg && !lost) return SDMM_OK;   // writes in flight on the tree's stream
    int hl = 0;
    if (seg) HIP_TRY(hipMemcpyAsync(seg, sdev, sizeof(int64_t) * (size_t)(nn + 1), hipMemcpyDeviceToHost, t->stream));
    HIP_TRY(hipMemcpyAsync(&hl, dlost, sizeof(int), hipMemcpyDeviceToHost, t->stream));
    HIP_TRY(hipStreamSynchronize(t->stream));
    if (lost) *lost = hl;
    return SDMM_OK;
}
