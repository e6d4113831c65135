// sdmm_amd.hpp -- C++ host-side mirror of the guiding interface the Mitsuba
// `sdmm` integrator plugin uses, layered over the C ABI (include/sdmm_gpu.h).
//
// The plugin (mitsuba/src/integrators/sdmm/volpath_sdmm.cpp, sdmm_proc.cpp)
// drives sdmm-lib through a handful of free functions on per-leaf contexts:
//   sdmm::initialize(sdmm, em, data, rng, n_spatial, dist)  volpath_sdmm.cpp:135
//   sdmm::em_step(sdmm, em, training_data)                  volpath_sdmm.cpp:220,304
//   sdmm::prepare(conditioner, sdmm)                        volpath_sdmm.cpp:237,307
//   sdmm::create_conditional(conditioner, cond, conditional) sdmm_proc.cpp:368
//   conditional.sample(rng, embedded, inv_jacobian, tangent) sdmm_proc.cpp:411-421
//   posterior + hsum_nested -> gmmPdf                        sdmm_proc.cpp:539-545
//   context.data.push_back(point6, normal3, weight)          sdmm_proc.cpp:894-902
// This header offers the same verbs with the same argument meaning, but the
// per-bounce calls are batched: a Mitsuba worker appends its bounce queries to
// a GuidingBatch and the whole wavefront is answered by one kernel launch.
// Errors surface as sdmm_amd::Error (the C ABI itself never throws).
#pragma once

#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <sstream>
#include <thread>
#include <unordered_set>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/sdmm_gpu.h"

namespace sdmm_amd {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

// The calling thread, for error reports (several render / optimisation
// threads call the library at once).
inline std::string thread_tag() {
    std::ostringstream o;
    o << std::this_thread::get_id();
    return o.str();
}

// SDMM_AMD_DEBUG_SYNC=1: every mixture call is followed by a synchronisation
// of the handle's stream, so an asynchronous fault (a kernel or copy the call
// enqueued) is reported by the call and the thread that caused it instead of
// by a later, unrelated call.  Debugging aid only (it serialises the stream).
inline bool debug_sync() {
    static const bool on = [] {
        const char* e = std::getenv("SDMM_AMD_DEBUG_SYNC");
        return e && *e && *e != '0';
    }();
    return on;
}

inline void check(int rc, const char* where) {
    if (rc != SDMM_OK) throw Error(rc, std::string(where) + " [thread " + thread_tag() + "]: " + sdmm_last_error());
}
// ... for a call on handle h: with SDMM_AMD_DEBUG_SYNC the enqueued work is
// checked before returning
inline void check(int rc, const char* where, sdmm_mix* h) {
    check(rc, where);
    if (h && debug_sync()) {
        const int r = sdmm_synchronize(h);
        if (r != SDMM_OK)
            throw Error(r, std::string(where) + " [debug sync, thread " + thread_tag() + "]: " + sdmm_last_error());
    }
}

// jmm::Samples / sdmm::Data: SoA training data, appended from many render
// threads (push_back_synchronized, samples.h:250-256), handed to em_step.
class TrainingData {
public:
    void reserve(size_t n) {
        for (auto& p : x_) p.reserve(n);
        w_.reserve(n);
        nrm_.reserve(3 * n);
    }
    // point = (normalised position, unit direction), normal, weight.
    // Zero weights are dropped like Samples::push_back (samples.h:281-283).
    bool push_back(const float point[6], const float normal[3], float weight) {
        if (weight == 0.0f) return false;
        std::lock_guard<std::mutex> lock(mutex_);
        for (int i = 0; i < 6; ++i) x_[i].push_back(point[i]);
        w_.push_back(weight);
        nrm_.insert(nrm_.end(), normal, normal + 3);
        return true;
    }
    size_t size() const { return w_.size(); }
    void clear() {
        for (auto& p : x_) p.clear();
        w_.clear();
        nrm_.clear();
    }
    sdmm_samples view() const {
        sdmm_samples s{};
        for (int i = 0; i < 6; ++i) s.x[i] = x_[i].data();
        s.w = w_.data();
        s.hpdf = nullptr;
        s.is_diffuse = nullptr;
        s.n = (int64_t)w_.size();
        return s;
    }
    const float* normals() const { return nrm_.data(); }
    const float* weights() const { return w_.data(); }
    const std::vector<float>& plane(int i) const { return x_[i]; }

private:
    std::vector<float> x_[6];
    std::vector<float> w_;
    std::vector<float> nrm_;
    std::mutex mutex_;
};

// One spatio-directional mixture + its stepwise EM state on one GPU
// (jmm::MixtureModel<6,K,3,...> + StepwiseTangentEM, i.e. sdmm::SDMM + sdmm::EM).
class Mixture {
    explicit Mixture(sdmm_mix* h) : h_(h) {}

public:
    explicit Mixture(int K, int device = 0, const sdmm_em_params* params = nullptr) {
        check(sdmm_create(K, params, device, &h_), "sdmm_create", h_);
    }
    ~Mixture() { sdmm_destroy(h_); }
    // take ownership of a handle (checkpoint loading)
    static std::unique_ptr<Mixture> adopt(sdmm_mix* h) { return std::unique_ptr<Mixture>(new Mixture(h)); }
    // jmm MixtureModel::save/load (mixture_model.h:315-326): canonical +
    // derived arrays and the stepwise state, restored bitwise
    void save_json(const std::string& path) const { check(sdmm_mix_save_json(h_, path.c_str()), "sdmm_mix_save_json"); }
    static std::unique_ptr<Mixture> load_json(const std::string& path, int device = 0) {
        sdmm_mix* h = nullptr;
        check(sdmm_mix_load_json(path.c_str(), device, &h), "sdmm_mix_load_json");
        return adopt(h);
    }
    Mixture(const Mixture&) = delete;
    Mixture& operator=(const Mixture&) = delete;

    int components() const { return sdmm_num_components(h_); }
    sdmm_mix* handle() { return h_; }
    void set_stream(void* hip_stream) { check(sdmm_set_stream(h_, hip_stream), "sdmm_set_stream", h_); }
    void synchronize() { check(sdmm_synchronize(h_), "sdmm_synchronize"); }

    // sdmm::initialize: seed positions = the first K/8 training points
    // (uniformHemisphereInit, mixture_model_init.h:139-141).
    void initialize(const TrainingData& data, float depth_prior, float spatial_distance, uint64_t seed) {
        const int n_pos = components() / 8;
        if ((int64_t)data.size() < n_pos) throw Error(SDMM_E_INVALID, "initialize: too few samples");
        std::vector<float> pos(3 * n_pos);
        for (int i = 0; i < n_pos; ++i)
            for (int d = 0; d < 3; ++d) pos[3 * i + d] = data.plane(d)[i];
        check(sdmm_init_hemisphere(h_, pos.data(), data.normals(), n_pos, depth_prior, spatial_distance, seed),
              "sdmm_init_hemisphere", h_);
    }

    // sdmm::em_step + sdmm::prepare on host-resident training data.
    void em_step(const TrainingData& data, int iterations = 1) {
        sdmm_samples s = data.view();
        check(sdmm_em_step_host(h_, &s, iterations), "sdmm_em_step_host", h_);
    }
    // ... or on device-resident SoA planes (no PCIe copy).
    void em_step_device(const sdmm_samples& device_samples, int iterations = 1) {
        check(sdmm_em_step(h_, &device_samples, iterations), "sdmm_em_step", h_);
    }

    // em.iterations_run (the plugin's 2-while-below-4 schedule, volpath_sdmm.cpp:299-302)
    int iterations_run() const {
        const sdmm_mix* h = h_;
        int it = 0;
        check(sdmm_iterations_run(&h, 1, &it), "sdmm_iterations_run", h_);
        return it;
    }

    // sdmm::save_json counterpart: export the canonical parameters.
    void params(std::vector<float>& weights, std::vector<float>& means, std::vector<float>& covs) const {
        const int K = sdmm_num_components(h_);
        weights.resize(K);
        means.resize(6 * K);
        covs.resize(25 * K);
        sdmm_params_out o{};
        o.weights = weights.data();
        o.mean = means.data();
        o.cov = covs.data();
        check(sdmm_get_params(h_, &o), "sdmm_get_params", h_);
    }

private:
    sdmm_mix* h_ = nullptr;
};

// The plugin's per-leaf optimisation loop (volpath_sdmm.cpp:287-311: one
// sdmm::em_step per tree leaf on a tev::ThreadPool) as one batched launch:
// leaves[i] takes `iterations` EM steps over samples [seg[i], seg[i+1]) of the
// device planes `device_samples` (the leaves' training data back to back).
// Bitwise the same as leaves[i]->em_step_device(leaf i) one by one.
inline void em_step_leaves(const std::vector<Mixture*>& leaves, const sdmm_samples& device_samples,
                           const std::vector<int64_t>& seg, int iterations = 1) {
    if (seg.size() != leaves.size() + 1) throw Error(SDMM_E_INVALID, "em_step_leaves: seg needs leaves + 1 offsets");
    std::vector<sdmm_mix*> h(leaves.size());
    for (size_t i = 0; i < leaves.size(); ++i) h[i] = leaves[i]->handle();
    check(sdmm_em_step_batched(h.data(), (int)h.size(), &device_samples, seg.data(), iterations),
          "sdmm_em_step_batched");
}
// ... on host-resident training data: the leaves' TrainingData concatenated.
inline void em_step_leaves(const std::vector<Mixture*>& leaves, const std::vector<const TrainingData*>& data,
                           int iterations = 1) {
    if (data.size() != leaves.size()) throw Error(SDMM_E_INVALID, "em_step_leaves: one TrainingData per leaf");
    std::vector<int64_t> seg(leaves.size() + 1, 0);
    for (size_t i = 0; i < data.size(); ++i) seg[i + 1] = seg[i] + data[i]->size();
    const int64_t n = seg.back();
    std::vector<float> planes[7];
    for (auto& p : planes) p.resize((size_t)n);
    for (size_t i = 0; i < data.size(); ++i)
        for (int d = 0; d < 7; ++d) {
            const float* src = d < 6 ? data[i]->plane(d).data() : data[i]->weights();
            std::copy(src, src + data[i]->size(), planes[d].begin() + seg[i]);
        }
    sdmm_samples s{};
    for (int d = 0; d < 6; ++d) s.x[d] = planes[d].data();
    s.w = planes[6].data();
    s.n = n;
    std::vector<sdmm_mix*> h(leaves.size());
    for (size_t i = 0; i < leaves.size(); ++i) h[i] = leaves[i]->handle();
    check(sdmm_em_step_batched_host(h.data(), (int)h.size(), &s, seg.data(), iterations),
          "sdmm_em_step_batched_host");
}

// ... with the plugin's per-leaf iteration counts (2 while iterations_run < 4,
// volpath_sdmm.cpp:299-305).
inline void em_step_leaves(const std::vector<Mixture*>& leaves, const std::vector<const TrainingData*>& data,
                           const std::vector<int>& iterations) {
    if (data.size() != leaves.size() || iterations.size() != leaves.size())
        throw Error(SDMM_E_INVALID, "em_step_leaves: one TrainingData and one iteration count per leaf");
    std::vector<int64_t> seg(leaves.size() + 1, 0);
    for (size_t i = 0; i < data.size(); ++i) seg[i + 1] = seg[i] + data[i]->size();
    const int64_t n = seg.back();
    std::vector<float> planes[7];
    for (auto& p : planes) p.resize((size_t)n);
    for (size_t i = 0; i < data.size(); ++i)
        for (int d = 0; d < 7; ++d) {
            const float* src = d < 6 ? data[i]->plane(d).data() : data[i]->weights();
            std::copy(src, src + data[i]->size(), planes[d].begin() + seg[i]);
        }
    sdmm_samples s{};
    for (int d = 0; d < 6; ++d) s.x[d] = planes[d].data();
    s.w = planes[6].data();
    s.n = n;
    std::vector<sdmm_mix*> h(leaves.size());
    for (size_t i = 0; i < leaves.size(); ++i) h[i] = leaves[i]->handle();
    check(sdmm_em_step_batched_host_iters(h.data(), (int)h.size(), &s, seg.data(), iterations.data()),
          "sdmm_em_step_batched_host_iters");
}

// Guide contexts shared by a renderer's worker threads (sdmm_guide_ctx_*):
// the reference's workers call the conditional concurrently
// (sdmm_proc.cpp:1086-1106); here each guided bounce leases a free context
// (its own stream and scratch on the published tree) for the duration of its
// copies + wavefront + synchronisation.  A pool smaller than the worker count
// keeps the device's hardware queues (GPU_MAX_HW_QUEUES, 4 by default) and
// copy engines from being oversubscribed by many small streams
// (tools/plugin_pattern_bench.py: 16 workers on 16 contexts ran slower than
// on 4).  Contexts are created on first use.
class GuideContextPool {
public:
    GuideContextPool(sdmm_stree* tree, int contexts) : tree_(tree), cap_(contexts > 0 ? contexts : 1) {}
    ~GuideContextPool() {
        for (sdmm_guide_ctx* c : all_) sdmm_guide_ctx_destroy(c);
    }
    GuideContextPool(const GuideContextPool&) = delete;
    GuideContextPool& operator=(const GuideContextPool&) = delete;

    class Lease {
    public:
        Lease(GuideContextPool* p, sdmm_guide_ctx* c) : pool_(p), ctx_(c) {}
        Lease(Lease&& o) noexcept : pool_(o.pool_), ctx_(o.ctx_) { o.ctx_ = nullptr; }
        Lease(const Lease&) = delete;
        Lease& operator=(const Lease&) = delete;
        ~Lease() {
            if (ctx_) pool_->release(ctx_);
        }
        sdmm_guide_ctx* get() const { return ctx_; }
        void* stream() const { return sdmm_guide_ctx_stream(ctx_); }

    private:
        GuideContextPool* pool_;
        sdmm_guide_ctx* ctx_;
    };

    // a free context (blocks while all `contexts` are leased)
    Lease acquire() {
        std::unique_lock<std::mutex> lock(mu_);
        cv_.wait(lock, [&] { return !free_.empty() || (int)all_.size() < cap_; });
        sdmm_guide_ctx* c = nullptr;
        if (!free_.empty()) {
            c = free_.back();
            free_.pop_back();
        } else {
            check(sdmm_guide_ctx_create(tree_, nullptr, &c), "sdmm_guide_ctx_create");
            all_.push_back(c);
        }
        return Lease(this, c);
    }

private:
    void release(sdmm_guide_ctx* c) {
        {
            std::lock_guard<std::mutex> lock(mu_);
            free_.push_back(c);
        }
        cv_.notify_one();
    }
    sdmm_stree* tree_;
    int cap_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<sdmm_guide_ctx*> all_, free_;
};

// Concurrent workers' guided bounces gathered into few large wavefronts
// (round 6).  The per-call cost of a guided wavefront (the leaf-major sort,
// the candidate and full-K kernels' tails, each copy's DMA set-up) is paid
// per CALL, so 16 workers each calling with its own tile run well below one
// call over their union (tools/plugin_pattern_bench.py).
//
// `slots` batches, each with its own guide context and pinned staging in
// batch layout (planes of stride cap).  serve() joins the open batch at the
// next free offset and copies its query planes into the batch's staging
// (host memcpy, the workers in parallel).  The first worker of a batch leads
// it: it waits until the batch holds `target` queries, or every thread that
// ever called serve() is inside serve() (nobody left to wait for), or
// `wait_us` passed; then it closes the batch (later arrivals take the next
// free one), waits for the members' copies and runs ONE
// sdmm_ctx_guide_pdf_host_batch over the staging -- one H2D, one wavefront,
// one D2H -- and wakes the members, who copy their outputs out.  Outputs are
// bitwise those of per-worker calls (every query is independent).
class GuideBatcher {
public:
    GuideBatcher(sdmm_stree* tree, int slots = 2, int64_t target = 1 << 18, int wait_us = 200)
        : tree_(tree), target_(target > 0 ? target : 1), wait_(wait_us > 0 ? wait_us : 0) {
        const int n = slots > 0 ? slots : 1;
        for (int i = 0; i < n; ++i) batches_.emplace_back(new Batch());
        for (auto& b : batches_) free_.push_back(b.get());
    }
    ~GuideBatcher() {
        for (auto& b : batches_) {
            if (b->ctx) sdmm_guide_ctx_destroy(b->ctx);
            sdmm_pinned_free(b->stage);
        }
    }
    GuideBatcher(const GuideBatcher&) = delete;
    GuideBatcher& operator=(const GuideBatcher&) = delete;

    // Blocks until r's outputs are in its host buffers; throws Error on failure.
    void serve(const sdmm_guide_host_req& r) {
        if (r.n <= 0) return;
        std::unique_lock<std::mutex> lock(mu_);
        callers_.insert(std::this_thread::get_id());
        ++inside_;
        // the open batch, if r fits; else close it and take a free one
        if (open_ && open_->n + r.n > open_->cap) close(open_);
        while (!open_) {
            if (free_.empty()) {
                cv_.wait(lock);
                continue;
            }
            Batch* b = free_.back();
            free_.pop_back();
            b->reset();
            if (b->cap < std::max(target_, r.n)) {
                // (idle batch: nothing reads its staging)
                const int64_t cap = std::max(target_, r.n) + std::max<int64_t>(r.n, 1 << 15);
                lock.unlock();
                sdmm_pinned_free(b->stage);
                b->stage = nullptr;
                b->cap = 0;
                void* p = nullptr;
                const int rc = sdmm_pinned_alloc((size_t)cap * kBytesPerQuery, &p);
                lock.lock();
                if (rc != SDMM_OK) {
                    free_.push_back(b);
                    --inside_;
                    cv_.notify_all();
                    throw Error(rc, std::string("GuideBatcher staging: ") + sdmm_last_error());
                }
                b->stage = (char*)p;
                b->cap = cap;
            }
            if (open_) {                      // (another thread opened one meanwhile)
                free_.push_back(b);
                if (open_->n + r.n > open_->cap) close(open_);
                continue;
            }
            open_ = b;
        }
        Batch* b = open_;
        const int64_t off = b->n;
        b->n += r.n;
        const bool leader = b->members++ == 0;
        ++b->copying;
        if (b->n >= target_ || inside_ >= callers_.size()) close(b);
        lock.unlock();
        copy_in(*b, off, r);
        lock.lock();
        if (--b->copying == 0) cv_.notify_all();
        if (leader) {
            const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(wait_);
            cv_.wait_until(lock, deadline, [&] { return b->closed; });
            if (!b->closed) close(b);
            cv_.wait(lock, [&] { return b->copying == 0; });
            const int64_t N = b->n;
            lock.unlock();
            int rc = SDMM_OK;
            std::string err;
            if (!b->ctx) rc = sdmm_guide_ctx_create(tree_, nullptr, &b->ctx);
            if (rc == SDMM_OK) {
                const sdmm_guide_host_req all{N, b->in(), b->cap, b->mode(), b->out(), b->cap, b->comp()};
                rc = sdmm_ctx_guide_pdf_host_batch(b->ctx, 1, &all);
            }
            if (rc != SDMM_OK) err = sdmm_last_error();
            lock.lock();
            b->rc = rc;
            b->err = err;
            b->done = true;
            cv_.notify_all();
        } else {
            cv_.wait(lock, [&] { return b->done; });
        }
        const int rc = b->rc;
        const std::string err = b->err;
        lock.unlock();
        if (rc == SDMM_OK) copy_out(*b, off, r);
        lock.lock();
        if (--b->members == 0) {              // the last one out frees the batch
            free_.push_back(b);
            cv_.notify_all();
        }
        --inside_;
        lock.unlock();
        if (rc != SDMM_OK) throw Error(rc, "sdmm_ctx_guide_pdf_host_batch (thread " + thread_tag() + "): " + err);
    }

private:
    // per query: 9 + 4 float planes, the int32 component, the mode byte
    static constexpr size_t kBytesPerQuery = 13 * sizeof(float) + sizeof(int32_t) + 1;
    struct Batch {
        sdmm_guide_ctx* ctx = nullptr;
        char* stage = nullptr;   // in 9 x cap floats | out 4 x cap floats | comp cap int32 | mode cap bytes
        int64_t cap = 0;
        int64_t n = 0;
        int members = 0, copying = 0;
        bool closed = false, done = false;
        int rc = SDMM_OK;
        std::string err;
        float* in() const { return (float*)stage; }
        float* out() const { return (float*)stage + 9 * cap; }
        int32_t* comp() const { return (int32_t*)((float*)stage + 13 * cap); }
        uint8_t* mode() const { return (uint8_t*)((float*)stage + 14 * cap); }
        void reset() {
            n = 0;
            members = copying = 0;
            closed = done = false;
            rc = SDMM_OK;
            err.clear();
        }
    };
    void close(Batch* b) {   // (mu_ held)
        b->closed = true;
        if (open_ == b) open_ = nullptr;
        cv_.notify_all();
    }
    static void copy_in(const Batch& b, int64_t off, const sdmm_guide_host_req& r) {
        for (int p = 0; p < 9; ++p)
            std::memcpy(b.in() + p * b.cap + off, r.in + p * r.in_stride, sizeof(float) * (size_t)r.n);
        std::memcpy(b.mode() + off, r.mode, (size_t)r.n);
    }
    static void copy_out(const Batch& b, int64_t off, const sdmm_guide_host_req& r) {
        for (int p = 0; p < 4; ++p)
            std::memcpy(r.out + p * r.out_stride, b.out() + p * b.cap + off, sizeof(float) * (size_t)r.n);
        std::memcpy(r.comp, b.comp() + off, sizeof(int32_t) * (size_t)r.n);
    }
    sdmm_stree* tree_;
    int64_t target_;
    int wait_;
    std::vector<std::unique_ptr<Batch>> batches_;
    std::vector<Batch*> free_;
    Batch* open_ = nullptr;
    std::mutex mu_;
    std::condition_variable cv_;
    std::unordered_set<std::thread::id> callers_;   // threads that ever called serve
    size_t inside_ = 0;                              // threads inside serve now
};

// A wavefront of guided-bounce queries against one mixture: the batched form
// of create_conditional + sample + posterior/hsum (sdmm_proc.cpp:368-545).
// Device SoA planes; capacity fixed at construction.
struct GuidingBatch {
    const float* c[3];   // condition (normalised position), device
    const float* u[3];   // uniforms: component choice, Box-Muller u1, u2, device
    float* d[3];         // sampled direction, device
    float* pdf;          // conditional mixture pdf at d (gmmPdf), device
    int32_t* comp;       // joint component used, -1 = invalid conditional, device
    int64_t n;
};

inline void sample_guided(const Mixture& m, const GuidingBatch& q) {
    check(sdmm_guide_batch(const_cast<Mixture&>(m).handle(), q.n, q.c, q.u, q.d, q.pdf, q.comp),
          "sdmm_guide_batch");
}

// The guiding accelerator (the plugin's m_accelerator STree: split_to_depth,
// split(threshold), find; volpath_sdmm.cpp:355-358,161,226, sdmm_proc.cpp:314)
// with one Mixture per node, and the guided wavefront over its leaves: every
// query is served by the mixture of the leaf its condition falls in
// (sampleSurface, sdmm_proc.cpp:309-421), BSDF-only (comp -1, pdf 0) where
// the leaf has none.
class SpatialTree {
public:
    SpatialTree(const float aabb_min[3], const float aabb_max[3], int device = 0) {
        check(sdmm_stree_create(aabb_min, aabb_max, device, &t_), "sdmm_stree_create");
    }
    ~SpatialTree() { sdmm_stree_destroy(t_); }
    SpatialTree(const SpatialTree&) = delete;
    SpatialTree& operator=(const SpatialTree&) = delete;

    sdmm_stree* handle() { return t_; }
    int nodes() const { return sdmm_stree_num_nodes(t_); }
    void set_stream(void* hip_stream) { check(sdmm_stree_set_stream(t_, hip_stream), "sdmm_stree_set_stream"); }
    void split_to_depth(int depth) { check(sdmm_stree_split_to_depth(t_, depth), "sdmm_stree_split_to_depth"); }
    // split(threshold) over host positions (the plugin's context.stats)
    void split(const float* const p[3], int64_t n, int threshold) {
        check(sdmm_stree_split(t_, p, n, threshold), "sdmm_stree_split");
    }
    bool is_leaf(int node) const {
        std::vector<int32_t> child(2 * (size_t)nodes());
        check(sdmm_stree_get_nodes(t_, nullptr, child.data(), nullptr), "sdmm_stree_get_nodes");
        return child[2 * (size_t)node] < 0;
    }
    // device points -> node ids (-1 outside)
    void find(int64_t n, const float* const p[3], int32_t* node_out) {
        check(sdmm_stree_find(t_, n, p, node_out), "sdmm_stree_find");
    }
    // one entry per node, nullptr where there is no trained mixture
    void bind(const std::vector<Mixture*>& node_mix) {
        if ((int)node_mix.size() != nodes()) throw Error(SDMM_E_INVALID, "bind: one mixture slot per node");
        std::vector<const sdmm_mix*> h(node_mix.size());
        for (size_t i = 0; i < h.size(); ++i) h[i] = node_mix[i] ? node_mix[i]->handle() : nullptr;
        check(sdmm_stree_bind_mixtures(t_, h.data()), "sdmm_stree_bind_mixtures");
    }
    // the wavefront against the bound mixtures; node_out optional
    void sample_guided(const GuidingBatch& q, int32_t* node_out = nullptr) {
        check(sdmm_guide_wavefront(t_, nullptr, q.n, q.c, q.u, q.d, q.pdf, q.comp, node_out),
              "sdmm_guide_wavefront");
    }
    void pdf_guided(int64_t n, const float* const c[3], const float* const d[3], float* pdf) {
        check(sdmm_pdf_wavefront(t_, nullptr, n, c, d, pdf), "sdmm_pdf_wavefront");
    }

    // sdmm::save_json(m_accelerator, path) (volpath_sdmm.cpp:125): the node
    // table plus every node's mixture (node_mix empty: the tree only)
    void save_json(const std::string& path, const std::vector<Mixture*>& node_mix = {}) const {
        std::vector<const sdmm_mix*> h;
        if (!node_mix.empty()) {
            if ((int)node_mix.size() != nodes()) throw Error(SDMM_E_INVALID, "save_json: one mixture slot per node");
            for (Mixture* m : node_mix) h.push_back(m ? m->handle() : nullptr);
        }
        check(sdmm_save_json(t_, h.empty() ? nullptr : h.data(), path.c_str()), "sdmm_save_json");
    }
    // the inverse: a new tree, node_mix[i] the node's mixture or null
    static std::unique_ptr<SpatialTree> load_json(const std::string& path, int device,
                                                  std::vector<std::unique_ptr<Mixture>>& node_mix) {
        int n = 0;
        check(sdmm_load_json(path.c_str(), device, nullptr, nullptr, 0, &n), "sdmm_load_json");
        std::vector<sdmm_mix*> h((size_t)n, nullptr);
        sdmm_stree* t = nullptr;
        check(sdmm_load_json(path.c_str(), device, &t, h.data(), n, &n), "sdmm_load_json");
        node_mix.clear();
        for (sdmm_mix* m : h) node_mix.push_back(m ? Mixture::adopt(m) : nullptr);
        return std::unique_ptr<SpatialTree>(new SpatialTree(t));
    }

private:
    explicit SpatialTree(sdmm_stree* t) : t_(t) {}
    sdmm_stree* t_ = nullptr;
};

// ---- run outputs the integrator writes next to the render ------------------
namespace detail {
inline std::string num(double v) {
    if (!std::isfinite(v)) return "null";   // nlohmann::json dumps non-finite numbers as null
    char b[40];
    std::snprintf(b, sizeof b, "%.17g", v);
    return b;
}
inline void make_dirs(const std::string& dir) {
    for (size_t i = 1; i <= dir.size(); ++i)
        if (i == dir.size() || dir[i] == '/') {
            const std::string d = dir.substr(0, i);
            if (::mkdir(d.c_str(), 0755) != 0 && errno != EEXIST) throw Error(SDMM_E_INVALID, "cannot create " + d);
        }
}
inline void write_text(const std::string& path, const std::string& text) {
    std::ofstream f(path);
    f << text;
    if (!f) throw Error(SDMM_E_INVALID, "cannot write " + path);
}
}  // namespace detail

// saveCheckpoint (volpath_sdmm.cpp:117-126): <dir>/checkpoints/model_%05i.asdmm
inline std::string save_checkpoint(const std::string& experiment_dir, int iteration, const SpatialTree& tree,
                                   const std::vector<Mixture*>& node_mix) {
    const std::string dir = experiment_dir + "/checkpoints";
    detail::make_dirs(dir);
    char name[32];
    std::snprintf(name, sizeof name, "/model_%05i.asdmm", iteration);
    tree.save_json(dir + name, node_mix);
    return dir + name;
}

// scene_norm.json (volpath_sdmm.cpp:340-351): the scene AABB's min corner and
// the largest extent, the normalisation of the guiding positions
inline void write_scene_norm(const std::string& path, const float scene_min[3], float spatial_norm) {
    detail::write_text(path, "{\n    \"scene_min\": [\n        " + detail::num(scene_min[0]) + ",\n        " +
                                 detail::num(scene_min[1]) + ",\n        " + detail::num(scene_min[2]) +
                                 "\n    ],\n    \"spatial_norm\": " + detail::num(spatial_norm) + "\n}\n");
}

// stats.json (volpath_sdmm.cpp:365, :421-428, :443-446): one record per render
// iteration, keys as the reference writes them (scripts/combine_renders.py and
// run_tests.py read total_elapsed_seconds / spp / mean_path_length)
class RunStats {
public:
    void push(int iteration, double elapsed_seconds, double total_elapsed_seconds, double mean_path_length,
              int spp, int total_spp) {
        rows_.push_back({iteration, elapsed_seconds, total_elapsed_seconds, mean_path_length, spp, total_spp});
    }
    size_t size() const { return rows_.size(); }
    void write(const std::string& path) const {   // std::setw(4) layout, keys sorted like nlohmann's
        std::string s = "[";
        for (size_t i = 0; i < rows_.size(); ++i) {
            const Row& r = rows_[i];
            s += i ? ",\n    {\n" : "\n    {\n";
            s += "        \"elapsed_seconds\": " + detail::num(r.elapsed) + ",\n";
            s += "        \"iteration\": " + std::to_string(r.iteration) + ",\n";
            s += "        \"mean_path_length\": " + detail::num(r.mean_path_length) + ",\n";
            s += "        \"spp\": " + std::to_string(r.spp) + ",\n";
            s += "        \"total_elapsed_seconds\": " + detail::num(r.total_elapsed) + ",\n";
            s += "        \"total_spp\": " + std::to_string(r.total_spp) + "\n    }";
        }
        s += rows_.empty() ? "]\n" : "\n]\n";
        detail::write_text(path, s);
    }

private:
    struct Row {
        int iteration;
        double elapsed, total_elapsed, mean_path_length;
        int spp, total_spp;
    };
    std::vector<Row> rows_;
};

// pdfSurface's mixing of BSDF and guiding densities (sdmm_proc.cpp:587-589):
// pdf = h * bsdfPdf + (1 - h) * gmmPdf, h = 0.5 (0.3 with product sampling).
// An analytic scene for the device Li (sdmm_scene_*): the description's
// arrays are only read during construction.
class Scene {
public:
    Scene(const sdmm_scene_desc& desc, int device = 0) { check(sdmm_scene_create(&desc, device, &h_), "sdmm_scene_create"); }
    ~Scene() { sdmm_scene_destroy(h_); }
    Scene(const Scene&) = delete;
    Scene& operator=(const Scene&) = delete;
    sdmm_scene* handle() { return h_; }
    // render() (volpath_sdmm.cpp:375-393): scene_norm.json values and the tree box
    void normalization(float scene_min[3], float* spatial_norm, float tree_min[3], float tree_max[3]) const {
        check(sdmm_scene_normalization(h_, scene_min, spatial_norm, tree_min, tree_max), "sdmm_scene_normalization");
    }

private:
    sdmm_scene* h_ = nullptr;
};

// The plugin's guiding state and schedule (SDMMVolumetricPathTracer,
// volpath_sdmm.cpp:132-312, :411-507) resident on the GPU (sdmm_guiding_*).
class GuidingModel {
public:
    GuidingModel(const float tree_min[3], const float tree_max[3], const sdmm_guiding_config* cfg = nullptr,
                 int device = 0) {
        sdmm_guiding_config c;
        sdmm_guiding_config_default(&c);
        if (cfg) c = *cfg;
        check(sdmm_guiding_create(tree_min, tree_max, &c, device, &h_), "sdmm_guiding_create");
    }
    ~GuidingModel() { sdmm_guiding_destroy(h_); }
    GuidingModel(const GuidingModel&) = delete;
    GuidingModel& operator=(const GuidingModel&) = delete;
    sdmm_guiding* handle() { return h_; }
    sdmm_stree* tree() { return sdmm_guiding_tree(h_); }
    int trained() const { return sdmm_guiding_trained(h_); }
    // Li's tail for a render pass, then optimize() (m_totalSpp += spp after)
    void push(const sdmm_path_vertices& v, uint64_t seed) { check(sdmm_guiding_push(h_, &v, seed), "sdmm_guiding_push"); }
    // optimizeAsync: optimize_async_wait_and_update (volpath_sdmm.cpp:227-242)
    void update() { check(sdmm_guiding_update(h_), "sdmm_guiding_update"); }
    sdmm_guiding_stats optimize(int spp) {
        sdmm_guiding_stats st{};
        check(sdmm_guiding_optimize(h_, spp, &st), "sdmm_guiding_optimize");
        return st;
    }
    // one pass of render()'s loop with the device Li (image: device, 3 planes)
    sdmm_guiding_stats iteration(Scene& scene, const sdmm_li_params& p, uint64_t push_seed, bool train, float* image,
                                 float* image_sqr = nullptr, sdmm_li_stats* li = nullptr) {
        sdmm_guiding_stats st{};
        check(sdmm_guiding_iteration(h_, scene.handle(), &p, push_seed, train ? 1 : 0, image, image_sqr, li, &st),
              "sdmm_guiding_iteration");
        return st;
    }

private:
    sdmm_guiding* h_ = nullptr;
};

// SDMMWorkResult::dumpIndividual (sdmm_wr.cpp:115-146): the pass's image and
// squared image as dir/iteration%05i.exr and dir/iteration_sqr%05i.exr (host
// planes [3][h][w]); returns the first path.
inline std::string dump_iteration(const std::string& dir, int iteration, int spp, float seconds, int width,
                                  int height, const float* rgb, const float* rgb_sqr) {
    detail::make_dirs(dir);
    char name[64];
    std::snprintf(name, sizeof(name), "/iteration%05i.exr", iteration);
    const std::string a = dir + name;
    check(sdmm_write_exr(a.c_str(), width, height, rgb, spp, iteration, seconds), "sdmm_write_exr");
    if (rgb_sqr) {
        std::snprintf(name, sizeof(name), "/iteration_sqr%05i.exr", iteration);
        const std::string b = dir + name;
        check(sdmm_write_exr(b.c_str(), width, height, rgb_sqr, spp, iteration, seconds), "sdmm_write_exr");
    }
    return a;
}

inline float mixed_pdf(float heuristicConditionalWeight, float bsdfPdf, float gmmPdf) {
    return heuristicConditionalWeight * bsdfPdf + (1.0f - heuristicConditionalWeight) * gmmPdf;
}

}  // namespace sdmm_amd
