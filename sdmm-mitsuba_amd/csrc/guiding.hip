// guiding.hip -- the plugin's guiding model (SDMMVolumetricPathTracer,
// volpath_sdmm.cpp:132-312, :411-507) on the device, behind sdmm_guiding_* in
// include/sdmm_gpu.h: the accelerator tree, one SDMM + stepwise EM state per
// trained leaf (SDMMContext, sdmm_proc.h:92-93), the leaves' training data
// and the per-iteration schedule.
//
// Data layout.  The reference keeps a Samples buffer per leaf context, filled
// under a mutex.  Here every leaf's records live in ONE device pool (SoA
// planes: point 6, normal 3, weight, leaf id), appended per render iteration
// in the producer's leaf order; optimize() orders the pool by leaf with a
// stable radix sort (a leaf's records stay in arrival order), so the leaves
// that can be optimised form one contiguous prefix that feeds the batched
// per-leaf EM directly, and are then dropped.  The leaves' stats positions
// (context.stats, used only for splitting) live in a second device pool of
// the same kind; only the positions of leaves that must split travel to the
// host, where the tree is built.
//
// Split leaves (split_leaf_recurse): records and stats positions move to the
// child leaf that holds them (a record outside the split leaf's subtree is
// dropped), and every new leaf starts from a copy of the parent's mixture and
// EM state -- jmm SNTree::createChildNode (sntree.h:172-205); sdmm-lib's tree,
// which the plugin instantiates, is absent (parity unpinned for this rule).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <numeric>
#include <vector>

#include "../../include/sdmm_gpu.h"

namespace sdmm_detail {
int set_error(int code, const char* msg);
int push_training_ex(sdmm_stree* t, const sdmm_path_vertices* v, int saved_per_path, uint64_t seed,
                     const sdmm_training_out* out, int64_t* n_out, int64_t* seg, int64_t* lost, bool reuse_counts,
                     int64_t known_count);
void destroy_many(sdmm_mix* const* ms, int n);
}  // namespace sdmm_detail

namespace {

constexpr int kPlanes = 10;   // x 6, normal 3, w

int fail(int code, const std::string& m) { return sdmm_detail::set_error(code, m.c_str()); }

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(SDMM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)
#define SDMM_TRY(expr)            \
    do {                          \
        const int r_ = (expr);    \
        if (r_) return r_;        \
    } while (0)

// key per record: its leaf for the ordering sort; `ready` leaves (flag) first
__global__ void pool_keys_kernel(const int32_t* __restrict__ node, int64_t n, const uint8_t* __restrict__ ready,
                                 int num_nodes, uint32_t* __restrict__ keys, int32_t* __restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int v = node[i];
    uint32_t k = 2u * (uint32_t)num_nodes;   // dropped records sort last
    if (v >= 0) k = ready && ready[v] ? (uint32_t)v : (uint32_t)(num_nodes + v);
    keys[i] = k;
    idx[i] = (int32_t)i;
}

__global__ void pool_gather_kernel(const float* __restrict__ src, float* __restrict__ dst, const int32_t* __restrict__ node_in,
                                   int32_t* __restrict__ node_out, const int32_t* __restrict__ perm, int64_t n,
                                   int64_t cap, int planes) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int64_t i = perm[j];
    for (int p = 0; p < planes; ++p) dst[p * cap + j] = src[p * cap + i];
    node_out[j] = node_in[i];
}

// the stats records (flag set) of a pushed batch appended to the stats pool:
// positions (planes 0..2 of the records) and the leaf id, in record order
__global__ void stats_append_kernel(const int32_t* __restrict__ sel, const int32_t* __restrict__ count,
                                    const float* __restrict__ rec, int64_t rcap, const int32_t* __restrict__ rnode,
                                    float* __restrict__ sp, int64_t scap, int32_t* __restrict__ snode) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= *count) return;
    const int i = sel[j];
    for (int f = 0; f < 3; ++f) sp[f * scap + j] = rec[f * rcap + i];
    snode[j] = rnode[i];
}

// first position with key >= v for v = 0 .. nk
__global__ void pool_seg_kernel(const uint32_t* __restrict__ keys, int64_t n, int nk, int64_t* __restrict__ seg) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v > nk) return;
    int64_t lo = 0, count = n;
    while (count > 0) {
        const int64_t step = count / 2, it = lo + step;
        if (keys[it] < (uint32_t)v) { lo = it + 1; count -= step + 1; }
        else count = step;
    }
    seg[v] = lo;
}

// records of split leaves: the leaf found in the new tree if it descends from
// the old one (parent table), else dropped (-1)
__global__ void pool_relabel_kernel(int32_t* __restrict__ node, const int32_t* __restrict__ found, int64_t n,
                                    const uint8_t* __restrict__ was_split, const int32_t* __restrict__ parent) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int v = node[i];
    if (v < 0 || !was_split[v]) return;
    int f = found[i];
    int a = f;
    while (a >= 0 && a != v) a = parent[a];
    node[i] = (a == v) ? f : -1;
}

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

// entries per leaf of a pool (dropped entries, node < 0, not counted): a
// block-private LDS histogram when the node count fits, else global atomics
constexpr int kCountBins = 16384;
constexpr int kCountPer = 16;   // entries per thread
__global__ void __launch_bounds__(256) pool_count_kernel(const int32_t* __restrict__ node, int64_t n, int nn,
                                                         unsigned long long* __restrict__ counts) {
    __shared__ unsigned h[kCountBins];
    const bool lds = nn <= kCountBins;
    if (lds)
        for (int i = threadIdx.x; i < nn; i += 256) h[i] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * 256 * kCountPer;
    for (int k = 0; k < kCountPer; ++k) {
        const int64_t i = base + (int64_t)k * 256 + threadIdx.x;
        if (i >= n) break;
        const int v = node[i];
        if (v < 0 || v >= nn) continue;
        if (lds) atomicAdd(&h[v], 1u);
        else atomicAdd(&counts[v], 1ull);
    }
    __syncthreads();
    if (lds)
        for (int i = threadIdx.x; i < nn; i += 256)
            if (h[i]) atomicAdd(&counts[i], (unsigned long long)h[i]);
}

// out[(i * npos + j) * 6 + f]: point (f < 3) / normal (f >= 3) of record starts[i] + j
__global__ void init_gather_kernel(const float* __restrict__ pool, int64_t cap, const int64_t* __restrict__ starts,
                                   int nf, int npos, float* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nf * npos) return;
    const int i = t / npos, j = t % npos;
    const int64_t r = starts[i] + j;
    for (int f = 0; f < 3; ++f) {
        out[(size_t)t * 6 + f] = pool[f * cap + r];
        out[(size_t)t * 6 + 3 + f] = pool[(6 + f) * cap + r];
    }
}

// SDMM_GUIDING_TIMING=1: host-clock phase times of optimize() on stderr
struct PhaseClock {
    bool on;
    hipStream_t st;
    std::chrono::steady_clock::time_point t;
    explicit PhaseClock(hipStream_t s) : on(std::getenv("SDMM_GUIDING_TIMING") != nullptr), st(s),
                                         t(std::chrono::steady_clock::now()) {}
    void lap(const char* what) {
        if (!on) return;
        (void)hipStreamSynchronize(st);
        const auto n = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[guiding] %-12s %8.2f ms\n", what,
                     std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};

}  // namespace

// SoA planes [planes][cap] + a leaf id per entry, double-buffered for the
// stable reorders
struct Pool {
    int planes = 0;
    float* p[2] = {nullptr, nullptr};
    int32_t* node[2] = {nullptr, nullptr};
    int cur = 0;
    int64_t n = 0, cap = 0;
    std::vector<int64_t> seg;   // after order(): per key range
    float* plane(int f) const { return p[cur] + (int64_t)f * cap; }
    int32_t* nodes() const { return node[cur]; }
};

struct sdmm_guiding {
    int device = 0;
    bool pool_held = false;     // raised the default pool's release threshold (pool_hold)
    sdmm_guiding_config cfg{};
    sdmm_stree* tree = nullptr;
    hipStream_t st = nullptr;
    std::vector<sdmm_mix*> mix;                 // per node (NULL: untrained / inner)
    int64_t total_spp = 0;
    int iteration = 0;
    Pool rec;     // training records: point 6, normal 3, weight
    Pool stat;    // stats positions (context.stats)
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    float* pinned = nullptr;   // host staging of the splitting leaves' positions
    size_t pinned_floats = 0;
    // optimizeAsync (volpath_sdmm.cpp:180-242): EM on its own stream while the
    // next pass renders with the conditioners (cond) of the previous update
    bool async = false;
    hipStream_t em_st = nullptr;
    hipEvent_t em_done = nullptr, copied = nullptr;
    std::vector<sdmm_mix*> cond;     // per node: the conditioner the renders use
    std::vector<int> pending;        // leaves stepped by the running EM
    bool running = false;
    float* tbuf = nullptr;           // the running EM's training data (7 planes)
    int64_t tcap = 0;
};

namespace {

int grow_pool(sdmm_guiding* g, Pool& P, int64_t need) {
    if (need <= P.cap) return SDMM_OK;
    // headroom for the next passes' records (every regrowth copies and
    // synchronises; HBM is plentiful)
    // (the first pass's pool takes 3x: the second pass adds as many records
    // again beside the first pass's untrained ones)
    int64_t cap = P.cap == 0 ? 3 * need : std::max<int64_t>(need + need / 2, P.cap * 2);
    cap = std::max<int64_t>(cap, 1 << 16);
    float* np[2] = {nullptr, nullptr};
    int32_t* nn[2] = {nullptr, nullptr};
    for (int b = 0; b < 2; ++b) {
        HIP_TRY(hipMalloc(&np[b], sizeof(float) * (size_t)P.planes * (size_t)cap));
        HIP_TRY(hipMalloc(&nn[b], sizeof(int32_t) * (size_t)cap));
    }
    if (P.n > 0) {
        for (int f = 0; f < P.planes; ++f)
            HIP_TRY(hipMemcpyAsync(np[0] + f * cap, P.plane(f), sizeof(float) * (size_t)P.n, hipMemcpyDeviceToDevice,
                                   g->st));
        HIP_TRY(hipMemcpyAsync(nn[0], P.nodes(), sizeof(int32_t) * (size_t)P.n, hipMemcpyDeviceToDevice, g->st));
    }
    HIP_TRY(hipStreamSynchronize(g->st));
    for (int b = 0; b < 2; ++b) {
        if (P.p[b]) HIP_TRY(hipFree(P.p[b]));
        if (P.node[b]) HIP_TRY(hipFree(P.node[b]));
        P.p[b] = np[b];
        P.node[b] = nn[b];
    }
    P.cur = 0;
    P.cap = cap;
    return SDMM_OK;
}

int grow_scratch(sdmm_guiding* g, size_t bytes) {
    if (bytes <= g->scratch_bytes) return SDMM_OK;
    HIP_TRY(hipStreamSynchronize(g->st));
    if (g->scratch) HIP_TRY(hipFree(g->scratch));
    g->scratch = nullptr;
    HIP_TRY(hipMalloc(&g->scratch, bytes));
    g->scratch_bytes = bytes;
    return SDMM_OK;
}

size_t al(size_t b) { return (b + 255) / 256 * 256; }

// Stable reorder of a pool by key (ready leaves first, then the other
// leaves, dropped entries last); P.seg over keys 0 .. 2 * num_nodes.
// order_pool's scratch for n entries over nn nodes
size_t order_scratch_bytes(int64_t n, int nn, int bits) {
    size_t tb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, bits);
    const size_t kb = al(sizeof(uint32_t) * (size_t)n);
    const size_t sb = al(sizeof(int64_t) * (size_t)(2 * nn + 1));
    const size_t rb = al((size_t)std::max(nn, 1));
    return 4 * kb + sb + rb + al(tb);
}

int order_pool(sdmm_guiding* g, Pool& P, const std::vector<uint8_t>& ready) {
    const int nn = sdmm_stree_num_nodes(g->tree);
    const int nk = 2 * nn;
    P.seg.assign((size_t)nk + 1, 0);
    if (P.n == 0) return SDMM_OK;
    int bits = 1;
    while ((1u << bits) <= (unsigned)nk) ++bits;
    size_t tb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, (int)P.n, 0, bits);
    const size_t kb = al(sizeof(uint32_t) * (size_t)P.n);
    const size_t sb = al(sizeof(int64_t) * (size_t)(nk + 1));
    const size_t rb = al((size_t)std::max(nn, 1));
    SDMM_TRY(grow_scratch(g, 4 * kb + sb + rb + al(tb)));
    char* b = (char*)g->scratch;
    uint32_t* k0 = (uint32_t*)b;
    uint32_t* k1 = (uint32_t*)(b + kb);
    int32_t* i0 = (int32_t*)(b + 2 * kb);
    int32_t* i1 = (int32_t*)(b + 3 * kb);
    int64_t* sdev = (int64_t*)(b + 4 * kb);
    uint8_t* rdev = (uint8_t*)(b + 4 * kb + sb);
    void* temp = b + 4 * kb + sb + rb;
    HIP_TRY(hipMemcpyAsync(rdev, ready.data(), (size_t)nn, hipMemcpyHostToDevice, g->st));
    hipLaunchKernelGGL(pool_keys_kernel, grid_for(P.n), dim3(256), 0, g->st, P.nodes(), P.n, rdev, nn, k0, i0);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(temp, tb, k0, k1, i0, i1, (int)P.n, 0, bits, g->st));
    hipLaunchKernelGGL(pool_gather_kernel, grid_for(P.n), dim3(256), 0, g->st, P.p[P.cur], P.p[1 - P.cur],
                       P.node[P.cur], P.node[1 - P.cur], i1, P.n, P.cap, P.planes);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(pool_seg_kernel, grid_for(nk + 1), dim3(256), 0, g->st, k1, P.n, nk, sdev);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(P.seg.data(), sdev, sizeof(int64_t) * (size_t)(nk + 1), hipMemcpyDeviceToHost, g->st));
    HIP_TRY(hipStreamSynchronize(g->st));   // (ready is a host temporary)
    P.cur = 1 - P.cur;
    P.n = P.seg[(size_t)nk];               // dropped entries are gone
    return SDMM_OK;
}

// entries per leaf of the record and stats pools (rc, sc: nn each) without
// reordering them: the one stable sort by `ready` that follows gives every
// leaf's entries the order a leaf sort before it would have kept
int pool_counts(sdmm_guiding* g, const Pool& R, const Pool& S, int nn, std::vector<int64_t>& rc,
                std::vector<int64_t>& sc) {
    rc.assign((size_t)nn, 0);
    sc.assign((size_t)nn, 0);
    if (nn == 0) return SDMM_OK;
    SDMM_TRY(grow_scratch(g, sizeof(int64_t) * 2 * (size_t)nn));
    unsigned long long* d = (unsigned long long*)g->scratch;
    HIP_TRY(hipMemsetAsync(d, 0, sizeof(int64_t) * 2 * (size_t)nn, g->st));
    const Pool* P[2] = {&R, &S};
    for (int q = 0; q < 2; ++q) {
        if (P[q]->n == 0) continue;
        const int64_t per = 256 * (int64_t)kCountPer;
        hipLaunchKernelGGL(pool_count_kernel, dim3((unsigned)((P[q]->n + per - 1) / per)), dim3(256), 0, g->st,
                           P[q]->nodes(), P[q]->n, nn, d + (size_t)q * nn);
        HIP_TRY(hipGetLastError());
    }
    std::vector<int64_t> h(2 * (size_t)nn);
    HIP_TRY(hipMemcpyAsync(h.data(), d, sizeof(int64_t) * h.size(), hipMemcpyDeviceToHost, g->st));
    HIP_TRY(hipStreamSynchronize(g->st));
    std::copy(h.begin(), h.begin() + nn, rc.begin());
    std::copy(h.begin() + nn, h.end(), sc.begin());
    return SDMM_OK;
}

// entries of split leaves: the leaf found in the new tree if it descends from
// the split leaf, else dropped
int relabel(sdmm_guiding* g, Pool& P, const uint8_t* dsplit, const int32_t* dparent) {
    if (P.n == 0) return SDMM_OK;
    int32_t* dfound = nullptr;
    HIP_TRY(hipMallocAsync((void**)&dfound, sizeof(int32_t) * (size_t)P.n, g->st));
    const float* pp[3] = {P.plane(0), P.plane(1), P.plane(2)};
    SDMM_TRY(sdmm_stree_find(g->tree, P.n, pp, dfound));
    hipLaunchKernelGGL(pool_relabel_kernel, grid_for(P.n), dim3(256), 0, g->st, P.nodes(), dfound, P.n, dsplit,
                       dparent);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipFreeAsync(dfound, g->st));
    return SDMM_OK;
}

// After a split: stats positions, pool records and mixtures of every split
// leaf move to its new leaves.  A new node's split leaf is its first ancestor
// that existed before (new nodes are numbered after every old one).
int redistribute(sdmm_guiding* g, int old_nodes) {
    PhaseClock clk(g->st);
    const int nn = sdmm_stree_num_nodes(g->tree);
    std::vector<int32_t> child(2 * (size_t)nn), parent((size_t)nn, -1);
    SDMM_TRY(sdmm_stree_get_nodes(g->tree, nullptr, child.data(), nullptr));
    for (int i = 0; i < nn; ++i)
        for (int c = 0; c < 2; ++c)
            if (child[2 * (size_t)i + c] >= 0) parent[(size_t)child[2 * (size_t)i + c]] = i;
    std::vector<uint8_t> was_split((size_t)nn, 0);
    for (int v = 0; v < old_nodes; ++v)   // records only ever name leaves: an old node with children was split
        if (child[2 * (size_t)v] >= 0) was_split[(size_t)v] = 1;
    std::vector<int> origin((size_t)nn, -1);   // new node -> the split leaf it came from
    for (int c = old_nodes; c < nn; ++c) {
        int a = parent[(size_t)c];
        while (a >= old_nodes) a = parent[(size_t)a];
        origin[(size_t)c] = a;
    }
    g->mix.resize((size_t)nn, nullptr);
    // mixtures: the split leaf's own handle moves to its first new leaf and
    // the others get copies (one slab); a split leaf whose mixture has no new
    // leaf to go to is destroyed.  Applied to the conditioners too (async).
    auto hand_down = [&](std::vector<sdmm_mix*>& tab, bool on_model_stream) -> int {
        tab.resize((size_t)nn, nullptr);
        std::vector<const sdmm_mix*> src;
        std::vector<int> dst;
        std::vector<uint8_t> moved((size_t)old_nodes, 0);
        for (int c = old_nodes; c < nn; ++c) {
            const int v = origin[(size_t)c];
            if (child[2 * (size_t)c] >= 0 || v < 0 || !tab[(size_t)v]) continue;
            if (!moved[(size_t)v]) {
                moved[(size_t)v] = 1;
                tab[(size_t)c] = tab[(size_t)v];
                continue;
            }
            src.push_back(tab[(size_t)v]);
            dst.push_back(c);
        }
        std::vector<sdmm_mix*> made(src.size(), nullptr);
        if (on_model_stream) {
            SDMM_TRY(sdmm_clone_many(src.data(), (int)src.size(), made.data()));
        } else {
            SDMM_TRY(sdmm_clone_many_on_stream(src.data(), (int)src.size(), (void*)g->st, made.data()));
        }
        for (size_t i = 0; i < dst.size(); ++i) tab[(size_t)dst[i]] = made[i];
        std::vector<sdmm_mix*> gone;
        for (int v = 0; v < old_nodes; ++v)
            if (was_split[(size_t)v] && tab[(size_t)v]) {
                if (!moved[(size_t)v]) gone.push_back(tab[(size_t)v]);
                tab[(size_t)v] = nullptr;
            }
        sdmm_detail::destroy_many(gone.data(), (int)gone.size());
        return SDMM_OK;
    };
    SDMM_TRY(hand_down(g->mix, true));
    clk.lap("redis:clone");
    if (g->async) SDMM_TRY(hand_down(g->cond, false));   // the conditioners follow their mixtures
    clk.lap("redis:destroy");
    // records and stats positions: relabelled on the device (order kept)
    uint8_t* dsplit = nullptr;
    int32_t* dparent = nullptr;
    HIP_TRY(hipMallocAsync((void**)&dsplit, (size_t)nn, g->st));
    HIP_TRY(hipMallocAsync((void**)&dparent, sizeof(int32_t) * (size_t)nn, g->st));
    HIP_TRY(hipMemcpyAsync(dsplit, was_split.data(), (size_t)nn, hipMemcpyHostToDevice, g->st));
    HIP_TRY(hipMemcpyAsync(dparent, parent.data(), sizeof(int32_t) * (size_t)nn, hipMemcpyHostToDevice, g->st));
    SDMM_TRY(relabel(g, g->rec, dsplit, dparent));
    SDMM_TRY(relabel(g, g->stat, dsplit, dparent));
    HIP_TRY(hipFreeAsync(dsplit, g->st));
    HIP_TRY(hipFreeAsync(dparent, g->st));
    HIP_TRY(hipStreamSynchronize(g->st));   // host tables above are temporaries
    return SDMM_OK;
}

// the renders' table: the mixtures themselves (sync) or their conditioners (async)
const std::vector<sdmm_mix*>& guide_table(const sdmm_guiding* g) { return g->async ? g->cond : g->mix; }

int bind(sdmm_guiding* g) {
    const auto& src = guide_table(g);
    std::vector<const sdmm_mix*> tab((size_t)sdmm_stree_num_nodes(g->tree), nullptr);
    for (size_t i = 0; i < src.size() && i < tab.size(); ++i) tab[i] = src[i];
    return sdmm_stree_bind_mixtures(g->tree, tab.data());
}

// optimize_async_wait_and_update (:227-242): wait for the running EM, then
// each stepped leaf's conditioner := its mixture (sdmm::prepare)
int update(sdmm_guiding* g) {
    if (!g->async || !g->running) return SDMM_OK;
    HIP_TRY(hipEventSynchronize(g->em_done));
    g->running = false;
    g->cond.resize(g->mix.size(), nullptr);
    std::vector<const sdmm_mix*> csrc, nsrc;
    std::vector<sdmm_mix*> cdst;
    std::vector<int> fresh;
    for (int v : g->pending) {
        const sdmm_mix* m = g->mix[(size_t)v];
        if (!m) continue;
        if (g->cond[(size_t)v]) {
            csrc.push_back(m);
            cdst.push_back(g->cond[(size_t)v]);
        } else {
            nsrc.push_back(m);
            fresh.push_back(v);
        }
    }
    g->pending.clear();
    SDMM_TRY(sdmm_copy_many(csrc.data(), cdst.data(), (int)csrc.size()));
    std::vector<sdmm_mix*> made(nsrc.size(), nullptr);
    SDMM_TRY(sdmm_clone_many_on_stream(nsrc.data(), (int)nsrc.size(), (void*)g->st, made.data()));
    for (size_t i = 0; i < fresh.size(); ++i) g->cond[(size_t)fresh[i]] = made[i];
    return bind(g);
}

// The default pool's release threshold, raised while any guiding model on
// the device lives and restored afterwards (it is shared with every other
// stream-ordered allocation of the host process).
struct PoolHold {
    int users = 0;
    uint64_t saved = 0;
    bool have_saved = false;
};
std::mutex g_pool_mu;
PoolHold g_pool_hold[64];

void pool_hold(int device) {
    if (device < 0 || device >= 64) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    PoolHold& h = g_pool_hold[device];
    if (h.users++ > 0) return;
    hipMemPool_t pool = nullptr;
    if (hipDeviceGetDefaultMemPool(&pool, device) != hipSuccess || !pool) return;
    h.have_saved = hipMemPoolGetAttribute(pool, hipMemPoolAttrReleaseThreshold, &h.saved) == hipSuccess;
    uint64_t keep = UINT64_MAX;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
}

void pool_release(int device) {
    if (device < 0 || device >= 64) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    PoolHold& h = g_pool_hold[device];
    if (h.users == 0 || --h.users > 0) return;
    hipMemPool_t pool = nullptr;
    if (!h.have_saved || hipDeviceGetDefaultMemPool(&pool, device) != hipSuccess || !pool) return;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &h.saved);
}

}  // namespace

extern "C" {

void sdmm_guiding_config_default(sdmm_guiding_config* c) {
    if (!c) return;
    c->K = 16;                  // SDMMProcess::NComponents of the built plugin
    c->split_depth = 2;         // split_to_depth(2), volpath_sdmm.cpp:398
    c->split_threshold = 4000;  // m_splitThreshold (:528)
    c->max_leaf_nodes = 2048;   // m_maxLeafNodes (:529)
    c->saved_per_path = 8;      // savedSamplesPerPath (:62)
    c->depth_prior = 0.01f;
    c->init_seed = 0x1A17;
    c->optimize_async = 0;      // optimizeAsync (:65; the test suite's XML default is true)
}

int sdmm_guiding_create(const float tree_min[3], const float tree_max[3], const sdmm_guiding_config* cfg,
                        int device, sdmm_guiding** out) {
    if (!tree_min || !tree_max || !cfg || !out || cfg->K < 8 || cfg->K % 8 || cfg->split_threshold < 1 ||
        cfg->saved_per_path < 1)
        return fail(SDMM_E_INVALID, "sdmm_guiding_create: invalid argument");
    *out = nullptr;
    sdmm_guiding* g = new (std::nothrow) sdmm_guiding();
    if (!g) return fail(SDMM_E_NOMEM, "out of host memory");
    g->device = device;
    g->cfg = *cfg;
    int r = sdmm_stree_create(tree_min, tree_max, device, &g->tree);
    if (!r) r = sdmm_stree_split_to_depth(g->tree, cfg->split_depth);
    if (!r) {
        hipError_t e = hipSetDevice(device);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->st, hipStreamNonBlocking);
        if (e != hipSuccess) r = fail(SDMM_E_HIP, std::string("sdmm_guiding_create: ") + hipGetErrorString(e));
    }
    if (!r) {
        // the per-leaf mixtures are stream-ordered allocations from the
        // device's default pool: keep its memory between synchronisations
        // (the default threshold returns it at every sync, so each new leaf
        // would grow the pool again)
        // -- a process-wide setting: the first live model raises it and the
        // last one restores the caller's value (pool_hold / pool_release)
        pool_hold(device);
        g->pool_held = true;
    }
    if (!r) r = sdmm_stree_set_stream(g->tree, (void*)g->st);
    g->async = cfg->optimize_async != 0;
    if (!r && g->async) {
        hipError_t e = hipStreamCreateWithFlags(&g->em_st, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&g->em_done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&g->copied, hipEventDisableTiming);
        if (e != hipSuccess) r = fail(SDMM_E_HIP, std::string("sdmm_guiding_create: ") + hipGetErrorString(e));
    }
    if (r) {
        sdmm_guiding_destroy(g);
        return r;
    }
    const int nn = sdmm_stree_num_nodes(g->tree);
    g->mix.assign((size_t)nn, nullptr);
    g->rec.planes = kPlanes;
    g->stat.planes = 3;
    *out = g;
    return SDMM_OK;
}

void sdmm_guiding_destroy(sdmm_guiding* g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    if (g->st) (void)hipStreamSynchronize(g->st);
    if (g->em_st) (void)hipStreamSynchronize(g->em_st);
    for (sdmm_mix* m : g->mix) sdmm_destroy(m);
    for (sdmm_mix* m : g->cond) sdmm_destroy(m);
    if (g->tbuf) (void)hipFree(g->tbuf);
    if (g->em_done) (void)hipEventDestroy(g->em_done);
    if (g->copied) (void)hipEventDestroy(g->copied);
    if (g->tree) sdmm_stree_destroy(g->tree);
    for (Pool* P : {&g->rec, &g->stat})
        for (int b = 0; b < 2; ++b) {
            if (P->p[b]) (void)hipFree(P->p[b]);
            if (P->node[b]) (void)hipFree(P->node[b]);
        }
    if (g->scratch) (void)hipFree(g->scratch);
    if (g->pinned) (void)hipHostFree(g->pinned);
    if (g->st) (void)hipStreamDestroy(g->st);
    if (g->em_st) (void)hipStreamDestroy(g->em_st);
    if (g->pool_held) pool_release(g->device);
    delete g;
}

sdmm_stree* sdmm_guiding_tree(sdmm_guiding* g) { return g ? g->tree : nullptr; }

int sdmm_guiding_node_mixtures(const sdmm_guiding* g, const sdmm_mix** out, int cap) {
    if (!g || !out) return fail(SDMM_E_INVALID, "invalid argument");
    const int nn = sdmm_stree_num_nodes(g->tree);
    if (cap < nn) return fail(SDMM_E_INVALID, "sdmm_guiding_node_mixtures: cap < num_nodes");
    const auto& t = guide_table(g);
    for (int i = 0; i < nn; ++i) out[i] = (size_t)i < t.size() ? t[(size_t)i] : nullptr;
    return SDMM_OK;
}

int sdmm_guiding_trained(const sdmm_guiding* g) {
    if (!g) return 0;
    int n = 0;
    for (const sdmm_mix* m : guide_table(g)) n += m ? 1 : 0;
    return n;
}

int sdmm_guiding_update(sdmm_guiding* g) {
    if (!g) return fail(SDMM_E_INVALID, "invalid argument");
    HIP_TRY(hipSetDevice(g->device));
    return update(g);
}

// push_back_data for a render pass's paths (Li's tail): records appended to
// the record pool, the own-leaf entries' positions to the stats pool
int sdmm_guiding_push(sdmm_guiding* g, const sdmm_path_vertices* v, uint64_t seed) {
    if (!g || !v) return fail(SDMM_E_INVALID, "invalid argument");
    HIP_TRY(hipSetDevice(g->device));
    PhaseClock clk(g->st);
    // the producer's count pass once (its offsets are reused by the write);
    // the pools are sized before anything is read back, so a push costs two
    // synchronisations: the record count and the stats count
    int64_t count = 0;
    SDMM_TRY(sdmm_detail::push_training_ex(g->tree, v, g->cfg.saved_per_path, seed, nullptr, &count, nullptr, nullptr,
                                           false, -1));
    clk.lap("push:count");
    if (count == 0) return SDMM_OK;
    if (count > INT32_MAX) return fail(SDMM_E_INVALID, "sdmm_guiding_push: too many records");
    Pool& R = g->rec;
    Pool& S = g->stat;
    SDMM_TRY(grow_pool(g, R, R.n + count));
    SDMM_TRY(grow_pool(g, S, S.n + count));   // the stats entries are a subset of the records
    {
        // the reorders' scratch sized with the pools (a regrowth inside
        // optimize() would free and synchronise there): the record pool's
        // capacity over the node count the leaf cap allows (x2 for the split's
        // overshoot), 17-bit keys
        const int nn_cap = std::max(sdmm_stree_num_nodes(g->tree), 4 * g->cfg.max_leaf_nodes + 64);
        SDMM_TRY(grow_scratch(g, order_scratch_bytes(R.cap, nn_cap, 17)));
    }
    size_t tb = 0;
    (void)hipcub::DeviceSelect::Flagged(nullptr, tb, hipcub::CountingInputIterator<int32_t>(0),
                                        (const uint8_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr, (int)count);
    char* tmp = nullptr;
    const size_t fb = al((size_t)count), sb = al(sizeof(int32_t) * (size_t)count);
    HIP_TRY(hipMallocAsync((void**)&tmp, fb + sb + 256 + al(tb), g->st));
    uint8_t* dstats = (uint8_t*)tmp;
    int32_t* sel = (int32_t*)(tmp + fb);
    int32_t* dcount = (int32_t*)(tmp + fb + sb);
    sdmm_training_out o{};
    for (int i = 0; i < 6; ++i) o.x[i] = R.plane(i) + R.n;
    for (int i = 0; i < 3; ++i) o.normal[i] = R.plane(6 + i) + R.n;
    o.w = R.plane(9) + R.n;
    o.stats = dstats;
    o.node = R.nodes() + R.n;
    o.capacity = count;
    int64_t got = 0;
    SDMM_TRY(sdmm_detail::push_training_ex(g->tree, v, g->cfg.saved_per_path, seed, &o, &got, nullptr, nullptr, true,
                                           count));
    clk.lap("push:write");
    // the stats entries in record order (leaf order, producer order inside)
    HIP_TRY(hipcub::DeviceSelect::Flagged(tmp + fb + sb + 256, tb, hipcub::CountingInputIterator<int32_t>(0), dstats,
                                          sel, dcount, (int)count, g->st));
    hipLaunchKernelGGL(stats_append_kernel, grid_for(count), dim3(256), 0, g->st, sel, dcount, R.plane(0) + R.n, R.cap,
                       R.nodes() + R.n, S.plane(0) + S.n, S.cap, S.nodes() + S.n);
    HIP_TRY(hipGetLastError());
    int32_t ns = 0;
    HIP_TRY(hipMemcpyAsync(&ns, dcount, sizeof(int32_t), hipMemcpyDeviceToHost, g->st));
    HIP_TRY(hipFreeAsync(tmp, g->st));
    HIP_TRY(hipStreamSynchronize(g->st));
    R.n += count;
    S.n += ns;
    clk.lap("push");
    return SDMM_OK;
}

// optimize() (volpath_sdmm.cpp:244-312) with the render loop's spp accounting
// (:495-506): split, canBeOptimized (:140-149), initialise new leaves
// (initializeSDMMContext with hmax(diagonal), :132-138, :291-293), 2 EM
// iterations while iterations_run < 4 else 1 (:299-305), drop their data,
// bind the trained leaves for the next render pass.
int sdmm_guiding_optimize(sdmm_guiding* g, int spp, sdmm_guiding_stats* out) {
    if (!g || spp < 0) return fail(SDMM_E_INVALID, "invalid argument");
    HIP_TRY(hipSetDevice(g->device));
    SDMM_TRY(update(g));   // async: no split while an EM runs
    PhaseClock clk(g->st);
    Pool& R = g->rec;
    Pool& S = g->stat;
    // (1) split_leaf_recurse(i, threshold) for every node while leaf_nodes() <=
    // the cap (:253-259), each leaf with its own stats positions in push order
    // (only a leaf holding more than the threshold can split)
    const int old_nodes = sdmm_stree_num_nodes(g->tree);
    if (sdmm_stree_leaf_nodes(g->tree) <= g->cfg.max_leaf_nodes) {
        std::vector<uint8_t> none((size_t)old_nodes, 0);
        SDMM_TRY(order_pool(g, S, none));
        std::vector<int32_t> ch(2 * (size_t)old_nodes), nodes;
        SDMM_TRY(sdmm_stree_get_nodes(g->tree, nullptr, ch.data(), nullptr));
        std::vector<int64_t> counts, starts;
        for (int v = 0; v < old_nodes; ++v) {
            const int64_t a = S.seg[(size_t)(old_nodes + v)], m = S.seg[(size_t)(old_nodes + v + 1)] - a;
            if (ch[2 * (size_t)v] >= 0 || m <= g->cfg.split_threshold) continue;
            nodes.push_back(v);
            counts.push_back(m);
            starts.push_back(a);
        }
        if (!nodes.empty()) {
            // the splitting leaves' stats positions stay on the device: the
            // split runs there (sdmm_stree_split_leaf_recurse_device, node
            // arrays identical to the host split's)
            clk.lap("split:order");
            const float* planes[3] = {S.plane(0), S.plane(1), S.plane(2)};
            SDMM_TRY(sdmm_stree_split_leaf_recurse_device(g->tree, (int)nodes.size(), nodes.data(), planes,
                                                          starts.data(), counts.data(), g->cfg.split_threshold));
        }
    }
    clk.lap("split");
    if (sdmm_stree_num_nodes(g->tree) != old_nodes) SDMM_TRY(redistribute(g, old_nodes));
    clk.lap("redistribute");
    const int nn = sdmm_stree_num_nodes(g->tree);
    std::vector<float> aabb(6 * (size_t)nn);
    std::vector<int32_t> child(2 * (size_t)nn);
    SDMM_TRY(sdmm_stree_get_nodes(g->tree, aabb.data(), child.data(), nullptr));
    // (2) records and stats per leaf: counted in place (the pools are reordered
    // once, by readiness, below; the stats pool at the next split)
    std::vector<uint8_t> ready((size_t)nn, 0);
    std::vector<int64_t> rcount, scount;
    SDMM_TRY(pool_counts(g, R, S, nn, rcount, scount));
    int n_ready = 0;
    for (int v = 0; v < nn; ++v) {
        const int64_t n_data = rcount[(size_t)v];
        const int64_t n_stats = scount[(size_t)v];
        if ((g->total_spp > 12 || n_data > 1000) && child[2 * (size_t)v] < 0 && n_stats >= 64 && n_data >= 8) {
            ready[(size_t)v] = 1;
            ++n_ready;
        }
    }
    clk.lap("order");
    g->total_spp += spp;
    if (out) {
        out->leaves = sdmm_stree_leaf_nodes(g->tree);
        out->optimized = n_ready;
        out->records = std::accumulate(rcount.begin(), rcount.end(), (int64_t)0);   // dropped ones not counted
    }
    ++g->iteration;
    if (n_ready == 0) return bind(g);
    // (3) the ready leaves' records as one prefix, in leaf order
    SDMM_TRY(order_pool(g, R, ready));
    clk.lap("init:order");
    std::vector<sdmm_mix*> mixes;
    std::vector<int64_t> bseg{0};
    const int K = g->cfg.K, npos = K / 8;
    float* P = R.p[R.cur];
    const int64_t cap = R.cap;
    // new leaves: initializeSDMMContext from the first K/8 records' positions
    // and normals (kMeansPlusPlus off, mixture_model_init.h:139-141), spatial
    // distance 3 hmax(diagonal) / (K/8) (:132-135); one gather, one init batch
    std::vector<int> fresh;
    std::vector<int64_t> starts;
    for (int v = 0; v < nn; ++v)
        if (ready[(size_t)v] && !g->mix[(size_t)v]) {
            fresh.push_back(v);
            starts.push_back(R.seg[(size_t)v]);
        }
    if (!fresh.empty()) {
        const int nf = (int)fresh.size();
        int64_t* dstart = nullptr;
        float* dinit = nullptr;
        HIP_TRY(hipMallocAsync((void**)&dstart, sizeof(int64_t) * (size_t)nf, g->st));
        HIP_TRY(hipMallocAsync((void**)&dinit, sizeof(float) * 6 * (size_t)npos * (size_t)nf, g->st));
        HIP_TRY(hipMemcpyAsync(dstart, starts.data(), sizeof(int64_t) * (size_t)nf, hipMemcpyHostToDevice, g->st));
        hipLaunchKernelGGL(init_gather_kernel, grid_for((int64_t)nf * npos), dim3(256), 0, g->st, P, cap, dstart,
                           nf, npos, dinit);
        HIP_TRY(hipGetLastError());
        std::vector<float> init(6 * (size_t)npos * (size_t)nf);
        HIP_TRY(hipMemcpyAsync(init.data(), dinit, sizeof(float) * init.size(), hipMemcpyDeviceToHost, g->st));
        HIP_TRY(hipFreeAsync(dstart, g->st));
        HIP_TRY(hipFreeAsync(dinit, g->st));
        HIP_TRY(hipStreamSynchronize(g->st));
        clk.lap("init:gather");
        std::vector<float> pos(3 * (size_t)npos * (size_t)nf), nrm(3 * (size_t)npos * (size_t)nf), dist((size_t)nf);
        std::vector<uint64_t> seeds((size_t)nf);
        std::vector<sdmm_mix*> made((size_t)nf, nullptr);
        sdmm_em_params ep;
        sdmm_em_params_default(&ep);
        int r = sdmm_create_many_on_stream(K, &ep, g->device, (void*)(g->async ? g->em_st : g->st), nf, made.data());
        if (r) return r;
        clk.lap("init:create");
        for (int i = 0; i < nf; ++i) {
            const int v = fresh[(size_t)i];
            for (int j = 0; j < npos; ++j)
                for (int f = 0; f < 3; ++f) {
                    const size_t o = ((size_t)i * npos + (size_t)j) * 6;
                    pos[((size_t)i * npos + (size_t)j) * 3 + (size_t)f] = init[o + (size_t)f];
                    nrm[((size_t)i * npos + (size_t)j) * 3 + (size_t)f] = init[o + 3 + (size_t)f];
                }
            float diag = 0.0f;
            for (int a3 = 0; a3 < 3; ++a3)
                diag = std::max(diag, aabb[6 * (size_t)v + 3 + a3] - aabb[6 * (size_t)v + a3]);
            // initializeSDMMContext(context, hmax(diag)) (:292); the async run
            // passes 0.1 * hmax(diag) (:218)
            const float maxd = g->async ? 0.1f * diag : diag;
            dist[(size_t)i] = (float)(3.0 * (double)maxd / (double)npos);
            seeds[(size_t)i] = g->cfg.init_seed + (uint64_t)v;
        }
        r = sdmm_init_hemisphere_batched(made.data(), nf, pos.data(), nrm.data(), g->cfg.depth_prior, dist.data(),
                                         seeds.data());
        if (r) {
            for (sdmm_mix* m : made) sdmm_destroy(m);
            return r;
        }
        for (int i = 0; i < nf; ++i) g->mix[(size_t)fresh[(size_t)i]] = made[(size_t)i];
        clk.lap("init:hemi");
    }
    for (int v = 0; v < nn; ++v) {
        if (!ready[(size_t)v]) continue;
        mixes.push_back(g->mix[(size_t)v]);
        bseg.push_back(R.seg[(size_t)v + 1]);
    }
    std::vector<int> iters(mixes.size(), 1);   // async: one em_step per leaf (:220)
    if (!g->async) {
        SDMM_TRY(sdmm_iterations_run(mixes.data(), (int)mixes.size(), iters.data()));
        for (int& it : iters) it = it < 4 ? 2 : 1;   // (:299-302)
    }
    clk.lap("init");
    const int64_t prefix = bseg.back();
    sdmm_samples smp{};
    if (!g->async) {
        for (int i = 0; i < 6; ++i) smp.x[i] = P + i * cap;
        smp.w = P + 9 * cap;
        smp.n = prefix;
        SDMM_TRY(sdmm_em_step_batched_iters(mixes.data(), (int)mixes.size(), &smp, bseg.data(), iters.data()));
    } else {
        // the swap to training_data (:208-212): the prefix moves to the EM's own
        // buffer (the pool keeps taking the next pass's records), the EM is
        // enqueued on its stream and runs beside the next pass (:214-223)
        if (prefix > g->tcap) {
            HIP_TRY(hipStreamSynchronize(g->em_st));
            if (g->tbuf) HIP_TRY(hipFree(g->tbuf));
            g->tbuf = nullptr;
            g->tcap = 0;
            const int64_t want = prefix + prefix / 2;
            HIP_TRY(hipMalloc((void**)&g->tbuf, sizeof(float) * 7 * (size_t)want));
            g->tcap = want;
        }
        for (int f = 0; f < 7; ++f)
            HIP_TRY(hipMemcpyAsync(g->tbuf + f * g->tcap, P + (f < 6 ? f : 9) * cap, sizeof(float) * (size_t)prefix,
                                   hipMemcpyDeviceToDevice, g->st));
        HIP_TRY(hipEventRecord(g->copied, g->st));
        HIP_TRY(hipStreamWaitEvent(g->em_st, g->copied, 0));
        for (int i = 0; i < 6; ++i) smp.x[i] = g->tbuf + i * g->tcap;
        smp.w = g->tbuf + 6 * g->tcap;
        smp.n = prefix;
        SDMM_TRY(sdmm_em_step_batched_iters(mixes.data(), (int)mixes.size(), &smp, bseg.data(), iters.data()));
        HIP_TRY(hipEventRecord(g->em_done, g->em_st));
        g->running = true;
        g->pending.clear();
        for (int v = 0; v < nn; ++v)
            if (ready[(size_t)v]) g->pending.push_back(v);
    }
    clk.lap("em");
    // (4) the optimised leaves' data is cleared (:308-309): drop the prefix
    if (prefix > 0) {
        const int64_t rest = R.n - prefix;
        float* Q = R.p[1 - R.cur];
        if (rest > 0) {
            for (int f = 0; f < kPlanes; ++f)
                HIP_TRY(hipMemcpyAsync(Q + f * cap, P + f * cap + prefix, sizeof(float) * (size_t)rest,
                                       hipMemcpyDeviceToDevice, g->st));
            HIP_TRY(hipMemcpyAsync(R.node[1 - R.cur], R.node[R.cur] + prefix, sizeof(int32_t) * (size_t)rest,
                                   hipMemcpyDeviceToDevice, g->st));
        }
        R.cur = 1 - R.cur;
        R.n = rest;
    }
    SDMM_TRY(bind(g));
    HIP_TRY(hipStreamSynchronize(g->st));
    clk.lap("drop+bind");
    return SDMM_OK;
}

// One iteration of render(): a render pass (guided once any leaf is trained,
// :311-316), its training data, then optimize() while training
// (m_still_training, :416, :495-501).
int sdmm_guiding_iteration(sdmm_guiding* g, sdmm_scene* scene, const sdmm_li_params* p, uint64_t push_seed,
                           int train, float* image, float* image_sqr, sdmm_li_stats* li_stats,
                           sdmm_guiding_stats* out) {
    if (!g || !scene || !p || !image) return fail(SDMM_E_INVALID, "invalid argument");
    sdmm_li_params q = *p;
    q.guided = sdmm_guiding_trained(g) > 0 ? 1 : 0;
    sdmm_path_vertices v{};
    SDMM_TRY(sdmm_li_render(scene, g->tree, nullptr, &q, image, image_sqr, train ? &v : nullptr, li_stats));
    if (train) SDMM_TRY(sdmm_guiding_push(g, &v, push_seed));
    SDMM_TRY(update(g));   // (:446-448, after every pass)
    if (!train) return SDMM_OK;
    return sdmm_guiding_optimize(g, p->spp * 1, out);
}

}  // extern "C"
