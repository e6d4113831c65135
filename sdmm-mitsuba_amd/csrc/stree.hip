// stree.hip -- device side of the spatial tree (jmm SNTree, sntree.h:93-299):
// the per-point leaf lookup of SNTreeNode::find (sntree.h:62-83) and the
// routing of a sample batch into leaf-contiguous order for the batched
// per-leaf EM (sdmm_em_step_batched).
//
// Node record (device, 8 x 32 bit): min[3], max[3], child0, child1 (-1 for a
// leaf).  find() in the reference recurses: a point outside a node's AABB
// (inclusive on both sides, Eigen::AlignedBox::contains) is not found there;
// a leaf returns itself; an inner node tries child 0, then child 1.  Children
// split the parent's box, so the recursion is a single descent here: the
// first child whose box contains the point.
#include "sdmm_device.h"

#include <hipcub/hipcub.hpp>

namespace sdmm {

// STNodeDev, box_contains, stree_find_point: sdmm_device.h (shared with guide.hip)

__global__ void stree_find_kernel(const STNodeDev* __restrict__ nodes, int64_t n, const float* __restrict__ p0,
                                  const float* __restrict__ p1, const float* __restrict__ p2,
                                  int32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = stree_find_point(nodes, p0[i], p1[i], p2[i]);
}

// key = node id, or num_nodes for points outside the tree (sorted last)
__global__ void stree_keys_kernel(const STNodeDev* __restrict__ nodes, int num_nodes, int n,
                                  const float* __restrict__ p0, const float* __restrict__ p1,
                                  const float* __restrict__ p2, uint32_t* __restrict__ keys,
                                  int32_t* __restrict__ idx) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int id = stree_find_point(nodes, p0[i], p1[i], p2[i]);
    keys[i] = (uint32_t)(id < 0 ? num_nodes : id);
    idx[i] = i;
}

// seg[v] = first sorted position with key >= v, v = 0..num_nodes (+ the end)
__global__ void stree_seg_kernel(const uint32_t* __restrict__ keys, int n, int num_nodes, int64_t* __restrict__ seg) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v > num_nodes) return;
    int lo = 0, count = n;
    while (count > 0) {
        const int step = count / 2, it = lo + step;
        if (keys[it] < (uint32_t)v) { lo = it + 1; count -= step + 1; }
        else count = step;
    }
    seg[v] = lo;
}

// out[j] = in[perm[j]] for the sample planes
__global__ void stree_gather_kernel(SamplesDev in, int n, const int32_t* __restrict__ perm, float* __restrict__ o0,
                                    float* __restrict__ o1, float* __restrict__ o2, float* __restrict__ o3,
                                    float* __restrict__ o4, float* __restrict__ o5, float* __restrict__ ow,
                                    float* __restrict__ oh, uint8_t* __restrict__ od) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int i = perm[j];
    o0[j] = in.x[0][i]; o1[j] = in.x[1][i]; o2[j] = in.x[2][i];
    o3[j] = in.x[3][i]; o4[j] = in.x[4][i]; o5[j] = in.x[5][i];
    ow[j] = in.w[i];
    if (oh) oh[j] = in.hpdf[i];
    if (od) od[j] = in.isDiffuse[i];
}

hipError_t launch_stree_find(const void* nodes, int64_t n, const float* p0, const float* p1, const float* p2,
                             int32_t* out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(stree_find_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       (const STNodeDev*)nodes, n, p0, p1, p2, out);
    return hipGetLastError();
}

size_t stree_route_temp_bytes(int n, int key_bits) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, n, 0, key_bits);
    return bytes;
}

// keys/idx: 2 x n each; seg_dev: num_nodes + 2 int64; out planes: n each
hipError_t launch_stree_route(const void* nodes, int num_nodes, int key_bits, const SamplesDev& in, int n,
                              uint32_t* keys0, uint32_t* keys1, int32_t* idx0, int32_t* idx1, void* temp,
                              size_t temp_bytes, int64_t* seg_dev, float* const out_x[6], float* out_w,
                              float* out_h, uint8_t* out_d, hipStream_t st) {
    const STNodeDev* nd = (const STNodeDev*)nodes;
    hipLaunchKernelGGL(stree_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, nd, num_nodes, n,
                       in.x[0], in.x[1], in.x[2], keys0, idx0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // stable: samples keep their batch order inside a leaf (deterministic EM input)
    e = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys0, keys1, idx0, idx1, n, 0, key_bits, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(stree_seg_kernel, dim3((unsigned)((num_nodes + 1 + 255) / 256)), dim3(256), 0, st, keys1, n,
                       num_nodes, seg_dev);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(stree_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, in, n, idx1,
                       out_x[0], out_x[1], out_x[2], out_x[3], out_x[4], out_x[5], out_w, out_h, out_d);
    return hipGetLastError();
}

}  // namespace sdmm

// ---------------------------------------------------------------------------
// split_leaf_recurse on device-resident positions (sdmm_stree_split_leaf_
// recurse_device; jmm SNTree::split, sntree.h:235-283, as the library's host
// split restates it).  The recursion runs level by level over "items" (a node
// being split with its samples, contiguous in a level buffer, in the parent's
// sample order); the host makes every per-node decision from the sums these
// kernels return, so the node arrays are those of the sequential recursion
// (renumbered to its creation order on the host).
namespace sdmm {

constexpr int kSplitChunk = 4096;   // samples per reduction chunk (= the host's split_sums)



// per chunk: the fp64 sums (p0, p1, p2, p0^2, p1^2, p2^2) in the canonical
// order: lane t sums samples t, t + 256, ... ; the 256 lane sums fold by a
// binary tree (stride 128 .. 1).  Products are separately rounded (no FMA),
// as on the host.
__global__ void __launch_bounds__(256)
split_sums_kernel(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                  const SplitChunkDev* __restrict__ chunks, double* __restrict__ partial) {
#pragma clang fp contract(off)
    __shared__ double red[6][256];
    const SplitChunkDev c = chunks[blockIdx.x];
    const int t = threadIdx.x;
    double a[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int j = t; j < c.len; j += 256) {
        const double p[3] = {(double)x[c.start + j], (double)y[c.start + j], (double)z[c.start + j]};
        for (int k = 0; k < 3; ++k) {
            a[k] = a[k] + p[k];
            const double sq = p[k] * p[k];
            a[3 + k] = a[3 + k] + sq;
        }
    }
    for (int k = 0; k < 6; ++k) red[k][t] = a[k];
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (t < s)
            for (int k = 0; k < 6; ++k) red[k][t] = red[k][t] + red[k][t + s];
        __syncthreads();
    }
    if (t < 6) partial[6 * (int64_t)blockIdx.x + t] = red[t][0];
}



// split_decide (the library's host split, sdmm_api.cpp) per item on the
// device: the chunk partials folded in chunk order from 0, the mean along the
// axis of largest variance (the first of equals), the children's boxes as
// st_child forms them.  IEEE fp64 / fp32 division, no contraction: bitwise
// the host's decision.
__global__ void __launch_bounds__(256)
split_decide_kernel(const SplitItemDev* __restrict__ items, int n_items, const double* __restrict__ partial,
                    int threshold, SplitCandDev* __restrict__ cand, SplitDecisionDev* __restrict__ dec) {
#pragma clang fp contract(off)
    const int it = blockIdx.x * blockDim.x + threadIdx.x;
    if (it >= n_items) return;
    const SplitItemDev I = items[it];
    SplitCandDev c;
    for (int a = 0; a < 3; ++a) c.mn0[a] = c.mx0[a] = c.mn1[a] = c.mx1[a] = 0.0f;
    c.active = 0;
    c.child_item[0] = c.child_item[1] = 0;
    c.pad = 0;
    c.start = I.start;
    c.n = I.n;
    c.out[0] = c.out[1] = 0;
    SplitDecisionDev d{0, 0, 0.0f, 0};
    if (I.n > threshold) {
        double s[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        for (int ch = I.c0; ch < I.c1; ++ch)
            for (int k = 0; k < 6; ++k) s[k] = s[k] + partial[6 * (int64_t)ch + k];
        float m[3], var[3];
        for (int a = 0; a < 3; ++a) {
            const double mu = s[a] / (double)I.n;
            m[a] = (float)mu;
            const double sq = mu * mu;
            var[a] = (float)(s[3 + a] / (double)I.n - sq);
        }
        int ax = 0;
        for (int a = 0; a < 3; ++a)
            if (var[a] > var[ax]) ax = a;
        const float split = (m[ax] - I.mn[ax]) / (I.mx[ax] - I.mn[ax]);
        if (split > 0.0f && split < 1.0f) {
            for (int a = 0; a < 3; ++a) {
                c.mn0[a] = c.mn1[a] = I.mn[a];
                c.mx0[a] = c.mx1[a] = I.mx[a];
            }
            const float diag = I.mx[ax] - I.mn[ax];
            const float d0 = split * diag;
            c.mn0[ax] = I.mn[ax] + d0;
            const float d1 = (1.0f - split) * diag;
            c.mx1[ax] = I.mx[ax] - d1;
            c.active = 1;
            d = SplitDecisionDev{1, ax, split, 0};
        }
    }
    cand[it] = c;
    dec[it] = d;
}

__device__ __forceinline__ bool split_in(const float* mn, const float* mx, float a, float b, float c) {
    return mn[0] <= a && a <= mx[0] && mn[1] <= b && b <= mx[1] && mn[2] <= c && c <= mx[2];
}

// children's sample counts of the candidate splits from the flags' exclusive
// scan: item it's child c holds rank[2 start + (c + 1) n] - rank[2 start + c n]
// (rank has 2 n_level + 1 entries: the last is the total)
__global__ void split_counts_kernel(const SplitCandDev* __restrict__ cand, int n_items,
                                    const int64_t* __restrict__ rank, long long* __restrict__ counts) {
    const int it = blockIdx.x * blockDim.x + threadIdx.x;
    if (it >= n_items) return;
    const SplitCandDev& c = cand[it];
    const int64_t b = 2 * c.start;
    counts[2 * it] = (long long)(rank[b + c.n] - rank[b]);
    counts[2 * it + 1] = (long long)(rank[b + 2 * c.n] - rank[b + c.n]);
}

// stable partition into the next level: item it's child-0 members then its
// child-1 members, each in the item's sample order.  flags[2 start + j] (c0),
// flags[2 start + n + j] (c1): the layout the exclusive scan turns into ranks.
__global__ void __launch_bounds__(256)
split_flags_kernel(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                   const int32_t* __restrict__ item, int64_t n, const SplitCandDev* __restrict__ cand,
                   int32_t* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SplitCandDev& c = cand[item[i]];
    const int64_t j = i - c.start;
    int f0 = 0, f1 = 0;
    if (c.active) {
        const float a = x[i], b = y[i], d = z[i];
        f0 = split_in(c.mn0, c.mx0, a, b, d) ? 1 : 0;
        f1 = split_in(c.mn1, c.mx1, a, b, d) ? 1 : 0;
    }
    flags[2 * c.start + j] = f0;
    flags[2 * c.start + c.n + j] = f1;
    if (i == n - 1) flags[2 * n] = 0;   // the scan's last entry: the total
}

// rank[] = exclusive scan of flags; the child's members land at its out
// offset + (rank - the item's rank at the child's first flag)
__global__ void __launch_bounds__(256)
split_scatter_kernel(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                     const int32_t* __restrict__ item, int64_t n, const SplitCandDev* __restrict__ cand,
                     const int32_t* __restrict__ flags, const int64_t* __restrict__ rank, float* __restrict__ ox,
                     float* __restrict__ oy, float* __restrict__ oz, int32_t* __restrict__ oitem) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int it = item[i];
    const SplitCandDev& c = cand[it];
    if (!c.active) return;
    const int64_t j = i - c.start;
    const int64_t e0 = 2 * c.start + j, e1 = 2 * c.start + c.n + j;
    const int64_t b0 = rank[2 * c.start], b1 = rank[2 * c.start + c.n];
    if (flags[e0]) {
        const int64_t o = c.out[0] + (rank[e0] - b0);
        ox[o] = x[i]; oy[o] = y[i]; oz[o] = z[i]; oitem[o] = c.child_item[0];
    }
    if (flags[e1]) {
        const int64_t o = c.out[1] + (rank[e1] - b1);
        ox[o] = x[i]; oy[o] = y[i]; oz[o] = z[i]; oitem[o] = c.child_item[1];
    }
}

// gather the splitting leaves' positions into the first level buffer
__global__ void __launch_bounds__(256)
split_load_kernel(const float* __restrict__ px, const float* __restrict__ py, const float* __restrict__ pz,
                  const int64_t* __restrict__ src_start, const int64_t* __restrict__ dst_start, int n_items,
                  int64_t total, float* __restrict__ ox, float* __restrict__ oy, float* __restrict__ oz,
                  int32_t* __restrict__ oitem) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int lo = 0, hi = n_items - 1;        // last item with dst_start <= i
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (dst_start[mid] <= i) lo = mid; else hi = mid - 1;
    }
    const int64_t s = src_start[lo] + (i - dst_start[lo]);
    ox[i] = px[s]; oy[i] = py[s]; oz[i] = pz[s]; oitem[i] = lo;
}

size_t split_scan_temp_bytes(int64_t n) {
    size_t b = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const int32_t*)nullptr, (int64_t*)nullptr, (int)n);
    return b;
}

static inline dim3 split_grid(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

hipError_t launch_split_load(const float* const p[3], const int64_t* src_start, const int64_t* dst_start, int n_items,
                             int64_t total, float* ox, float* oy, float* oz, int32_t* oitem, hipStream_t st) {
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(split_load_kernel, split_grid(total), dim3(256), 0, st, p[0], p[1], p[2], src_start, dst_start,
                       n_items, total, ox, oy, oz, oitem);
    return hipGetLastError();
}

hipError_t launch_split_sums(const float* x, const float* y, const float* z, const void* chunks, int n_chunks,
                             double* partial, hipStream_t st) {
    if (n_chunks <= 0) return hipSuccess;
    hipLaunchKernelGGL(split_sums_kernel, dim3((unsigned)n_chunks), dim3(256), 0, st, x, y, z,
                       (const SplitChunkDev*)chunks, partial);
    return hipGetLastError();
}

// flags + exclusive scan (2 n + 1 entries) + the children's counts per item
hipError_t launch_split_flags(const float* x, const float* y, const float* z, const int32_t* item, int64_t n,
                              const void* cand, int n_items, int32_t* flags, int64_t* rank, void* temp,
                              size_t temp_bytes, long long* counts, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(split_flags_kernel, split_grid(n), dim3(256), 0, st, x, y, z, item, n,
                       (const SplitCandDev*)cand, flags);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, flags, rank, (int)(2 * n + 1), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(split_counts_kernel, split_grid(n_items), dim3(256), 0, st, (const SplitCandDev*)cand,
                       n_items, rank, counts);
    return hipGetLastError();
}

hipError_t launch_split_decide(const void* items, int n_items, const double* partial, int threshold, void* cand,
                               void* dec, hipStream_t st) {
    if (n_items <= 0) return hipSuccess;
    hipLaunchKernelGGL(split_decide_kernel, split_grid(n_items), dim3(256), 0, st, (const SplitItemDev*)items,
                       n_items, partial, threshold, (SplitCandDev*)cand, (SplitDecisionDev*)dec);
    return hipGetLastError();
}

// the stable partition of the accepted splits into the next level
hipError_t launch_split_scatter(const float* x, const float* y, const float* z, const int32_t* item, int64_t n,
                                const void* cand, const int32_t* flags, const int64_t* rank, float* ox, float* oy,
                                float* oz, int32_t* oitem, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(split_scatter_kernel, split_grid(n), dim3(256), 0, st, x, y, z, item, n,
                       (const SplitCandDev*)cand, flags, rank, ox, oy, oz, oitem);
    return hipGetLastError();
}

size_t split_cand_bytes() { return sizeof(SplitCandDev); }
size_t split_chunk_bytes() { return sizeof(SplitChunkDev); }
int split_chunk_samples() { return kSplitChunk; }

}  // namespace sdmm
