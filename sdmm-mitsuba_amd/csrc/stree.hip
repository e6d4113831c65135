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
