// kmeanspp.hip -- kMeansPPInit (dmm/jmm/mixture_model_init.h:244-330) on the
// device: the k-means++ choice of a leaf's n_pos seed positions / normals,
// which uniformHemisphereInit (:79-242) expands into K = 8 n_pos components
// when kMeansPlusPlus is set (:130-138).
//
// One workgroup (1024 lanes) per leaf; the n_pos draws are sequential inside
// it.  Draw i is one pass over the leaf's samples -- fold in the distances to
// the position chosen by draw i-1 (:306-328), form the weight (metric^2 for
// i == 0, else minDist^5 * metric unless the sample lies within both
// thresholds of a chosen position, :266-289), sum -- and a partial pass of
// tile-ordered inclusive scans that stops at the first sample whose prefix
// reaches u * S.  Sample j is always handled by lane j mod 1024, so the
// per-sample state (three float minima + the fp64 weight) never crosses lanes.
//
// Arithmetic (oracle/sdmm_oracle_kmeans.c, mode 1): distances in float exactly
// as the reference (no contraction, acos as (float) acos((double) x)); the
// weights and their sums in fp64 instead of the reference's float CDF (the
// choice differs only when u lies within the float CDF's rounding of a
// boundary); uniform fallback j = ceil(u n) - 1 (:292-299).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <mutex>
#include <vector>

#include "../../include/sdmm_gpu.h"
#include "host_xfer.h"

#pragma clang fp contract(off)

namespace sdmm_detail {
int set_error(int code, const char* msg);
}  // namespace sdmm_detail

namespace {

constexpr int KB = 1024;        // lanes per leaf
constexpr int KW = KB / 64;     // waves
constexpr double NORMAL_T = 0.2 * 0.2;     // NORMAL_DISTANCE_TRHESHOLD (:76)
constexpr double SPATIAL_T = 2e-2 * 2e-2;  // SPATIAL_DISTANCE_THRESHOLD (:77)

struct KmppLeaf {
    int64_t s0, n;
};

__device__ inline float metric_of(float w) { return fminf(fmaxf(w, 1e-3f), 3.0f); }   // (:120)

__device__ inline double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

// deterministic block sum (fixed tree), broadcast to every lane
__device__ double block_sum(double v, double* lds) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) lds[wv] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < KW; ++i) s += lds[i];
    return s;
}

__device__ int64_t block_max_i64(int64_t v, int64_t* lds) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t t = __shfl_down(v, o, 64);
        v = t > v ? t : v;
    }
    __syncthreads();
    if (lane == 0) lds[wv] = v;
    __syncthreads();
    int64_t m = lds[0];
    for (int i = 1; i < KW; ++i) m = lds[i] > m ? lds[i] : m;
    return m;
}

// inclusive scan over the workgroup in lane order; *total = the last lane's value
__device__ double block_scan(double v, double* lds, double* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
        const double t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    __syncthreads();
    if (lane == 63) lds[wv] = v;
    __syncthreads();
    double off = 0.0;
    for (int i = 0; i < wv; ++i) off += lds[i];
    double tot = 0.0;
    for (int i = 0; i < KW; ++i) tot += lds[i];
    *total = tot;
    return off + v;
}

__global__ __launch_bounds__(KB) void kmeanspp_kernel(const float* __restrict__ x0, const float* __restrict__ x1,
                                                      const float* __restrict__ x2, const float* __restrict__ n0,
                                                      const float* __restrict__ n1, const float* __restrict__ n2,
                                                      const float* __restrict__ w, const KmppLeaf* __restrict__ leaves,
                                                      int n_pos, const float* __restrict__ u,
                                                      float* __restrict__ mins, double* __restrict__ pdf, int64_t base0,
                                                      int64_t ntot, int64_t* __restrict__ out_idx,
                                                      float* __restrict__ out_pn) {
    __shared__ double lds_d[KW];
    __shared__ int64_t lds_i[KW];
    __shared__ int first;
    const KmppLeaf L = leaves[blockIdx.x];
    const int t = threadIdx.x;
    const int64_t off = L.s0 - base0;
    float* md = mins + off;
    float* msd = mins + ntot + off;
    float* msnd = mins + 2 * ntot + off;
    double* pd = pdf + off;
    float p0 = 0, p1 = 0, p2 = 0, q0 = 0, q1 = 0, q2 = 0;
    for (int pi = 0; pi < n_pos; ++pi) {
        double part = 0.0, rem = 0.0;
        int64_t last_pos = -1;
        for (int64_t j = t; j < L.n; j += KB) {
            const int64_t g = L.s0 + j;
            const double m = (double)metric_of(w[g]);
            double v;
            if (pi == 0) {
                md[j] = msd[j] = msnd[j] = INFINITY;
                v = m * m;
                rem += 1.0;
            } else {
                // min distances to the position of draw pi-1 (:306-328)
                float dot = n0[g] * q0 + n1[g] * q1 + n2[g] * q2;
                dot = fminf(1.0f, fmaxf(-1.0f, dot));
                const float nd = (float)((double)(float)acos((double)dot) / 3.14159265358979323846);
                const float nd2 = nd * nd;
                const float d0 = x0[g] - p0, d1 = x1[g] - p1, d2 = x2[g] - p2;
                const float sd2 = d0 * d0 + d1 * d1 + d2 * d2;
                const float dist = sd2 + nd2;
                float a = md[j], b = msd[j], c = msnd[j];
                if (dist < a) a = dist;
                if ((double)nd2 < NORMAL_T && sd2 < b) {
                    c = nd2;
                    b = sd2;
                }
                md[j] = a; msd[j] = b; msnd[j] = c;
                if ((double)c < NORMAL_T && (double)b < SPATIAL_T) {
                    v = 0.0;
                } else {
                    const double d = (double)a;
                    const double dd = d * d;
                    v = dd * dd * d * m;
                    rem += 1.0;
                }
            }
            pd[j] = v;
            part += v;
            if (v > 0.0) last_pos = j;
        }
        const double S = block_sum(part, lds_d);
        const double R = block_sum(rem, lds_d);
        const int64_t LP = block_max_i64(last_pos, lds_i);
        const float uf = u[(int64_t)blockIdx.x * n_pos + pi];
        int64_t chosen;
        if (R > 0.0 && S > 0.0) {
            const double target = (double)uf * S;
            double run = 0.0;
            chosen = -1;
            for (int64_t tb = 0; tb < L.n; tb += KB) {
                const int64_t j = tb + t;
                const double v = j < L.n ? pd[j] : 0.0;
                double tot;
                const double c = block_scan(v, lds_d, &tot);
                if (t == 0) first = KB;
                __syncthreads();
                if (j < L.n && run + c >= target) atomicMin(&first, t);
                __syncthreads();
                const int f = first;
                __syncthreads();
                if (f < KB) {
                    chosen = tb + f;
                    break;
                }
                run += tot;
            }
            if (chosen < 0) chosen = LP;
        } else {
            const double c = ceil((double)uf * (double)L.n) - 1.0;
            chosen = c < 0.0 ? 0 : (c > (double)(L.n - 1) ? L.n - 1 : (int64_t)c);
        }
        const int64_t g = L.s0 + chosen;
        p0 = x0[g]; p1 = x1[g]; p2 = x2[g];
        q0 = n0[g]; q1 = n1[g]; q2 = n2[g];
        if (t == 0) {
            const int64_t o = (int64_t)blockIdx.x * n_pos + pi;
            out_idx[o] = chosen;
            float* pn = out_pn + 6 * o;
            pn[0] = p0; pn[1] = p1; pn[2] = p2;
            pn[3] = q0; pn[4] = q1; pn[5] = q2;
        }
    }
}

int kfail(int code, const std::string& msg) { return sdmm_detail::set_error(code, msg.c_str()); }

}  // namespace

extern "C" {

int sdmm_kmeanspp_select(const sdmm_samples* s, const float* const normals[3], const int64_t* seg, int n_leaves,
                         int n_pos, const float* uniforms, int device, void* hip_stream, int64_t* out_index,
                         float* out_positions, float* out_normals) {
    if (!s || !normals || !seg || n_leaves < 0 || n_pos <= 0 || (n_leaves > 0 && (!uniforms || !out_index)))
        return kfail(SDMM_E_INVALID, "sdmm_kmeanspp_select: invalid argument");
    if (n_leaves == 0) return SDMM_OK;
    for (int i = 0; i < 3; ++i)
        if (!s->x[i] || !normals[i]) return kfail(SDMM_E_INVALID, "sdmm_kmeanspp_select: NULL plane");
    if (!s->w) return kfail(SDMM_E_INVALID, "sdmm_kmeanspp_select: NULL weights");
    std::vector<KmppLeaf> lv((size_t)n_leaves);
    for (int l = 0; l < n_leaves; ++l) {
        if (seg[l + 1] <= seg[l]) return kfail(SDMM_E_INVALID, "sdmm_kmeanspp_select: a leaf without samples");
        if (seg[l] < 0 || seg[l + 1] > s->n) return kfail(SDMM_E_INVALID, "sdmm_kmeanspp_select: segment outside");
        lv[(size_t)l] = KmppLeaf{seg[l], seg[l + 1] - seg[l]};
    }
    const int64_t base0 = seg[0], ntot = seg[n_leaves] - seg[0];
    hipStream_t st = (hipStream_t)hip_stream;
    hipError_t e = hipSetDevice(device);
    // scratch: the leaf table, the draws, three float minima and the fp64
    // weight per sample, the chosen indices
    const size_t o_u = ((sizeof(KmppLeaf) * (size_t)n_leaves + 255) / 256) * 256;
    const size_t nu = (size_t)n_leaves * (size_t)n_pos;
    const size_t o_min = o_u + ((sizeof(float) * nu + 255) / 256) * 256;
    const size_t o_pdf = o_min + ((sizeof(float) * 3 * (size_t)ntot + 255) / 256) * 256;
    const size_t o_idx = o_pdf + sizeof(double) * (size_t)ntot;
    const size_t o_pn = o_idx + ((sizeof(int64_t) * nu + 255) / 256) * 256;
    const size_t total = o_pn + sizeof(float) * 6 * nu;
    // the scratch: the (device, stream) pool entry, held until the stream sync
    // below; host data moves through the thread's pinned bounce buffer (host
    // transfer rules, sdmm_api.cpp)
    if (device < 0) return kfail(SDMM_E_INVALID, "sdmm_kmeanspp_select: device index out of range");
    sdmm_detail::StreamScratch* sc = nullptr;
    std::unique_lock<std::mutex> hold = sdmm_detail::stream_scratch(device, st, &sc);
    if (e == hipSuccess) e = sdmm_detail::scratch_reserve(*sc, total);
    char* d = sc->p;
    const size_t o_hu = ((sizeof(KmppLeaf) * lv.size() + 15) / 16) * 16;   // pinned: leaves, draws
    const size_t o_hi = o_hu + ((sizeof(float) * nu + 15) / 16) * 16;       // then the results back
    const size_t o_hp = o_hi + ((sizeof(int64_t) * nu + 15) / 16) * 16;
    char* pin = nullptr;
    if (e == hipSuccess) e = sdmm_detail::bounce_buf(o_hp + sizeof(float) * 6 * nu, &pin);
    if (e == hipSuccess) {
        std::memcpy(pin, lv.data(), sizeof(KmppLeaf) * lv.size());
        std::memcpy(pin + o_hu, uniforms, sizeof(float) * nu);
        e = hipMemcpyAsync(d, pin, sizeof(KmppLeaf) * lv.size(), hipMemcpyHostToDevice, st);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(d + o_u, pin + o_hu, sizeof(float) * nu, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(kmeanspp_kernel, dim3((unsigned)n_leaves), dim3(KB), 0, st, s->x[0], s->x[1], s->x[2],
                           normals[0], normals[1], normals[2], s->w, (const KmppLeaf*)d, n_pos,
                           (const float*)(d + o_u), (float*)(d + o_min), (double*)(d + o_pdf), base0, ntot,
                           (int64_t*)(d + o_idx), (float*)(d + o_pn));
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(pin + o_hi, d + o_idx, sizeof(int64_t) * nu, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess && (out_positions || out_normals))
        e = hipMemcpyAsync(pin + o_hp, d + o_pn, sizeof(float) * 6 * nu, hipMemcpyDeviceToHost, st);
    {   // always: the scratch and the bounce buffer are reused only when idle
        const hipError_t es = hipStreamSynchronize(st);
        if (e == hipSuccess) e = es;
    }
    if (e != hipSuccess) return kfail(SDMM_E_HIP, std::string("sdmm_kmeanspp_select: ") + hipGetErrorString(e));
    std::memcpy(out_index, pin + o_hi, sizeof(int64_t) * nu);
    const float* pn = (const float*)(pin + o_hp);
    for (size_t i = 0; i < nu; ++i)
        for (int a = 0; a < 3; ++a) {
            if (out_positions) out_positions[3 * i + a] = pn[6 * i + a];
            if (out_normals) out_normals[3 * i + a] = pn[6 * i + 3 + a];
        }
    return SDMM_OK;
}

}  // extern "C"
