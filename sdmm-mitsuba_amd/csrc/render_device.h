// render_device.h -- records shared by the device Li / training producer
// (render.hip) and their host launchers (render_api.cpp, sdmm_api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdmm {

// ---- counter-based RNG (host + device; oracle/sdmm_oracle_train.c restates) ----
__host__ __device__ __forceinline__ uint64_t rng_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// uniform in [0, 1): 24 random bits, exact in float
__host__ __device__ __forceinline__ float rng_uniform(uint64_t seed, uint64_t path, uint32_t stream, uint32_t dim) {
    const uint64_t k = rng_mix(rng_mix(seed ^ (path * 0xD1B54A32D192ED03ull)) + (((uint64_t)stream << 16) | dim));
    return (float)(uint32_t)(k >> 40) * (1.0f / 16777216.0f);
}
// streams: 0 camera; 1 + b bounce b (dims: 0-1 BSDF sample, 2 BSDF/guide
// choice, 3-5 guide sample, 6 roulette); kJitterStream + d: vertex d's jitters
constexpr uint32_t kJitterStream = 1024;

constexpr int kVertexFields = 16;          // weight 3, throughput 3, pdf, point 6, normal 3

struct QuadDev {
    float p0[3], e1[3], e2[3];   // corner and edges (world)
    float n[3];                  // unit normal (flipNormals applied)
    float g1[3], g2[3];          // dual vectors: (p - p0).g1, (p - p0).g2 in [0, 1] on the quad
    int bsdf, emitter;           // emitter -1: none
};

// Per-BSDF parameters beside the diffuse reflectance (kBsdfParams floats per
// BSDF): [0] kind (0 diffuse, 1 smooth plastic, 2 rough conductor).
// Plastic: [1..3] specular reflectance, [4] eta = intIOR / extIOR, [5] 1 /
// eta^2, [6] the internal diffuse Fresnel reflectance fdrInt, [7] the
// specular sampling weight sAvg / (dAvg + sAvg) (bsdfs/plastic.cpp:159-200).
// Rough conductor: [1..3] specular reflectance, [4] eta, [5] k (a gray
// conductor), [6] the Beckmann alpha, [7] unused (bsdfs/roughconductor.cpp).
constexpr int kBsdfParams = 8;
constexpr int kBsdfDiffuse = 0;
constexpr int kBsdfPlastic = 1;
constexpr int kBsdfConductor = 2;

struct SceneDev {
    const QuadDev* quads;
    int n_quads;
    const float* refl;    // 3 per BSDF (plastic: its diffuseReflectance)
    const float* bpar;    // kBsdfParams per BSDF; null: every BSDF diffuse
    const float* lmodel;  // kLearnedStride per BSDF: [M, M SDMM4 records] (learned_bsdf.h); null: none
    const float* rad;     // 3 per emitter
    float cam[12];        // camera-to-world 3x4 (row major)
    float tanx, aspect, near_clip;
    int width, height;
    float smin[3], snorm;
};

struct PathsDev {
    float *px, *py, *pz;     // current hit point
    float *dx, *dy, *dz;     // direction of the ray that reached it
    float *tr, *tg, *tb;     // throughput
    float *lr, *lg, *lb;     // Li
    int* depth;              // rRec.depth; -1 once the path has ended
    int* quad;               // hit quad
    int* nv;                 // saved vertices
    int* nray;               // traced bounce rays (a delta bounce saves no vertex)
    float* rec;              // vertex records: rec[(f * V + v) * P + p]
    int V;
    int64_t P;
};

struct QueryDev {
    float *c0, *c1, *c2;     // condition
    float *u0, *u1, *u2;     // guide sample
    float *b0, *b1, *b2;     // BSDF direction (world)
    uint8_t* mode;           // 1: BSDF chosen (pdf query), 0: guide sample
    float *d0, *d1, *d2;     // wavefront outputs (compact: query j = path idx[j])
    float* pdf;
    int32_t* comp;
    // compaction of the live guided queries: flag per path, the selected
    // path ids, each path's compact slot (-1: no query), compact inputs
    uint8_t* live;
    int32_t* idx;
    int32_t* slot;
    float *k_c0, *k_c1, *k_c2, *k_u0, *k_u1, *k_u2, *k_b0, *k_b1, *k_b2;
    uint8_t* k_mode;
    // product sampling (sampleProduct): the BSDF/guide draw per path (the
    // wavefront decides with the query's own h), and per compact query the
    // shading frame (row-major, columns s t n), the material and h out
    float* ch;
    float* k_ch;
    float* k_F[9];
    int32_t* k_mat;
    float* hq;
    // the loop head's BSDF sample for the shade kernel (non-diffuse BSDFs):
    // sampled lobe delta (1) or smooth (0), its weight (RGB) and pdf
    uint8_t* bdelta;
    float *bw0, *bw1, *bw2, *bpdf;
    // product with a rough conductor's learned BSDF: compact query j's lobes
    // (weights, local means, covariances) at row lrow0 + j of the render's
    // extended learned-BSDF table (lM lobes a row); lw null: no such material
    float *lw, *lm, *lc;
    int lrow0, lM;
};

}  // namespace sdmm
