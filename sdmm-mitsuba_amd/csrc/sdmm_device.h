// sdmm_device.h -- device-side layouts and helpers shared by the gfx950 kernels.
//
// HBM layouts (all SoA so a wave's 64 lanes touch consecutive addresses):
//   samples      x0..x5, w, [hpdf], [isDiffuse]  one plane per field, N each
//   E-step param ep[f * Kp + k], f < EP_FIELDS    (component k on lane k / CPL)
//   guide param  gp[k * GP_STRIDE + f], f < GP_FIELDS (AoS, see below)
//   stats        compact double [H, wsum, W(K), M(5K), Clow(15K)]  (2 + 21K)
//   partials     float [G][PSTRIDE], one row per E-step workgroup
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sdmm {

// ---- E-step component record (per component k, SoA over k) -----------------
// mu_p (3) | L^{-1} lower 5x5 row-major (15) | to rows 0..2 (9) | detInv | pi
// (pi = 0 for dead/padded components).  The pdf is evaluated in the
// reference's factor order NORM5*exp(-q/2) -> *detInv*J -> *pi so that, with
// the kernel in FTZ/DAZ mode, underflow flushes where the reference's
// flushDenormals=true build flushes (volpath_sdmm.cpp:88-90).
enum : int {
    EP_MU0 = 0, EP_MU1, EP_MU2,
    EP_L00, EP_L10, EP_L11, EP_L20, EP_L21, EP_L22,
    EP_L30, EP_L31, EP_L32, EP_L33,
    EP_L40, EP_L41, EP_L42, EP_L43, EP_L44,
    EP_R00, EP_R01, EP_R02, EP_R10, EP_R11, EP_R12, EP_R20, EP_R21, EP_R22,
    EP_DI, EP_PI,
    // folded forms for the responsibility kernel (no tangent vector needed):
    //   u3 = L30 tp0 + L31 tp1 + L32 tp2 + a (A . d),  A = L33 R0
    //   u4 = L40 tp0 + L41 tp1 + L42 tp2 + a (B . d),  B = L43 R0 + L44 R1
    //   pi pdf = NORM5 exp(-q/2) * a * (detInv pi)
    EP_A0, EP_A1, EP_A2, EP_B0, EP_B1, EP_B2, EP_DIPI,
    // origin-shifted spatial rows for the responsibility kernel:
    //   u_m = sum_j L_mj (p_j - o) + NC_m,  NC_m = -sum_j L_mj (mu_j - o)  (fp64 -> f32)
    // with o = kOrigin (the centre of the normalised scene box), so the
    // subtraction p - mu costs nothing per pair
    EP_NC0, EP_NC1, EP_NC2, EP_NC3, EP_NC4,
    // (1 - |R2|^2) / 2 in fp64, rounded: the component half of the cancellation-free
    // 1 + cos(theta) of the statistics kernels (estep.hip one_plus_c)
    EP_CN,
    EP_FIELDS
};
constexpr float kOrigin = 0.5f;

// ---- guide record (per joint component) -------------------------------------
enum : int {
    GP_W = 0,                            // mixture weight pi_k
    GP_MU0, GP_MU1, GP_MU2,              // spatial mean (marginal mean)
    GP_ML00, GP_ML10, GP_ML11, GP_ML20, GP_ML21, GP_ML22,  // marginal LLT lower
    GP_MDI,                              // marginal detInv
    GP_P00, GP_P01, GP_P02, GP_P10, GP_P11, GP_P12,        // muPremult 2x3
    GP_T00, GP_T01, GP_T02, GP_T10, GP_T11, GP_T12, GP_T20, GP_T21, GP_T22, // to
    GP_CL00, GP_CL10, GP_CL11,           // conditional LLT (2x2 lower)
    GP_CI00, GP_CI01, GP_CI10, GP_CI11,  // conditional L^{-1}
    GP_CDI,                              // conditional detInv
    // RN64(1 / ML_ii) as doubles (two float slots each, 8-byte aligned): the
    // float division r / ML_ii of the marginal's triangular solve is exactly
    // (float)((double) r * RN64(1 / ML_ii)) -- see div_exact in guide.hip
    GP_RML00 = 34, GP_RML11 = 36, GP_RML22 = 38,
    GP_FIELDS = 40
};
// The guide record is AoS, gp[k * GP_STRIDE + f]: a query thread walks the
// components in order with wave-uniform k, so one component's fields come in
// a few wide scalar loads (s_load_dwordx8/x16) instead of one load per field.
constexpr int GP_STRIDE = 40;
static_assert(GP_FIELDS <= GP_STRIDE, "guide record stride");

// Per-component sufficient statistics accumulated by the E-step.
enum : int {
    ST_W = 0, ST_M0, ST_M1, ST_M2, ST_M3, ST_M4,
    ST_C00, ST_C10, ST_C11, ST_C20, ST_C21, ST_C22,
    ST_C30, ST_C31, ST_C32, ST_C33, ST_C40, ST_C41, ST_C42, ST_C43, ST_C44,
    ST_FIELDS  // 21
};

// Canonical per-component arrays (same names/widths as the oracle's or_mixture,
// oracle/sdmm_oracle.h) kept on the device for export and the M-step.
struct CanonDev {
    float* weights;    // K
    float* cdf;        // K
    float* mean;       // K*6
    float* cov;        // K*25
    float* to;         // K*9
    float* cholL;      // K*25
    float* cholLInv;   // K*25
    float* detInv;     // K
    float* muPremult;  // K*6
    float* condCov;    // K*4
    float* margL;      // K*9
    float* margDetInv; // K
    float* condL;      // K*4
    float* condLInv;   // K*4
    float* condDetInv; // K
    int* valid;        // K
};

// Stepwise EM state (stepwise_tangent.h:181-210), device resident, fp64.
struct EmStateDev {
    double* scalars;   // [0]=heuristicTotalWeight [1]=sgH [2]=normalization
                       // [3]=iterationsRun [4]=alpha [5]=niPriorMinusOne
                       // [6]=decreasePrior [7]=trainingCutoff [8]=last status
    double* T;         // K   totalWeightForMixture
    double* sgW;       // K
    double* sgM;       // K*5
    double* sgC;       // K*25 (full, the reference keeps full 5x5)
    float* bPriors;    // K*25
    float* bDepth;     // K*9
};

enum : int {
    SC_HTW = 0, SC_SGH, SC_NORM, SC_IT, SC_ALPHA, SC_NI, SC_DECP, SC_CUT, SC_STATUS, SC_COUNT
};

// The bits of a float VALUE.  Never write __builtin_bit_cast(T, v.y) or
// (T, v[j]) on an ext_vector element: hipcc (ROCm 7.2, clang) lowers a bit
// cast of a vector-element lvalue as a read of element 0 (checked in the IR;
// tests/test_gpu_parity.py test_rare_angle_every_lane_slot is the regression).
__device__ __forceinline__ uint32_t fbits(float x) { return __builtin_bit_cast(uint32_t, x); }

// jmm Coordinates (utils.h:32-48) in float: rows t1, t2, n of the tangent
// frame of the unit vector n
__device__ __forceinline__ void coordinates_f(const float n[3], float to[9]) {
#pragma clang fp contract(off)   // (the header precedes the sources' own pragma)
    float sign = copysignf(1.0f, n[2]);
    const float a = -1.0f / (sign + n[2]);
    const float b = n[0] * n[1] * a;
    to[0] = 1.0f + sign * n[0] * n[0] * a; to[1] = sign * b; to[2] = -sign * n[0];
    to[3] = b; to[4] = sign + n[1] * n[1] * a; to[5] = -n[1];
    to[6] = n[0]; to[7] = n[1]; to[8] = n[2];
}

struct SamplesDev {
    const float* x[6];
    const float* w;
    const float* hpdf;          // nullable
    const uint8_t* isDiffuse;   // nullable
};

// ---- batched per-leaf EM (sdmm_em_step_batched) ------------------------------
// One leaf of the plugin's spatial tree = one mixture with its own contiguous
// sample range of the batch planes (volpath_sdmm.cpp:287-311 runs em_step per
// leaf).  The E-step of leaf i is the single-mixture launch (same chunking,
// same partial rows) relocated to rows [row0, row0 + rows) of a shared buffer.
struct LeafDesc {
    const float* ep;   // E-step record of the leaf's mixture
    double* stats;     // its compact stats [H, wsum, W, M, Clow]
    int64_t s0, n;     // samples [s0, s0 + n) of the batch planes
    int64_t chunk;     // samples per wave (the single-mixture split)
    int row0, rows;    // its partial rows
};
// M-step operands of one mixture (mstep_batched_kernel: one workgroup each)
struct MixDesc {
    CanonDev C;
    EmStateDev S;
    float* ep;
    float* gp;
    const double* stats;
    double* wmean;
    double* wcov;
    int64_t n;
    const double* ncount;   // non-null: the sample count is *ncount (all-reduced over ranks)
};

// scratch of the coherent (Morton) ordering of a guided batch
struct GuideSortScratch {
    uint32_t* keys[2];
    int32_t* idx[2];
    void* temp;
    size_t temp_bytes;
};

// grow-only scratch of the product wavefronts (guide.hip): the thread path's
// per-query pair cache and the full-K wave kernel's per-workgroup pair slices;
// owned by the mixture / tree handle, released with it
struct ProductScratch {
    float* base;
    size_t bytes;
};

// ---- spatial tree node (stree.hip, guide.hip) ------------------------------
// min[3], max[3], child0, child1 (-1 for a leaf).
// device split of the spatial tree (stree.hip, sdmm_stree_split_leaf_recurse_device)
struct SplitChunkDev {
    int64_t start;   // level-buffer index of the chunk's first sample
    int32_t len;
    int32_t pad;
};

// per item: the candidate children's boxes (child 0 = the upper part), or
// inactive (the item is a final leaf: its samples leave the recursion)
struct SplitCandDev {
    float mn0[3], mx0[3], mn1[3], mx1[3];
    int32_t active;
    int32_t child_item[2];   // next-level item ids (final pass)
    int32_t pad;
    int64_t start, n;        // the item's range in the level buffer
    int64_t out[2];          // the children's first index in the next level buffer
};

// per item of a split level, for the decision on the device: the node's box,
// its range in the level buffer and its chunks [c0, c1) of the level's sums
struct SplitItemDev {
    float mn[3], mx[3];
    int64_t start, n;
    int32_t c0, c1;
};
// the decision per item (active 0: at most threshold samples, or degenerate)
struct SplitDecisionDev {
    int32_t active, axis;
    float split;
    int32_t pad;
};

struct STNodeDev {
    float mn[3], mx[3];
    int c0, c1;
};
static_assert(sizeof(STNodeDev) == 32, "node record");

__device__ __forceinline__ bool box_contains(const STNodeDev& n, float x, float y, float z) {
    return n.mn[0] <= x && x <= n.mx[0] && n.mn[1] <= y && y <= n.mx[1] && n.mn[2] <= z && z <= n.mx[2];
}

// SNTreeNode::find (jmm/sntree.h:62-83): depth first, child 0 before child 1,
// into every child whose (inclusive) box holds the point, BACKTRACKING when a
// subtree holds no leaf box with the point (split planes computed as
// min + s diag and max - (1 - s) diag can leave an ulp gap between siblings).
// The greedy descent is the common case; only a dead end restarts as the full
// depth-first search, with the pending siblings on a small stack.
constexpr int kFindStack = 64;
__device__ __forceinline__ int stree_find_point(const STNodeDev* __restrict__ nodes, float x, float y, float z) {
    STNodeDev n = nodes[0];
    if (!box_contains(n, x, y, z)) return -1;
    int id = 0;
    for (int guard = 0; guard < 4096; ++guard) {
        if (n.c0 < 0) return id;
        const STNodeDev a = nodes[n.c0];
        if (box_contains(a, x, y, z)) { id = n.c0; n = a; continue; }
        const int c1 = n.c1;
        const STNodeDev b = nodes[c1];
        if (box_contains(b, x, y, z)) { id = c1; n = b; continue; }
        // dead end below a node that holds the point: the reference's search
        int stack[kFindStack];
        int sp = 0;
        stack[sp++] = 0;
        while (sp > 0) {
            const int i = stack[--sp];
            const STNodeDev m = nodes[i];
            if (m.c0 < 0) return i;
            const STNodeDev m0 = nodes[m.c0], m1 = nodes[m.c1];
            if (box_contains(m1, x, y, z) && sp < kFindStack) stack[sp++] = m.c1;
            if (box_contains(m0, x, y, z) && sp < kFindStack) stack[sp++] = m.c0;
        }
        return -1;
    }
    return -1;
}

constexpr float kHeuristicWeight = 0.5f;     // mixture_model.h:398
constexpr double kPi = 3.14159265358979323846;

// Constant address space: uniform loads from it become scalar (SMEM) loads.
typedef const float __attribute__((address_space(4)))* cfloat_p;
typedef const uint8_t __attribute__((address_space(4)))* cu8_p;

// ---- wave-level helpers (wave64) -------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
        0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}

// Sum over aligned groups of G lanes (G in {8, 16, 32, 64}); every lane of the
// group receives the group sum.  quad_perm/mirror DPP reduce within rows of
// 16 lanes; rows are then combined through v_readlane (SGPR) reads.  (The
// gfx950 permlane16/32 swaps would save two instructions, but ROCm 7.2 folds
// swap(x, x) into x + x, so they are not used.)
template <int G>
__device__ __forceinline__ float group_sum(float x) {
    x += dpp<0xB1>(x);   // quad_perm [1,0,3,2]  (xor 1)
    x += dpp<0x4E>(x);   // quad_perm [2,3,0,1]  (xor 2)
    x += dpp<0x141>(x);  // row_half_mirror      (pairs within 8)
    if constexpr (G == 8) return x;
    x += dpp<0x140>(x);  // row_mirror           (pairs within 16)
    if constexpr (G == 64) {
        const int xi = __builtin_bit_cast(int, x);
        const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(xi, 0));
        const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(xi, 16));
        const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(xi, 32));
        const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(xi, 48));
        x = (r0 + r1) + (r2 + r3);
    } else if constexpr (G == 32) {
        const int xi = __builtin_bit_cast(int, x);
        const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(xi, 0));
        const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(xi, 16));
        const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(xi, 32));
        const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(xi, 48));
        x = ((threadIdx.x & 63) < 32) ? (r0 + r1) : (r2 + r3);
    }
    return x;
}

}  // namespace sdmm
