// valu_rates.hip -- issue-rate microbenchmark for the VALU instructions the
// E-step kernels are built from (gfx950).  Each variant runs a long loop of
// independent instructions (8 chains per lane) with a chip-full of waves
// (--wps per SIMD), so the measured rate is throughput, not latency.
// Output: SIMD-cycles per wave-instruction at the clock given by --mhz.
//
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/_bin/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

#define SCALAR_KERNEL(NAME, ASM, INIT)                                                    \
__global__ void NAME(float* out, int iters, float b, float c) {                           \
    float a[8];                                                                           \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * (j + 1) * INIT;   \
    for (int i = 0; i < iters; ++i) {                                                     \
        _Pragma("unroll") for (int r = 0; r < 2; ++r)                                     \
        _Pragma("unroll") for (int j = 0; j < 8; ++j)                                     \
            asm volatile(ASM : "+v"(a[j]) : "v"(b), "v"(c));                              \
    }                                                                                     \
    float s = 0;                                                                          \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) s += a[j];                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                       \
}

SCALAR_KERNEL(k_fma, "v_fma_f32 %0, %1, %2, %0", 1e-3f)
SCALAR_KERNEL(k_mul, "v_mul_f32 %0, %1, %0", 1e-3f)
SCALAR_KERNEL(k_max, "v_max_f32 %0, %1, %0", 1e-3f)
SCALAR_KERNEL(k_exp, "v_exp_f32 %0, %0", 1e-5f)
SCALAR_KERNEL(k_rsq, "v_rsq_f32 %0, %0", 1e-3f)
SCALAR_KERNEL(k_cnd, "v_cmp_gt_f32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %2, vcc", 1e-3f)

__global__ void k_pkfma(float* out, int iters, float b, float c) {
    f2 a[8];
    const f2 bb = {b, b + 1}, cc = {c, c + 1};
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = f2{threadIdx.x * (j + 1) * 1e-3f, (float)j};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(bb), "v"(cc));
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j].x + a[j].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// packed FMA with a wave-uniform SGPR-pair operand broadcast to both halves
__global__ void k_pkfma_s(float* out, int iters, float b, float c) {
    f2 a[8];
    const f2 cc = {c, c + 1};
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = f2{threadIdx.x * (j + 1) * 1e-3f, (float)j};
    const f2 sb = {b, b};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(a[j]) : "s"(sb), "v"(cc));
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j].x + a[j].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 3 FMA : 1 exp, the E-step's rough mix of plain and transcendental VALU
__global__ void k_mix(float* out, int iters, float b, float c) {
    float a[8], e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = threadIdx.x * (j + 1) * 1e-3f; e[j] = a[j] * 1e-2f; }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            asm volatile("v_fma_f32 %0, %2, %3, %0\n\tv_fma_f32 %0, %2, %3, %0\n\t"
                         "v_fma_f32 %0, %2, %3, %0\n\tv_exp_f32 %1, %1"
                         : "+v"(a[j]), "+v"(e[j]) : "v"(b), "v"(c));
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + e[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(float*, int, float, float);

int main(int argc, char** argv) {
    double mhz = 2400;
    int wps = 8;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--mhz") && i + 1 < argc) mhz = atof(argv[++i]);
        if (!strcmp(argv[i], "--wps") && i + 1 < argc) wps = atoi(argv[++i]);
    }
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int threads = 256;          // 4 waves per block: one per SIMD
    const int blocks = cus * wps;     // -> wps waves per SIMD
    const int iters = 4096;
    float* out;
    CHECK(hipMalloc(&out, sizeof(float) * blocks * threads));
    struct { const char* name; kfn f; int insts; } vs[] = {
        {"v_fma_f32", k_fma, 16},
        {"v_mul_f32", k_mul, 16},
        {"v_max_f32", k_max, 16},
        {"v_pk_fma_f32", k_pkfma, 16},
        {"v_pk_fma_f32 (sgpr bcast)", k_pkfma_s, 16},
        {"v_exp_f32", k_exp, 16},
        {"v_rsq_f32", k_rsq, 16},
        {"v_cmp + v_cndmask (2 insts)", k_cnd, 32},
        {"3 v_fma + 1 v_exp", k_mix, 32},
    };
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    printf("CUs %d, %d waves/SIMD, clock assumed %.0f MHz\n", cus, wps, mhz);
    for (auto& v : vs) {
        hipLaunchKernelGGL(v.f, dim3(blocks), dim3(threads), 0, 0, out, 64, 1.0001f, 1e-4f);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(v.f, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0001f, 1e-4f);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double wave_insts = (double)blocks * (threads / 64) * iters * v.insts;
        const double simd_cycles = ms * 1e-3 * mhz * 1e6 * cus * 4;
        printf("%-30s %8.3f ms  %.3f SIMD-cycles per wave-instruction\n", v.name, ms,
               simd_cycles / wave_insts);
    }
    CHECK(hipFree(out));
    return 0;
}
