// store_bw.hip -- write-bandwidth ceiling for the responsibility E-step's
// output stream (537 MB of [N][K] fp32 rows at N = 2^20, K = 128): how fast
// can the chip write that many bytes with no compute at all?
//   plain / nt      : grid-stride 16-B-per-lane stores, 1 KB per wave-instruction
//   rows            : the split kernel's shape -- a wave writes a 16-row x 512-B
//                     tile as 4 stores of four 256-B half rows per instruction
// Build: hipcc -O3 --offload-arch=gfx950 tools/store_bw.hip -o /tmp/store_bw
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void __launch_bounds__(256) fill_kernel(f4* __restrict__ out, long n4, float v) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const f4 x = f4{v, v + 1.0f, v + 2.0f, (float)i};
        if (NT) __builtin_nontemporal_store(x, out + i);
        else out[i] = x;
    }
}

// tile t = 16 rows of 128 floats; lane (g = lane >> 4, col = lane & 15)
template <bool NT>
__global__ void __launch_bounds__(256) rows_kernel(float* __restrict__ out, long tiles, long nwaves, float v) {
    const int lane = threadIdx.x & 63;
    const long wave = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int g = lane >> 4, col = lane & 15;
    for (long t = wave; t < tiles; t += nwaves) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int rw = g + 4 * i;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int ch = 16 * h + col;
                const f4 x = f4{v, (float)rw, (float)ch, (float)t};
                f4* p = (f4*)(out + (16 * t + rw) * 128 + 4 * ch);
                if (NT) __builtin_nontemporal_store(x, p);
                else *p = x;
            }
        }
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
    const long N = 1L << 20, K = 128;
    const long bytes = N * K * 4;
    float* out;
    CK(hipMalloc(&out, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto launch) -> int {
        for (int w = 0; w < 3; ++w) launch();
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        std::vector<float> ms;
        for (int r = 0; r < 20; ++r) {
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float t;
            hipEventElapsedTime(&t, a, b);
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const float med = ms[ms.size() / 2];
        printf("{\"case\": \"%s\", \"us_median\": %.1f, \"us_min\": %.1f, \"TBps_median\": %.3f}\n", name, med * 1e3,
               ms[0] * 1e3, bytes / (med * 1e-3) / 1e12);
        return 0;
    };
    const long n4 = bytes / 16, tiles = N / 16;
    char nm[96];
    for (int wpc : {4, 8, 12, 16, 32}) {
        const int blocks = 256 * wpc / 4;
        snprintf(nm, sizeof nm, "plain %d waves/CU", wpc);
        if (timeit(nm, [&] { hipLaunchKernelGGL(fill_kernel<false>, dim3(blocks), dim3(256), 0, 0, (f4*)out, n4, 1.0f); })) return 1;
        snprintf(nm, sizeof nm, "nt %d waves/CU", wpc);
        if (timeit(nm, [&] { hipLaunchKernelGGL(fill_kernel<true>, dim3(blocks), dim3(256), 0, 0, (f4*)out, n4, 1.0f); })) return 1;
        const long nwaves = (long)blocks * 4;
        snprintf(nm, sizeof nm, "rows nt %d waves/CU", wpc);
        if (timeit(nm, [&] { hipLaunchKernelGGL(rows_kernel<true>, dim3(blocks), dim3(256), 0, 0, out, tiles, nwaves, 1.0f); })) return 1;
        snprintf(nm, sizeof nm, "rows plain %d waves/CU", wpc);
        if (timeit(nm, [&] { hipLaunchKernelGGL(rows_kernel<false>, dim3(blocks), dim3(256), 0, 0, out, tiles, nwaves, 1.0f); })) return 1;
    }
    CK(hipFree(out));
    return 0;
}
