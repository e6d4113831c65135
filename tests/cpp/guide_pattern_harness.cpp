// guide_pattern_harness.cpp -- the drop-in plugin's guided bounce in the
// reference's threading pattern: every render worker serves its own tiles'
// bounces concurrently (sdmm_proc.cpp:1086-1106; the plugin's guideWavefront,
// plugin/volpath_sdmm_amd.cpp), each through its own guide context on the
// published tree -- pinned H2D of the tile's query planes, one
// sdmm_ctx_guide_pdf_wavefront, D2H of the outputs, a stream synchronise.
//
// usage: guide_pattern_harness model.asdmm queries.bin out.bin threads tile reps
//   queries.bin: int64 n, float c[3][n], u[3][n], dgiven[3][n], uint8 mode[n]
//   out.bin    : float d[3][n], pdf[n], int32 comp[n] (the last repetition)
//   stdout     : one JSON line {threads, tile, reps, queries, seconds, queries_per_s}
// Threads take tiles t = i, i + threads, ... (a fixed assignment, so the
// pinned staging of a thread's tiles is filled once, outside the timing).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sdmm_gpu.h"

namespace {

void die(const std::string& what) {
    std::fprintf(stderr, "%s\n", what.c_str());
    std::exit(1);
}
void ck(int rc, const char* what) {
    if (rc != SDMM_OK) die(std::string(what) + ": " + sdmm_last_error());
}
void hk(hipError_t e, const char* what) {
    if (e != hipSuccess) die(std::string(what) + ": " + hipGetErrorString(e));
}

struct Worker {
    sdmm_guide_ctx* ctx = nullptr;
    hipStream_t st = nullptr;
    std::vector<int64_t> tiles;   // first query of each of this worker's tiles
    // pinned: per tile 9 float planes + mode in, 4 float planes + comp out
    float* h_in = nullptr;
    uint8_t* h_mode = nullptr;
    float* h_out = nullptr;
    int32_t* h_comp = nullptr;
    float* d_in = nullptr;
    uint8_t* d_mode = nullptr;
    float* d_out = nullptr;
    int32_t* d_comp = nullptr;
};

}  // namespace

int main(int argc, char** argv) {
    if (argc != 7) die("usage: guide_pattern_harness model.asdmm queries.bin out.bin threads tile reps");
    const int T = std::atoi(argv[4]);
    const int64_t tile = std::atoll(argv[5]);
    const int reps = std::atoi(argv[6]);
    if (T < 1 || tile < 1 || reps < 1) die("threads, tile, reps must be positive");

    FILE* f = std::fopen(argv[2], "rb");
    if (!f) die("cannot open queries");
    int64_t n = 0;
    if (std::fread(&n, 8, 1, f) != 1 || n <= 0) die("bad queries header");
    std::vector<float> q(9 * (size_t)n);
    std::vector<uint8_t> mode((size_t)n);
    if (std::fread(q.data(), 4, q.size(), f) != q.size() || std::fread(mode.data(), 1, mode.size(), f) != mode.size())
        die("short queries file");
    std::fclose(f);

    int nn = 0;
    ck(sdmm_load_json(argv[1], 0, nullptr, nullptr, 0, &nn), "sdmm_load_json (size)");
    sdmm_stree* tree = nullptr;
    std::vector<sdmm_mix*> mix((size_t)nn, nullptr);
    ck(sdmm_load_json(argv[1], 0, &tree, mix.data(), nn, &nn), "sdmm_load_json");
    std::vector<const sdmm_mix*> cmix(mix.begin(), mix.end());
    ck(sdmm_stree_publish(tree, cmix.data()), "sdmm_stree_publish");

    const int64_t ntiles = (n + tile - 1) / tile;
    std::vector<Worker> W((size_t)T);
    for (int i = 0; i < T; ++i) {
        Worker& w = W[(size_t)i];
        for (int64_t t = i; t < ntiles; t += T) w.tiles.push_back(t * tile);
        const size_t k = w.tiles.size() ? w.tiles.size() : 1;
        const size_t m = k * (size_t)tile;
        ck(sdmm_guide_ctx_create(tree, nullptr, &w.ctx), "sdmm_guide_ctx_create");
        w.st = (hipStream_t)sdmm_guide_ctx_stream(w.ctx);
        hk(hipHostMalloc((void**)&w.h_in, 4 * 9 * m, hipHostMallocDefault), "hipHostMalloc");
        hk(hipHostMalloc((void**)&w.h_mode, m, hipHostMallocDefault), "hipHostMalloc");
        hk(hipHostMalloc((void**)&w.h_out, 4 * 4 * m, hipHostMallocDefault), "hipHostMalloc");
        hk(hipHostMalloc((void**)&w.h_comp, 4 * m, hipHostMallocDefault), "hipHostMalloc");
        hk(hipMalloc((void**)&w.d_in, 4 * 9 * (size_t)tile), "hipMalloc");
        hk(hipMalloc((void**)&w.d_mode, (size_t)tile), "hipMalloc");
        hk(hipMalloc((void**)&w.d_out, 4 * 4 * (size_t)tile), "hipMalloc");
        hk(hipMalloc((void**)&w.d_comp, 4 * (size_t)tile), "hipMalloc");
        // the worker's tiles in its pinned staging (what its path tracing
        // would have written there), planes of stride `tile` per tile
        for (size_t j = 0; j < w.tiles.size(); ++j) {
            const int64_t a = w.tiles[j], e = std::min(a + tile, n);
            for (int p = 0; p < 9; ++p)
                std::memcpy(w.h_in + (j * 9 + p) * tile, q.data() + p * n + a, 4 * (size_t)(e - a));
            std::memcpy(w.h_mode + j * tile, mode.data() + a, (size_t)(e - a));
        }
    }

    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<std::string> err((size_t)T);
    auto body = [&](int i) {
        Worker& w = W[(size_t)i];
        ++ready;
        while (!go.load()) std::this_thread::yield();
        for (int r = 0; r < reps && err[(size_t)i].empty(); ++r)
            for (size_t j = 0; j < w.tiles.size(); ++j) {
                const int64_t a = w.tiles[j], nq = std::min(a + tile, n) - a;
                float* hi = w.h_in + j * 9 * tile;
                for (int p = 0; p < 9; ++p)
                    if (hipMemcpyAsync(w.d_in + p * tile, hi + p * tile, 4 * (size_t)nq, hipMemcpyHostToDevice,
                                       w.st) != hipSuccess) { err[(size_t)i] = "upload"; return; }
                if (hipMemcpyAsync(w.d_mode, w.h_mode + j * tile, (size_t)nq, hipMemcpyHostToDevice, w.st) !=
                    hipSuccess) { err[(size_t)i] = "upload"; return; }
                const float* c[3] = {w.d_in, w.d_in + tile, w.d_in + 2 * tile};
                const float* u[3] = {w.d_in + 3 * tile, w.d_in + 4 * tile, w.d_in + 5 * tile};
                const float* dg[3] = {w.d_in + 6 * tile, w.d_in + 7 * tile, w.d_in + 8 * tile};
                float* d[3] = {w.d_out, w.d_out + tile, w.d_out + 2 * tile};
                if (sdmm_ctx_guide_pdf_wavefront(w.ctx, nq, c, u, dg, w.d_mode, d, w.d_out + 3 * tile, w.d_comp,
                                                 nullptr) != SDMM_OK) {
                    err[(size_t)i] = std::string("sdmm_ctx_guide_pdf_wavefront: ") + sdmm_last_error();
                    return;
                }
                float* ho = w.h_out + j * 4 * tile;
                for (int p = 0; p < 4; ++p)
                    if (hipMemcpyAsync(ho + p * tile, w.d_out + p * tile, 4 * (size_t)nq, hipMemcpyDeviceToHost,
                                       w.st) != hipSuccess) { err[(size_t)i] = "download"; return; }
                if (hipMemcpyAsync(w.h_comp + j * tile, w.d_comp, 4 * (size_t)nq, hipMemcpyDeviceToHost, w.st) !=
                    hipSuccess) { err[(size_t)i] = "download"; return; }
                if (hipStreamSynchronize(w.st) != hipSuccess) { err[(size_t)i] = "hipStreamSynchronize"; return; }
            }
    };
    std::vector<std::thread> th;
    for (int i = 0; i < T; ++i) th.emplace_back(body, i);
    while (ready.load() < T) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    go = true;
    for (auto& x : th) x.join();
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int i = 0; i < T; ++i)
        if (!err[(size_t)i].empty()) die("worker " + std::to_string(i) + ": " + err[(size_t)i]);

    // the outputs in query order
    std::vector<float> d(3 * (size_t)n), pdf((size_t)n);
    std::vector<int32_t> comp((size_t)n);
    for (const Worker& w : W)
        for (size_t j = 0; j < w.tiles.size(); ++j) {
            const int64_t a = w.tiles[j], e = std::min(a + tile, n);
            for (int p = 0; p < 3; ++p)
                std::memcpy(d.data() + p * n + a, w.h_out + (j * 4 + p) * tile, 4 * (size_t)(e - a));
            std::memcpy(pdf.data() + a, w.h_out + (j * 4 + 3) * tile, 4 * (size_t)(e - a));
            std::memcpy(comp.data() + a, w.h_comp + j * tile, 4 * (size_t)(e - a));
        }
    FILE* o = std::fopen(argv[3], "wb");
    if (!o) die("cannot write output");
    std::fwrite(d.data(), 4, d.size(), o);
    std::fwrite(pdf.data(), 4, pdf.size(), o);
    std::fwrite(comp.data(), 4, comp.size(), o);
    std::fclose(o);

    const double total = (double)n * reps;
    std::printf("{\"threads\": %d, \"tile\": %lld, \"reps\": %d, \"queries\": %lld, \"seconds\": %.6f, "
                "\"queries_per_s\": %.1f}\n",
                T, (long long)tile, reps, (long long)n, sec, total / sec);
    for (Worker& w : W) {
        sdmm_guide_ctx_destroy(w.ctx);
        (void)hipHostFree(w.h_in); (void)hipHostFree(w.h_mode); (void)hipHostFree(w.h_out); (void)hipHostFree(w.h_comp);
        (void)hipFree(w.d_in); (void)hipFree(w.d_mode); (void)hipFree(w.d_out); (void)hipFree(w.d_comp);
    }
    for (sdmm_mix* m : mix) sdmm_destroy(m);
    sdmm_stree_destroy(tree);
    return 0;
}
