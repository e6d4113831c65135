// guide_pattern_harness.cpp -- the drop-in plugin's guided bounce in the
// reference's threading pattern: every render worker serves its own tiles'
// bounces concurrently (sdmm_proc.cpp:1086-1106; the plugin's guideWavefront,
// plugin/volpath_sdmm_amd.cpp), each through its own guide context on the
// published tree -- pinned H2D of the tile's query planes, one
// sdmm_ctx_guide_pdf_wavefront, D2H of the outputs, a stream synchronise.
//
// usage: guide_pattern_harness model.asdmm queries.bin out.bin threads tile reps [contexts] [resident|batch[:T:W]]
//   contexts: guide contexts shared by the threads through
//             sdmm_amd::GuideContextPool (0 or absent: one per thread)
//   resident: the tiles' queries stay in device memory (no copies: the
//             device-resident rate of the same calls, for comparison)
//   batch   : the workers' bounces gathered by sdmm_amd::GuideBatcher into
//             wavefronts of up to T queries (default 262144), a batch's
//             leader waiting at most W us (default 200) for more; contexts =
//             the batches in flight
//   queries.bin: int64 n, float c[3][n], u[3][n], dgiven[3][n], uint8 mode[n]
//   out.bin    : float d[3][n], pdf[n], int32 comp[n] (the last repetition)
//   stdout     : one JSON line {threads, tile, reps, queries, seconds, queries_per_s}
// Threads take tiles t = i, i + threads, ... (a fixed assignment, so the
// pinned staging of a thread's tiles is filled once, outside the timing).
// One untimed pass over the tiles precedes the timed `reps` passes.
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

#include "sdmm_amd.hpp"

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

// The staging of one tile, as the plugin lays it out (Staging): the 9 query
// planes (stride `tile`) then the mode bytes in ONE block, and the 4 output
// planes then the component indices in one block, so that a bounce is one
// H2D and one D2H copy.
struct Worker {
    std::vector<int64_t> tiles;   // first query of each of this worker's tiles
    char* h_in = nullptr;         // pinned, per tile: in block, then out block
    char* d_in = nullptr;         // device: one tile's in block (resident: every tile's)
    char* d_out = nullptr;        // device: one tile's out block
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 7 || argc > 9)
        die("usage: guide_pattern_harness model.asdmm queries.bin out.bin threads tile reps [contexts] "
            "[resident|batch[:T:W]]");
    const int contexts_arg = argc >= 8 ? std::atoi(argv[7]) : 0;
    const std::string mode_arg = argc == 9 ? argv[8] : "";
    const bool resident = mode_arg == "resident";
    const bool batch = mode_arg.rfind("batch", 0) == 0;
    if (!mode_arg.empty() && !resident && !batch) die("mode: resident or batch[:T:W]");
    int64_t batch_target = 1 << 18;
    int batch_wait = 200;
    if (batch && mode_arg.size() > 5) {
        if (std::sscanf(mode_arg.c_str(), "batch:%lld:%d", (long long*)&batch_target, &batch_wait) != 2)
            die("batch:T:W expects two integers");
    }
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
    const size_t in_bytes = (36 + 1) * (size_t)tile, out_bytes = (16 + 4) * (size_t)tile;
    std::vector<Worker> W((size_t)T);
    for (int i = 0; i < T; ++i) {
        Worker& w = W[(size_t)i];
        for (int64_t t = i; t < ntiles; t += T) w.tiles.push_back(t * tile);
        const size_t k = w.tiles.size() ? w.tiles.size() : 1;
        hk(hipHostMalloc((void**)&w.h_in, (in_bytes + out_bytes) * k, hipHostMallocDefault), "hipHostMalloc");
        hk(hipMalloc((void**)&w.d_in, in_bytes * (resident ? k : 1)), "hipMalloc");
        hk(hipMalloc((void**)&w.d_out, out_bytes), "hipMalloc");
        // the worker's tiles in its pinned staging (what its path tracing
        // would have written there)
        for (size_t j = 0; j < w.tiles.size(); ++j) {
            const int64_t a = w.tiles[j], e = std::min(a + tile, n);
            float* hi = (float*)(w.h_in + (in_bytes + out_bytes) * j);
            for (int p = 0; p < 9; ++p) std::memcpy(hi + p * tile, q.data() + p * n + a, 4 * (size_t)(e - a));
            std::memcpy((char*)(hi + 9 * tile), mode.data() + a, (size_t)(e - a));
            if (resident)
                hk(hipMemcpy(w.d_in + in_bytes * j, hi, in_bytes, hipMemcpyHostToDevice), "hipMemcpy");
        }
    }

    const int contexts = contexts_arg > 0 ? contexts_arg : T;
    sdmm_amd::GuideContextPool pool(tree, contexts);
    sdmm_amd::GuideBatcher batcher(tree, contexts, batch_target, batch_wait);
    std::vector<std::string> err((size_t)T);
    // one pass of every thread over its tiles, `nrep` times; returns seconds
    auto run = [&](int nrep) {
        std::atomic<int> ready{0};
        std::atomic<bool> go{false};
        auto body = [&](int i) {
            Worker& w = W[(size_t)i];
            ++ready;
            while (!go.load()) std::this_thread::yield();
            for (int r = 0; r < nrep && err[(size_t)i].empty(); ++r)
                for (size_t j = 0; j < w.tiles.size(); ++j) {
                    const int64_t a = w.tiles[j], nq = std::min(a + tile, n) - a;
                    char* hb = w.h_in + (in_bytes + out_bytes) * j;
                    if (batch) {
                        // the staging as the request: 9 planes (stride tile) + modes
                        // in, 4 planes + components out
                        const sdmm_guide_host_req rq{nq, (const float*)hb, tile, (const uint8_t*)(hb + 36 * tile),
                                                     (float*)(hb + in_bytes), tile,
                                                     (int32_t*)(hb + in_bytes + 16 * tile)};
                        try {
                            batcher.serve(rq);
                        } catch (const std::exception& e) {
                            err[(size_t)i] = e.what();
                            return;
                        }
                        continue;
                    }
                    const sdmm_amd::GuideContextPool::Lease lease = pool.acquire();
                    const hipStream_t st = (hipStream_t)lease.stream();
                    float* din = (float*)(resident ? w.d_in + in_bytes * j : w.d_in);
                    if (!resident && hipMemcpyAsync(din, hb, in_bytes, hipMemcpyHostToDevice, st) != hipSuccess) {
                        err[(size_t)i] = "upload";
                        return;
                    }
                    const float* c[3] = {din, din + tile, din + 2 * tile};
                    const float* u[3] = {din + 3 * tile, din + 4 * tile, din + 5 * tile};
                    const float* dg[3] = {din + 6 * tile, din + 7 * tile, din + 8 * tile};
                    float* dout = (float*)w.d_out;
                    float* d[3] = {dout, dout + tile, dout + 2 * tile};
                    if (sdmm_ctx_guide_pdf_wavefront(lease.get(), nq, c, u, dg, (const uint8_t*)(din + 9 * tile), d,
                                                     dout + 3 * tile, (int32_t*)(dout + 4 * tile), nullptr) != SDMM_OK) {
                        err[(size_t)i] = std::string("sdmm_ctx_guide_pdf_wavefront: ") + sdmm_last_error();
                        return;
                    }
                    if (!resident || r == nrep - 1)
                        if (hipMemcpyAsync(hb + in_bytes, w.d_out, out_bytes, hipMemcpyDeviceToHost, st) != hipSuccess) {
                            err[(size_t)i] = "download";
                            return;
                        }
                    if (hipStreamSynchronize(st) != hipSuccess) { err[(size_t)i] = "hipStreamSynchronize"; return; }
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
        return sec;
    };
    // an untimed pass first: the pool's contexts are created on first use and
    // a context's scratch grows on its first calls (once per render pass in
    // the plugin, where a pass serves a whole frame of tiles)
    (void)run(1);
    const double sec = run(reps);

    // the outputs in query order
    std::vector<float> d(3 * (size_t)n), pdf((size_t)n);
    std::vector<int32_t> comp((size_t)n);
    for (const Worker& w : W)
        for (size_t j = 0; j < w.tiles.size(); ++j) {
            const int64_t a = w.tiles[j], e = std::min(a + tile, n);
            const float* ho = (const float*)(w.h_in + (in_bytes + out_bytes) * j + in_bytes);
            for (int p = 0; p < 3; ++p) std::memcpy(d.data() + p * n + a, ho + p * tile, 4 * (size_t)(e - a));
            std::memcpy(pdf.data() + a, ho + 3 * tile, 4 * (size_t)(e - a));
            std::memcpy(comp.data() + a, ho + 4 * tile, 4 * (size_t)(e - a));
        }
    FILE* o = std::fopen(argv[3], "wb");
    if (!o) die("cannot write output");
    std::fwrite(d.data(), 4, d.size(), o);
    std::fwrite(pdf.data(), 4, pdf.size(), o);
    std::fwrite(comp.data(), 4, comp.size(), o);
    std::fclose(o);

    const double total = (double)n * reps;
    std::printf("{\"threads\": %d, \"contexts\": %d, \"tile\": %lld, \"reps\": %d, \"queries\": %lld, "
                "\"resident\": %s, \"batch\": %s, \"batch_target\": %lld, \"batch_wait_us\": %d, "
                "\"seconds\": %.6f, \"queries_per_s\": %.1f}\n",
                T, contexts, (long long)tile, reps, (long long)n, resident ? "true" : "false", batch ? "true" : "false",
                (long long)batch_target, batch_wait, sec, total / sec);
    for (Worker& w : W) {
        (void)hipHostFree(w.h_in);
        (void)hipFree(w.d_in);
        (void)hipFree(w.d_out);
    }
    for (sdmm_mix* m : mix) sdmm_destroy(m);
    sdmm_stree_destroy(tree);
    return 0;
}
