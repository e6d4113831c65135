// plugin_harness.cpp -- drives the C ABI through the C++ mirror header the way
// the Mitsuba sdmm plugin drives sdmm-lib: one mixture per spatial-tree leaf,
// per-leaf EM on worker threads (tev::ThreadPool::parallelFor,
// volpath_sdmm.cpp:287-311), 3 optimize() calls with 2 EM iterations per call
// while iterations_run < 4 else 1 (:299-305) -- 2, 2, 1 -- training data
// pushed from host threads (sdmm_proc.cpp:894-902).
//
// usage: plugin_harness in.bin out.bin [batched]
//   batched: the leaves are stepped by ONE sdmm_em_step_batched_host call per
//   plugin call (the C++ mirror's em_step_leaves) instead of a thread each;
//   the output must be bitwise the same
//   in.bin : int64 N, int32 K, int32 leaves, float x[6][N], w[N], normals[N][3]
//   out.bin: per leaf: float weights[K], means[K][6], covs[K][25]
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <thread>
#include <vector>

#include "sdmm_amd.hpp"

int main(int argc, char** argv) {
    if (argc != 3 && argc != 4) { std::fprintf(stderr, "usage: %s in.bin out.bin [batched]\n", argv[0]); return 2; }
    const bool batched = argc == 4;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    int64_t N; int32_t K, L;
    if (std::fread(&N, 8, 1, f) != 1 || std::fread(&K, 4, 1, f) != 1 || std::fread(&L, 4, 1, f) != 1) return 2;
    std::vector<float> x(6 * N), w(N), nrm(3 * N);
    if (std::fread(x.data(), 4, 6 * N, f) != (size_t)(6 * N) || std::fread(w.data(), 4, N, f) != (size_t)N ||
        std::fread(nrm.data(), 4, 3 * N, f) != (size_t)(3 * N)) return 2;
    std::fclose(f);

    std::vector<std::vector<float>> outW(L), outM(L), outC(L);
    std::vector<std::string> errors(L);
    auto leaf_data = [&](int l, sdmm_amd::TrainingData& data) {
        const int64_t a = N * l / L, b = N * (l + 1) / L;
        data.reserve(b - a);
        for (int64_t i = a; i < b; ++i) {
            float p[6];
            for (int d = 0; d < 6; ++d) p[d] = x[d * N + i];
            data.push_back(p, &nrm[3 * i], w[i]);
        }
    };
    if (batched) {
        try {
            std::vector<sdmm_amd::TrainingData> data(L);
            std::vector<std::unique_ptr<sdmm_amd::Mixture>> mixes;
            std::vector<sdmm_amd::Mixture*> ptrs;
            std::vector<const sdmm_amd::TrainingData*> dptrs;
            for (int l = 0; l < L; ++l) {
                leaf_data(l, data[l]);
                mixes.emplace_back(new sdmm_amd::Mixture(K));
                mixes.back()->initialize(data[l], 0.01f, 0.1f, 0x1A17u + (uint64_t)l);
                ptrs.push_back(mixes.back().get());
                dptrs.push_back(&data[l]);
            }
            for (int call = 0; call < 3; ++call) {
                std::vector<int> iters;   // 2 while iterations_run < 4, else 1 (volpath_sdmm.cpp:299-305)
                for (auto* m : ptrs) iters.push_back(m->iterations_run() < 4 ? 2 : 1);
                sdmm_amd::em_step_leaves(ptrs, dptrs, iters);
            }
            for (int l = 0; l < L; ++l) mixes[l]->params(outW[l], outM[l], outC[l]);
        } catch (const std::exception& e) {
            std::fprintf(stderr, "batched: %s\n", e.what());
            return 1;
        }
    } else {
        auto leaf = [&](int l) {
            try {
                sdmm_amd::TrainingData data;
                leaf_data(l, data);
                sdmm_amd::Mixture m(K);
                m.initialize(data, 0.01f, 0.1f, 0x1A17u + (uint64_t)l);
                for (int call = 0; call < 3; ++call) m.em_step(data, m.iterations_run() < 4 ? 2 : 1);
                m.params(outW[l], outM[l], outC[l]);
            } catch (const std::exception& e) {
                errors[l] = e.what();
            }
        };
        std::vector<std::thread> pool;
        for (int l = 0; l < L; ++l) pool.emplace_back(leaf, l);
        for (auto& t : pool) t.join();
        for (int l = 0; l < L; ++l)
            if (!errors[l].empty()) { std::fprintf(stderr, "leaf %d: %s\n", l, errors[l].c_str()); return 1; }
    }
    FILE* o = std::fopen(argv[2], "wb");
    for (int l = 0; l < L; ++l) {
        std::fwrite(outW[l].data(), 4, outW[l].size(), o);
        std::fwrite(outM[l].data(), 4, outM[l].size(), o);
        std::fwrite(outC[l].data(), 4, outC[l].size(), o);
    }
    std::fclose(o);
    return 0;
}
