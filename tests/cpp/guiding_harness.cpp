// guiding_harness.cpp -- the plugin's render() loop (volpath_sdmm.cpp:411-507)
// in C++ over the C ABI, through the C++ mirror (sdmm_amd::Scene,
// sdmm_amd::GuidingModel): sampleCount spp rendered samplesPerIteration at a
// time, training (push + optimize) while samplesRendered < sampleCount / 4,
// guided once a leaf is trained.  Writes each pass's image and the guiding
// stats, for the bitwise comparison with the Python driver of the same loop.
//
// usage: guiding_harness scene.bin out.bin [exr_dir|-] [async]
//   exr_dir: also dump iteration%05i.exr / iteration_sqr%05i.exr per pass
//            (SDMMWorkResult::dumpIndividual, sdmm_wr.cpp:115-146)
//   async  : optimizeAsync (volpath_sdmm.cpp:65, :180-242)
//   scene.bin: int32 n_quads, n_bsdfs, n_emitters, width, height, spp_total, spp_it;
//              float quads[9 n_quads]; int32 flip[n_quads], bsdf[n_quads], emitter[n_quads];
//              float reflectance[3 n_bsdfs], radiance[3 n_emitters], cam[16], fov
//   out.bin  : per pass: int32 trained, leaves, optimized; float image[3 * width * height]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "sdmm_amd.hpp"

template <class T>
static bool rd(FILE* f, T* p, size_t n) { return std::fread(p, sizeof(T), n, f) == n; }

int main(int argc, char** argv) {
    if (argc < 3 || argc > 5) {
        std::fprintf(stderr, "usage: %s scene.bin out.bin [exr_dir|-] [async]\n", argv[0]);
        return 2;
    }
    const bool dump = argc >= 4 && std::strcmp(argv[3], "-") != 0;
    const bool async = argc == 5 && std::strcmp(argv[4], "async") == 0;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t hdr[7];
    if (!rd(f, hdr, 7)) return 2;
    const int nq = hdr[0], nb = hdr[1], ne = hdr[2], W = hdr[3], H = hdr[4], spp_total = hdr[5], spp_it = hdr[6];
    std::vector<float> quads(9 * (size_t)nq), refl(3 * (size_t)nb), rad(3 * (size_t)ne), cam(16);
    std::vector<int32_t> flip(nq), bsdf(nq), emitter(nq);
    float fov = 0;
    if (!rd(f, quads.data(), quads.size()) || !rd(f, flip.data(), flip.size()) || !rd(f, bsdf.data(), bsdf.size()) ||
        !rd(f, emitter.data(), emitter.size()) || !rd(f, refl.data(), refl.size()) || !rd(f, rad.data(), rad.size()) ||
        !rd(f, cam.data(), 16) || !rd(f, &fov, 1))
        return 2;
    std::fclose(f);
    try {
        sdmm_scene_desc d{};
        d.n_quads = nq; d.quads = quads.data(); d.flip_normals = flip.data(); d.bsdf = bsdf.data();
        d.n_bsdfs = nb; d.reflectance = refl.data(); d.emitter = emitter.data(); d.n_emitters = ne;
        d.radiance = rad.data();
        for (int i = 0; i < 16; ++i) d.camera_to_world[i] = cam[(size_t)i];
        d.fov_x_deg = fov; d.near_clip = 1e-2f; d.width = W; d.height = H;
        sdmm_amd::Scene scene(d);
        float smin[3], norm, tmin[3], tmax[3];
        scene.normalization(smin, &norm, tmin, tmax);
        sdmm_guiding_config cfg;
        sdmm_guiding_config_default(&cfg);                       // split_to_depth(2), K = 16, 4000, 2048
        cfg.optimize_async = async ? 1 : 0;
        sdmm_amd::GuidingModel model(tmin, tmax, &cfg);
        float* image = nullptr;
        float* image_sqr = nullptr;
        if (hipMalloc(&image, sizeof(float) * 3 * (size_t)W * H) != hipSuccess ||
            hipMalloc(&image_sqr, sizeof(float) * 3 * (size_t)W * H) != hipSuccess)
            return 1;
        std::vector<float> host(3 * (size_t)W * H), host_sqr(3 * (size_t)W * H);
        FILE* o = std::fopen(argv[2], "wb");
        int it = 0;
        for (int done = 0; done < spp_total; done += spp_it, ++it) {
            const bool train = done < spp_total / 4;           // m_still_training (:416)
            sdmm_li_params p{};
            p.spp = spp_it; p.max_depth = 10; p.rr_depth = 10; p.bsdf_fraction = 0.5f; p.saved_vertices = 9;
            p.seed = 1 + (uint64_t)it; p.pixel_begin = 0; p.pixel_end = (int64_t)W * H;
            const sdmm_guiding_stats st = model.iteration(scene, p, 1001 + (uint64_t)it, train, image, image_sqr);
            if (hipDeviceSynchronize() != hipSuccess ||
                hipMemcpy(host.data(), image, sizeof(float) * host.size(), hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(host_sqr.data(), image_sqr, sizeof(float) * host.size(), hipMemcpyDeviceToHost) != hipSuccess)
                return 1;
            if (dump) sdmm_amd::dump_iteration(argv[3], it, spp_it, 0.0f, W, H, host.data(), host_sqr.data());
            const int32_t rec[3] = {model.trained(), train ? st.leaves : -1, train ? st.optimized : -1};
            std::fwrite(rec, 4, 3, o);
            std::fwrite(host.data(), 4, host.size(), o);
        }
        std::fclose(o);
        (void)hipFree(image);
        (void)hipFree(image_sqr);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "guiding_harness: %s\n", e.what());
        return 1;
    }
    return 0;
}
