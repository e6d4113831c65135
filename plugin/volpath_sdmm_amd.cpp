/*
 * volpath_sdmm_amd.cpp -- the `sdmm` integrator plugin (the SDMM volumetric
 * path tracer of Mitsuba 0.6) with its guiding model on an MI355X through the
 * C ABI of include/sdmm_gpu.h.  It builds as the plugin named `sdmm` -- the
 * SharedLibrary('sdmm', ...) entry of mitsuba/src/integrators/SConscript:44-55,
 * with this one source in place of volpath_sdmm.cpp + sdmm_proc.cpp +
 * sdmm_wr.cpp + sdmm_wu.cpp -- so scenes that say <integrator type="sdmm">
 * (test-suite/scenes/_integrators/sdmm.xml:14) load it unchanged; it links
 * libsdmm_amd.so.
 *
 * NOT COMPILED in this repository: Mitsuba 0.6 and its dependencies are not in
 * the image.  Every guiding call below is exercised by the tests through the
 * same entry points (tests/test_gpu_li.py, tests/test_gpu_harness.py,
 * tests/cpp/guiding_harness.cpp).
 *
 * What stays as in the reference plugin (mitsuba/src/integrators/sdmm/):
 *   - the properties (volpath_sdmm.cpp:52-91) and their checks;
 *   - the render() loop (:334-516): scene_norm.json, the tree box (getAABB,
 *     :314-332), split_to_depth(2), sampleCount / samplesPerIteration passes,
 *     training while samplesRendered < sampleCount / 4, optimizeAsync,
 *     per-pass iteration%05i.exr dumps, stats.json, the final checkpoint;
 *   - the film: each pass added with weight spp / sampleCount
 *     (SDMMProcess::develop, sdmm_proc.cpp:1142-1158);
 *   - Li (sdmm_proc.cpp:592-871): no NEE; the guide is queried for every
 *     BSDF that is not all-delta (:297) and the BSDF/guide choice is taken
 *     first with heuristicConditionalWeight 0.5 (:383-392); a BSDF-chosen
 *     delta lobe returns weight / h with pdf * h (:401-405), a smooth one
 *     (weight * pdf) / pdfSurface, the guide's direction eval / pdfSurface
 *     with pdf = h bsdfPdf + (1-h) gmmPdf (:587-589); saved vertices with
 *     clamped pdf only for non-delta samples (`cacheable`, :764, :821-846)
 *     with the normal flipped to the wi side (:765-767); recordRadiance
 *     (:615-637); strict normals on wi and wo (:688-691, :777-780); medium
 *     transitions, index-matched (ENull) passes and
 *     rayIntersectAndLookForEmitter's transmittance through null surfaces
 *     (:788-800, :988-1050); Russian roulette after rrDepth with q =
 *     min(max(throughput) eta^2, 0.95) (:788, :858-868);
 *   - sampleProduct (:327-392): the BSDF's learned DMM (getDMM, :327-329;
 *     the diffuse case re-centres slice 0 on the wi-side normal, :335-339,
 *     otherwise rotate_to_wo(wi), :341-354 -- sdmm-lib calls the maintainer's
 *     build keeps) is handed to sdmm_guide_product_wavefront as one table row
 *     per query (lobes in the local frame, the shading frame per query),
 *     which multiplies it with the leaf's conditional, picks h = 0.3 (0.5
 *     without a usable product) and the BSDF/guide choice against that h;
 *   - bsdfOnly: no training (:416), so no leaf ever holds an initialised
 *     context and every bounce takes the BSDF-only branch (:316-323); the
 *     learned-BSDF-only branch (:331, :384, :410-413) is unreachable in the
 *     reference for the same reason and is not reproduced.
 * What changes:
 *   - the guiding state (tree, per-leaf SDMM + EM, training data, optimize)
 *     lives on the GPU: one sdmm_guiding handle;
 *   - Li runs bounce-synchronously over a tile of paths (a wavefront): the
 *     CPU threads intersect and evaluate Mitsuba's BSDFs, and ONE
 *     sdmm_ctx_guide_pdf_wavefront call per bounce and tile builds every
 *     vertex's conditional once and samples it or evaluates its pdf; each
 *     bounce leases a guide context (stream + scratch) on the tree published
 *     once per pass, from a pool shared by the workers (property
 *     guideContexts, 4), so the workers' bounces run concurrently, as the
 *     reference's per-thread calls do (sdmm_proc.cpp:1086-1106);
 *   - push_back_data (:876-965) is one sdmm_guiding_push per tile.
 */
#include <algorithm>
#include <atomic>
#include <cmath>
#include <fstream>
#include <iomanip>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include <mitsuba/core/plugin.h>
#include <mitsuba/core/timer.h>
#include <mitsuba/render/scene.h>

#include <hip/hip_runtime.h>

#include "sdmm_gpu.h"
#include "sdmm_amd.hpp"   // GuideContextPool (sdmm-mitsuba_amd/host)

MTS_NAMESPACE_BEGIN

// learned-BSDF lobes per product query (a row of the per-tile table); a
// learned DMM with more slices is an error
constexpr int kMaxLobes = 32;

namespace {

void check_sdmm(int rc, const char* what) {
    if (rc != SDMM_OK) SLog(EError, "%s failed (%i): %s", what, rc, sdmm_last_error());
}

void check_hip(hipError_t e, const char* what) {
    if (e != hipSuccess) SLog(EError, "%s failed: %s", what, hipGetErrorString(e));
}

// Pinned host + device staging of one worker's wavefront (SoA planes).
struct Staging {
    int64_t cap = 0;
    int V = 0;
    // query planes: c 3, u 3, dgiven 3 (float); mode (u8); outputs d 3, pdf (float), comp (int32)
    float* h_in = nullptr;
    uint8_t* h_mode = nullptr;
    float* h_out = nullptr;
    int32_t* h_comp = nullptr;
    float* d_in = nullptr;
    uint8_t* d_mode = nullptr;
    float* d_out = nullptr;
    int32_t* d_comp = nullptr;
    // sampleProduct: per query its learned-BSDF row (weights, local means,
    // 2x2 covs, diffuse flag), material = its own row (-1: none), the
    // shading frame (9 planes), the BSDF/guide draw, and h out
    float* h_bw = nullptr;
    float* h_bmean = nullptr;
    float* h_bcov = nullptr;
    uint8_t* h_bdiff = nullptr;
    int32_t* h_mat = nullptr;
    float* h_pf = nullptr;       // frame 9 planes, choice, h
    float* d_bw = nullptr;
    float* d_bmean = nullptr;
    float* d_bcov = nullptr;
    uint8_t* d_bdiff = nullptr;
    int32_t* d_mat = nullptr;
    float* d_pf = nullptr;
    // saved-vertex records of the tile's paths (sdmm_path_vertices layout)
    float* h_rec = nullptr;
    int32_t* h_nv = nullptr;
    float* d_rec = nullptr;
    int32_t* d_nv = nullptr;
    void allocate(int64_t n, int vslots, bool product) {
        release();
        cap = n;
        V = vslots;
        if (product) {
            const size_t L = (size_t)n * kMaxLobes;
            check_hip(hipHostMalloc((void**)&h_bw, sizeof(float) * L, hipHostMallocDefault), "hipHostMalloc");
            check_hip(hipHostMalloc((void**)&h_bmean, sizeof(float) * 3 * L, hipHostMallocDefault), "hipHostMalloc");
            check_hip(hipHostMalloc((void**)&h_bcov, sizeof(float) * 4 * L, hipHostMallocDefault), "hipHostMalloc");
            check_hip(hipHostMalloc((void**)&h_bdiff, n, hipHostMallocDefault), "hipHostMalloc");
            check_hip(hipHostMalloc((void**)&h_mat, sizeof(int32_t) * n, hipHostMallocDefault), "hipHostMalloc");
            check_hip(hipHostMalloc((void**)&h_pf, sizeof(float) * 11 * n, hipHostMallocDefault), "hipHostMalloc");
            check_hip(hipMalloc((void**)&d_bw, sizeof(float) * L), "hipMalloc");
            check_hip(hipMalloc((void**)&d_bmean, sizeof(float) * 3 * L), "hipMalloc");
            check_hip(hipMalloc((void**)&d_bcov, sizeof(float) * 4 * L), "hipMalloc");
            check_hip(hipMalloc((void**)&d_bdiff, n), "hipMalloc");
            check_hip(hipMalloc((void**)&d_mat, sizeof(int32_t) * n), "hipMalloc");
            check_hip(hipMalloc((void**)&d_pf, sizeof(float) * 11 * n), "hipMalloc");
        }
        check_hip(hipHostMalloc((void**)&h_in, sizeof(float) * 9 * n, hipHostMallocDefault), "hipHostMalloc");
        check_hip(hipHostMalloc((void**)&h_mode, n, hipHostMallocDefault), "hipHostMalloc");
        check_hip(hipHostMalloc((void**)&h_out, sizeof(float) * 4 * n, hipHostMallocDefault), "hipHostMalloc");
        check_hip(hipHostMalloc((void**)&h_comp, sizeof(int32_t) * n, hipHostMallocDefault), "hipHostMalloc");
        check_hip(hipHostMalloc((void**)&h_rec, sizeof(float) * 16 * V * n, hipHostMallocDefault), "hipHostMalloc");
        check_hip(hipHostMalloc((void**)&h_nv, sizeof(int32_t) * n, hipHostMallocDefault), "hipHostMalloc");
        check_hip(hipMalloc((void**)&d_in, sizeof(float) * 9 * n), "hipMalloc");
        check_hip(hipMalloc((void**)&d_mode, n), "hipMalloc");
        check_hip(hipMalloc((void**)&d_out, sizeof(float) * 4 * n), "hipMalloc");
        check_hip(hipMalloc((void**)&d_comp, sizeof(int32_t) * n), "hipMalloc");
        check_hip(hipMalloc((void**)&d_rec, sizeof(float) * 16 * V * n), "hipMalloc");
        check_hip(hipMalloc((void**)&d_nv, sizeof(int32_t) * n), "hipMalloc");
    }
    void release() {
        for (void* p : {(void*)h_in, (void*)h_mode, (void*)h_out, (void*)h_comp, (void*)h_rec, (void*)h_nv,
                        (void*)h_bw, (void*)h_bmean, (void*)h_bcov, (void*)h_bdiff, (void*)h_mat, (void*)h_pf})
            if (p) (void)hipHostFree(p);
        for (void* p : {(void*)d_in, (void*)d_mode, (void*)d_out, (void*)d_comp, (void*)d_rec, (void*)d_nv,
                        (void*)d_bw, (void*)d_bmean, (void*)d_bcov, (void*)d_bdiff, (void*)d_mat, (void*)d_pf})
            if (p) (void)hipFree(p);
        h_bw = h_bmean = h_bcov = h_pf = d_bw = d_bmean = d_bcov = d_pf = nullptr;
        h_bdiff = d_bdiff = nullptr;
        h_mat = d_mat = nullptr;
        h_in = h_out = d_in = d_out = h_rec = d_rec = nullptr;
        h_mode = d_mode = nullptr;
        h_comp = d_comp = h_nv = d_nv = nullptr;
        cap = 0;
    }
    ~Staging() { release(); }
    float& rec(int f, int v, int64_t p, int64_t n) { return h_rec[((int64_t)f * V + v) * n + p]; }
};

// One path of a tile's wavefront.
struct PathState {
    RayDifferential ray;
    Intersection its;
    Spectrum throughput, Li;
    int depth;           // rRec.depth; -1 = finished
    Point2 samplePos;
    int64_t query;       // index into this bounce's query planes, -1 = BSDF only
    // the BSDF sample drawn before the query (its direction is the pdf query's)
    Spectrum bsdfWeight;
    Float bsdfPdf;
    bool pdfMode;        // the BSDF was chosen (rnd <= h; with sampleProduct the wavefront decides, comp -2)
    Float eta;           // relative IOR along the path (:604, :788)
    const Medium* medium;   // rRec.medium (:788-790)
    bool emission;       // rRec.type still has EEmittedRadiance (camera ray, or index-matched passes before a scatter)
    bool scattered;      // (:645, :870)
};

}  // namespace

class SDMMAmdPathTracer : public Integrator {
public:
    SDMMAmdPathTracer(const Properties& props) : Integrator(props) {
        // the reference's properties (volpath_sdmm.cpp:52-65)
        m_strictNormals = props.getBoolean("strictNormals", true);
        m_maxDepth = props.getInteger("maxDepth", -1);
        m_rrDepth = props.getInteger("rrDepth", 5);
        m_samplesPerIteration = props.getInteger("samplesPerIteration", 8);
        m_sampleProduct = props.getBoolean("sampleProduct", false);
        m_bsdfOnly = props.getBoolean("bsdfOnly", false);
        m_savedSamplesPerPath = props.getInteger("savedSamplesPerPath", 8);
        m_optimizeAsync = props.getBoolean("optimizeAsync", true);
        (void)props.getBoolean("flushDenormals", true);   // the device flushes f32 denormals
        // this port's own
        m_device = props.getInteger("hipDevice", 0);
        m_tileSize = props.getInteger("wavefrontTile", 64);
        m_guideContexts = props.getInteger("guideContexts", 4);
        m_guideBatch = props.getInteger("guideBatch", 1 << 18);
        m_guideBatchBelow = props.getInteger("guideBatchBelow", 1 << 14);
        if (m_rrDepth <= 0) Log(EError, "'rrDepth' must be set to a value greater than zero!");
        if (m_maxDepth <= 0 && m_maxDepth != -1)
            Log(EError, "'maxDepth' must be set to -1 (infinite) or a value greater than zero!");
        if (m_maxDepth != m_rrDepth) Log(EError, "'maxDepth' must match 'rrDepth' for the SDMM integrator!");
    }

    SDMMAmdPathTracer(Stream* stream, InstanceManager* manager) : Integrator(stream, manager) {
        m_strictNormals = stream->readBool();
        m_maxDepth = stream->readInt();
        m_rrDepth = stream->readInt();
        m_samplesPerIteration = stream->readInt();
        m_sampleProduct = stream->readBool();
        m_bsdfOnly = stream->readBool();
        m_savedSamplesPerPath = stream->readInt();
        m_optimizeAsync = stream->readBool();
        m_device = stream->readInt();
        m_tileSize = stream->readInt();
        m_guideContexts = stream->readInt();
        m_guideBatch = stream->readInt();
        m_guideBatchBelow = stream->readInt();
    }

    ~SDMMAmdPathTracer() {
        m_batch.reset();   // (their contexts read the model's tree)
        m_pool.reset();
        if (m_guiding) sdmm_guiding_destroy(m_guiding);
    }

    void serialize(Stream* stream, InstanceManager* manager) const override {
        Integrator::serialize(stream, manager);
        stream->writeBool(m_strictNormals);
        stream->writeInt(m_maxDepth);
        stream->writeInt(m_rrDepth);
        stream->writeInt(m_samplesPerIteration);
        stream->writeBool(m_sampleProduct);
        stream->writeBool(m_bsdfOnly);
        stream->writeInt(m_savedSamplesPerPath);
        stream->writeBool(m_optimizeAsync);
        stream->writeInt(m_device);
        stream->writeInt(m_tileSize);
        stream->writeInt(m_guideContexts);
        stream->writeInt(m_guideBatch);
        stream->writeInt(m_guideBatchBelow);
    }

    bool preprocess(const Scene* scene, RenderQueue* queue, const RenderJob* job, int sceneResID, int sensorResID,
                    int samplerResID) override {
        Integrator::preprocess(scene, queue, job, sceneResID, sensorResID, samplerResID);
        if (scene->getSubsurfaceIntegrators().size() > 0)
            Log(EError, "Subsurface integrators are not supported by the SDMM path tracer!");
        return true;
    }

    void cancel() override { m_cancelled = true; }

    bool render(Scene* scene, RenderQueue* queue, const RenderJob* job, int, int, int) override {
        ref<Sensor> sensor = scene->getSensor();
        Film* film = sensor->getFilm();
        const Vector2i size = film->getCropSize();
        const size_t sampleCount = scene->getSampler()->getSampleCount();
        const int nCores = std::max(1, (int)std::thread::hardware_concurrency());
        if (sampleCount % m_samplesPerIteration != 0)
            Log(EWarn, "sampleCount %% samplesPerIteration (" SIZE_T_FMT " %% %i) != 0", sampleCount,
                m_samplesPerIteration);
        const fs::path outDir = scene->getDestinationFile().parent_path();

        // scene normalisation and the tree box (:375-396)
        const AABB sceneBox = scene->getAABBWithoutCamera();
        const Vector extents = sceneBox.getExtents();
        m_sceneMin = sceneBox.min;
        m_spatialNorm = std::max(extents[0], std::max(extents[1], extents[2]));
        {
            std::ofstream f((outDir / "scene_norm.json").string());
            f << std::setprecision(9) << "{\n    \"scene_min\": [" << m_sceneMin[0] << ", " << m_sceneMin[1] << ", "
              << m_sceneMin[2] << "],\n    \"spatial_norm\": " << m_spatialNorm << "\n}\n";
        }
        float tmin[3], tmax[3];
        for (int a = 0; a < 3; ++a) {
            tmin[a] = -1e-5f;
            tmax[a] = (float)((sceneBox.max[a] - sceneBox.min[a]) / m_spatialNorm) + 1e-5f;
        }
        sdmm_guiding_config cfg;
        sdmm_guiding_config_default(&cfg);             // K 16, split_to_depth(2), 4000, 2048
        cfg.saved_per_path = m_savedSamplesPerPath;
        cfg.optimize_async = m_optimizeAsync ? 1 : 0;
        m_batch.reset();   // (a previous render's model and its contexts)
        m_pool.reset();
        if (m_guiding) {
            sdmm_guiding_destroy(m_guiding);
            m_guiding = nullptr;
        }
        check_sdmm(sdmm_guiding_create(tmin, tmax, &cfg, m_device, &m_guiding), "sdmm_guiding_create");
        m_stream = (hipStream_t)sdmm_stree_get_stream(sdmm_guiding_tree(m_guiding));

        ref<Timer> timer = new Timer();
        std::ostringstream stats;
        stats << "[\n";
        Float totalElapsed = 0;
        bool success = true;
        const int nPasses = (int)((sampleCount + m_samplesPerIteration - 1) / m_samplesPerIteration);
        film->clear();
        for (int samplesRendered = 0, it = 0; samplesRendered < (int)sampleCount;
             samplesRendered += m_samplesPerIteration, ++it) {
            const bool training = !m_bsdfOnly && samplesRendered < (int)sampleCount / 4;   // (:416)
            timer->reset();
            std::vector<float> mean(3 * (size_t)size.x * size.y), sqr(mean.size());
            int64_t pathLength = 0, paths = 0;
            success = renderPass(scene, sensor.get(), size, it, training, nCores, mean, sqr, pathLength, paths);
            if (!success) break;
            // optimize_async_wait_and_update after the pass (:446-448)
            check_sdmm(sdmm_guiding_update(m_guiding), "sdmm_guiding_update");
            const Float elapsed = timer->getSeconds();
            totalElapsed += elapsed;
            // the film: this pass with weight spp / sampleCount (sdmm_proc.cpp:1142-1158)
            ref<Bitmap> bmp = new Bitmap(Bitmap::ERGB, Bitmap::EFloat32, size);
            float* px = bmp->getFloat32Data();
            const size_t plane = (size_t)size.x * size.y;
            for (size_t i = 0; i < plane; ++i)
                for (int ch = 0; ch < 3; ++ch) px[3 * i + ch] = mean[ch * plane + i];
            film->addBitmap(bmp, (Float)1 / (Float)nPasses);
            queue->signalRefresh(job);
            // dumpIndividual (sdmm_wr.cpp:115-146)
            char name[64];
            std::snprintf(name, sizeof(name), "iteration%05i.exr", it);
            check_sdmm(sdmm_write_exr((outDir / name).string().c_str(), size.x, size.y, mean.data(),
                                      m_samplesPerIteration, it, (float)elapsed),
                       "sdmm_write_exr");
            std::snprintf(name, sizeof(name), "iteration_sqr%05i.exr", it);
            check_sdmm(sdmm_write_exr((outDir / name).string().c_str(), size.x, size.y, sqr.data(),
                                      m_samplesPerIteration, it, (float)elapsed),
                       "sdmm_write_exr");
            // optimize() / optimize_async_run() while training (:495-501)
            timer->reset();
            sdmm_guiding_stats gs{};
            if (training) check_sdmm(sdmm_guiding_optimize(m_guiding, m_samplesPerIteration, &gs), "optimize");
            const Float trainingSeconds = timer->getSeconds();
            stats << (it ? ",\n" : "") << "    {\"iteration\": " << it << ", \"elapsed_seconds\": " << elapsed
                  << ", \"total_elapsed_seconds\": " << totalElapsed << ", \"training_seconds\": " << trainingSeconds
                  << ", \"mean_path_length\": " << (paths ? (double)pathLength / (double)paths : 0.0)
                  << ", \"spp\": " << m_samplesPerIteration
                  << ", \"total_spp\": " << samplesRendered + m_samplesPerIteration
                  << ", \"leaf_nodes_count\": " << sdmm_stree_leaf_nodes(sdmm_guiding_tree(m_guiding))
                  << ", \"optimized_nodes_count\": " << (training ? gs.optimized : 0) << "}";
            if (m_cancelled) { success = false; break; }
        }
        check_sdmm(sdmm_guiding_update(m_guiding), "sdmm_guiding_update");
        stats << "\n]\n";
        std::ofstream((outDir / "stats.json").string()) << stats.str();
        saveCheckpoint(outDir, nPasses);
        return success;
    }

    MTS_DECLARE_CLASS()

private:
    // saveCheckpoint (:121-130): checkpoints/model_%05i.asdmm
    void saveCheckpoint(const fs::path& dir, int iteration) {
        const fs::path cdir = dir / "checkpoints";
        if (!fs::exists(cdir)) fs::create_directories(cdir);
        char name[64];
        std::snprintf(name, sizeof(name), "model_%05i.asdmm", iteration);
        sdmm_stree* tree = sdmm_guiding_tree(m_guiding);
        std::vector<const sdmm_mix*> mix((size_t)sdmm_stree_num_nodes(tree));
        check_sdmm(sdmm_guiding_node_mixtures(m_guiding, mix.data(), (int)mix.size()), "node_mixtures");
        check_sdmm(sdmm_save_json(tree, mix.data(), (cdir / name).string().c_str()), "sdmm_save_json");
    }

    // One render pass over all tiles on nCores threads.
    bool renderPass(Scene* scene, Sensor* sensor, const Vector2i& size, int iteration, bool training, int nCores,
                    std::vector<float>& mean, std::vector<float>& sqr, int64_t& pathLength, int64_t& paths) {
        const int T = m_tileSize;
        const int tx = (size.x + T - 1) / T, ty = (size.y + T - 1) / T;
        std::atomic<int> next{0};
        std::atomic<int64_t> len{0}, cnt{0};
        const bool guided = sdmm_guiding_trained(m_guiding) > 0;   // m_iteration != 0 (:311-316)
        // the render phase reads the tree and its leaves' conditionals from
        // every worker at once (sdmm_proc.cpp:1086-1106): publish them once,
        // then each worker guides through its own context, with no lock
        // then each bounce leases a guide context (stream + scratch) from a
        // pool shared by the workers (sdmm_amd::GuideContextPool)
        // -- or, for a plain (non-product) bounce of fewer than guideBatchBelow
        // queries with guideBatch > 0 (late bounces, small tiles), the
        // workers' bounces are gathered into shared wavefronts of up to
        // guideBatch queries (sdmm_amd::GuideBatcher, two in flight)
        // (both kept across passes: the tree object is the model's for its
        // lifetime, a republished tree serves the same contexts, and their
        // scratch stays allocated)
        if (guided) {
            check_sdmm(sdmm_stree_publish(sdmm_guiding_tree(m_guiding), nullptr), "sdmm_stree_publish");
            if (!m_pool) m_pool.reset(new sdmm_amd::GuideContextPool(sdmm_guiding_tree(m_guiding), m_guideContexts));
            if (!m_batch && m_guideBatch > 0 && !(m_sampleProduct && !m_bsdfOnly))
                m_batch.reset(new sdmm_amd::GuideBatcher(sdmm_guiding_tree(m_guiding), 2, m_guideBatch));
        }
        m_ctxPool = guided ? m_pool.get() : nullptr;
        m_batcher = guided ? m_batch.get() : nullptr;
        auto worker = [&](int wid) {
            ref<Sampler> sampler = static_cast<Sampler*>(scene->getSampler()->clone().get());
            Staging st;
            const int V = std::max(1, m_maxDepth > 0 ? std::min(m_maxDepth - 1, 10) : 10);
            st.allocate((int64_t)T * T * m_samplesPerIteration, V, m_sampleProduct && !m_bsdfOnly);
            for (int t = next++; t < tx * ty && !m_cancelled; t = next++) {
                const int x0 = (t % tx) * T, y0 = (t / tx) * T;
                const int w = std::min(T, size.x - x0), h = std::min(T, size.y - y0);
                int64_t l = 0, c = 0;
                renderTile(scene, sensor, sampler, st, size, x0, y0, w, h, iteration, training, guided, mean, sqr,
                           l, c);
                len += l;
                cnt += c;
            }
        };
        std::vector<std::thread> workers;
        for (int i = 0; i < nCores; ++i) workers.emplace_back(worker, i);
        for (auto& th : workers) th.join();
        m_ctxPool = nullptr;
        m_batcher = nullptr;
        pathLength = len;
        paths = cnt;
        return !m_cancelled;
    }

    // One tile's paths as a wavefront (Li, sdmm_proc.cpp:592-871).  The
    // bounce loop draws its numbers from the worker's sampler in wavefront
    // order (every path's bounce b before any path's bounce b+1): use the
    // independent sampler, as the test suite's scenes do.
    void renderTile(Scene* scene, Sensor* sensor, Sampler* sampler, Staging& st, const Vector2i& size, int x0,
                    int y0, int w, int h, int iteration, bool training, bool guided, std::vector<float>& mean,
                    std::vector<float>& sqr, int64_t& pathLength, int64_t& pathCount) {
        const int spp = m_samplesPerIteration;
        const int64_t n = (int64_t)w * h * spp;
        const int V = st.V;
        const Float hWeight = 0.5f;                            // heuristicConditionalWeight (:383)
        std::vector<PathState> P((size_t)n);
        std::vector<int> nv((size_t)n, 0);
        // camera rays and the first hit (:641-677)
        for (int64_t p = 0; p < n; ++p) {
            const int64_t pix = p / spp;
            const Point2i xy(x0 + (int)(pix % w), y0 + (int)(pix / w));
            if (p % spp == 0) sampler->generate(xy);
            PathState& s = P[(size_t)p];
            s.samplePos = Point2((Float)xy.x, (Float)xy.y) + sampler->next2D();
            s.throughput = sensor->sampleRayDifferential(s.ray, s.samplePos, Point2(0.5f), 0.5f);
            s.Li = Spectrum(0.0f);
            s.depth = -1;
            s.query = -1;
            s.eta = 1.0f;
            s.medium = sensor->getMedium();
            s.emission = true;
            s.scattered = false;
            if (scene->rayIntersect(s.ray, s.its)) {
                if (s.its.isEmitter()) s.Li += s.throughput * s.its.Le(-s.ray.d);
                s.depth = 1;
            } else {                               // (:653-665): attenuated by the camera's medium
                Spectrum v = s.throughput * scene->evalEnvironment(s.ray);
                if (s.medium) v *= s.medium->evalTransmittance(s.ray, sampler);
                s.Li += v;
            }
            sampler->advance();
        }
        std::vector<std::unique_ptr<BSDFSamplingRecord>> brecs((size_t)n);
        for (int bounce = 0;; ++bounce) {
            // loop head (:649-691): emission / environment after index-matched
            // passes, the depth cap, strict normals on wi; then sampleSurface's
            // first half (:275-392): the guide is queried for every BSDF that is
            // not all-delta (:297); the BSDF sample is drawn up front (its
            // direction is the pdf query's when the BSDF is chosen, and it is
            // the whole answer when the leaf has no valid conditional)
            int64_t nq = 0, live = 0;
            for (int64_t p = 0; p < n; ++p) {
                PathState& s = P[(size_t)p];
                s.query = -1;
                if (s.depth < 0) continue;
                if (!s.its.isValid()) {                // (:653-665), only reached after an index-matched pass
                    if (s.emission) {
                        Spectrum v = s.throughput * scene->evalEnvironment(s.ray);
                        if (s.medium) v *= s.medium->evalTransmittance(s.ray, sampler);
                        s.Li += v;
                        recordRadiance(st, p, n, nv[(size_t)p], v);
                    }
                    s.depth = -1;
                    continue;
                }
                if (bounce > 0 && s.emission && s.its.isEmitter()) {   // (:668-672)
                    const Spectrum v = s.throughput * s.its.Le(-s.ray.d);
                    s.Li += v;
                    recordRadiance(st, p, n, nv[(size_t)p], v);
                }
                if (m_maxDepth >= 0 && s.depth >= m_maxDepth) { s.depth = -1; continue; }
                const Float wiDotGeoN = -dot(s.its.geoFrame.n, s.ray.d), wiDotShN = Frame::cosTheta(s.its.wi);
                if (wiDotGeoN * wiDotShN < 0 && m_strictNormals) { s.depth = -1; continue; }   // (:688-691)
                const BSDF* bsdf = s.its.getBSDF(s.ray);
                brecs[(size_t)p].reset(new BSDFSamplingRecord(s.its, sampler, ERadiance));
                BSDFSamplingRecord& bRec = *brecs[(size_t)p];
                const unsigned type = bsdf->getType();
                const bool allDelta = (type & BSDF::EDelta) == (type & BSDF::EAll);
                ++live;
                if (!guided || allDelta) {              // (:297-302, :316-323)
                    s.bsdfWeight = bsdf->sample(bRec, s.bsdfPdf, sampler->next2D());
                    continue;
                }
                const Float choice = sampler->next1D();    // rRec.nextSample1D() (:383)
                s.bsdfWeight = bsdf->sample(bRec, s.bsdfPdf, sampler->next2D());
                s.pdfMode = choice <= hWeight;
                const Vector dB = s.its.toWorld(bRec.wo);
                const int64_t q = nq++;
                if (st.h_mat) learnedRow(st, bsdf, bRec, s.its, q, n, (float)choice);
                float* in = st.h_in;
                const Point c((s.its.p - m_sceneMin) / m_spatialNorm);        // createCondition (:263-273)
                in[0 * n + q] = (float)c.x; in[1 * n + q] = (float)c.y; in[2 * n + q] = (float)c.z;
                in[3 * n + q] = (float)sampler->next1D();
                in[4 * n + q] = (float)sampler->next1D();
                in[5 * n + q] = (float)sampler->next1D();
                in[6 * n + q] = (float)dB.x; in[7 * n + q] = (float)dB.y; in[8 * n + q] = (float)dB.z;
                st.h_mode[q] = s.pdfMode ? 1 : 0;
                s.query = q;
            }
            if (live == 0) break;
            if (nq > 0) guideWavefront(st, n, nq);
            const bool productBounce = nq > 0 && st.h_mat != nullptr;
            // sampleSurface's second half (:392-507) and the loop body (:759-871)
            for (int64_t p = 0; p < n; ++p) {
                PathState& s = P[(size_t)p];
                if (s.depth < 0) continue;
                const BSDF* bsdf = s.its.getBSDF(s.ray);
                BSDFSamplingRecord& bRec = *brecs[(size_t)p];
                const int32_t comp = s.query >= 0 ? st.h_comp[s.query] : -1;
                Spectrum weight(0.0f);
                Float pdf = 0;
                if (comp == -1) {
                    // BSDF only, h = 1 (:298-302, :316-323, :392-405)
                    weight = s.bsdfWeight;
                    pdf = s.bsdfPdf;
                } else {
                    const Float gmmPdf = st.h_out[3 * n + s.query];
                    // h: 0.5, or the product query's own 0.3 / 0.5 (:383-392)
                    const Float hq = productBounce ? (Float)st.h_pf[10 * n + s.query] : hWeight;
                    if (comp == -2) {
                        // the BSDF sample was chosen (:392-407)
                        if (!s.bsdfWeight.isZero()) {
                            if (bRec.sampledType & BSDF::EDelta) {
                                // a delta lobe: gmmPdf = 0, pdf *= h, weight / h (:401-405)
                                pdf = s.bsdfPdf * hq;
                                weight = s.bsdfWeight / hq;
                            } else {
                                const Float bsdfPdf = bsdf->pdf(bRec);   // pdfSurface (:510-534, :587-589)
                                pdf = (bsdfPdf > 0 && std::isfinite(bsdfPdf)) ? hq * bsdfPdf + (1 - hq) * gmmPdf : 0;
                                if (pdf != 0) weight = (s.bsdfWeight * s.bsdfPdf) / pdf;
                            }
                        }
                    } else {
                        // the guide's direction: a fresh record's lobe state
                        // (nothing was sampled, :410-463) and bsdf->eval / pdfSurface
                        bRec.sampledType = 0;
                        bRec.sampledComponent = -1;
                        bRec.eta = 1.0f;
                        const Vector d(st.h_out[0 * n + s.query], st.h_out[1 * n + s.query],
                                       st.h_out[2 * n + s.query]);
                        if (!d.isZero()) {
                            bRec.wo = s.its.toLocal(d);
                            const Float bsdfPdf = bsdf->pdf(bRec);
                            pdf = (bsdfPdf > 0 && std::isfinite(bsdfPdf)) ? hq * bsdfPdf + (1 - hq) * gmmPdf : 0;
                            if (pdf != 0) weight = bsdf->eval(bRec) / pdf;
                        }
                    }
                }
                const bool cacheable = !(bRec.sampledType & BSDF::EDelta);   // (:764)
                if (weight.isZero() || !weight.isValid()) { s.depth = -1; continue; }   // (:759-774)
                const Vector wo = s.its.toWorld(bRec.wo);
                const Float woDotGeoN = dot(s.its.geoFrame.n, wo);
                if (woDotGeoN * Frame::cosTheta(bRec.wo) <= 0 && m_strictNormals) { s.depth = -1; continue; }
                // the vertex normal on the wi side (:650-651, :765-767)
                const Normal n_s = Frame::cosTheta(bRec.wi) < 0 ? Normal(-s.its.shFrame.n) : s.its.shFrame.n;
                const Point o = s.its.p;
                const Point cnd((o - m_sceneMin) / m_spatialNorm);
                s.ray = RayDifferential(o, wo, s.ray.time);
                s.throughput *= weight;
                s.eta *= bRec.eta;                     // (:788)
                if (s.its.isMediumTransition()) s.medium = s.its.getTargetMedium(s.ray.d);   // (:789-790)
                if (bRec.sampledType == BSDF::ENull) {
                    // an index-matched medium transition (:792-800): continue
                    // through it, no vertex, no roulette; emission is seen
                    // again only if the path has not scattered yet
                    s.emission = !s.scattered;
                    scene->rayIntersect(s.ray, s.its);
                    ++s.depth;
                    continue;
                }
                // trace and look for an emitter through index-matched surfaces
                // (rayIntersectAndLookForEmitter, :803, :988-1050); no NEE: MIS
                // weight 1 (:811-816)
                Spectrum value(0.0f);
                const int maxInteractions = m_maxDepth >= 0 ? m_maxDepth - s.depth - 1 : -1;
                const bool hit = lookForEmitter(scene, sampler, s.medium, maxInteractions, s.ray, s.its, value);
                int& k = nv[(size_t)p];
                if (!value.isZero()) {
                    const Spectrum rad = s.throughput * value;
                    s.Li += rad;
                    recordRadiance(st, p, n, k, rad);
                }
                if (cacheable && k < V) {             // the saved vertex (:821-846)
                    const Float clamped = std::max(pdf, (Float)0.1f);
                    Float rgb[3], thr[3];
                    value.toLinearRGB(rgb[0], rgb[1], rgb[2]);
                    s.throughput.toLinearRGB(thr[0], thr[1], thr[2]);
                    for (int ch = 0; ch < 3; ++ch) {
                        st.rec(ch, k, p, n) = (float)(rgb[ch] / clamped);
                        st.rec(3 + ch, k, p, n) = (float)thr[ch];
                    }
                    st.rec(6, k, p, n) = (float)clamped;
                    st.rec(7, k, p, n) = (float)cnd.x; st.rec(8, k, p, n) = (float)cnd.y;
                    st.rec(9, k, p, n) = (float)cnd.z;
                    st.rec(10, k, p, n) = (float)wo.x; st.rec(11, k, p, n) = (float)wo.y;
                    st.rec(12, k, p, n) = (float)wo.z;
                    st.rec(13, k, p, n) = (float)n_s.x; st.rec(14, k, p, n) = (float)n_s.y;
                    st.rec(15, k, p, n) = (float)n_s.z;
                    ++k;
                }
                s.emission = false;                    // rRec.type = ERadianceNoEmission (:850)
                if (!hit) { s.depth = -1; continue; }   // the next loop head would end it (:653-665)
                if (s.depth >= m_rrDepth) {             // Russian roulette (:858-868)
                    const Float qq = std::min(s.throughput.max() * s.eta * s.eta, (Float)0.95f);
                    if (sampler->next1D() >= qq) { s.depth = -1; continue; }
                    s.throughput /= qq;
                }
                ++s.depth;
                s.scattered = true;
            }
        }
        // the pixels' pass mean and mean of squares (box filter, sample order)
        const size_t plane = (size_t)size.x * size.y;
        for (int64_t pix = 0; pix < (int64_t)w * h; ++pix) {
            Float acc[3] = {0, 0, 0}, sq[3] = {0, 0, 0};
            for (int sidx = 0; sidx < spp; ++sidx) {
                Float rgb[3];
                P[(size_t)(pix * spp + sidx)].Li.toLinearRGB(rgb[0], rgb[1], rgb[2]);
                for (int ch = 0; ch < 3; ++ch) { acc[ch] += rgb[ch]; sq[ch] += rgb[ch] * rgb[ch]; }
            }
            const size_t o = (size_t)(y0 + pix / w) * size.x + (size_t)(x0 + pix % w);
            for (int ch = 0; ch < 3; ++ch) {
                mean[ch * plane + o] = (float)(acc[ch] / spp);
                sqr[ch * plane + o] = (float)(sq[ch] / spp);
            }
        }
        for (int64_t p = 0; p < n; ++p) pathLength += nv[(size_t)p];
        pathCount += n;
        // push_back_data + the jittered neighbour leaves for the tile (:876-965)
        if (training) {
            for (int64_t p = 0; p < n; ++p) st.h_nv[p] = nv[(size_t)p];
            const int64_t path0 = ((int64_t)y0 * size.x + x0) * spp;   // the jitter's counter RNG (tile-unique)
            std::lock_guard<std::mutex> lock(m_gpuMutex);
            check_hip(hipMemcpyAsync(st.d_rec, st.h_rec, sizeof(float) * 16 * V * n, hipMemcpyHostToDevice, m_stream),
                      "upload vertices");
            check_hip(hipMemcpyAsync(st.d_nv, st.h_nv, sizeof(int32_t) * n, hipMemcpyHostToDevice, m_stream),
                      "upload vertex counts");
            sdmm_path_vertices v{n, V, path0, st.d_rec, st.d_nv};
            check_sdmm(sdmm_guiding_push(m_guiding, &v, 0x5D33u + (uint64_t)iteration), "sdmm_guiding_push");
        }
    }

    // rayIntersectAndLookForEmitter (sdmm_proc.cpp:988-1050): intersect, and
    // through a chain of index-matched (ENull) surfaces keep tracing while
    // accumulating the medium transmittance and the null BSDFs' discrete
    // eval, until an occluder, a light source or maxInteractions; value gets
    // the attenuated emission of an emitter (or the environment on a miss).
    // _its receives the FIRST surface hit (the path continues from there).
    // Returns whether a surface was hit.
    static bool lookForEmitter(const Scene* scene, Sampler* sampler, const Medium* medium, int maxInteractions,
                               Ray ray, Intersection& _its, Spectrum& value) {
        Intersection its2, *its = &_its;
        Spectrum transmittance(1.0f);
        bool surface = false, first = true, firstHit = false;
        int interactions = 0;
        while (true) {
            surface = scene->rayIntersect(ray, *its);
            if (first) { firstHit = surface; first = false; }
            if (medium) transmittance *= medium->evalTransmittance(Ray(ray, 0, its->t), sampler);
            if (surface && (interactions == maxInteractions || !(its->getBSDF()->getType() & BSDF::ENull) ||
                            its->isEmitter()))
                break;                              // an occluder or a light source
            if (!surface) break;
            if (transmittance.isZero()) return firstHit;
            if (its->isMediumTransition()) medium = its->getTargetMedium(ray.d);
            const Vector wo = its->shFrame.toLocal(ray.d);
            BSDFSamplingRecord bRec(*its, -wo, wo, ERadiance);
            bRec.typeMask = BSDF::ENull;
            transmittance *= its->getBSDF()->eval(bRec, EDiscrete);
            ray.o = ray(its->t);
            ray.mint = Epsilon;
            its = &its2;
            if (++interactions > 100) return firstHit;   // round-off guard (:1035-1038)
        }
        if (surface) {
            if (its->isEmitter()) value = transmittance * its->Le(-ray.d);
        } else {
            const Emitter* env = scene->getEnvironmentEmitter();
            if (env) value = transmittance * env->evalEnvironment(RayDifferential(ray));
        }
        return firstHit;
    }

    // recordRadiance (:628-637): every saved vertex of the path gets the
    // radiance divided by its throughput and sampling pdf
    static void recordRadiance(Staging& st, int64_t p, int64_t n, int k, const Spectrum& rad) {
        Float r[3];
        rad.toLinearRGB(r[0], r[1], r[2]);
        for (int v = 0; v < k; ++v) {
            const float pdf = st.rec(6, v, p, n);
            for (int ch = 0; ch < 3; ++ch) {
                const float thr = st.rec(3 + ch, v, p, n);
                if (thr > 1e-4f) st.rec(ch, v, p, n) += (float)(r[ch] / (thr * pdf));
            }
        }
    }

    // sampleProduct: query q's learned-BSDF row (:327-356).  getDMM / the
    // diffuse re-centring / rotate_to_wo are the BSDF's and sdmm-lib's calls
    // (the maintainer's build has both); the lobes go over in the local
    // shading frame with the frame F = [s t n] per query -- the kernel forms
    // mean F m and frame Coordinates(m) F^T (:348-355).  A diffuse BSDF keeps
    // its lobes as loaded and is flagged: the kernel re-centres slice 0 on
    // F's third column (the shading normal; getDMM fails from the back side,
    // so no flip is needed) exactly as set_mean does (:335-339).
    void learnedRow(Staging& st, const BSDF* bsdf, BSDFSamplingRecord& bRec, const Intersection& its, int64_t q,
                    int64_t n, float choice) {
        st.h_mat[q] = -1;
        for (int f = 0; f < 3; ++f)
            for (int c = 0; c < 3; ++c) {
                const Vector col = c == 0 ? its.shFrame.s : (c == 1 ? its.shFrame.t : its.shFrame.n);
                st.h_pf[(size_t)(3 * f + c) * n + q] = (float)col[f];
            }
        st.h_pf[9 * n + q] = choice;
        BSDF::DMM learned;
        if (!bsdf->getDMM(bRec, learned)) return;          // no learned BSDF: the plain conditional (h 0.5)
        const auto type = bsdf->getType();
        const bool diffuse = (type & BSDF::EDiffuseReflection) == (type & BSDF::EAll);
        if (!diffuse) enoki::packet(learned.tangent_space, 0).rotate_to_wo({bRec.wi[0], bRec.wi[1], bRec.wi[2]});
        const size_t M = enoki::slices(learned);
        if (M > (size_t)kMaxLobes) Log(EError, "learned BSDF with %i lobes (max %i)", (int)M, kMaxLobes);
        float* w = st.h_bw + (size_t)q * kMaxLobes;
        float* mean = st.h_bmean + (size_t)q * kMaxLobes * 3;
        float* cov = st.h_bcov + (size_t)q * kMaxLobes * 4;
        for (int j = 0; j < kMaxLobes; ++j) {
            w[j] = (size_t)j < M ? (float)enoki::slice(learned.weight.pmf, j) : 0.0f;   // 0: skipped
            if ((size_t)j >= M) continue;
            auto lobe = enoki::slice(learned.tangent_space, j);
            for (int a = 0; a < 3; ++a) mean[3 * j + a] = (float)lobe.mean(a);
            auto c2 = enoki::slice(learned.cov, j);
            for (int a = 0; a < 4; ++a) cov[4 * j + a] = (float)c2(a / 2, a % 2);
        }
        st.h_bdiff[q] = diffuse ? 1 : 0;
        st.h_mat[q] = (int32_t)q;
    }

    // One guided bounce of a tile's wavefront: sampleSurface / pdfSurface for
    // nq queries (query planes of stride n) in one call on a leased guide
    // context and its stream -- the workers run at once, as the reference's
    // render threads do (sdmm_proc.cpp:1086-1106).
    void guideWavefront(Staging& st, int64_t n, int64_t nq) {
        if (m_batcher && !st.h_mat && nq < m_guideBatchBelow) {
            // the staging is the request (pinned planes of stride n); the
            // batch's leader copies, launches and synchronises
            const sdmm_guide_host_req rq{nq, st.h_in, n, st.h_mode, st.h_out, n, st.h_comp};
            try {
                m_batcher->serve(rq);
            } catch (const sdmm_amd::Error& e) {
                SLog(EError, "%s", e.what());
            }
            return;
        }
        const sdmm_amd::GuideContextPool::Lease lease = m_ctxPool->acquire();
        const hipStream_t wst = (hipStream_t)lease.stream();
        for (int f = 0; f < 9; ++f)
            check_hip(hipMemcpyAsync(st.d_in + f * n, st.h_in + f * n, sizeof(float) * nq, hipMemcpyHostToDevice,
                                     wst), "upload queries");
        check_hip(hipMemcpyAsync(st.d_mode, st.h_mode, nq, hipMemcpyHostToDevice, wst), "upload modes");
        const float* c[3] = {st.d_in, st.d_in + n, st.d_in + 2 * n};
        const float* u[3] = {st.d_in + 3 * n, st.d_in + 4 * n, st.d_in + 5 * n};
        const float* dg[3] = {st.d_in + 6 * n, st.d_in + 7 * n, st.d_in + 8 * n};
        float* d[3] = {st.d_out, st.d_out + n, st.d_out + 2 * n};
        if (st.h_mat) {
            // sampleProduct: the per-query table rows, frames and draws
            const size_t L = (size_t)nq * kMaxLobes;
            check_hip(hipMemcpyAsync(st.d_bw, st.h_bw, sizeof(float) * L, hipMemcpyHostToDevice, wst), "upload");
            check_hip(hipMemcpyAsync(st.d_bmean, st.h_bmean, sizeof(float) * 3 * L, hipMemcpyHostToDevice, wst),
                      "upload");
            check_hip(hipMemcpyAsync(st.d_bcov, st.h_bcov, sizeof(float) * 4 * L, hipMemcpyHostToDevice, wst),
                      "upload");
            check_hip(hipMemcpyAsync(st.d_bdiff, st.h_bdiff, nq, hipMemcpyHostToDevice, wst), "upload");
            check_hip(hipMemcpyAsync(st.d_mat, st.h_mat, sizeof(int32_t) * nq, hipMemcpyHostToDevice, wst),
                      "upload");
            for (int f = 0; f < 10; ++f)
                check_hip(hipMemcpyAsync(st.d_pf + f * n, st.h_pf + f * n, sizeof(float) * nq, hipMemcpyHostToDevice,
                                         wst), "upload");
            const sdmm_bsdf_table tab{st.d_bw, st.d_bmean, st.d_bcov, (int)nq, kMaxLobes, st.d_bdiff};
            const float* F[9];
            for (int f = 0; f < 9; ++f) F[f] = st.d_pf + f * n;
            check_sdmm(sdmm_ctx_guide_product_wavefront(lease.get(), nq, c, u, st.d_pf + 9 * n, dg, &tab, st.d_mat, F, d,
                                                        st.d_out + 3 * n, st.d_comp, st.d_pf + 10 * n, nullptr),
                       "sdmm_ctx_guide_product_wavefront");
            check_hip(hipMemcpyAsync(st.h_pf + 10 * n, st.d_pf + 10 * n, sizeof(float) * nq, hipMemcpyDeviceToHost,
                                     wst), "download h");
        } else {
            check_sdmm(sdmm_ctx_guide_pdf_wavefront(lease.get(), nq, c, u, dg, st.d_mode, d, st.d_out + 3 * n, st.d_comp,
                                                    nullptr),
                       "sdmm_ctx_guide_pdf_wavefront");
        }
        for (int f = 0; f < 4; ++f)
            check_hip(hipMemcpyAsync(st.h_out + f * n, st.d_out + f * n, sizeof(float) * nq, hipMemcpyDeviceToHost,
                                     wst), "download directions");
        check_hip(hipMemcpyAsync(st.h_comp, st.d_comp, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, wst),
                  "download components");
        check_hip(hipStreamSynchronize(wst), "hipStreamSynchronize");
    }

    bool m_strictNormals = true;
    int m_maxDepth = -1, m_rrDepth = 5, m_samplesPerIteration = 8, m_savedSamplesPerPath = 8;
    bool m_sampleProduct = false, m_bsdfOnly = false, m_optimizeAsync = true;
    int m_device = 0, m_tileSize = 64;
    Point m_sceneMin;
    Float m_spatialNorm = 1;
    sdmm_guiding* m_guiding = nullptr;
    hipStream_t m_stream = nullptr;   // the model's (training-data pushes, under m_gpuMutex)
    int m_guideContexts = 4;          // guide contexts shared by the workers (one per hardware queue)
    sdmm_amd::GuideContextPool* m_ctxPool = nullptr;   // the pass's (renderPass)
    int m_guideBatch = 1 << 18;       // queries per gathered wavefront (0: each worker calls alone)
    // bounces with fewer queries than this are gathered, larger ones go
    // through the context pool (16 x 32 K-query tiles: contexts 298 M/s,
    // batcher 212-240; 4 K-query tiles: batcher 85 M/s, contexts 14;
    // profiles/round6_plugin_pattern_final.json)
    int m_guideBatchBelow = 1 << 14;
    sdmm_amd::GuideBatcher* m_batcher = nullptr;       // the pass's (renderPass)
    std::unique_ptr<sdmm_amd::GuideContextPool> m_pool;   // created at the first guided pass
    std::unique_ptr<sdmm_amd::GuideBatcher> m_batch;
    std::mutex m_gpuMutex;
    std::atomic<bool> m_cancelled{false};
};

MTS_IMPLEMENT_CLASS_S(SDMMAmdPathTracer, false, Integrator)
MTS_EXPORT_PLUGIN(SDMMAmdPathTracer, "SDMM volumetric path tracer (MI355X guiding)");
MTS_NAMESPACE_END
