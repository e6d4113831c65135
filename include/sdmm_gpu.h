/*
 * sdmm_gpu.h -- C ABI of the MI355X-native SDMM path-guiding hot path.
 *
 * This is the drop-in boundary the Mitsuba `sdmm` integrator plugin calls in
 * place of the (absent) sdmm-lib submodule.  Every entry point names the
 * reference interface it replaces (paths relative to anadodik/sdmm-mitsuba):
 *
 *   sdmm_create / sdmm_destroy    SDMMContext construction
 *                                 (mitsuba/src/integrators/sdmm/sdmm_proc.h:92-93)
 *   sdmm_init_hemisphere          sdmm::initialize  (volpath_sdmm.cpp:132-138);
 *                                 math: jmm uniformHemisphereInit
 *                                 (dmm/jmm/mixture_model_init.h:79-242)
 *   sdmm_em_step                  sdmm::em_step     (volpath_sdmm.cpp:220, :304)
 *                                 + sdmm::prepare   (volpath_sdmm.cpp:237, :307);
 *                                 math: jmm StepwiseTangentEM::optimize
 *                                 (dmm/jmm/opt/stepwise_tangent.h:597-1053)
 *   sdmm_em_step_batched          the plugin's per-leaf optimisation loop: one
 *                                 sdmm::em_step per tree leaf, run on a thread
 *                                 pool (volpath_sdmm.cpp:244-312, leaf filter
 *                                 :140-149), as ONE batched device launch
 *   sdmm_estep_stats/sdmm_mstep   the same EM step split around the
 *                                 sufficient-statistics all-reduce (multi-GPU)
 *   sdmm_responsibilities         MixtureModel::posteriorAndLog over a batch
 *                                 (dmm/jmm/mixture_model.h:146-192)
 *   sdmm_guide_batch              sdmm::create_conditional + conditional.sample
 *                                 + posterior/hsum_nested (sdmm_proc.cpp:368,
 *                                 :411-421, :539-545); math: jmm
 *                                 MixtureModel::conditional/sample/pdf
 *                                 (mixture_model.h:235-304, :72-75, :113-121)
 *   sdmm_pdf_batch                pdfSurface's gmmPdf (sdmm_proc.cpp:510-590)
 *   sdmm_get_params/set_params    sdmm::save_json / load_json
 *                                 (volpath_sdmm.cpp:121-130; bsdfs/diffuse.cpp:101-114)
 *
 * Conventions: plain C types only; every function returns SDMM_OK (0) or a
 * negative SDMM_E* code and sets a thread-local message (sdmm_last_error).
 * No C++ exception crosses the ABI.  Pointers documented "device" must be
 * HBM-resident allocations on the handle's device; "host" pointers are
 * ordinary memory, read-only during the call.  A handle is re-entrant
 * against other handles; calls on one handle must be serialised by the
 * caller.  Work is enqueued on the handle's HIP stream (sdmm_set_stream);
 * functions that return data to host memory synchronise that stream.
 * Host threads may call the library at once on distinct handles (the
 * reference's per-leaf worker threads, volpath_sdmm.cpp:287-311, and render
 * threads, sdmm_proc.cpp:1086-1106): host data moves through the calling
 * thread's pinned bounce buffer (never a DMA from caller memory), per-call
 * device scratch is pooled per (device, stream), and no buffer is freed
 * before the stream that used it has been synchronised.
 */
#ifndef SDMM_GPU_H
#define SDMM_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDMM_ABI_VERSION 1

enum {
    SDMM_OK = 0,
    SDMM_E_INVALID = -1,   /* bad argument / unsupported K */
    SDMM_E_HIP = -2,       /* HIP runtime error */
    SDMM_E_STATE = -3,     /* handle not initialised */
    SDMM_E_NOMEM = -4
};

typedef struct sdmm_mix sdmm_mix;

/* StepwiseTangentEM constructor arguments (stepwise_tangent.h:221-252). */
typedef struct {
    float alpha;              /* 0.9   stepwise exponent */
    float bprior[5];          /* 1e-5  diagonal covariance prior (overwritten by init) */
    float ni_prior_minus_one; /* 6e-5  weight prior */
    double epsilon;           /* 1e-100 depth-prior diagonal (as float: 0) */
    int decrease_prior;       /* 1 */
} sdmm_em_params;

/* SoA sample batch, one plane per field (Samples<6,float>, samples.h:32-46). */
typedef struct {
    const float* x[6];          /* normalised position (3) + unit direction (3) */
    const float* w;             /* weight */
    const float* hpdf;          /* heuristic pdf, may be NULL */
    const uint8_t* is_diffuse;  /* heuristic flag, may be NULL */
    int64_t n;
} sdmm_samples;

/* Fill p with the reference defaults. */
void sdmm_em_params_default(sdmm_em_params* p);

/* Create a K-component mixture (1 <= K <= 512) on HIP device `device`. */
int sdmm_create(int K, const sdmm_em_params* params, int device, sdmm_mix** out);
/* Stream-ordered creation: the allocation (hipMallocAsync) and initialisation
 * are enqueued on hip_stream, which the handle then uses; nothing waits on the
 * host.  For the many small per-leaf mixtures of a guiding tree.  The stream
 * must outlive the handle (its memory is freed on it). */
int sdmm_create_on_stream(int K, const sdmm_em_params* params, int device, void* hip_stream, sdmm_mix** out);
/* n such handles from ONE stream-ordered slab (one allocation, one
 * initialisation launch for all); the slab is freed with its last handle. */
int sdmm_create_many_on_stream(int K, const sdmm_em_params* params, int device, void* hip_stream, int n,
                               sdmm_mix** out);
void sdmm_destroy(sdmm_mix* m);
int sdmm_num_components(const sdmm_mix* m);
/* Diagnostics: E-step kernel layouts (components per lane, lanes per sample)
 * of the responsibility and statistics kernels.  Any pointer may be NULL. */
int sdmm_layout(const sdmm_mix* m, int* resp_cpl, int* resp_lps, int* stats_cpl, int* stats_lps);
/* Diagnostics: name of the kernel the handle launches for the responsibility
 * (which = 0) or statistics (which = 1) E-step; "" for a NULL handle. */
const char* sdmm_kernel_name(const sdmm_mix* m, int which);
/* Guided queries keep a per-query list of at most `cap` candidate components
 * (default 40, maximum 64); queries that do not fit take the full-K path.
 * Results are identical for every cap; 0 sends every query down the full-K
 * path (a testing knob).  A tree wavefront uses the smallest cap of the
 * mixtures bound to it (read when the table is bound / passed). */
int sdmm_set_guide_capacity(sdmm_mix* m, int cap);
/* coherent != 0 (default): guided batches of >= 16384 queries are served in
 * Morton order of their condition position (a device radix sort of the
 * batch), so the queries of a wave touch the same components.  Outputs are
 * written at each query's own index and are identical either way. */
int sdmm_set_guide_order(sdmm_mix* m, int coherent);
/* Diagnostics: how many queries of the handle's last guided call (guide, pdf,
 * product) took the full-K fallback path.  Synchronises the handle's stream. */
int sdmm_guide_fallback_count(const sdmm_mix* m, int* count);
/* Work is enqueued on this hipStream_t, taken literally (NULL = the HIP null
 * stream).  A new handle starts on its own non-blocking stream, whose value
 * sdmm_get_stream returns before any sdmm_set_stream call. */
int sdmm_set_stream(sdmm_mix* m, void* hip_stream);
void* sdmm_get_stream(const sdmm_mix* m);
int sdmm_synchronize(sdmm_mix* m);

/* uniformHemisphereInit with given seed positions/normals (host, n_pos*3 each);
 * K must equal 8 * n_pos.  depth_prior / min_spatial_distance in normalised
 * scene units; seed drives the PCG32 direction jitter. */
int sdmm_init_hemisphere(sdmm_mix* m, const float* positions, const float* normals, int n_pos,
                         float depth_prior, float min_spatial_distance, uint64_t seed);

/* sdmm_init_hemisphere for n mixtures of one K at once (mixture i: K/8
 * positions / normals at positions + 3 (K/8) i, its own spatial distance and
 * seed): one host synchronisation for the whole set (the guiding model's new
 * leaves). */
int sdmm_init_hemisphere_batched(sdmm_mix* const* mixes, int n, const float* positions, const float* normals,
                                 float depth_prior, const float* min_spatial_distance, const uint64_t* seeds);

/* kMeansPPInit (dmm/jmm/mixture_model_init.h:244-330) on the device: for each
 * of n_leaves leaves -- samples [seg[l], seg[l+1]) of the device planes s->x[0..2]
 * (positions), normals[0..2] and s->w -- the k-means++ choice of n_pos seed
 * samples, draw i using uniforms[l * n_pos + i] (the rng() calls, in order).
 * out_index (host, n_leaves * n_pos): leaf-relative sample indices;
 * out_positions / out_normals (host, 3 per draw, may be NULL): the chosen
 * samples' positions and normals.  Weights
 * and their sums in fp64 (the reference forms a float CDF; the choice differs
 * only where a draw falls within its rounding of a boundary).  One workgroup
 * per leaf on hip_stream; returns after the indices are on the host. */
int sdmm_kmeanspp_select(const sdmm_samples* s, const float* const normals[3], const int64_t* seg, int n_leaves,
                         int n_pos, const float* uniforms, int device, void* hip_stream, int64_t* out_index,
                         float* out_positions, float* out_normals);

/* uniformHemisphereInit with kMeansPlusPlus = true (:130-138) for n mixtures
 * of one K: mixture i's K/8 positions / normals chosen by sdmm_kmeanspp_select
 * over samples [seg[i], seg[i+1]); its PCG32 stream (seeds[i]) gives the
 * K/8 k-means++ draws and then the direction jitter. */
int sdmm_init_hemisphere_kmeanspp_batched(sdmm_mix* const* mixes, int n, const sdmm_samples* s,
                                          const float* const normals[3], const int64_t* seg, float depth_prior,
                                          const float* min_spatial_distance, const uint64_t* seeds);

/* Host-only variant (no device, no handle): writes the initial component
 * parameters, for data generators and tests.  Arrays sized K=8*n_pos. */
int sdmm_hemisphere_init_host(const float* positions, const float* normals, int n_pos,
                              float depth_prior, float min_spatial_distance, uint64_t seed,
                              float* weights /*K*/, float* means /*K*6*/, float* covs /*K*25*/,
                              float* bpriors /*K*25*/, float* bdepth /*K*9*/);

/* One stepwise EM iteration (`iterations` times) over device-resident samples. */
int sdmm_em_step(sdmm_mix* m, const sdmm_samples* device_samples, int iterations);
/* Same with host-resident samples (staged through the handle's buffers). */
int sdmm_em_step_host(sdmm_mix* m, const sdmm_samples* host_samples, int iterations);

/* Batched per-leaf EM (the spatial tree's leaves, each its own mixture):
 * mixes[i] takes one stepwise EM iteration (`iterations` times) over samples
 * [seg[i], seg[i+1]) of the device planes `device_samples` (the leaves' data
 * stored back to back).  seg: host, n_mix + 1 non-decreasing offsets within
 * [0, device_samples->n]; a leaf with no samples is left unchanged (like
 * sdmm_em_step with n = 0).  All handles must share K and the device and be
 * distinct; the work runs on mixes[0]'s stream (the other handles' streams
 * are synchronised on entry and wait for the batch on exit).  Results are
 * bitwise those of sdmm_em_step(mixes[i], leaf i) called one by one. */
int sdmm_em_step_batched(sdmm_mix* const* mixes, int n_mix, const sdmm_samples* device_samples,
                         const int64_t* seg, int iterations);
/* Per-leaf iteration counts (the built plugin's optimize(): 2 EM iterations
 * for a leaf while its em.iterations_run < 4, else 1, volpath_sdmm.cpp:299-305):
 * round t steps every leaf with iterations[i] > t; bitwise the same as
 * sdmm_em_step(mixes[i], leaf i, iterations[i]) one by one. */
int sdmm_em_step_batched_iters(sdmm_mix* const* mixes, int n_mix, const sdmm_samples* device_samples,
                               const int64_t* seg, const int* iterations);
/* Same with host-resident planes (staged through mixes[0]'s buffers; returns
 * after the batch, so the host planes may be reused). */
int sdmm_em_step_batched_host(sdmm_mix* const* mixes, int n_mix, const sdmm_samples* host_samples,
                              const int64_t* seg, int iterations);
int sdmm_em_step_batched_host_iters(sdmm_mix* const* mixes, int n_mix, const sdmm_samples* host_samples,
                                    const int64_t* seg, const int* iterations);

/* Split-phase EM step for sample-sharded multi-GPU runs:
 *   sdmm_estep_stats  writes this shard's fp64 sufficient statistics,
 *                     layout [H, weightSum, W(K), M(5K), C_lower(15K)],
 *                     sdmm_stats_len(K) doubles, into `stats` (device);
 *   (caller all-reduces `stats` with a SUM over ranks, e.g. ncclAllReduce)
 *   sdmm_mstep        consumes the global statistics; n_total = global sample
 *                     count (samples.size() of the reference).              */
size_t sdmm_stats_len(int K);
int sdmm_estep_stats(sdmm_mix* m, const sdmm_samples* device_samples, double* stats);
int sdmm_mstep(sdmm_mix* m, const double* stats, int64_t n_total);

/* Multi-GPU.  One process per GPU; a communicator joins the ranks
 * that train the same mixtures.  Transports:
 *   RCCL   sdmm_comm_unique_id on one rank, the 128 bytes shared by the caller
 *          (MPI, a file, torch.distributed), then sdmm_comm_init_rccl on every
 *          rank (collectives on the mixtures' HIP streams, over xGMI);
 *   host   sdmm_comm_init_host with the caller's own collective on HOST buffers
 *          (allreduce: in-place SUM of count doubles; broadcast: in-place from
 *          rank root); the library stages through pinned memory.  Callbacks
 *          return 0 on success.
 * Every rank must make the same sequence of sharded calls.
 *   sdmm_em_step_sharded   sample-sharded StepwiseTangentEM::optimize
 *                          (stepwise_tangent.h:597-1053): this rank's shard's
 *                          statistics, ONE all-reduce (sum) of [H, wsum, W, M,
 *                          Clow, n] fp64, then the same M-step on every rank
 *                          (identical parameters everywhere, no broadcast).
 *                          The reference's own sharded-statistics pattern is the
 *                          legacy jmm/opt/stepwise.h:248-396 (threads + mutex).
 *   sdmm_em_step_batched_sharded  the per-leaf EM with every rank holding
 *                          samples of every leaf: the batched statistics of all
 *                          leaves (+ counts) in ONE all-reduce per iteration
 *                          round, then the batched M-step on every rank.
 *   sdmm_mix_broadcast     leaf-sharded EM: after each rank stepped the leaves it
 *                          owns (owner[i] == rank, e.g. sdmm_em_step_batched on
 *                          that subset), every leaf's parameters and stepwise
 *                          state are broadcast from its owner (RCCL: one fused
 *                          group), so all ranks hold all leaves for guiding. */
typedef struct sdmm_comm sdmm_comm;
#define SDMM_COMM_ID_BYTES 128
typedef int (*sdmm_host_allreduce_f64)(double* buf, size_t count, void* user);
typedef int (*sdmm_host_broadcast)(void* buf, size_t bytes, int root, void* user);
int sdmm_comm_unique_id(void* id /* SDMM_COMM_ID_BYTES */);
int sdmm_comm_init_rccl(const void* id, int nranks, int rank, int device, sdmm_comm** out);
int sdmm_comm_init_host(int nranks, int rank, int device, sdmm_host_allreduce_f64 allreduce,
                        sdmm_host_broadcast broadcast, void* user, sdmm_comm** out);
void sdmm_comm_destroy(sdmm_comm* c);
int sdmm_comm_rank(const sdmm_comm* c);
int sdmm_comm_size(const sdmm_comm* c);
/* in-place SUM of count device doubles over the ranks, on hip_stream */
int sdmm_comm_allreduce_f64(sdmm_comm* c, double* buf, size_t count, void* hip_stream);
int sdmm_em_step_sharded(sdmm_mix* m, sdmm_comm* c, const sdmm_samples* device_shard, int iterations);
int sdmm_em_step_batched_sharded(sdmm_mix* const* mixes, int n_mix, sdmm_comm* c, const sdmm_samples* device_samples,
                                 const int64_t* seg, const int* iterations);
int sdmm_mix_broadcast(sdmm_mix* const* mixes, int n_mix, const int32_t* owner, sdmm_comm* c);

/* Posterior (responsibility) of every sample: resp[n*K + k], device, fp32. */
int sdmm_responsibilities(sdmm_mix* m, const sdmm_samples* device_samples, float* resp);

/* Guided bounce for nq queries (device SoA planes):
 *   c[3]   normalised condition position     u[3]  uniforms (cdf, Box-Muller)
 *   d[3]   sampled world direction (out)     pdf   conditional mixture pdf at d
 *   comp   joint component index used (-1: no valid conditional -> BSDF only) */
int sdmm_guide_batch(const sdmm_mix* m, int64_t nq, const float* const c[3], const float* const u[3],
                     float* const d[3], float* pdf, int32_t* comp);
/* gmmPdf of given directions d (device SoA). */
int sdmm_pdf_batch(const sdmm_mix* m, int64_t nq, const float* const c[3], const float* const d[3],
                   float* pdf);
/* Product sampling with a learned BSDF -- sampleSurface / pdfSurface with
 * sampleProduct (sdmm_proc.cpp:327-392, :474-486): the query's conditional
 * times the learned-BSDF lobes of its material (sdmm::product, absent;
 * restated from jmm MixtureModel::multiply, mixture_model.h:345-370, and
 * MVTN::multiply, multivariate_tangent_normal.h:555-617), then sample / pdf
 * of the product.  Device arrays:
 *   bsdf      B materials x M (<= 64) directional lobes in the LOCAL shading
 *             frame, already oriented for wi (sdmm-lib's rotate_to_wo is the
 *             caller's): weights [B][M], unit means [B][M][3], 2x2 covariances
 *             [B][M][4] in each lobe's tangent frame Coordinates(mean)
 *   material  per query; < 0 (or >= B): no learned BSDF
 *   frame[9]  per-query to-world matrix F, row-major, columns s, t, n
 *             (sdmm_proc.cpp:348-352); lobes go to world as mean F m,
 *             frame to F^T (:353-356)
 *   heuristic (nullable) per query heuristicConditionalWeight (:383-392):
 *             0.3 product, 0.5 plain conditional (no BSDF / empty product),
 *             1 no valid conditional (BSDF only)
 * comp = k * M + j (joint component k, lobe j) for product samples, the
 * joint index for plain-conditional samples, -1 for BSDF only.  Bit-exact
 * against oracle/sdmm_oracle_product.inc in comp; pdf of given directions
 * d with sdmm_pdf_product_batch. */
typedef struct {
    const float* weights;
    const float* means;
    const float* covs;
    int B, M;
    /* per material (nullable): 1 = a diffuse BSDF.  The plugin's diffuse case
     * (sdmm_proc.cpp:335-339) re-centres only slice 0 on the shading normal
     * (set_mean(normal): mean = F's third column, frame Coordinates(mean));
     * slices >= 1 are then used as stored, in world coordinates. */
    const uint8_t* diffuse;
} sdmm_bsdf_table;
int sdmm_guide_product_batch(const sdmm_mix* m, int64_t nq, const float* const c[3], const float* const u[3],
                             const sdmm_bsdf_table* bsdf, const int32_t* material, const float* const frame[9],
                             float* const d[3], float* pdf, int32_t* comp, float* heuristic);
int sdmm_pdf_product_batch(const sdmm_mix* m, int64_t nq, const float* const c[3], const float* const d[3],
                           const sdmm_bsdf_table* bsdf, const int32_t* material, const float* const frame[9],
                           float* pdf, float* heuristic);
/* lower_bound + tie walk of utils.h:104-115 on a caller CDF (device). */
int sdmm_sample_discrete_cdf(const sdmm_mix* m, const float* cdf, int n, const float* u, int64_t nq,
                             int32_t* out);

/* Export the mixture (host outputs, any may be NULL): the canonical MVTN
 * parameters plus every derived array, in the oracle's or_mixture layout. */
typedef struct {
    float* weights;    /* K */
    float* cdf;        /* K */
    float* mean;       /* K*6 */
    float* cov;        /* K*25 */
    float* to;         /* K*9 */
    float* cholL;      /* K*25 */
    float* cholLInv;   /* K*25 */
    float* detInv;     /* K */
    float* muPremult;  /* K*6 */
    float* condCov;    /* K*4 */
    float* margL;      /* K*9 */
    float* margDetInv; /* K */
    float* condL;      /* K*4 */
    float* condLInv;   /* K*4 */
    float* condDetInv; /* K */
    int32_t* valid;    /* K */
    float* normalization; /* 1 */
} sdmm_params_out;
int sdmm_get_params(const sdmm_mix* m, const sdmm_params_out* out);
/* Replace the mixture by (weights, means, covs) host arrays; runs MVTN::set. */
int sdmm_set_params(sdmm_mix* m, const float* weights, const float* means, const float* covs);

/* Stepwise state export/import (checkpointing, tests).  Host buffers:
 * scalars[9] = {heuristicTotalWeight, sgH, normalization, iterationsRun,
 * alpha, niPriorMinusOne, decreasePrior, trainingCutoff, lastStatus};
 * T[K], sgW[K], sgM[5K], sgC[25K] (double); bpriors[25K], bdepth[9K] (float). */
/* iterations_run of n mixtures (StepwiseTangentEM::iterationsRun, the
 * plugin's 2-while-below-4 schedule, volpath_sdmm.cpp:299-302), one wait. */
int sdmm_iterations_run(const sdmm_mix* const* mixes, int n, int* out);
int sdmm_get_state(const sdmm_mix* m, double* scalars, double* T, double* sgW, double* sgM,
                   double* sgC, float* bpriors, float* bdepth);
int sdmm_set_state(sdmm_mix* m, const double* scalars, const double* T, const double* sgW,
                   const double* sgM, const double* sgC, const float* bpriors, const float* bdepth);

/* Spatial tree (the plugin's accelerator: sdmm-lib DMMSTree, sdmm_proc.h:91,
 * absent; restated from jmm SNTree, dmm/jmm/sntree.h:93-299, spatial part).
 * Node ids are the reference's m_nodes indices; child 0 is the upper part of
 * a split.  Construction is host work (as in the reference); find and route
 * run on the device, on the tree's own stream.
 *   sdmm_stree_create          root = the AABB enlarged to a cube (:101-106)
 *   sdmm_stree_split_to_depth  split_to_depth (:195-233); the built plugin
 *                              calls split_to_depth(2) (sdmm/volpath_sdmm.cpp:398)
 *   sdmm_stree_split           split(threshold) (:235-283) on HOST position
 *                              planes p[3] (n points): every leaf, no leaf cap
 *   sdmm_stree_find            STree.find(key) (sdmm_proc.cpp:314, :923, :954)
 *                              for n DEVICE points -> node id or -1 (outside);
 *                              depth first with backtracking (sntree.h:62-83)
 *   sdmm_stree_route           device samples -> device planes `out` (same n,
 *                              same optional planes) in leaf-contiguous order,
 *                              stable within a leaf; seg (host, num_nodes + 1):
 *                              node v's samples are [seg[v], seg[v+1]), points
 *                              outside the tree follow seg[num_nodes].  `seg`
 *                              with the leaves' mixtures feeds
 *                              sdmm_em_step_batched directly. Synchronous. */
typedef struct sdmm_stree sdmm_stree;
int sdmm_stree_create(const float aabb_min[3], const float aabb_max[3], int device, sdmm_stree** out);
void sdmm_stree_destroy(sdmm_stree* t);
int sdmm_stree_split_to_depth(sdmm_stree* t, int max_depth);
int sdmm_stree_split(sdmm_stree* t, const float* const p[3], int64_t n, int threshold);
int sdmm_stree_num_nodes(const sdmm_stree* t);
/* The built plugin's tree calls (sdmm/volpath_sdmm.cpp):
 *   sdmm_stree_leaf_nodes          m_accelerator->leaf_nodes() (:182, :253)
 *   sdmm_stree_split_leaf_recurse  split_leaf_recurse(node_i, threshold)
 *                                  (:184, :257): node's samples p (host planes,
 *                                  the node's stats positions); a leaf holding
 *                                  more than threshold is split and its children
 *                                  recursively; an inner node is left alone
 *   sdmm_stree_split_leaves        the whole splitting block of optimize() /
 *                                  optimize_async_run() (:181-186, :253-260):
 *                                  if leaf_nodes() <= max_leaf_nodes (2048,
 *                                  :529), split_leaf_recurse(i, threshold (4000,
 *                                  :528)) for every node, the samples routed to
 *                                  the leaves by find. */
int sdmm_stree_leaf_nodes(const sdmm_stree* t);
int sdmm_stree_split_leaf_recurse(sdmm_stree* t, int node, const float* const p[3], int64_t n, int threshold);
int sdmm_stree_split_leaves(sdmm_stree* t, const float* const p[3], int64_t n, int threshold, int max_leaf_nodes);
/* split_leaf_recurse for n nodes at once (increasing ids), node i with its
 * own counts[i] positions at planes p[3i..3i+2]: leaves split on parallel host
 * threads, the new nodes numbered exactly as n sequential calls would. */
int sdmm_stree_split_leaf_recurse_many(sdmm_stree* t, int n, const int32_t* nodes, const float* const* p,
                                       const int64_t* counts, int threshold);
/* The same on DEVICE-resident positions: node i's counts[i] positions are
 * entries [starts[i], starts[i] + counts[i]) of the device planes p[0..2].
 * The recursion runs on the device level by level (fp64 sums in the same
 * fixed order as the host split's, the per-node decisions on the host, a
 * stable partition per level); the node arrays are identical to
 * sdmm_stree_split_leaf_recurse_many's.  On the tree's stream; synchronous. */
int sdmm_stree_split_leaf_recurse_device(sdmm_stree* t, int n, const int32_t* nodes, const float* const p[3],
                                         const int64_t* starts, const int64_t* counts, int threshold);
/* aabb[6 * i] = min(3), max(3); child[2 * i] = children (-1, -1 for a leaf);
 * axis[i]: split axis.  Any output may be NULL. */
int sdmm_stree_get_nodes(const sdmm_stree* t, float* aabb, int32_t* child, int32_t* axis);
int sdmm_stree_find(sdmm_stree* t, int64_t n, const float* const p[3], int32_t* node_out);
int sdmm_stree_route(sdmm_stree* t, const sdmm_samples* device_samples, const sdmm_samples* out, int64_t* seg);
/* The tree's HIP stream, taken literally (NULL = the HIP null stream); before
 * any sdmm_stree_set_stream call the tree uses its own non-blocking stream.  A
 * wavefront waits (events) for pending work of the bound mixtures on their own
 * streams, so an EM step enqueued before it is complete when it reads the
 * mixtures; its outputs are ready once the tree's stream is. */
int sdmm_stree_set_stream(sdmm_stree* t, void* hip_stream);
void* sdmm_stree_get_stream(const sdmm_stree* t);

/* Guided wavefront over the tree's leaves -- SDMMRenderer::sampleSurface for
 * a batch of bounces (sdmm_proc.cpp:309-421): per query, node =
 * STree.find(c) (:314), that node's mixture node_mix[node] (host array of
 * sdmm_stree_num_nodes handles; NULL or uninitialised = no trained context,
 * and a query outside the tree: BSDF only, :316-323), then conditional /
 * sample / pdf exactly as sdmm_guide_batch against that mixture (outputs
 * bitwise equal to it; comp -1 and pdf 0 when there is no valid conditional).
 * node_out (nullable): node id per query (-1 outside).  Runs on the tree's
 * stream; the mixtures must have no pending work on other streams.
 * node_mix NULL: use the table bound by sdmm_stree_bind_mixtures (the
 * plugin binds once per training iteration, after the per-leaf EM; the
 * table re-uploads only when a handle/K changes).
 *   sdmm_pdf_wavefront   pdfSurface's gmmPdf of given directions d
 *                        (sdmm_proc.cpp:510-590) per query's own leaf. */
int sdmm_stree_bind_mixtures(sdmm_stree* t, const sdmm_mix* const* node_mix);
int sdmm_guide_wavefront(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
                         const float* const u[3], float* const d[3], float* pdf, int32_t* comp,
                         int32_t* node_out);
int sdmm_pdf_wavefront(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
                       const float* const d[3], float* pdf);
/* One guided bounce of a whole wavefront, sampleSurface + pdfSurface with the
 * plugin's BSDF/guide mixing (sdmm_proc.cpp:383-421, :474-502): the per-query
 * conditional is built ONCE; query q then either samples it (pdf_mode[q] == 0:
 * d, pdf, comp exactly as sdmm_guide_wavefront) or evaluates its gmmPdf at the
 * BSDF-sampled direction dgiven[q] (pdf_mode[q] != 0: pdf exactly as
 * sdmm_pdf_wavefront, d[q] = dgiven[q], comp[q] = -2 when the conditional is
 * valid, -1 when not -- the reference's validConditional, :368-392). */
int sdmm_guide_pdf_wavefront(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
                             const float* const u[3], const float* const dgiven[3], const uint8_t* pdf_mode,
                             float* const d[3], float* pdf, int32_t* comp, int32_t* node_out);

/* Product sampling over the spatial tree's leaves -- sampleSurface /
 * pdfSurface with sampleProduct for a wavefront of bounces (sdmm_proc.cpp:
 * 309-392, :474-502): per query, node = STree.find(c), that node's mixture
 * (node_mix or the table bound by sdmm_stree_bind_mixtures; none: BSDF only,
 * h = 1, comp -1, pdf 0), then exactly sdmm_guide_product_batch /
 * sdmm_pdf_product_batch against it (outputs bitwise equal).
 *   choice (nullable, device): the mixed bounce -- query q's BSDF/guide draw;
 *          with it, dgiven (device, 3 planes: the BSDF-sampled directions) is
 *          required and query q becomes a pdf query at dgiven[q] when
 *          choice[q] <= h[q] (the reference's rRec.nextSample1D() <=
 *          heuristicConditionalWeight, :392, with h 0.3 for a usable product,
 *          0.5 for the plain conditional): d = dgiven, pdf = the used
 *          mixture's pdf there, comp = -2.  Without choice, every query samples.
 *   heuristic (nullable): per query h (0.3 / 0.5 / 1); node_out (nullable). */
int sdmm_guide_product_wavefront(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
                                 const float* const u[3], const float* choice, const float* const dgiven[3],
                                 const sdmm_bsdf_table* bsdf, const int32_t* material, const float* const frame[9],
                                 float* const d[3], float* pdf, int32_t* comp, float* heuristic, int32_t* node_out);
int sdmm_pdf_product_wavefront(sdmm_stree* t, const sdmm_mix* const* node_mix, int64_t nq, const float* const c[3],
                               const float* const d[3], const sdmm_bsdf_table* bsdf, const int32_t* material,
                               const float* const frame[9], float* pdf, float* heuristic);

/* Concurrent guided bounces from many render threads -- the reference's
 * render workers call create_conditional / sample / pdf at once, each with
 * thread_local scratch (sdmm_proc.cpp:1086-1106, volpath_sdmm.cpp:411-507).
 *   sdmm_stree_publish   make the tree's current state readable from guide
 *                        contexts: uploads the nodes and the mixture table
 *                        (node_mix, or the bound one when NULL) and waits for
 *                        the bound mixtures' pending work.  Call it from one
 *                        thread after any change to the tree, the binding or
 *                        the bound mixtures (once per render pass); a later
 *                        change un-publishes the tree (context calls then fail
 *                        with SDMM_E_STATE).
 *   sdmm_guide_ctx_*     one render worker's context: its own HIP stream
 *                        (hip_stream NULL: a new non-blocking stream the
 *                        context owns) and its own guided-batch / product
 *                        scratch.  Contexts of one tree run at once from
 *                        different host threads with no lock; calls on ONE
 *                        context must be serialised by the caller.
 *   sdmm_ctx_guide_pdf_wavefront / sdmm_ctx_guide_product_wavefront
 *                        sdmm_guide_pdf_wavefront / sdmm_guide_product_wavefront
 *                        against the published tree on the context's stream
 *                        (outputs bitwise equal; asynchronous -- synchronise
 *                        the context's stream before reading them). */
typedef struct sdmm_guide_ctx sdmm_guide_ctx;
int sdmm_stree_publish(sdmm_stree* t, const sdmm_mix* const* node_mix);
int sdmm_guide_ctx_create(sdmm_stree* t, void* hip_stream, sdmm_guide_ctx** out);
void sdmm_guide_ctx_destroy(sdmm_guide_ctx* g);
void* sdmm_guide_ctx_stream(const sdmm_guide_ctx* g);
int sdmm_ctx_guide_pdf_wavefront(sdmm_guide_ctx* g, int64_t nq, const float* const c[3], const float* const u[3],
                                 const float* const dgiven[3], const uint8_t* pdf_mode, float* const d[3], float* pdf,
                                 int32_t* comp, int32_t* node_out);
int sdmm_ctx_guide_product_wavefront(sdmm_guide_ctx* g, int64_t nq, const float* const c[3], const float* const u[3],
                                     const float* choice, const float* const dgiven[3], const sdmm_bsdf_table* bsdf,
                                     const int32_t* material, const float* const frame[9], float* const d[3],
                                     float* pdf, int32_t* comp, float* heuristic, int32_t* node_out);
/* Several render workers' guided bounces served as ONE wavefront (round 6):
 * the requests' queries, in request order, go through a single
 * sdmm_ctx_guide_pdf_wavefront on the context -- each query's outputs are
 * bitwise those of a call on its own request (queries are independent) --
 * with the copies done here: per request one strided H2D of its nine query
 * planes and one of its mode bytes, one strided D2H of its four output planes
 * and one of its components.  Synchronous (the context's stream is
 * synchronised before returning).  Host buffers must be pinned
 * (hipHostMalloc / hipHostRegister): checked, SDMM_E_INVALID otherwise.  The
 * C++ mirror's sdmm_amd::GuideBatcher gathers concurrent workers' requests
 * into these calls.
 *   in   : planes c0 c1 c2 u0 u1 u2 dgiven0 dgiven1 dgiven2 (as
 *          sdmm_guide_pdf_wavefront), plane p at in + p * in_stride
 *   mode : n bytes (pdf_mode)
 *   out  : planes d0 d1 d2 pdf, plane p at out + p * out_stride
 *   comp : n int32 */
typedef struct sdmm_guide_host_req {
    int64_t n;
    const float* in;
    int64_t in_stride;
    const uint8_t* mode;
    float* out;
    int64_t out_stride;
    int32_t* comp;
} sdmm_guide_host_req;
int sdmm_ctx_guide_pdf_host_batch(sdmm_guide_ctx* g, int nreq, const sdmm_guide_host_req* reqs);
/* Page-locked host memory for such requests (hipHostMalloc / hipHostFree on
 * the library's side, so that host code needs no HIP headers). */
int sdmm_pinned_alloc(size_t bytes, void** out);
void sdmm_pinned_free(void* p);
/* Checkpoints (.asdmm, JSON; schema in DESIGN.md section 9).
 *   sdmm_save_json      the accelerator: sdmm::save_json(m_accelerator, path),
 *                       volpath_sdmm.cpp:117-126 (model_%05i.asdmm, once per
 *                       render iteration, :441).  Writes the tree's node table
 *                       and, for every node with a non-NULL node_mix entry
 *                       (node_mix may be NULL: tree only), that mixture's
 *                       canonical + derived arrays and its stepwise-EM state.
 *   sdmm_load_json      the inverse.  tree_out NULL: size query, only
 *                       *num_nodes_out is set.  Otherwise node_mix_out (cap >=
 *                       num_nodes) receives one new handle per saved mixture and
 *                       NULL elsewhere; restored mixtures are bitwise the saved
 *                       ones (guide outputs, later EM steps).  A malformed file
 *                       creates nothing and returns SDMM_E_INVALID.
 *   sdmm_mix_save_json / sdmm_mix_load_json   one mixture: jmm
 *                       MixtureModel::save/load (mixture_model.h:315-326).
 *   sdmm_get_em_params  the constructor arguments the handle was created with.
 *   sdmm_restore_params exact inverse of sdmm_get_params (every array required;
 *                       no MVTN::set re-derivation).
 *   sdmm_stree_set_nodes replace the node table (as sdmm_stree_get_nodes
 *                       returns it; children must follow their parent). */
int sdmm_save_json(const sdmm_stree* t, const sdmm_mix* const* node_mix, const char* path);
int sdmm_load_json(const char* path, int device, sdmm_stree** tree_out, sdmm_mix** node_mix_out, int cap,
                   int* num_nodes_out);
int sdmm_mix_save_json(const sdmm_mix* m, const char* path);
int sdmm_mix_load_json(const char* path, int device, sdmm_mix** out);
int sdmm_get_em_params(const sdmm_mix* m, sdmm_em_params* p);
/* A new handle holding a copy of m's mixture and stepwise EM state (device to
 * device, on m's stream; the new handle uses m's stream) -- a split leaf's
 * children start from their parent's distribution and optimizer (jmm
 * SNTree::createChildNode, sntree.h:172-205). */
int sdmm_clone(const sdmm_mix* m, sdmm_mix** out);
/* sdmm_clone of n handles of one K into one slab (on src[0]'s stream, or on
 * hip_stream: the new handles then use it). */
int sdmm_clone_many(const sdmm_mix* const* src, int n, sdmm_mix** out);
int sdmm_clone_many_on_stream(const sdmm_mix* const* src, int n, void* hip_stream, sdmm_mix** out);
/* dst[i] := src[i] (mixture + EM state), one kernel on dst[0]'s stream after
 * the sources' pending work -- sdmm::prepare(conditioner, sdmm) of the async
 * update (volpath_sdmm.cpp:227-242) when conditioners are separate handles. */
int sdmm_copy_many(const sdmm_mix* const* src, sdmm_mix* const* dst, int n);
int sdmm_restore_params(sdmm_mix* m, const sdmm_params_out* in);
int sdmm_stree_set_nodes(sdmm_stree* t, int n, const float* aabb, const int32_t* child, const int32_t* axis);

/* ---- Guided path tracing on the device (SDMMRenderer::Li) ----------------
 * An analytic scene of parallelograms (Mitsuba rectangles; a cube is six) with
 * diffuse BSDFs and one-sided area emitters, rendered by a wavefront path
 * tracer whose every bounce goes through sdmm_guide_pdf_wavefront -- the
 * plugin's per-bounce sampleSurface / pdfSurface (sdmm_proc.cpp:275-590,
 * :592-871) on the device.  The Cornell Box of the test suite
 * (test-suite/scenes/cornell-box/cornell-box.xml:75-143) is this kind of
 * scene (sdmm-mitsuba_amd/scenes.py).
 *
 *   sdmm_scene_create   quads: 9 floats each (corner, edge1, edge2, world);
 *                       normal = normalize(edge1 x edge2), negated where
 *                       flip_normals[q] (nullable); bsdf[q] indexes
 *                       reflectance (3 per BSDF); emitter[q] (nullable, -1 =
 *                       none) indexes radiance (3 per emitter, Le on the
 *                       normal side); camera_to_world row major 4x4 (Mitsuba's
 *                       toWorld, camera looks along +z), fov along x.
 *   sdmm_scene_normalization  render() (volpath_sdmm.cpp:375-393): the scene
 *                       AABB without the camera gives scene_min and
 *                       spatial_norm = its largest extent (scene_norm.json),
 *                       the tree box = [0, extent / norm] -+ 1e-5 (getAABB).
 *   sdmm_li_render      spp samples for pixels [pixel_begin, pixel_end) (row
 *                       major), one path per sample; image (device, 3 planes
 *                       of width * height floats) receives each pixel's mean
 *                       radiance, image_sqr (nullable) the mean of the squared
 *                       samples (the reference's m_blockSqr, sdmm_wr.cpp:144).  guided = 0: BSDF sampling only (iteration
 *                       0, :311-323); otherwise every bounce queries the
 *                       leaves' mixtures (node_mix, or the table bound to t)
 *                       with the BSDF/guide choice of probability
 *                       bsdf_fraction (0.5, :383).  Conditions are
 *                       (p - scene_min) / spatial_norm (createCondition,
 *                       :263-273).  Runs on the tree's stream.  The saved
 *                       vertices (Li's Vertex records, :606-637, :815-846)
 *                       stay in the scene's buffers; *vertices_out (nullable)
 *                       points at them until the next sdmm_li_render.
 * Random numbers are counter based: sample (path, stream, dimension) of a
 * path are fixed, whatever runs beside it (render_device.h). */
typedef struct sdmm_scene sdmm_scene;
/* A glossy material's learned BSDF: the reference's BSDF::SDMM4
 * (include/mitsuba/render/bsdf.h:310-314), a mixture over (theta_i, alpha) x
 * direction loaded per material by sdmm::load_json (roughconductor.cpp:
 * 230-245).  M <= 8 components; host arrays
 *   weights[M]
 *   means[M][5]  (theta, alpha, x, y, z): the condition's mean and the unit
 *                direction in the canonical local frame (z = normal, wi at
 *                azimuth 0)
 *   covs[M][16]  row major over the tangent coordinates (theta, alpha, t1,
 *                t2), t at the component's direction in its
 *                Coordinates(mean) frame (sdmm_bsdf_table's convention).
 * getDMM (roughconductor.cpp:182-194) conditions it on (theta_i =
 * acos(min(1, cos theta_i)), alpha) with create_conditional_pruned(..., 2):
 * this library's reading of that sdmm-lib call (absent from the snapshot) is
 * in sdmm-mitsuba_amd/csrc/learned_bsdf.h and DESIGN.md section 10. */
typedef struct sdmm_learned_bsdf4 {
    int M;
    const float* weights;
    const float* means;
    const float* covs;
} sdmm_learned_bsdf4;
/* getDMM + rotate_to_wo on the host for the local incident direction
 * wi_local (wi_local[2] > 0; the plugin's learnedRow): *n_out (<= keep)
 * lobes weights[n], means[n][3] (local, unit), covs[n][4] (2x2 in each
 * mean's Coordinates frame); *n_out = 0: no valid conditional.  The device
 * render forms the same lobes bitwise. */
int sdmm_learned4_conditional(const sdmm_learned_bsdf4* m, float alpha, const float wi_local[3], int keep,
                              int* n_out, float* weights, float* means, float* covs);
/* The same for nq local incident directions on the device (wi_local: 3
 * device planes; outputs device: weights[nq][keep], means[nq][keep][3],
 * covs[nq][keep][4], n_out[nq] the lobes per query, unused lobes weight 0),
 * asynchronous on hip_stream -- a plugin's whole wavefront of getDMM calls
 * in one launch. */
int sdmm_learned4_conditional_device(const sdmm_learned_bsdf4* m, float alpha, int64_t nq,
                                     const float* const wi_local[3], int keep, float* weights, float* means,
                                     float* covs, int32_t* n_out, void* hip_stream);
/* sdmm::load_json / save_json of a learned BSDF (the material's .sdmm file,
 * roughconductor.cpp:230-245) in this library's JSON form (DESIGN.md section
 * 9): load with cap 0 is a size query (*M_out only); otherwise the arrays
 * hold cap components. */
int sdmm_learned4_save_json(const sdmm_learned_bsdf4* m, const char* path);
int sdmm_learned4_load_json(const char* path, int cap, int* M_out, float* weights, float* means, float* covs);
typedef struct {
    int n_quads;
    const float* quads;
    const int32_t* flip_normals;
    const int32_t* bsdf;
    int n_bsdfs;
    const float* reflectance;
    const int32_t* emitter;
    int n_emitters;
    const float* radiance;
    float camera_to_world[16];
    float fov_x_deg;
    float near_clip;
    int width, height;
    /* nullable (every BSDF diffuse): 8 floats per BSDF -- [0] kind (0
     * diffuse, 1 smooth plastic: bsdfs/plastic.cpp, its diffuseReflectance in
     * `reflectance`), [1..3] specularReflectance, [4] eta = intIOR / extIOR,
     * [5] 1 / eta^2, [6] fdrInt (the internal diffuse Fresnel reflectance,
     * fresnelDiffuseReflectance(1 / eta)), [7] the specular sampling weight
     * sAvg / (dAvg + sAvg) (plastic.cpp:188-196).  A plastic bounce queries
     * the guide like any BSDF with a smooth lobe; a delta lobe chosen by the
     * BSDF sample returns weight / h with pdf * h and saves no vertex
     * (sdmm_proc.cpp:297, :383-409, :764).  Kind 2, rough conductor
     * (bsdfs/roughconductor.cpp; `reflectance` unused): [1..3]
     * specularReflectance, [4] eta, [5] k (a gray conductor), [6] the
     * Beckmann alpha (isotropic, sampleVisible = false), [7] unused. */
    const float* bsdf_params;
    /* nullable: n_bsdfs entries (appended in round 6) -- a rough conductor's
     * learned BSDF, the material's SDMM4 (roughconductor.cpp:182-194,
     * :230-245); M = 0 (or the array NULL): none, so getDMM fails and the
     * product falls back to the plain conditional (sdmm_proc.cpp:327-392).
     * Only rough conductors read theirs. */
    const struct sdmm_learned_bsdf4* learned_models;
} sdmm_scene_desc;
/* The descriptor has grown across ABI revisions (bsdf_params was appended):
 * zero-initialise it (`sdmm_scene_desc d = {0};` / `memset`) before filling
 * the fields you use, so an older caller's unset trailing pointer is NULL --
 * sdmm_scene_create reads every field. */
typedef struct {
    int spp;
    int max_depth;            /* maxDepth (:649, :684), -1 = unbounded (capped by the vertex slots) */
    int rr_depth;             /* rrDepth (:858) */
    int guided;
    float bsdf_fraction;      /* heuristicConditionalWeight (0.5) */
    int saved_vertices;       /* vertex slots per path (>= max_depth - 1; the reference's array holds 10) */
    uint64_t seed;
    int64_t pixel_begin, pixel_end;
    /* sampleProduct (volpath_sdmm.cpp:60, sdmm_proc.cpp:327-392): guided
     * bounces sample the product of the leaf's conditional with the hit
     * material's learned BSDF (learned_bsdf row = the quad's bsdf index; for
     * a diffuse BSDF set diffuse[b], the plugin's slice-0 rule) through
     * sdmm_guide_product_wavefront, with h = 0.3 (0.5 when the product is
     * unusable) and the BSDF/guide choice taken against that h.  A rough
     * conductor's row is not read: each bounce conditions the conductor's
     * learned model (sdmm_scene_desc.learned_models: getDMM on theta_i and
     * alpha, pruned to 2 lobes -- none or no valid conditional: the plain
     * conditional) then rotate_to_wo(wi) and the shading frame to world,
     * sdmm_proc.cpp:340-355; the component index is then k * max(M, 2) + j
     * with a conductor in the scene.  0: the plain
     * conditional with bsdf_fraction.  (bsdfOnly never trains, :416, so it
     * is the guided = 0 render; its learned-BSDF branch, :331/:384/:410, is
     * unreachable in the reference.) */
    int sample_product;
    sdmm_bsdf_table learned_bsdf;   /* device arrays */
} sdmm_li_params;
/* Vertex records of the last render (device): field f of vertex v of path p
 * at rec[(f * max_vertices + v) * n_paths + p]; f: 0-2 weight (RGB), 3-5
 * throughput, 6 clamped sampling pdf, 7-12 point (condition, world
 * direction), 13-15 normal; nv[p] vertices per path; path p's global index
 * (the RNG's path counter) is path0 + p. */
typedef struct {
    int64_t n_paths;
    int max_vertices;
    int64_t path0;
    const float* rec;
    const int32_t* nv;
} sdmm_path_vertices;
typedef struct {
    int64_t paths;           /* paths started (pixels x spp) */
    int64_t segments;        /* bounce rays traced after the camera rays (a delta lobe's saves no vertex) */
    int64_t guided_queries;  /* live bounces that queried the guide (compacted wavefront sizes summed) */
    int64_t fallback_queries;   /* of those, served by the full-K path (the candidate list overflowed) */
} sdmm_li_stats;
int sdmm_scene_create(const sdmm_scene_desc* desc, int device, sdmm_scene** out);
void sdmm_scene_destroy(sdmm_scene* s);
int sdmm_scene_normalization(const sdmm_scene* s, float scene_min[3], float* spatial_norm, float tree_min[3],
                             float tree_max[3]);
int sdmm_li_render(sdmm_scene* s, sdmm_stree* t, const sdmm_mix* const* node_mix, const sdmm_li_params* p,
                   float* image, float* image_sqr, sdmm_path_vertices* vertices_out, sdmm_li_stats* stats);

/* Training-data producer: the tail of Li (sdmm_proc.cpp:876-965) for a batch
 * of paths' saved vertices.  Per path, vertices nv-1 down to
 * max(nv - saved_per_path, 0): the vertex's leaf (STree.find with its box,
 * :921-930) gets (point, normal, average weight) plus a stats entry when the
 * average is finite (push_back_data, :880-914); then 1 (last vertex) + 1
 * (average > 1000) jittered copies go to the leaf at point + (u - 1/2) x leaf
 * diagonal, a draw outside the tree or in the same leaf retried while fewer
 * than 8 draws failed (:932-964); u from stream 1024 + vertex of the path's
 * counter RNG under `seed`.  Output (device planes, capacity records): the
 * records in leaf order, a leaf's records in (path, push) order; node = leaf
 * id, source = p * max_vertices + v, stats = 1 for the vertex's own leaf.
 * *n_out = number of records (also when it exceeds capacity: then nothing is
 * written and SDMM_E_INVALID is returned; out NULL: count only); seg (host, nullable,
 * num_nodes + 1): leaf v's records are [seg[v], seg[v+1]).  lost (nullable):
 * vertices outside the tree (the reference throws).  Synchronous. */
typedef struct {
    float* x[6];
    float* normal[3];        /* nullable (all three) */
    float* w;
    uint8_t* stats;          /* nullable */
    int32_t* node;           /* nullable */
    int64_t* source;         /* nullable */
    int64_t capacity;
} sdmm_training_out;
int sdmm_push_training(sdmm_stree* t, const sdmm_path_vertices* v, int saved_per_path, uint64_t seed,
                       const sdmm_training_out* out, int64_t* n_out, int64_t* seg, int64_t* lost);

/* ---- The plugin's guiding model (SDMMVolumetricPathTracer) ----------------
 * volpath_sdmm.cpp:132-312, :411-507 on the device: the accelerator tree
 * (split_to_depth(split_depth) at creation, :398), one SDMM + EM state per
 * trained leaf, the leaves' training data and the per-iteration schedule.
 *   sdmm_guiding_push      Li's tail for a render pass (sdmm_push_training):
 *                          records appended to the leaves' data, own-leaf
 *                          positions to their stats (:894-902)
 *   sdmm_guiding_optimize  optimize() (:244-312): split every leaf by its stats
 *                          (split_leaf_recurse(threshold) under the leaf cap,
 *                          :253-259; a split leaf's data, stats and mixture go
 *                          to its new leaves -- jmm sntree.h:172-205), then per
 *                          leaf canBeOptimized (:140-149, with m_totalSpp of the
 *                          previous passes), initializeSDMMContext on first use
 *                          (K/8 positions = the leaf's first records, spatial
 *                          distance 3 hmax(diagonal) / (K/8), :132-138, :291),
 *                          2 EM iterations while iterations_run < 4 else 1
 *                          (:299-305) as ONE batched launch, the optimised
 *                          leaves' data cleared (:308-309); the trained leaves
 *                          are bound to the tree for the next pass.  spp: the
 *                          pass's samples per pixel (m_totalSpp += spp after).
 *   sdmm_guiding_iteration one pass of render()'s loop (:411-507): sdmm_li_render
 *                          (guided once a leaf is trained, :311-316), then
 *                          push + optimize when train (m_still_training).
 * Everything runs on the model's stream (= its tree's); calls return when
 * the host-side state is updated. */
typedef struct sdmm_guiding sdmm_guiding;
typedef struct {
    int K;                  /* components per leaf (16, SDMMProcess::NComponents) */
    int split_depth;        /* 2 */
    int split_threshold;    /* 4000 */
    int max_leaf_nodes;     /* 2048 */
    int saved_per_path;     /* 8 */
    float depth_prior;      /* 0.01 (sdmm-lib initialize is absent: jmm uniformHemisphereInit's) */
    uint64_t init_seed;     /* leaf v's hemisphere init seed = init_seed + v */
    int optimize_async;     /* optimizeAsync (volpath_sdmm.cpp:65, :180-242): one EM step per leaf (0.1 x
                               hmax(diagonal) at init) on the model's EM stream, overlapping the next pass;
                               renders use each leaf's conditioner, updated after the pass (sdmm_guiding_update) */
} sdmm_guiding_config;
typedef struct {
    int leaves;             /* leaf_nodes() after the split */
    int optimized;          /* leaves stepped this call */
    int64_t records;        /* pool records before the optimised leaves' were dropped */
} sdmm_guiding_stats;
void sdmm_guiding_config_default(sdmm_guiding_config* c);
int sdmm_guiding_create(const float tree_min[3], const float tree_max[3], const sdmm_guiding_config* cfg,
                        int device, sdmm_guiding** out);
void sdmm_guiding_destroy(sdmm_guiding* g);
sdmm_stree* sdmm_guiding_tree(sdmm_guiding* g);
int sdmm_guiding_node_mixtures(const sdmm_guiding* g, const sdmm_mix** out, int cap);
int sdmm_guiding_trained(const sdmm_guiding* g);
int sdmm_guiding_push(sdmm_guiding* g, const sdmm_path_vertices* v, uint64_t seed);
int sdmm_guiding_optimize(sdmm_guiding* g, int spp, sdmm_guiding_stats* out);
/* async: optimize_async_wait_and_update (:227-242) -- wait for the running EM,
 * copy each stepped leaf's mixture into its conditioner; no-op otherwise. */
int sdmm_guiding_update(sdmm_guiding* g);
int sdmm_guiding_iteration(sdmm_guiding* g, sdmm_scene* scene, const sdmm_li_params* p, uint64_t push_seed,
                           int train, float* image, float* image_sqr, sdmm_li_stats* li_stats,
                           sdmm_guiding_stats* out);

/* SDMMWorkResult::dumpIndividual (sdmm_wr.cpp:115-146): an RGB float OpenEXR
 * file (uncompressed scanlines, channels B G R, attributes spp / iteration
 * (int) and time (float) as Bitmap::setMetadata writes them) from HOST planes
 * rgb[3][height][width].  The plugin writes iteration%05i.exr (the pass's
 * mean) and iteration_sqr%05i.exr (its mean of squares) per render pass. */
int sdmm_write_exr(const char* path, int width, int height, const float* rgb, int spp, int iteration, float time);

const char* sdmm_last_error(void);
int sdmm_abi_version(void);

/* Library teardown (no reference counterpart: sdmm-lib holds no device state
 * outside its contexts).  Frees the per-(device, stream) scratch pool that
 * init / clone / k-means++ calls keep between calls.  Call only when no other
 * thread is inside the library; later calls regrow the pool on demand. */
int sdmm_release_cached_scratch(void);

#ifdef __cplusplus
}
#endif
#endif /* SDMM_GPU_H */
