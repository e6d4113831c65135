/*
 * sdmm_oracle_train.c -- CPU ORACLE (test infrastructure only): the host-routed
 * reference of the training-data producer, the tail of SDMMRenderer::Li
 * (mitsuba/src/integrators/sdmm/sdmm_proc.cpp:876-965), for the checker of
 * sdmm_push_training.  Restated from the reference as text:
 *
 *   :876-878   no saved vertex -> nothing
 *   :917-918   vertices d = depth-1 down to max(depth - savedSamplesPerPath, 0)
 *   :919-930   key = the vertex's position; find(key, aabb) (the leaf and its
 *              box; the reference throws when there is none: counted in *lost)
 *   :880-914   push_back_data: average RGB weight (Spectrum::average, sum *
 *              (1/3)); pushed (point, normal, average) only if valid (jmm
 *              isValidSample: finite, opt/stepwise_tangent.h:445-460); the
 *              vertex's own leaf also gets a stats entry
 *   :932-935   nJitters = (d >= depth-1) + (average > 1000)
 *   :937-964   per jitter a draw of 3 uniforms: position + (u - 1/2) x leaf
 *              diagonal; no leaf or the same leaf (equal box min) -> ++attempts,
 *              the jitter retried while attempts < 8; else pushed there
 *
 * The uniforms are the library's counter-based numbers (render_device.h),
 * restated below: draw k of vertex d of path p = (u(3k), u(3k+1), u(3k+2)) on
 * stream 1024 + d.  Records are emitted in (path, push) order; the checker
 * sorts them stably by leaf, which is the order sdmm_push_training returns.
 */
#include <math.h>
#include <stdint.h>

int or_stree_find(const float* mn, const float* mx, const int* child, const float p[3]);

static uint64_t rng_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

float or_rng_uniform(uint64_t seed, uint64_t path, uint32_t stream, uint32_t dim) {
    const uint64_t k = rng_mix(rng_mix(seed ^ (path * 0xD1B54A32D192ED03ull)) + (((uint64_t)stream << 16) | dim));
    return (float)(uint32_t)(k >> 40) * (1.0f / 16777216.0f);
}

/* rec: field f of vertex v of path p at rec[(f * V + v) * P + p] (fields:
 * 0-2 weight, 3-5 throughput, 6 pdf, 7-12 point, 13-15 normal).  Writes at
 * most cap records; returns the number of records. */
int64_t or_push_training(const float* mn, const float* mx, const int* child, const float* rec, const int32_t* nv,
                         int64_t P, int V, int64_t path0, int saved, uint64_t seed, int32_t* node,
                         int64_t* source, uint8_t* stats, float* w, int64_t cap, int64_t* lost) {
#define VREC(f, v, p) rec[((int64_t)(f) * V + (v)) * P + (p)]
    int64_t n = 0;
    *lost = 0;
    for (int64_t p = 0; p < P; ++p) {
        const int depth = nv[p];
        const int first = depth - saved > 0 ? depth - saved : 0;
        for (int d = depth - 1; d >= first; --d) {
            const float pos[3] = {VREC(7, d, p), VREC(8, d, p), VREC(9, d, p)};
            const int leaf = or_stree_find(mn, mx, child, pos);
            if (leaf < 0) {
                ++*lost;
                continue;
            }
            const float* bmn = mn + 3 * leaf;
            const float* bmx = mx + 3 * leaf;
            const float avg = (VREC(0, d, p) + VREC(1, d, p) + VREC(2, d, p)) * (1.0f / 3.0f);
            const int ok = isfinite(avg);
            const int64_t src = p * V + d;
            if (ok) {
                if (n < cap) { node[n] = leaf; source[n] = src; stats[n] = 1; w[n] = avg; }
                ++n;
            }
            const int jitters = (d >= depth - 1 ? 1 : 0) + (avg > 1000.0f ? 1 : 0);
            int attempts = 0, draw = 0;
            const float diag[3] = {bmx[0] - bmn[0], bmx[1] - bmn[1], bmx[2] - bmn[2]};
            for (int j = 0; j < jitters; ++j) {
                float jp[3];
                for (int a = 0; a < 3; ++a) {
                    const float off = (or_rng_uniform(seed, (uint64_t)(path0 + p), 1024u + (uint32_t)d,
                                                      (uint32_t)(3 * draw + a)) - 0.5f) * diag[a];
                    jp[a] = pos[a] + off;
                }
                ++draw;
                const int nb = or_stree_find(mn, mx, child, jp);
                int same = nb < 0;
                if (!same)
                    same = mn[3 * nb] == bmn[0] && mn[3 * nb + 1] == bmn[1] && mn[3 * nb + 2] == bmn[2];
                if (same) {
                    ++attempts;
                    if (attempts < 8) --j;
                    continue;
                }
                if (ok) {
                    if (n < cap) { node[n] = nb; source[n] = src; stats[n] = 0; w[n] = avg; }
                    ++n;
                }
            }
        }
    }
    return n;
#undef VREC
}
