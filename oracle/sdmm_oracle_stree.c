/*
 * sdmm_oracle_stree.c -- CPU ORACLE (test infrastructure only): the spatial
 * tree of the plugin's guiding accelerator, restated from jmm SNTree
 * (mitsuba/src/integrators/dmm/jmm/sntree.h:93-299).  sdmm-lib's DMMSTree,
 * which the plugin actually instantiates (sdmm_proc.h:91), is absent from
 * the snapshot, so parity with it is unpinned; SNTree is its readable
 * counterpart.  Spatial part only (one value per leaf, no NGridNode normal
 * cells).  Checker for sdmm_stree_* in sdmm-mitsuba_amd (device find/route
 * and the host-built tree).
 *
 *   SNTree ctor (:101-106)        root = AABB enlarged to a cube
 *   SNTreeNode::find (:62-83)     inclusive box test (Eigen AlignedBox), leaf
 *                                 returns, inner node tries child 0 then 1
 *   createChildNode (:172-192)    child 0 = UPPER part (min += s * diag),
 *                                 child 1 = lower (max -= (1 - s) * diag),
 *                                 child axis = (axis + 1) % 3; a child gets
 *                                 every parent sample its box contains
 *   split_to_depth (:195-233)     midpoint splits, depth advances after z
 *   split / getSplitLocation      leaf with > threshold samples: split at the
 *   (:141-170, :235-283)          mean along the max-variance axis (strict >),
 *                                 children recursively, child 0 first
 * Stated choices (the reference leaves them open): mean/variance summed in
 * double in sample order; a split at s <= 0, s >= 1 or one that leaves all
 * samples in a child is skipped (the reference would recurse forever).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    float* mn;
    float* mx;
    int* axis;
    int* child;
    int n, cap;
} st_tree;

static int st_push(st_tree* t, const float mn[3], const float mx[3], int axis) {
    if (t->n >= t->cap) return -1;
    const int i = t->n++;
    for (int a = 0; a < 3; ++a) { t->mn[3 * i + a] = mn[a]; t->mx[3 * i + a] = mx[a]; }
    t->axis[i] = axis;
    t->child[2 * i] = t->child[2 * i + 1] = -1;
    return i;
}

static int st_in(const st_tree* t, int i, float x, float y, float z) {
    const float* a = t->mn + 3 * i;
    const float* b = t->mx + 3 * i;
    return a[0] <= x && x <= b[0] && a[1] <= y && y <= b[1] && a[2] <= z && z <= b[2];
}

/* child c of node i split along axis `ax` at s (createChildNode) */
static void st_child_box(const st_tree* t, int i, int ax, int c, float s, float mn[3], float mx[3]) {
    for (int a = 0; a < 3; ++a) { mn[a] = t->mn[3 * i + a]; mx[a] = t->mx[3 * i + a]; }
    const float diag = t->mx[3 * i + ax] - t->mn[3 * i + ax];
    if (c == 0) {
        const float d = s * diag;
        mn[ax] = t->mn[3 * i + ax] + d;
    } else {
        const float d = (1.0f - s) * diag;
        mx[ax] = t->mx[3 * i + ax] - d;
    }
}

static int st_depth(st_tree* t, int i, int depth, int max_depth) {
    const int next = (t->axis[i] == 2) ? depth + 1 : depth;
    if (t->child[2 * i] >= 0) {
        for (int c = 0; c < 2; ++c)
            if (st_depth(t, t->child[2 * i + c], next, max_depth)) return -1;
        return 0;
    }
    if (depth < max_depth) {
        for (int c = 0; c < 2; ++c) {
            float mn[3], mx[3];
            st_child_box(t, i, t->axis[i], c, 0.5f, mn, mx);
            const int id = st_push(t, mn, mx, (t->axis[i] + 1) % 3);
            if (id < 0) return -1;
            t->child[2 * i + c] = id;
        }
        for (int c = 0; c < 2; ++c)
            if (st_depth(t, t->child[2 * i + c], next, max_depth)) return -1;
    }
    return 0;
}

/* SNTreeNode::find (jmm/sntree.h:62-83): recursive, child 0 before child 1,
 * entering only nodes whose box contains the point; a subtree without a leaf
 * box holding the point returns nullptr and the search goes on (backtracks). */
static int st_find_rec(const st_tree* t, int i, const float p[3]) {
    if (!st_in(t, i, p[0], p[1], p[2])) return -1;
    if (t->child[2 * i] < 0) return i;
    for (int c = 0; c < 2; ++c) {
        const int f = st_find_rec(t, t->child[2 * i + c], p);
        if (f >= 0) return f;
    }
    return -1;
}

int or_stree_find(const float* mn, const float* mx, const int* child, const float p[3]) {
    st_tree t = {(float*)mn, (float*)mx, NULL, (int*)child, 0, 0};
    return st_find_rec(&t, 0, p);
}

/* The split's fp64 sums over a node's samples in the library's one fixed
 * order (sdmm_api.cpp split_sums_host, stree.hip split_sums_kernel): chunks
 * of 4096 consecutive samples; in a chunk lane t of 256 sums samples t,
 * t + 256, ... in order (products separately rounded); the lane sums fold
 * pairwise (stride 128 .. 1); the chunk sums are added in chunk order.  jmm
 * itself sums in float in an unspecified (Eigen) order. */
static void st_sums(const int64_t* idx, int64_t n, const float* px, const float* py, const float* pz,
                    double mean[3], double sq[3]) {
    static const int64_t C = 4096;
    double lane[256][6];
    for (int a = 0; a < 3; ++a) { mean[a] = 0.0; sq[a] = 0.0; }
    for (int64_t c0 = 0; c0 < n; c0 += C) {
        const int64_t len = (n - c0 < C) ? n - c0 : C;
        memset(lane, 0, sizeof(lane));
        for (int64_t j = 0; j < len; ++j) {
            double* a = lane[j % 256];
            const int64_t i = idx[c0 + j];
            const double p[3] = {px[i], py[i], pz[i]};
            for (int k = 0; k < 3; ++k) {
                a[k] = a[k] + p[k];
                a[3 + k] = a[3 + k] + p[k] * p[k];
            }
        }
        for (int st = 128; st > 0; st >>= 1)
            for (int tt = 0; tt < st; ++tt)
                for (int k = 0; k < 6; ++k) lane[tt][k] = lane[tt][k] + lane[tt + st][k];
        for (int k = 0; k < 3; ++k) {
            mean[k] = mean[k] + lane[0][k];
            sq[k] = sq[k] + lane[0][3 + k];
        }
    }
}

static int st_split(st_tree* t, int i, int64_t* idx, int64_t n, const float* px, const float* py,
                    const float* pz, int threshold) {
    if (n <= threshold) return 0;
    double mean[3], sq[3];
    st_sums(idx, n, px, py, pz, mean, sq);
    float m[3], var[3];
    for (int a = 0; a < 3; ++a) {
        const double mu = mean[a] / (double)n;
        m[a] = (float)mu;
        var[a] = (float)(sq[a] / (double)n - mu * mu);
    }
    int ax = 0;
    for (int a = 1; a < 3; ++a)
        if (var[a] > var[ax]) ax = a;
    const float s = (m[ax] - t->mn[3 * i + ax]) / (t->mx[3 * i + ax] - t->mn[3 * i + ax]);
    if (!(s > 0.0f && s < 1.0f)) return 0;
    float cmn[2][3], cmx[2][3];
    int64_t* sub[2];
    int64_t cnt[2] = {0, 0};
    for (int c = 0; c < 2; ++c) {
        st_child_box(t, i, ax, c, s, cmn[c], cmx[c]);
        sub[c] = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
        for (int64_t j = 0; j < n; ++j) {
            const float x = px[idx[j]], y = py[idx[j]], z = pz[idx[j]];
            if (cmn[c][0] <= x && x <= cmx[c][0] && cmn[c][1] <= y && y <= cmx[c][1] && cmn[c][2] <= z &&
                z <= cmx[c][2])
                sub[c][cnt[c]++] = idx[j];
        }
    }
    int rc = 0;
    if (cnt[0] == n || cnt[1] == n) goto done;   /* would not separate the samples */
    t->axis[i] = ax;
    for (int c = 0; c < 2; ++c) {
        const int id = st_push(t, cmn[c], cmx[c], (ax + 1) % 3);
        if (id < 0) { rc = -1; goto done; }
        t->child[2 * i + c] = id;
    }
    for (int c = 0; c < 2 && rc == 0; ++c)
        rc = st_split(t, t->child[2 * i + c], sub[c], cnt[c], px, py, pz, threshold);
done:
    free(sub[0]);
    free(sub[1]);
    return rc;
}

/* Build: root cube, split_to_depth(depth), then split(threshold) over the n
 * points (each first placed in its leaf by find).  Node arrays of capacity
 * cap.  Returns the node count, or -1 when cap is exceeded. */
int or_stree_build(const float aabb_min[3], const float aabb_max[3], int depth, const float* px,
                   const float* py, const float* pz, int64_t n, int threshold, int cap, float* mn, float* mx,
                   int* axis, int* child) {
    st_tree t = {mn, mx, axis, child, 0, cap};
    float size = 0.0f, rmn[3], rmx[3];
    for (int a = 0; a < 3; ++a) {
        const float e = aabb_max[a] - aabb_min[a];
        if (e > size) size = e;
    }
    for (int a = 0; a < 3; ++a) { rmn[a] = aabb_min[a]; rmx[a] = aabb_min[a] + size; }
    if (st_push(&t, rmn, rmx, 0) < 0) return -1;
    if (st_depth(&t, 0, 0, depth)) return -1;
    if (n > 0 && threshold > 0) {
        const int n0 = t.n;
        int64_t** per = (int64_t**)calloc((size_t)n0, sizeof(int64_t*));
        int64_t* cnt = (int64_t*)calloc((size_t)n0, sizeof(int64_t));
        for (int64_t j = 0; j < n; ++j) {
            const float p[3] = {px[j], py[j], pz[j]};
            const int id = or_stree_find(mn, mx, child, p);
            if (id < 0) continue;
            if (!per[id]) per[id] = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
            per[id][cnt[id]++] = j;
        }
        int rc = 0;
        for (int id = 0; id < n0 && rc == 0; ++id)
            if (child[2 * id] < 0 && per[id]) rc = st_split(&t, id, per[id], cnt[id], px, py, pz, threshold);
        for (int id = 0; id < n0; ++id) free(per[id]);
        free(per);
        free(cnt);
        if (rc) return -1;
    }
    return t.n;
}
