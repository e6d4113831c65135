"""CPU ORACLE wrapper (test infrastructure only).

ctypes binding of oracle/_build/liboracle.so, the plain-C restatement of the
jmm stepwise tangent-space EM and guided sampling (see sdmm_oracle.h for the
reference file:line map).  Only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may import this module; the product path never
does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liboracle.so"

_f = C.POINTER(C.c_float)
_d = C.POINTER(C.c_double)
_i = C.POINTER(C.c_int)


class _Mixture(C.Structure):
    _fields_ = [
        ("K", C.c_int), ("heuristicWeight", C.c_float), ("normalization", C.c_float),
        ("weights", _f), ("cdf", _f), ("mean", _f), ("cov", _f), ("to", _f),
        ("cholL", _f), ("cholLInv", _f), ("detInv", _f), ("muPremult", _f),
        ("condCov", _f), ("margL", _f), ("margDetInv", _f), ("condL", _f),
        ("condLInv", _f), ("condDetInv", _f), ("valid", _i),
    ]


class _EmState(C.Structure):
    _fields_ = [
        ("K", C.c_int), ("iterationsRun", C.c_int), ("decreasePrior", C.c_int),
        ("trainingCutoff", C.c_int), ("alpha", C.c_double), ("niPriorMinusOne", C.c_double),
        ("heuristicTotalWeight", C.c_double), ("sgH", C.c_double),
        ("totalWeight", _d), ("sgW", _d), ("sgM", _d), ("sgC", _d),
        ("bPriors", _f), ("bDepth", _f),
    ]


class _Samples(C.Structure):
    _fields_ = [
        ("n", C.c_int64), ("x", _f * 6), ("w", _f), ("hpdf", _f),
        ("isDiffuse", C.POINTER(C.c_uint8)),
    ]


def build() -> Path:
    """Compile the oracle with its committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        L.or_pcg32_next_float.restype = C.c_float
        L.or_pcg32_next_uint.restype = C.c_uint32
        L.or_sinc_pi.restype = C.c_float
        L.or_sinc_pi.argtypes = [C.c_float]
        L.or_mvtn_pdf_and_log.restype = C.c_float
        L.or_marginal_pdf.restype = C.c_float
        L.or_conditional_pdf.restype = C.c_float
        L.or_uniform_hemisphere_init.argtypes = [
            C.c_void_p, C.c_void_p, _f, _f, C.c_int, C.c_float, C.c_float, C.c_uint64, C.c_int]
        L.or_em_state_init.argtypes = [C.c_void_p, C.c_int, C.c_double, _d, C.c_double,
                                       C.c_double, C.c_int]
        L.or_mstep_f32.argtypes = [C.c_void_p, C.c_void_p, _d, C.c_int64]
        L.or_mstep_f64.argtypes = [C.c_void_p, C.c_void_p, _d, C.c_int64]
        L.or_mstep_x64.argtypes = [C.c_void_p, C.c_void_p, _d, C.c_int64]
        L.or_guide_batch.argtypes = [C.c_void_p, C.c_int64, _f, _f, _f, _f,
                                     C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.or_pdf_batch.argtypes = [C.c_void_p, C.c_int64, _f, _f, _f]
        L.or_sample_discrete_cdf.argtypes = [_f, C.c_int, C.c_float]
        L.or_is_positive_definite_f64.argtypes = [_d, C.c_int]
        L.or_is_positive_definite_f32.argtypes = [_f, C.c_int]
        L.or_ts_log.argtypes = [_f, _f, _f, _f]
        L.or_ts_exp.argtypes = [_f, _f, _f, _f]
        L.or_coordinates.argtypes = [_f, _f]
        L.or_component_set.argtypes = [C.c_void_p, C.c_int, _d, _d, C.c_int]
        L.or_guide_product_batch.argtypes = [C.c_void_p, C.c_int64, _f, _f, C.POINTER(C.c_int32), _f, _f, _f,
                                             _f, C.c_int, C.POINTER(C.c_uint8), _f, _f, _f, _f,
                                             C.POINTER(C.c_int32), _f]
        _l = C.POINTER(C.c_int64)
        L.or_kmeanspp_select.argtypes = [_f, _f, _f, _f, _f, _f, _f, C.c_int64, C.c_int, _f, C.c_int, _l]
        L.or_uniform_hemisphere_init_kmeanspp.argtypes = [
            C.c_void_p, C.c_void_p, _f, _f, _f, _f, _f, _f, _f, C.c_int64, C.c_int, C.c_float, C.c_float,
            C.c_uint64, C.c_int, C.c_int, _l]
        L.or_mvtn_multiply.restype = C.c_float
        L.or_mvtn_multiply.argtypes = [_f, _f, _f, _f, _f]
        _lib = L
    return _lib


def _fp(a):
    return a.ctypes.data_as(_f)


def _dp(a):
    return a.ctypes.data_as(_d)


MIX_FIELDS = {
    "weights": 1, "cdf": 1, "mean": 6, "cov": 25, "to": 9, "cholL": 25, "cholLInv": 25,
    "detInv": 1, "muPremult": 6, "condCov": 4, "margL": 9, "margDetInv": 1, "condL": 4,
    "condLInv": 4, "condDetInv": 1,
}


class Mixture:
    """jmm::MixtureModel<6,K,3,float,...> held in numpy arrays."""

    def __init__(self, K: int):
        self.K = K
        self.arr = {k: np.zeros(K * w, np.float32) for k, w in MIX_FIELDS.items()}
        self.valid = np.zeros(K, np.int32)
        self.s = _Mixture()
        self.s.K = K
        self.s.heuristicWeight = 0.5
        self.s.normalization = 1.0
        for k, a in self.arr.items():
            setattr(self.s, k, _fp(a))
        self.s.valid = self.valid.ctypes.data_as(_i)

    @property
    def ptr(self):
        return C.byref(self.s)

    def __getattr__(self, name):
        if name in MIX_FIELDS:
            w = MIX_FIELDS[name]
            a = self.__dict__["arr"][name]
            return a if w == 1 else a.reshape(self.K, -1)
        raise AttributeError(name)

    def set_component(self, k, mean6, cov25, mode=1):
        m = np.ascontiguousarray(mean6, np.float64)
        c = np.ascontiguousarray(np.asarray(cov25, np.float64).reshape(25))
        return lib().or_component_set(self.ptr, k, _dp(m), _dp(c), mode)

    def configure(self):
        return lib().or_mixture_configure(self.ptr)

    def copy_params_from(self, params: dict):
        """Load exported derived params (dict of arrays named like MIX_FIELDS)."""
        for k in MIX_FIELDS:
            if k in params:
                self.arr[k][:] = np.asarray(params[k], np.float32).reshape(-1)
        if "normalization" in params:
            self.s.normalization = float(params["normalization"])
        self.valid[:] = 1


class EmState:
    def __init__(self, K, alpha=0.9, bprior=1e-5, ni=6e-5, epsilon=1e-100, decrease_prior=True):
        self.K = K
        self.d = {"totalWeight": np.zeros(K), "sgW": np.zeros(K), "sgM": np.zeros(K * 5),
                  "sgC": np.zeros(K * 25)}
        self.bPriors = np.zeros(K * 25, np.float32)
        self.bDepth = np.zeros(K * 9, np.float32)
        self.s = _EmState()
        for k, a in self.d.items():
            setattr(self.s, k, _dp(a))
        self.s.bPriors = _fp(self.bPriors)
        self.s.bDepth = _fp(self.bDepth)
        bp = np.full(5, bprior, np.float64)
        lib().or_em_state_init(C.byref(self.s), K, alpha, _dp(bp), ni, epsilon, int(decrease_prior))

    @property
    def ptr(self):
        return C.byref(self.s)


class Samples:
    def __init__(self, x: np.ndarray, w: np.ndarray, hpdf=None, is_diffuse=None):
        self.x = [np.ascontiguousarray(x[i], np.float32) for i in range(6)]
        self.w = np.ascontiguousarray(w, np.float32)
        self.hpdf = None if hpdf is None else np.ascontiguousarray(hpdf, np.float32)
        self.isd = None if is_diffuse is None else np.ascontiguousarray(is_diffuse, np.uint8)
        self.s = _Samples()
        self.s.n = len(self.w)
        for i in range(6):
            self.s.x[i] = _fp(self.x[i])
        self.s.w = _fp(self.w)
        self.s.hpdf = _fp(self.hpdf) if self.hpdf is not None else _f()
        self.s.isDiffuse = (self.isd.ctypes.data_as(C.POINTER(C.c_uint8))
                            if self.isd is not None else C.POINTER(C.c_uint8)())

    @property
    def ptr(self):
        return C.byref(self.s)


def hemisphere_init(K_positions, positions, normals, depth_prior, min_dist, seed, mode=1,
                    with_state=True, **em_kw):
    K = K_positions * 8
    m = Mixture(K)
    st = EmState(K, **em_kw) if with_state else None
    pos = np.ascontiguousarray(positions, np.float32).reshape(-1)
    nrm = np.ascontiguousarray(normals, np.float32).reshape(-1)
    lib().or_uniform_hemisphere_init(m.ptr, st.ptr if st else None, _fp(pos), _fp(nrm),
                                     K_positions, depth_prior, min_dist, seed, mode)
    return m, st


def kmeanspp_select(x, normals, w, n_pos, u, mode=1):
    """kMeansPPInit (mixture_model_init.h:244-330): the sample indices of the
    n_pos seed positions for the draws u.  mode 0: the reference's float CDF;
    mode 1: the device rule (fp64 weights and sums), see sdmm_oracle_kmeans.c."""
    xs = [np.ascontiguousarray(x[i], np.float32) for i in range(3)]
    ns = [np.ascontiguousarray(normals[i], np.float32) for i in range(3)]
    ww = np.ascontiguousarray(w, np.float32)
    uu = np.ascontiguousarray(u, np.float32)
    assert uu.size >= n_pos
    out = np.zeros(n_pos, np.int64)
    r = lib().or_kmeanspp_select(*[_fp(a) for a in xs + ns], _fp(ww), ww.size, n_pos, _fp(uu), mode,
                                 out.ctypes.data_as(C.POINTER(C.c_int64)))
    assert r == 0, r
    return out


def hemisphere_init_kmeanspp(K_positions, x, normals, w, depth_prior, min_dist, seed, mode=1, select_mode=1):
    """uniformHemisphereInit with kMeansPlusPlus = true (:130-138): one PCG32
    stream for the k-means++ draws and then the direction jitter."""
    K = K_positions * 8
    m = Mixture(K)
    st = EmState(K)
    xs = [np.ascontiguousarray(x[i], np.float32) for i in range(3)]
    ns = [np.ascontiguousarray(normals[i], np.float32) for i in range(3)]
    ww = np.ascontiguousarray(w, np.float32)
    idx = np.zeros(K_positions, np.int64)
    r = lib().or_uniform_hemisphere_init_kmeanspp(m.ptr, st.ptr, *[_fp(a) for a in xs + ns], _fp(ww), ww.size,
                                                  K_positions, depth_prior, min_dist, seed, mode, select_mode,
                                                  idx.ctypes.data_as(C.POINTER(C.c_int64)))
    return m, st, idx, r


def stats_len(K):
    return 2 + 31 * K


_SFX = {"faithful": "f32", "accurate": "f64", "exact": "x64", True: "f64", False: "f32"}


def _mode(accurate):
    """accurate: True/False (accurate/faithful) or 'faithful'|'accurate'|'exact'."""
    return _SFX[accurate]


def calculate_stats(m: Mixture, s: Samples, accurate=True):
    out = np.zeros(stats_len(m.K))
    getattr(lib(), "or_calculate_stats_" + _mode(accurate))(m.ptr, s.ptr, _dp(out))
    return out


def mstep(m: Mixture, st: EmState, stats: np.ndarray, n_samples: int, accurate=True):
    st_ = np.ascontiguousarray(stats, np.float64)
    return getattr(lib(), "or_mstep_" + _mode(accurate))(m.ptr, st.ptr, _dp(st_), n_samples)


def optimize(m: Mixture, st: EmState, s: Samples, accurate=True):
    return getattr(lib(), "or_optimize_" + _mode(accurate))(m.ptr, st.ptr, s.ptr)


def responsibilities(m: Mixture, s: Samples):
    out = np.zeros((s.s.n, m.K), np.float32)
    lib().or_responsibilities(m.ptr, s.ptr, _fp(out))
    return out


def guide_batch(m: Mixture, c: np.ndarray, u: np.ndarray):
    c = np.ascontiguousarray(c, np.float32)
    u = np.ascontiguousarray(u, np.float32)
    nq = c.shape[0]
    d = np.zeros((nq, 3), np.float32)
    pdf = np.zeros(nq, np.float32)
    comp = np.zeros(nq, np.int32)
    slot = np.zeros(nq, np.int32)
    I32 = C.POINTER(C.c_int32)
    lib().or_guide_batch(m.ptr, nq, _fp(c), _fp(u), _fp(d), _fp(pdf),
                         comp.ctypes.data_as(I32), slot.ctypes.data_as(I32))
    return d, pdf, comp, slot


def guide_product_batch(m: Mixture, c, u, material, frames, bw, bmean, bcov, dgiven=None, diffuse=None,
                        choice=None):
    """Product sampling with a learned-BSDF table (sdmm_oracle_product.inc).
    c, u: (nq, 3); material: (nq,) int (-1: none); frames: (nq, 9) row-major
    to-world [s t n] columns; bw (B, M), bmean (B, M, 3) local, bcov (B, M, 4).
    diffuse (B,) flags: the plugin's diffuse case (slice 0 on the normal);
    choice (nq,) with dgiven: the mixed bounce (pdf query where choice <= h).
    Returns dir (nq, 3), pdf, comp (k * M + j for product samples, -2 for
    pdf queries of the mixed bounce), h."""
    c = np.ascontiguousarray(c, np.float32)
    u = np.ascontiguousarray(u, np.float32)
    nq = c.shape[0]
    material = np.ascontiguousarray(material, np.int32)
    frames = np.ascontiguousarray(frames, np.float32)
    bw = np.ascontiguousarray(bw, np.float32)
    M = bw.shape[1]
    bmean = np.ascontiguousarray(bmean, np.float32)
    bcov = np.ascontiguousarray(bcov, np.float32)
    d = np.zeros((nq, 3), np.float32)
    pdf = np.zeros(nq, np.float32)
    comp = np.zeros(nq, np.int32)
    h = np.zeros(nq, np.float32)
    I32 = C.POINTER(C.c_int32)
    dg = None if dgiven is None else np.ascontiguousarray(dgiven, np.float32)
    df = None if diffuse is None else np.ascontiguousarray(diffuse, np.uint8)
    ch = None if choice is None else np.ascontiguousarray(choice, np.float32)
    lib().or_guide_product_batch(m.ptr, nq, _fp(c), _fp(u), material.ctypes.data_as(I32), _fp(frames), _fp(bw),
                                 _fp(bmean), _fp(bcov), M,
                                 None if df is None else df.ctypes.data_as(C.POINTER(C.c_uint8)),
                                 None if ch is None else _fp(ch), None if dg is None else _fp(dg), _fp(d),
                                 _fp(pdf), comp.ctypes.data_as(I32), _fp(h))
    return d, pdf, comp, h


def mvtn_multiply(e, ci, mj, cj):
    """MVTN::multiply test hook: (weight, product mean (3), L (2x2), Linv (2x2), detInv)."""
    out = np.zeros(13, np.float32)
    f = lambda a: np.ascontiguousarray(a, np.float32)
    e, ci, mj, cj = f(e), f(ci), f(mj), f(cj)
    lib().or_mvtn_multiply(_fp(e), _fp(ci), _fp(mj), _fp(cj), _fp(out))
    return float(out[0]), out[1:4].copy(), out[4:8].reshape(2, 2).copy(), out[8:12].reshape(2, 2).copy(), float(out[12])


def pdf_batch(m: Mixture, c: np.ndarray, d: np.ndarray):
    c = np.ascontiguousarray(c, np.float32)
    d = np.ascontiguousarray(d, np.float32)
    out = np.zeros(c.shape[0], np.float32)
    lib().or_pdf_batch(m.ptr, c.shape[0], _fp(c), _fp(d), _fp(out))
    return out


def sample_discrete_cdf(cdf, u):
    cdf = np.ascontiguousarray(cdf, np.float32)
    return lib().or_sample_discrete_cdf(_fp(cdf), len(cdf), float(u))


def is_pd(A, single=False):
    if single:
        a = np.ascontiguousarray(A, np.float32)
        return bool(lib().or_is_positive_definite_f32(_fp(a), a.shape[0]))
    a = np.ascontiguousarray(A, np.float64)
    return bool(lib().or_is_positive_definite_f64(_dp(a), a.shape[0]))


def ts_log(to, emb):
    to = np.ascontiguousarray(to, np.float32).reshape(9)
    emb = np.ascontiguousarray(emb, np.float32).reshape(6)
    t = np.zeros(5, np.float32)
    j = np.zeros(1, np.float32)
    ok = lib().or_ts_log(_fp(to), _fp(emb), _fp(t), _fp(j))
    return ok, t, float(j[0])


def ts_exp(to, tangent):
    to = np.ascontiguousarray(to, np.float32).reshape(9)
    t = np.ascontiguousarray(tangent, np.float32).reshape(5)
    e = np.zeros(6, np.float32)
    j = np.zeros(1, np.float32)
    ok = lib().or_ts_exp(_fp(to), _fp(t), _fp(e), _fp(j))
    return ok, e, float(j[0])


def coordinates(n):
    n = np.ascontiguousarray(n, np.float32)
    to = np.zeros(9, np.float32)
    lib().or_coordinates(_fp(n), _fp(to))
    return to.reshape(3, 3)


def pcg32_floats(seed, n, seq=0xda3e39cb94b95bdb):
    class R(C.Structure):
        _fields_ = [("state", C.c_uint64), ("inc", C.c_uint64)]
    r = R()
    lib().or_pcg32_seed(C.byref(r), C.c_uint64(seed), C.c_uint64(seq))
    return np.array([lib().or_pcg32_next_float(C.byref(r)) for _ in range(n)], np.float32)


def stree_build(aabb_min, aabb_max, depth, p, threshold, cap=1 << 16):
    """jmm SNTree (spatial part) restated in C: returns (aabb[n,6], child[n,2], axis[n])."""
    p = [np.ascontiguousarray(x, np.float32) for x in p]
    n = p[0].shape[0]
    mn = np.zeros(3 * cap, np.float32)
    mx = np.zeros(3 * cap, np.float32)
    ax = np.zeros(cap, np.int32)
    ch = np.zeros(2 * cap, np.int32)
    lo = np.ascontiguousarray(aabb_min, np.float32)
    hi = np.ascontiguousarray(aabb_max, np.float32)
    f = lib().or_stree_build
    f.restype = C.c_int
    cnt = f(_fp(lo), _fp(hi), C.c_int(depth), _fp(p[0]), _fp(p[1]), _fp(p[2]), C.c_int64(n),
            C.c_int(threshold), C.c_int(cap), _fp(mn), _fp(mx), ax.ctypes.data_as(C.c_void_p),
            ch.ctypes.data_as(C.c_void_p))
    assert cnt > 0, "oracle tree capacity exceeded"
    aabb = np.concatenate([mn[:3 * cnt].reshape(-1, 3), mx[:3 * cnt].reshape(-1, 3)], 1)
    return aabb, ch[:2 * cnt].reshape(-1, 2).copy(), ax[:cnt].copy()


def stree_find(aabb, child, pts):
    """SNTreeNode::find for points (n, 3) on a tree from stree_build."""
    mn = np.ascontiguousarray(aabb[:, :3].reshape(-1), np.float32)
    mx = np.ascontiguousarray(aabb[:, 3:].reshape(-1), np.float32)
    ch = np.ascontiguousarray(child.reshape(-1), np.int32)
    f = lib().or_stree_find
    f.restype = C.c_int
    out = np.empty(len(pts), np.int32)
    for i, q in enumerate(np.ascontiguousarray(pts, np.float32)):
        out[i] = f(_fp(mn), _fp(mx), ch.ctypes.data_as(C.c_void_p), _fp(q))
    return out


def rng_uniform(seed, path, stream, dim):
    """The library's counter-based uniform (render_device.h), restated in C."""
    f = lib().or_rng_uniform
    f.restype = C.c_float
    f.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32]
    return f(seed, path, stream, dim)


def push_training(aabb, child, rec, nv, V, path0, saved, seed):
    """Host-routed training records of Li's tail (sdmm_proc.cpp:876-965) in
    (path, push) order: dict node, source, stats, w (+ lost)."""
    mn = np.ascontiguousarray(aabb[:, :3].reshape(-1), np.float32)
    mx = np.ascontiguousarray(aabb[:, 3:].reshape(-1), np.float32)
    ch = np.ascontiguousarray(child.reshape(-1), np.int32)
    rec = np.ascontiguousarray(rec, np.float32)
    nv = np.ascontiguousarray(nv, np.int32)
    P = int(nv.shape[0])
    cap = int(nv.sum()) * 3 + 1
    node = np.empty(cap, np.int32)
    src = np.empty(cap, np.int64)
    st = np.empty(cap, np.uint8)
    w = np.empty(cap, np.float32)
    lost = C.c_int64(0)
    f = lib().or_push_training
    f.restype = C.c_int64
    n = f(_fp(mn), _fp(mx), ch.ctypes.data_as(C.c_void_p), _fp(rec), nv.ctypes.data_as(C.c_void_p),
          C.c_int64(P), C.c_int(V), C.c_int64(path0), C.c_int(saved), C.c_uint64(seed),
          node.ctypes.data_as(C.c_void_p), src.ctypes.data_as(C.c_void_p), st.ctypes.data_as(C.c_void_p),
          _fp(w), C.c_int64(cap), C.byref(lost))
    assert n <= cap
    return {"node": node[:n].copy(), "source": src[:n].copy(), "stats": st[:n].copy(), "w": w[:n].copy(),
            "lost": int(lost.value)}


L4_MAX, L4_REC = 8, 22
L4_STRIDE = 1 + L4_MAX * L4_REC


def pack_learned_models(models, n_bsdfs):
    """desc["learned_models"] (per BSDF None or (weights[M], means[M][5],
    covs[M][16])) as the oracle's packed table: L4_STRIDE floats per BSDF,
    [M, M records of (w, mean 5, cov 16)]; None when there are none."""
    if not models:
        return None
    out = np.zeros((n_bsdfs, L4_STRIDE), np.float32)
    for b, m in enumerate(models):
        if m is None:
            continue
        w, mu, cv = (np.asarray(x, np.float32) for x in m)
        M = len(w)
        out[b, 0] = M
        rec = np.concatenate([w.reshape(M, 1), mu.reshape(M, 5), cv.reshape(M, 16)], axis=1)
        out[b, 1:1 + M * L4_REC] = rec.reshape(-1)
    return np.ascontiguousarray(out)


def learned4_conditional(model, alpha, wl, keep=2):
    """or_learned4_conditional: the conductor's lobes (weights, local means,
    2x2 covariances) of one SDMM4 at local incident direction wl."""
    w, mu, cv = (np.asarray(x, np.float32) for x in model)
    M = len(w)
    rec = np.ascontiguousarray(np.concatenate([w.reshape(M, 1), mu.reshape(M, 5), cv.reshape(M, 16)], axis=1),
                               np.float32)
    ow = np.zeros(L4_MAX, np.float32)
    om = np.zeros((L4_MAX, 3), np.float32)
    oc = np.zeros((L4_MAX, 4), np.float32)
    wl = np.ascontiguousarray(wl, np.float32)
    f = lib().or_learned4_conditional
    f.restype = C.c_int
    vp = lambda a: a.ctypes.data_as(C.c_void_p)
    n = f(vp(rec), C.c_int(M), C.c_float(alpha), vp(wl), C.c_int(keep), vp(ow), vp(om), vp(oc))
    return ow[:n], om[:n], oc[:n]


def li_render(desc: dict, aabb, child, node_mix=None, guided=False, spp=1, max_depth=10, rr_depth=10, h=0.5,
              V=9, seed=0, pixels=None, learned=None, threads=1):
    """SDMMRenderer::Li restated on the CPU (sdmm_oracle_li.inc) for a
    scene description (scenes.cornell_box() fields), the tree (aabb (n, 6),
    child (n, 2)) and per-node oracle Mixtures (None: no trained context).
    learned: (weights (B, M), means (B, M, 3), covs (B, M, 4), diffuse (B,))
    for sampleProduct.  Returns dict image (3, H, W), image_sqr, rec
    (16, V, P), nv (P,), comps (bounces, P)."""
    W, H = int(desc["width"]), int(desc["height"])
    lo, hi = (0, W * H) if pixels is None else pixels
    P = (hi - lo) * spp
    f32 = lambda a: np.ascontiguousarray(a, np.float32)
    i32 = lambda a: np.ascontiguousarray(a, np.int32)
    quads, flip, bsdf = f32(desc["quads"]), i32(desc["flip_normals"]), i32(desc["bsdf"])
    refl, em, rad = f32(desc["reflectance"]), i32(desc["emitter"]), f32(desc["radiance"])
    cam = f32(desc["camera_to_world"])
    mn = np.ascontiguousarray(np.asarray(aabb)[:, :3].reshape(-1), np.float32)
    mx = np.ascontiguousarray(np.asarray(aabb)[:, 3:].reshape(-1), np.float32)
    ch = np.ascontiguousarray(np.asarray(child).reshape(-1), np.int32)
    nn = len(mn) // 3
    tab = (C.c_void_p * nn)()
    kmax = 1
    if node_mix is not None:
        for i, m in enumerate(node_mix):
            if m is not None:
                tab[i] = C.cast(m.ptr, C.c_void_p)
                kmax = max(kmax, m.K)
    image = np.zeros((3, H, W), np.float32)
    image_sqr = np.zeros((3, H, W), np.float32)
    rec = np.zeros((16, V, P), np.float32)
    nv = np.zeros(P, np.int32)
    bounces = max_depth - 1 if max_depth > 0 else V
    comps = np.full((bounces, P), -9, np.int32)
    if learned is not None:
        bw, bm, bc, bd = f32(learned[0]), f32(learned[1]), f32(learned[2]), np.ascontiguousarray(learned[3], np.uint8)
        M = bw.shape[1]
    else:
        bw = bm = bc = np.zeros(1, np.float32)
        bd = np.zeros(1, np.uint8)
        M = 0
    f = lib().or_li_render
    f.restype = C.c_int
    vp = lambda a: a.ctypes.data_as(C.c_void_p)
    bpar = f32(desc["bsdf_params"]) if "bsdf_params" in desc else None
    lmod = pack_learned_models(desc.get("learned_models"), len(refl) // 3)
    rc = f(vp(quads), vp(flip), vp(bsdf), C.c_int(len(bsdf)), vp(refl), vp(bpar) if bpar is not None else None,
           vp(em), vp(rad), vp(cam),
           C.c_float(desc["fov_x_deg"]), C.c_float(desc["near_clip"]), C.c_int(W), C.c_int(H), vp(mn), vp(mx),
           vp(ch), tab, C.c_int(int(guided)), C.c_int(spp), C.c_int(max_depth), C.c_int(rr_depth), C.c_float(h),
           C.c_int(V), C.c_uint64(seed), C.c_int64(lo), C.c_int64(hi), C.c_int(1 if learned is not None else 0),
           vp(bw), vp(bm), vp(bc), vp(bd), C.c_int(M), C.c_int(kmax), vp(image), vp(image_sqr), vp(rec), vp(nv),
           vp(comps), C.c_int(threads), vp(lmod) if lmod is not None else None)
    assert rc == 0, "or_li_render failed"
    return {"image": image, "image_sqr": image_sqr, "rec": rec, "nv": nv, "comps": comps}
