"""CPU: analytic known-answer tests pinning the oracle (SURVEY.md 8(c) KATs 1-8).

The reference ships no golden vectors for this path and cannot be built here
(Eigen/Boost/enoki/sdmm-lib absent), so the oracle is pinned by these KATs; the
committed fixtures in tests/golden/ are regression vectors of the oracle.
"""
import ctypes as C

import numpy as np
import pytest


def _pcg(oracle, seed, seq):
    class R(C.Structure):
        _fields_ = [("state", C.c_uint64), ("inc", C.c_uint64)]
    r = R()
    oracle.lib().or_pcg32_seed(C.byref(r), C.c_uint64(seed), C.c_uint64(seq))
    return r


def test_pcg32_published_vector(oracle):
    # pcg32_srandom(42u, 54u) (pcg-c basic demo) -- the generator enoki::PCG32
    # implements (sdmm_proc.h:87, RNG = enoki::PCG32<float, 1>).
    r = _pcg(oracle, 42, 54)
    got = [oracle.lib().or_pcg32_next_uint(C.byref(r)) for _ in range(6)]
    assert got == [0xa15c02b7, 0x7b47f409, 0xba1d3330, 0x83d2f293, 0xbfa4784b, 0xcbed606e]


def _rand_unit(rng, n):
    v = rng.normal(size=(n, 3))
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


def test_kat2_coordinates_orthonormal(oracle):
    rng = np.random.default_rng(1)
    ns = np.concatenate([_rand_unit(rng, 200), np.float32([[0, 0, 1], [0, 0, -1], [1, 0, 0]])])
    for n in ns:
        to = oracle.coordinates(n).astype(np.float64)
        np.testing.assert_allclose(to @ to.T, np.eye(3), atol=2e-6)
        np.testing.assert_array_equal(to[2], n)          # row 2 == n
        assert np.linalg.det(to) > 0


def test_kat1_log_exp_identities(oracle):
    rng = np.random.default_rng(2)
    for _ in range(300):
        n = _rand_unit(rng, 1)[0]
        to = oracle.coordinates(n)
        # exp(log(x)) == x for unit directions not antipodal to the mean
        d = _rand_unit(rng, 1)[0]
        if float(to[2] @ d) < -0.99:
            continue
        emb = np.concatenate([rng.normal(size=3).astype(np.float32), d])
        ok, t, jac = oracle.ts_log(to, emb)
        assert ok
        ok2, e2, _ = oracle.ts_exp(to, t)
        assert ok2
        np.testing.assert_allclose(e2[3:], d, atol=2e-5)
        np.testing.assert_array_equal(e2[:3], emb[:3])
        # log(exp(v)) == v for |v_t| < pi
        v = np.concatenate([rng.normal(size=3), rng.uniform(-1.5, 1.5, 2)]).astype(np.float32)
        ok3, e3, _ = oracle.ts_exp(to, v)
        ok4, v4, _ = oracle.ts_log(to, e3)
        assert ok3 and ok4
        np.testing.assert_allclose(v4, v, atol=5e-5)


def test_log_failure_modes(oracle):
    to = oracle.coordinates(np.float32([0, 0, 1]))
    assert oracle.ts_log(to, np.float32([0, 0, 0, 0, 0, 0]))[0] == 0       # d == 0
    assert oracle.ts_log(to, np.float32([0, 0, 0, 0, 0, -1]))[0] == 0      # antipode (c <= -1)
    ok, t, jac = oracle.ts_log(to, np.float32([0, 0, 0, 0, 0, 1]))        # at the pole
    assert ok and jac == 1.0 and (t == 0).all()
    # sin(angle) < 1e-3 quirk: angle/sin replaced by 1 (mvtn.h:164)
    ok, t, jac = oracle.ts_log(to, np.float32([0, 0, 0, 5e-4, 0, np.sqrt(1 - 25e-8)]))
    assert ok and jac == 1.0
    # exp fails for |t| >= pi
    assert oracle.ts_exp(to, np.float32([0, 0, 0, 3.2, 0]))[0] == 0


def _single(oracle, mean6, cov):
    m = oracle.Mixture(1)
    m.set_component(0, np.asarray(mean6, np.float64), np.asarray(cov, np.float64), mode=1)
    m.weights[:] = 1.0
    m.configure()
    return m


def _pdf(oracle, m, pts):
    f = oracle.lib().or_mvtn_pdf_and_log
    t = np.zeros(5, np.float32)
    out = np.empty(len(pts))
    for i, p in enumerate(np.ascontiguousarray(pts, np.float32)):
        out[i] = f(m.ptr, 0, p.ctypes.data_as(C.POINTER(C.c_float)), t.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def test_kat3_component_pdf_integrates_to_one(oracle):
    """MC over a position box x S^2 (uniform directions): E[pdf] * volume ~= 1."""
    rng = np.random.default_rng(3)
    mean = [0.5, 0.4, 0.6, 0.0, 0.6, 0.8]
    cov = np.diag([1e-3, 2e-3, 1.5e-3, 0.3, 0.2])
    cov[0, 1] = cov[1, 0] = 5e-4
    cov[3, 4] = cov[4, 3] = 0.05
    m = _single(oracle, mean, cov)
    n = 200_000
    half = 6 * np.sqrt(np.diag(cov)[:3])
    p = rng.uniform(-1, 1, size=(n, 3)) * half + np.array(mean[:3])
    d = _rand_unit(rng, n)
    pts = np.concatenate([p, d], 1)
    vals = _pdf(oracle, m, pts)
    vol = np.prod(2 * half) * 4 * np.pi
    est = vals.mean() * vol
    se = vals.std() * vol / np.sqrt(n)
    # tangent-space mass outside |t| < pi is ~exp(-pi^2/(2*0.3)) ~ 7e-8: negligible
    assert abs(est - 1.0) < 5 * se + 1e-3, (est, se)


def test_kat4_posterior_sums_to_one(oracle, synth):
    b = synth.em_batch(2000, 128)
    pos, nrm = synth.model_seed_points(b, 128)
    m, _ = oracle.hemisphere_init(16, pos, nrm, 0.01, 0.1, 7, mode=1)
    s = oracle.Samples(b["x"], b["w"], b["hpdf"], b["is_diffuse"])
    r = oracle.responsibilities(m, s)
    live = r.sum(1) > 0
    assert live.mean() > 0.5   # far samples underflow every component (FTZ)
    np.testing.assert_allclose(r.sum(1)[live], 1.0, atol=1e-5)
    # heuristic: posterior sums to (1-h) * sum / (...) + h * hpdf * invSum == 1
    bh = synth.em_batch(2000, 128, heuristic=True)
    sh = oracle.Samples(bh["x"], bh["w"], bh["hpdf"], bh["is_diffuse"])
    rh = oracle.responsibilities(m, sh)
    assert (rh.sum(1)[bh["is_diffuse"] == 1] < 1.0 + 1e-6).all()


def test_kat5_single_component_em_step(oracle):
    """One EM step of a 1-component mixture on w=1 samples returns the sample
    mean / covariance of the tangent vectors plus the exact prior terms."""
    rng = np.random.default_rng(5)
    mean = [0.5, 0.5, 0.5, 0.0, 0.0, 1.0]
    cov = np.diag([2e-3, 2e-3, 2e-3, 0.2, 0.2])
    m = _single(oracle, mean, cov)
    st = oracle.EmState(1)
    N = 5000
    L = np.linalg.cholesky(cov)
    z = rng.normal(size=(N, 5)) @ L.T
    to = m.to.reshape(3, 3)
    x = np.zeros((6, N), np.float32)
    for i in range(N):
        ok, e, _ = oracle.ts_exp(to, np.concatenate([z[i, :3] + mean[:3], z[i, 3:]]))
        x[:, i] = e
    w = np.ones(N, np.float32)
    s = oracle.Samples(x, w)
    # tangent vectors as the E-step sees them (component frame)
    taus = np.zeros((N, 5))
    for i in range(N):
        ok, t, _ = oracle.ts_log(to, x[:, i] - np.float32(mean[:3] + [0, 0, 0]))
        taus[i] = t
        taus[i, :3] += mean[:3]
    assert oracle.optimize(m, st, s, accurate=True) == 1
    mu = taus.mean(0)
    C = taus.T @ taus / N - np.outer(mu, mu)
    # decreasePrior at it=0: a = 100/K = 100, B = a * bPrior = 1e-3 I, ni = 6e-5
    expected = (C + 100 * np.float32(1e-5) * np.eye(5)) / (0.05 * 100 + 1.0)
    np.testing.assert_allclose(m.cov[0].reshape(5, 5), expected, rtol=2e-5, atol=1e-9)
    np.testing.assert_allclose(m.mean[0, :3], mu[:3], atol=1e-6)
    assert m.weights[0] == 1.0


def test_kat6_em_converges_on_known_mixture(oracle, synth):
    """EM on 2^16 samples of a K=16 generator: log-likelihood rises and the
    fitted mixture explains the data about as well as the generator."""
    b = synth.em_batch(1 << 16, 16, guards=False)
    g = b["generator"]
    pos, nrm = synth.model_seed_points(b, 16)
    m, st = oracle.hemisphere_init(2, pos, nrm, 0.01, 0.1, 11, mode=1)
    s = oracle.Samples(b["x"], b["w"])
    gm = oracle.Mixture(16)
    for k in range(16):
        gm.set_component(k, g["mean"][k].astype(np.float64), g["cov"][k].astype(np.float64))
    gm.weights[:] = g["weights"]
    gm.configure()

    def loglik(mix):
        f = oracle.lib().or_mvtn_pdf_and_log
        t = np.zeros(5, np.float32)
        idx = np.random.default_rng(0).choice(b["x"].shape[1], 4000, replace=False)
        ll = 0.0
        for i in idx:
            p = np.ascontiguousarray(b["x"][:, i])
            pp = p.ctypes.data_as(C.POINTER(C.c_float))
            tp = t.ctypes.data_as(C.POINTER(C.c_float))
            v = sum(mix.weights[k] * f(mix.ptr, k, pp, tp) for k in range(mix.K))
            ll += np.log(max(v, 1e-300))
        return ll / len(idx)

    lls = [loglik(m)]
    for _ in range(12):
        oracle.optimize(m, st, s, accurate=True)
        lls.append(loglik(m))
    assert lls[-1] > lls[0] + 1.0
    assert lls[-1] > loglik(gm) - 0.5, (lls, loglik(gm))


def test_kat7_sample_discrete_cdf_lower_bound_and_tie_walk(oracle):
    rng = np.random.default_rng(7)
    for n in (1, 2, 5, 33):
        w = rng.random(n).astype(np.float32)
        w[rng.random(n) < 0.4] = 0
        if w.sum() == 0:
            w[-1] = 1
        cdf = np.cumsum(w / w.sum(), dtype=np.float32)
        for u in np.concatenate([rng.random(200), cdf, [0.0]]).astype(np.float32):
            i = int(np.searchsorted(cdf, u, side="left"))
            if i == n:
                i -= 1
                while i > 0 and cdf[i] == cdf[i - 1]:
                    i -= 1
            assert oracle.sample_discrete_cdf(cdf, u) == i
    # u beyond the last cdf value walks back over the trailing zero-weight run
    cdf = np.float32([0.25, 0.5, 0.999, 0.999, 0.999])
    assert oracle.sample_discrete_cdf(cdf, np.float32(0.9995)) == 2


def test_kat8_box_muller_order(oracle):
    """MVTN::sample: z = r * (sin(theta), cos(theta)) (sincos res0=sin, res1=cos)."""
    mean = [0.5, 0.5, 0.5, 0.0, 0.0, 1.0]
    cov = np.diag([1e-3, 1e-3, 1e-3, 0.25, 0.09])
    m = _single(oracle, mean, cov)
    c = np.float32([[0.5, 0.5, 0.5]])
    for u1, u2 in [(0.3, 0.1), (0.7, 0.35), (0.01, 0.9)]:
        u = np.float32([[0.5, u1, u2]])
        d, pdf, comp, slot = oracle.guide_batch(m, c, u)
        r = np.sqrt(-2 * np.log(1 - np.float32(u1)))
        th = 2 * np.pi * np.float32(u2)
        z = r * np.array([np.sin(th), np.cos(th)])
        L = m.condL[0].reshape(2, 2)
        v = L @ z
        to = oracle.coordinates(np.float32(mean[3:]))
        ok, e, _ = oracle.ts_exp(to, np.float32([0, 0, 0, v[0], v[1]]))
        np.testing.assert_allclose(d[0], e[3:], atol=1e-5)
        assert comp[0] == 0 and pdf[0] > 0


def test_faithful_and_accurate_modes_agree_to_reference_noise(oracle, synth):
    b = synth.em_batch(8192, 128)
    pos, nrm = synth.model_seed_points(b, 128)
    s = oracle.Samples(b["x"], b["w"])
    ma, sa = oracle.hemisphere_init(16, pos, nrm, 0.01, 0.1, 3, mode=1)
    mf, sf = oracle.hemisphere_init(16, pos, nrm, 0.01, 0.1, 3, mode=0)
    for _ in range(3):
        oracle.optimize(ma, sa, s, accurate=True)
        oracle.optimize(mf, sf, s, accurate=False)
    np.testing.assert_allclose(mf.weights, ma.weights, rtol=2e-3, atol=1e-6)
    np.testing.assert_allclose(mf.mean, ma.mean, rtol=1e-3, atol=1e-4)


def test_pd_check(oracle):
    rng = np.random.default_rng(9)
    for _ in range(100):
        A = rng.normal(size=(5, 5))
        S = A @ A.T + 1e-3 * np.eye(5)
        assert oracle.is_pd(S) and oracle.is_pd(S.astype(np.float32), single=True)
        S2 = S.copy()
        S2[2, 2] = -1.0
        assert not oracle.is_pd(S2)
    # only the lower triangle is read (SelfAdjointEigenSolver)
    S = np.eye(5)
    S[0, 4] = 100.0
    assert oracle.is_pd(S)


def test_float_division_by_double_reciprocal_is_exact():
    """The guide kernel's div_exact (guide.hip): IEEE float x / d equals
    (float)((double)x * RN64(1 / d)) -- checked here on 4M pairs, including
    divisors whose significands are all ones / powers of two and quotients that
    are exact, near overflow of the significand, or tiny."""
    rng = np.random.default_rng(11)
    n = 1 << 22
    x = (rng.standard_normal(n) * np.exp(rng.uniform(-20, 20, n))).astype(np.float32)
    d = np.abs(rng.standard_normal(n) * np.exp(rng.uniform(-10, 10, n))).astype(np.float32) + np.float32(1e-30)
    special = np.array([1.0, 2.0, 0.5, np.nextafter(np.float32(2), np.float32(0)), np.float32(1.9999999),
                        np.float32(3.0), np.float32(0.1), np.float32(7.0)], np.float32)
    d[:special.size * 1000] = np.repeat(special, 1000)
    x[:4000] = (d[:4000] * np.float32(3)).astype(np.float32)          # exact quotients
    with np.errstate(over="ignore", under="ignore"):
        ref = x / d
        got = (x.astype(np.float64) * (1.0 / d.astype(np.float64))).astype(np.float32)
    ok = np.isfinite(ref) & (np.abs(ref) >= np.finfo(np.float32).tiny)
    np.testing.assert_array_equal(got[ok], ref[ok])
