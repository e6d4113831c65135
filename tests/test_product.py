"""CPU: the oracle's product sampling with a learned BSDF
(oracle/sdmm_oracle_product.inc: jmm MixtureModel::multiply,
mixture_model.h:345-370, MVTN::multiply, multivariate_tangent_normal.h:555-617;
plugin path sdmm_proc.cpp:327-392).  sdmm-lib's sdmm::product is absent and
the learned-BSDF `.sdmm` files are LFS pointers, so these analytic known-answer
tests pin the restatement (parity against sdmm-lib unpinned):

  P1  equal means, equal covariances: product mean = the mean, covariance =
      Sigma / 2, weight = N(0; 0, 2 Sigma) = 1 / (2 pi sqrt(det 2 Sigma));
  P2  small covariances: the tangent-plane (Euclidean) Gaussian product;
  P3  the product mixture pdf integrates to 1 over S^2 (Monte Carlo);
  P4  batch rules: no learned BSDF -> the plain conditional (h = 0.5), bitwise
      equal to or_guide_batch; no valid conditional -> BSDF only (h = 1);
  P5  sampled directions follow the product pdf (sample mean vs pdf mean).
"""
import numpy as np
import pytest


def _iso(s2):
    return np.float32([s2, 0, 0, s2])


def test_p1_equal_lobes(oracle):
    rng = np.random.default_rng(3)
    for _ in range(20):
        e = rng.normal(size=3)
        e = (e / np.linalg.norm(e)).astype(np.float32)
        s2 = np.float32(rng.uniform(0.01, 0.2))
        w, mean, L, Linv, detInv = oracle.mvtn_multiply(e, _iso(s2), e, _iso(s2))
        np.testing.assert_allclose(mean, e, atol=1e-6)
        cov = L @ L.T
        np.testing.assert_allclose(cov, np.diag([s2 / 2, s2 / 2]), rtol=1e-4, atol=1e-7)
        np.testing.assert_allclose(w, 1.0 / (2 * np.pi * 2 * s2), rtol=1e-4)
        np.testing.assert_allclose(Linv @ L, np.eye(2), atol=1e-5)
        np.testing.assert_allclose(detInv, 1.0 / np.linalg.det(L), rtol=1e-5)


def test_p2_small_angle_is_the_euclidean_product(oracle):
    """Both lobes near the north pole with small covariances: the tangent
    planes nearly coincide, so the product is the Euclidean Gaussian product
    mu = S2 (S1 + S2)^-1 mu1 + S1 (S1 + S2)^-1 mu2, S = S1 (S1 + S2)^-1 S2 and
    weight N(mu1 - mu2; 0, S1 + S2)."""
    e = np.float32([0, 0, 1])
    for mu2, S1, S2 in [((0.01, 0.0), [4e-4, 0, 0, 1e-4], [1e-4, 0, 0, 1e-4]),
                        ((0.004, -0.006), [2e-4, 5e-5, 5e-5, 3e-4], [3e-4, -4e-5, -4e-5, 1e-4])]:
        t = np.array(mu2)
        th = np.linalg.norm(t)
        mj = np.float32([t[0] / th * np.sin(th), t[1] / th * np.sin(th), np.cos(th)])
        # the second lobe's covariance lives in ITS frame Coordinates(mj); near
        # the pole it is the same plane up to O(th) rotation
        S1m, S2m = np.array(S1).reshape(2, 2), np.array(S2).reshape(2, 2)
        w, mean, L, Linv, detInv = oracle.mvtn_multiply(e, np.float32(S1), mj, np.float32(S2))
        Ssum = S1m + S2m
        mu = S1m @ np.linalg.solve(Ssum, t)
        S = S1m @ np.linalg.solve(Ssum, S2m)
        # tangent of the product mean at the pole
        np.testing.assert_allclose(mean[:2], mu, rtol=0.03, atol=2e-5)
        np.testing.assert_allclose(L @ L.T, S, rtol=0.05, atol=2e-6)
        wref = np.exp(-0.5 * t @ np.linalg.solve(Ssum, t)) / (2 * np.pi * np.sqrt(np.linalg.det(Ssum)))
        np.testing.assert_allclose(w, wref, rtol=0.03)


def _fitted(oracle, synth, K=16, iters=3):
    b = synth.em_batch(8192, 128)
    pos, nrm = synth.model_seed_points(b, K)
    m, st = oracle.hemisphere_init(K // 8, pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, 5, mode=1)
    s = oracle.Samples(b["x"], b["w"])
    for _ in range(iters):
        oracle.optimize(m, st, s, accurate=True)
    return b, m


def _uniform_sphere(rng, n):
    v = rng.normal(size=(n, 3))
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


def test_p3_product_pdf_integrates_to_one(oracle, synth):
    b, m = _fitted(oracle, synth)
    bw, bmean, bcov = synth.bsdf_table(2, 3)
    c, _ = synth.sample_queries_near(b, 6)
    F = synth.shading_frames(6)
    rng = np.random.default_rng(1)
    n = 100000
    d = _uniform_sphere(rng, n)
    for q in range(6):
        cq = np.repeat(c[:, q][None], n, 0)
        Fq = np.repeat(F[q][None], n, 0)
        mat = np.full(n, q % 2, np.int32)
        _, pdf, _, h = oracle.guide_product_batch(m, cq, np.zeros((n, 3)), mat, Fq, bw, bmean, bcov, dgiven=d)
        if h[0] != np.float32(0.3):
            continue
        integral = pdf.mean() * 4 * np.pi
        # tangent Gaussians with sd up to 0.6 lose a little mass past the
        # antipode and through the exp-map Jacobian; the product is narrower
        assert abs(integral - 1.0) < 0.05, integral


def test_p4_batch_rules(oracle, synth):
    b, m = _fitted(oracle, synth)
    bw, bmean, bcov = synth.bsdf_table(3, 4)
    nq = 600
    c, u = synth.sample_queries_near(b, nq // 2)
    c2, u2 = synth.queries(nq // 2)
    c = np.concatenate([c, c2], 1).T
    u = np.concatenate([u, u2], 1).T
    F = synth.shading_frames(nq)
    none = np.full(nq, -1, np.int32)
    d, pdf, comp, h = oracle.guide_product_batch(m, c, u, none, F, bw, bmean, bcov)
    dr, pr, cr, _ = oracle.guide_batch(m, c, u)
    valid = cr >= 0
    np.testing.assert_array_equal(comp, cr)
    np.testing.assert_array_equal(pdf, pr)
    np.testing.assert_array_equal(d, dr)
    np.testing.assert_array_equal(h, np.where(valid, 0.5, 1.0).astype(np.float32))
    mat = (np.arange(nq) % 3).astype(np.int32)
    d, pdf, comp, h = oracle.guide_product_batch(m, c, u, mat, F, bw, bmean, bcov)
    assert set(np.unique(h).tolist()) <= {float(np.float32(0.3)), 0.5, 1.0}
    assert (h == np.float32(0.3)).mean() > 0.4
    assert ((h == 1.0) == ~valid).all()
    prod = h == np.float32(0.3)
    M = bw.shape[1]
    assert (comp[prod] >= 0).all() and (comp[prod] % M < M).all() and (comp[prod] // M < m.K).all()
    np.testing.assert_allclose(np.linalg.norm(d[prod], axis=1), 1.0, atol=1e-5)
    assert (pdf[prod] > 0).all()
    # pdf of the given (sampled) directions == the pdf returned with the sample
    _, pg, _, hg = oracle.guide_product_batch(m, c, u, mat, F, bw, bmean, bcov, dgiven=d)
    np.testing.assert_array_equal(hg, h)
    np.testing.assert_array_equal(pg[prod], pdf[prod])


def test_p5_samples_follow_the_pdf(oracle, synth):
    b, m = _fitted(oracle, synth)
    bw, bmean, bcov = synth.bsdf_table(1, 3, seed=11)
    c, _ = synth.sample_queries_near(b, 4, seed=3)
    F = synth.shading_frames(4, seed=5)
    rng = np.random.default_rng(2)
    n = 40000
    for q in range(4):
        cq = np.repeat(c[:, q][None], n, 0)
        Fq = np.repeat(F[q][None], n, 0)
        mat = np.zeros(n, np.int32)
        u = rng.uniform(0, 1, size=(n, 3)).astype(np.float32)
        d, pdf, comp, h = oracle.guide_product_batch(m, cq, u, mat, Fq, bw, bmean, bcov)
        if h[0] != np.float32(0.3):
            continue
        # E[d] from the samples vs from importance-weighted uniform directions
        du = _uniform_sphere(rng, 400000)
        _, pu, _, _ = oracle.guide_product_batch(m, np.repeat(c[:, q][None], len(du), 0), np.zeros((len(du), 3)),
                                                 np.zeros(len(du), np.int32), np.repeat(F[q][None], len(du), 0),
                                                 bw, bmean, bcov, dgiven=du)
        ref = (du * pu[:, None]).mean(0) * 4 * np.pi / ((pu.mean()) * 4 * np.pi)
        np.testing.assert_allclose(d.mean(0), ref, atol=0.02)
