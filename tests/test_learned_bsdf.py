"""A glossy material's learned BSDF (sdmm_learned_bsdf4, csrc/learned_bsdf.h):
the reference's BSDF::SDMM4 (bsdf.h:310-314) conditioned per bounce by
RoughConductor::getDMM on (theta_i, alpha) with
sdmm::create_conditional_pruned(..., 2) (roughconductor.cpp:182-194), then
rotate_to_wo(wi) (sdmm_proc.cpp:340-355).  sdmm-lib is absent, so the
semantics are this library's stated reading; these CPU tests pin the library's
host path (sdmm_learned4_conditional, the same code the device runs) against
the oracle's C restatement bitwise, and both against analytic known answers
(a Gaussian conditional computed in float64 here), plus the JSON loader.
Parity against sdmm-lib itself: unpinned (no fixture exists)."""
import numpy as np
import pytest


def _coords(n):
    n = np.asarray(n, np.float64)
    s = np.copysign(1.0, n[2])
    a = -1.0 / (s + n[2])
    b = n[0] * n[1] * a
    return np.array([[1 + s * n[0] * n[0] * a, s * b, -s * n[0]], [b, s + n[1] * n[1] * a, -n[1]], n])


def _wi(rng, n):
    th = rng.uniform(0.0, 1.55, n)
    ph = rng.uniform(0.0, 2 * np.pi, n)
    return np.stack([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)], 1).astype(np.float32)


def test_json_round_trip(pkg, scenes, tmp_path):
    m = scenes.load_learned()
    L = pkg.LearnedBSDF(*m)
    for a, b in zip(L.arrays(), pkg.LearnedBSDF.load_json(scenes.LEARNED_CONDUCTOR).arrays()):
        np.testing.assert_array_equal(a, b)
    L.save_json(tmp_path / "m.sdmm4.json")
    for a, b in zip(L.arrays(), pkg.LearnedBSDF.load_json(tmp_path / "m.sdmm4.json").arrays()):
        np.testing.assert_array_equal(a, b)
    (tmp_path / "bad.json").write_text('{"format": "sdmm-amd.asdmm", "version": 1}')
    with pytest.raises(pkg.SDMMError):
        pkg.LearnedBSDF.load_json(tmp_path / "bad.json")


@pytest.mark.parametrize("keep", [1, 2, 4])
def test_host_conditional_equals_oracle_bitwise(pkg, oracle, scenes, keep):
    m = scenes.load_learned()
    L = pkg.LearnedBSDF(*m)
    rng = np.random.default_rng(keep)
    W = _wi(rng, 1500)
    counts = np.zeros(keep + 1, int)
    for i, wl in enumerate(W):
        alpha = float((0.03, 0.2, 0.6)[i % 3])
        a = L.conditional(alpha, wl, keep)
        b = oracle.learned4_conditional(m, alpha, wl, keep)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
        counts[len(a[0])] += 1
        if len(a[0]):
            np.testing.assert_allclose(a[0].sum(), 1.0, rtol=2e-6)
            np.testing.assert_allclose(np.linalg.norm(a[1], axis=1), 1.0, rtol=2e-6)
            assert (a[2][:, 0] > 0).all() and (a[2][:, 0] * a[2][:, 3] - a[2][:, 1] ** 2 > 0).all()
            assert (np.diff(a[0]) <= 0).all()          # pruned in decreasing weight
    assert counts[keep] == len(W)                       # the synthetic model covers every condition


def test_conditional_known_answers(pkg, oracle):
    """One component with a full 4x4 covariance: weight 1; the mean is the
    exponential map at mu_d of S_dc S_cc^-1 (x - mu_c), rotated onto wi's
    azimuth; the covariance is S_dd - S_dc S_cc^-1 S_cd (float64 here)
    carried to Coordinates(mean') by parallel transport -- an isometry, so its
    eigenvalues are the conditional's."""
    th0, al0 = 0.6, 0.2
    mu = np.float32([-np.sin(0.6), 0.0, np.cos(0.6)])
    A = np.float64([[0.3, 0, 0, 0], [0.05, 0.1, 0, 0], [-0.25, 0.02, 0.15, 0], [0.03, -0.01, 0.02, 0.12]])
    cov = (A @ A.T).astype(np.float32)
    model = (np.float32([1.0]), np.float32([[th0, al0, *mu]]), cov.reshape(1, 16))
    L = pkg.LearnedBSDF(*model)
    for th, al in ((0.6, 0.2), (0.75, 0.25), (0.4, 0.1)):
        wl = np.float32([np.sin(th), 0.0, np.cos(th)])   # azimuth 0: rotate_to_wo is the identity
        w, mean, c = L.conditional(al, wl, 2)
        assert len(w) == 1 and w[0] == 1.0
        C = cov.astype(np.float64)
        Scc, Sdc, Sdd = C[:2, :2], C[2:, :2], C[2:, 2:]
        shift = Sdc @ np.linalg.solve(Scc, np.float64([th - th0, al - al0]))
        T = _coords(mu)
        ln = np.linalg.norm(shift)
        d = np.cos(ln) * mu + (np.sin(ln) / ln if ln > 0 else 1.0) * (shift[0] * T[0] + shift[1] * T[1])
        np.testing.assert_allclose(mean[0], d, atol=2e-6)
        # S'_dd in Coordinates(mean') from mu's axes parallel-transported
        cond = Sdd - Sdc @ np.linalg.solve(Scc, Sdc.T)
        if ln > 0:
            u = shift / ln
            u3 = u[0] * T[0] + u[1] * T[1]
            g = (np.cos(ln) - 1) * u3 - np.sin(ln) * T[2]
            E = np.stack([T[0] + u[0] * g, T[1] + u[1] * g])
        else:
            E = T[:2]
        Td = _coords(d / np.linalg.norm(d))
        B = Td[:2] @ E.T
        want = B @ cond @ B.T
        got = np.float64([[c[0, 0], c[0, 1]], [c[0, 2], c[0, 3]]])
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(np.linalg.eigvalsh(got), np.linalg.eigvalsh(cond), rtol=1e-5)
        b = oracle.learned4_conditional(model, al, wl, 2)
        for x, y in zip((w, mean, c), b):
            np.testing.assert_array_equal(x, y)


def test_conditional_pruning_and_invalid(pkg):
    """Two identical components: the tie keeps the lower index first, both at
    weight 1/2; a condition far outside every component (densities underflow
    to 0), a non-PD S_cc, or cos theta_i <= 0: no valid conditional."""
    mu = np.float32([0.0, 0.0, 1.0])
    cov = np.diag(np.float32([0.01, 0.01, 0.04, 0.04])).reshape(16)
    two = pkg.LearnedBSDF(np.float32([0.5, 0.5]), np.float32([[0.3, 0.2, *mu]] * 2), np.stack([cov, cov]))
    w, m, c = two.conditional(0.2, np.float32([np.sin(0.3), 0, np.cos(0.3)]), 2)
    assert len(w) == 2 and (w == np.float32(0.5)).all()
    assert len(two.conditional(0.2, np.float32([np.sin(0.3), 0, np.cos(0.3)]), 1)[0]) == 1
    tight = np.diag(np.float32([1e-6, 1e-6, 0.04, 0.04])).reshape(16)
    far = pkg.LearnedBSDF(np.float32([1.0]), np.float32([[0.1, 0.1, *mu]]), tight[None])
    assert len(far.conditional(0.9, np.float32([np.sin(1.2), 0, np.cos(1.2)]), 2)[0]) == 0
    bad = cov.copy().reshape(4, 4)
    bad[0, 1] = bad[1, 0] = 0.02                      # |rho| > 1: S_cc not PD
    npd = pkg.LearnedBSDF(np.float32([1.0]), np.float32([[0.3, 0.2, *mu]]), bad.reshape(1, 16))
    assert len(npd.conditional(0.2, np.float32([0.2, 0, 0.97]), 2)[0]) == 0
    assert len(two.conditional(0.2, np.float32([0.2, 0, -0.97]), 2)[0]) == 0


def test_scene_rejects_invalid_learned_model(pkg, scenes):
    desc = scenes.cornell_box(32, 18, conductor=("Floor",))
    w, mu, cv = scenes.load_learned()
    mu = mu.copy()
    mu[0, 2:] *= 1.5                                  # a non-unit direction
    f = list(scenes._BSDFS).index("Floor")
    desc["learned_models"][f] = (w, mu, cv)
    with pytest.raises(pkg.SDMMError):
        pkg.Scene(desc)
