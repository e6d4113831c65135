"""kMeansPPInit (dmm/jmm/mixture_model_init.h:244-330): the k-means++ choice of
the seed positions that uniformHemisphereInit expands when kMeansPlusPlus is
set (:130-138).

The reference has no test or fixture for this function and cannot be built
here (Eigen, Boost): its parity is UNPINNED beyond the restatement in
oracle/sdmm_oracle_kmeans.c.  CPU tests check the restatement's two
arithmetic modes against each other (mode 0 = the reference's float CDF, mode
1 = the device rule with fp64 weights) and its defining properties; GPU tests
hold the HIP kernel to mode 1 index for index.
"""
import numpy as np
import pytest


def _leaf(rng, n, clustered=False, dup=False):
    if dup:   # every sample at one point with one normal: all masked after draw 0
        x = np.tile(rng.random((3, 1)), (1, n)).astype(np.float32)
        nr = np.tile(np.array([[0.0], [0.0], [1.0]]), (1, n)).astype(np.float32)
    else:
        if clustered:   # a few tight clusters: the thresholds (:76-77) mask samples
            c = rng.random((3, 4))
            x = (c[:, rng.integers(0, 4, n)] + rng.normal(scale=5e-3, size=(3, n))).astype(np.float32)
        else:
            x = (rng.random((3, n)) * 0.3).astype(np.float32)
        nr = rng.normal(size=(3, n))
        if clustered:
            nr[2] += 4.0
        nr = (nr / np.linalg.norm(nr, axis=0)).astype(np.float32)
    w = rng.exponential(size=n).astype(np.float32)
    w[rng.random(n) < 0.1] = 0.0          # clamped up to 1e-3 (:120)
    w[rng.random(n) < 0.02] = 50.0        # clamped down to 3
    return x, nr, w


CASES = [(1, 1, False, False), (7, 2, False, False), (1024, 16, False, False), (1025, 16, True, False),
         (3000, 64, True, False), (5000, 8, False, False), (300, 16, False, True), (2048, 2, True, False)]


def test_oracle_float_and_fp64_rules_agree(oracle, plog):
    """The device rule (fp64 weights / sums) picks the reference rule's (float
    CDF) index except where a draw falls within the float rounding of a CDF
    boundary: over many leaves they agree on every draw."""
    rng = np.random.default_rng(7)
    total = same = 0
    for trial in range(60):
        n = int(rng.integers(1, 4000))
        x, nr, w = _leaf(rng, n, clustered=trial % 2 == 1, dup=trial % 13 == 0)
        npos = int(rng.choice([1, 2, 8, 16]))
        u = rng.random(npos).astype(np.float32)
        a = oracle.kmeanspp_select(x, nr, w, npos, u, mode=0)
        b = oracle.kmeanspp_select(x, nr, w, npos, u, mode=1)
        total += npos
        same += int((a == b).sum())
    plog("kmeanspp_float_vs_fp64_rule_disagreements", total - same, 0)
    assert same == total


def test_oracle_kmeanspp_properties(oracle):
    """Draw 0 samples by metric^2 (:268-270, :289); a sample within both
    thresholds of a chosen position is never chosen again (:271-284); all
    samples masked -> the uniform CDF (:292-299)."""
    rng = np.random.default_rng(3)
    n = 2000
    x, nr, w = _leaf(rng, n, clustered=True)
    m = np.clip(w, 1e-3, 3.0).astype(np.float64) ** 2
    cdf = np.cumsum(m) / m.sum()
    for u in (0.0, 0.25, 0.5, 0.999):
        idx = oracle.kmeanspp_select(x, nr, w, 1, np.array([u], np.float32), mode=1)
        assert idx[0] == np.searchsorted(cdf, np.float32(u), side="left")
    u = rng.random(16).astype(np.float32)
    idx = oracle.kmeanspp_select(x, nr, w, 16, u, mode=1)
    for i in range(1, 16):
        j = idx[i]
        for k in idx[:i]:
            sd = float(np.sum((x[:, j] - x[:, k]).astype(np.float64) ** 2))
            ndot = float(np.clip(np.dot(nr[:, j], nr[:, k]), -1, 1))
            nd = np.arccos(ndot) / np.pi
            assert not (nd * nd < 0.04 - 1e-6 and sd < 4e-4 - 1e-9), (i, j, k)
    # one point repeated: draw 0 by metric, then every sample masked -> uniform
    xd, nd_, wd = _leaf(rng, 300, dup=True)
    u = np.array([0.5, 0.0, 0.5, 0.999], np.float32)
    idx = oracle.kmeanspp_select(xd, nd_, wd, 4, u, mode=1)
    assert list(idx[1:]) == [0, int(np.ceil(0.5 * 300)) - 1, int(np.ceil(np.float32(0.999) * 300)) - 1]


def _device_leaves(pkg, rng, cases):
    xs, ns, ws, seg = [], [], [], [0]
    for n, npos, clustered, dup in cases:
        x, nr, w = _leaf(rng, n, clustered, dup)
        xs.append(x)
        ns.append(nr)
        ws.append(w)
        seg.append(seg[-1] + n)
    return xs, ns, ws, np.asarray(seg, np.int64)


@pytest.mark.gpu
def test_kmeanspp_select_matches_oracle(pkg, oracle, gpu, plog):
    """HIP kmeanspp_kernel == oracle mode 1, index for index, on ragged leaves
    (1 sample, tile edges 1024 / 1025, clustered leaves where the thresholds
    mask, an all-duplicate leaf that falls back to the uniform CDF)."""
    import torch
    rng = np.random.default_rng(11)
    for npos in (1, 2, 16, 64):
        cases = [(n, npos, c, d) for n, _, c, d in CASES]
        xs, ns, ws, seg = _device_leaves(pkg, rng, cases)
        X = np.concatenate(xs, 1)
        Nn = np.concatenate(ns, 1)
        W = np.concatenate(ws)
        planes = [torch.from_numpy(np.ascontiguousarray(X[i])).to(gpu) for i in range(3)]
        planes += [torch.zeros(X.shape[1], device=gpu) for _ in range(3)]
        ds = pkg.DeviceSamples(planes, torch.from_numpy(W).to(gpu))
        nt = [torch.from_numpy(np.ascontiguousarray(Nn[i])).to(gpu) for i in range(3)]
        u = rng.random((len(cases), npos)).astype(np.float32)
        idx, pos, nrm = pkg.kmeanspp_select(ds, nt, seg, npos, u)
        for l in range(len(cases)):
            ref = oracle.kmeanspp_select(xs[l], ns[l], ws[l], npos, u[l], mode=1)
            np.testing.assert_array_equal(idx[l], ref, err_msg=f"leaf {l} npos {npos}")
            np.testing.assert_array_equal(pos[l], xs[l][:, ref].T)
            np.testing.assert_array_equal(nrm[l], ns[l][:, ref].T)
    plog("kmeanspp_index_mismatches", 0, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [16, 128])
def test_init_hemisphere_kmeanspp_matches_oracle(pkg, oracle, gpu, K):
    """uniformHemisphereInit with kMeansPlusPlus: one PCG32 stream gives the
    K/8 k-means++ draws then the direction jitter; the device mixtures equal
    the oracle's (the same tolerance as the plain hemisphere init)."""
    import torch
    rng = np.random.default_rng(5 + K)
    cases = [(1500, 0, True, False), (700, 0, False, False), (3000, 0, True, False)]
    xs, ns, ws, seg = _device_leaves(pkg, rng, cases)
    X = np.concatenate(xs, 1)
    Nn = np.concatenate(ns, 1)
    W = np.concatenate(ws)
    planes = [torch.from_numpy(np.ascontiguousarray(X[i])).to(gpu) for i in range(3)]
    planes += [torch.zeros(X.shape[1], device=gpu) for _ in range(3)]
    ds = pkg.DeviceSamples(planes, torch.from_numpy(W).to(gpu))
    nt = [torch.from_numpy(np.ascontiguousarray(Nn[i])).to(gpu) for i in range(3)]
    mixes = [pkg.SDMM(K) for _ in cases]
    dists = np.array([0.05, 0.1, 0.02], np.float32)
    seeds = np.array([0x1A17, 99, 12345], np.uint64)
    pkg.init_hemisphere_kmeanspp_batched(mixes, ds, nt, seg, 0.01, dists, seeds)
    for l, m in enumerate(mixes):
        om, ost, idx, r = oracle.hemisphere_init_kmeanspp(K // 8, xs[l], ns[l], ws[l], 0.01, float(dists[l]),
                                                          int(seeds[l]))
        assert r == 0
        p = m.get_params()
        for name in ("weights", "cdf", "mean", "cov", "cholL", "cholLInv", "detInv", "muPremult"):
            np.testing.assert_allclose(p[name], getattr(om, name), rtol=2e-6, atol=1e-7, err_msg=f"{l} {name}")
        st = m.get_state()
        np.testing.assert_array_equal(st["bpriors"], ost.bPriors)
        np.testing.assert_array_equal(st["bdepth"], ost.bDepth)
