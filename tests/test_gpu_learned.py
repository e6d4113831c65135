"""GPU: the conductor's learned BSDF conditioned on the device
(sdmm_learned4_conditional_device; the same learned_bsdf.h code the render's
product bounces run in li_compact_kernel) -- getDMM on (theta_i, alpha),
pruned to 2, rotate_to_wo (roughconductor.cpp:182-194, sdmm_proc.cpp:340-355)
-- BITWISE the oracle's C restatement (oracle/sdmm_oracle_li.inc
li_learned_conditional) and the host ABI, lobe counts, weights, means and
covariances, over incident directions on and below the horizon."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("keep", [2, 3])
def test_device_learned_conditional_equals_oracle(pkg, oracle, scenes, gpu, plog, keep):
    import torch
    m = scenes.load_learned()
    L = pkg.LearnedBSDF(*m)
    rng = np.random.default_rng(11 + keep)
    nq = 1 << 16
    th = rng.uniform(0.0, 1.75, nq)                      # some below the horizon: no valid getDMM
    ph = rng.uniform(0.0, 2 * np.pi, nq)
    W = np.stack([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)]).astype(np.float32)
    Wt = [torch.from_numpy(W[i].copy()).to(gpu) for i in range(3)]
    mism = 0
    for alpha in (0.05, 0.2, 0.6):
        w, mean, cov, n = L.conditional_device(alpha, Wt, keep)
        torch.cuda.synchronize()
        w, mean, cov, n = (x.cpu().numpy() for x in (w, mean, cov, n))
        assert (n[W[2] <= 0] == 0).all() and (n[W[2] > 0] == keep).all()
        for q in rng.choice(nq, 3000, replace=False):
            ow, om, oc = oracle.learned4_conditional(m, alpha, W[:, q], keep)
            k = len(ow)
            assert n[q] == k
            same = (np.array_equal(w[q, :k], ow) and np.array_equal(mean[q, :k], om) and
                    np.array_equal(cov[q, :k], oc))
            mism += 0 if same else 1
            if q % 7 == 0:
                hw, hm, hc = L.conditional(alpha, W[:, q], keep)
                np.testing.assert_array_equal(hw, ow)
                np.testing.assert_array_equal(hm, om)
                np.testing.assert_array_equal(hc, oc)
    plog(f"learned4_device_vs_oracle_mismatches_keep{keep}", mism, 0)
    assert mism == 0
