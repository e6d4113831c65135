"""CPU: the oracle reproduces the committed golden fixtures bit for bit.

tests/golden/*.npz were produced by tests/golden/make_golden.py from the oracle
(the reference has no golden vectors for this path -- SURVEY.md 8(c)); this
test pins the oracle against regressions.  tests/test_gpu_golden.py checks the
HIP path against the same fixtures."""
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"


def _load(name):
    return dict(np.load(GOLDEN / name))


@pytest.mark.parametrize("K", [16, 128])
def test_golden_estep(oracle, K):
    g = _load(f"golden_estep_K{K}.npz")
    m, st = oracle.hemisphere_init(K // 8, g["seed_pos"], g["seed_nrm"], 0.01, 0.1, 0x1A17, mode=1)
    for f in ("weights", "mean", "cov", "to", "cholLInv", "detInv", "muPremult", "condL", "margL"):
        np.testing.assert_array_equal(np.asarray(getattr(m, f)), g["init_" + f], err_msg=f)
    s = oracle.Samples(g["x"], g["w"], g["hpdf"], g["is_diffuse"])
    np.testing.assert_array_equal(oracle.responsibilities(m, s), g["resp"])
    for mode in ("faithful", "accurate", "exact"):
        np.testing.assert_array_equal(oracle.calculate_stats(m, s, accurate=mode), g["stats_" + mode])


def test_golden_em_and_guide(oracle):
    g = _load("golden_em_K16.npz")
    K = 16
    s = oracle.Samples(g["x"], g["w"])
    for mode in ("exact", "faithful"):
        m, st = oracle.hemisphere_init(K // 8, g["seed_pos"], g["seed_nrm"], 0.01, 0.1, 0x1A17,
                                       mode=0 if mode == "faithful" else 1)
        for _ in range(3):
            assert oracle.optimize(m, st, s, accurate=mode) == 1
        for f in ("weights", "cdf", "mean", "cov", "cholLInv", "condLInv"):
            np.testing.assert_array_equal(np.asarray(getattr(m, f)), g[f"em_{mode}_" + f], err_msg=f)
        if mode == "exact":
            d, pdf, comp, slot = oracle.guide_batch(m, g["q_c"].T, g["q_u"].T)
            np.testing.assert_array_equal(comp, g["q_comp"])
            np.testing.assert_array_equal(slot, g["q_slot"])
            np.testing.assert_array_equal(d, g["q_dir"])
            np.testing.assert_array_equal(pdf, g["q_pdf"])
            np.testing.assert_array_equal(oracle.pdf_batch(m, g["q_c"].T, d), g["pdf_at_dir"])


def test_golden_fixture_sanity():
    g = _load("golden_em_K16.npz")
    w = g["em_exact_weights"]
    assert abs(float(w.sum()) - 1.0) < 1e-5 and (w >= 0).all()
    assert (g["q_comp"] >= -1).all() and (g["q_comp"] < 16).all()
    ok = g["q_comp"] >= 0
    np.testing.assert_allclose(np.linalg.norm(g["q_dir"][ok], axis=1), 1.0, atol=1e-5)
    e = _load("golden_estep_K128.npz")
    live = e["resp"].sum(1) > 0
    assert live.mean() > 0.5
