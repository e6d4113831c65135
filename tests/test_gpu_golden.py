"""GPU vs the committed golden fixtures (tests/golden/, made by the oracle)."""
from pathlib import Path

import numpy as np
import pytest

from helpers import estep_f64, posterior_f64
from test_gpu_parity import check_explained

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"


def _load(name):
    return dict(np.load(GOLDEN / name))


@pytest.mark.parametrize("K", [16, 128])
def test_gpu_estep_vs_golden(pkg, gpu, plog, K):
    import torch
    g = _load(f"golden_estep_K{K}.npz")
    mix = pkg.SDMM(K)
    mix.init_hemisphere(g["seed_pos"], g["seed_nrm"], 0.01, 0.1, 0x1A17)
    p = mix.get_params()
    for f in ("weights", "mean", "cov", "to", "detInv"):
        np.testing.assert_allclose(p[f], g["init_" + f], rtol=2e-6, atol=1e-7, err_msg=f)
    ds = pkg.DeviceSamples.from_numpy(g["x"], g["w"], g["hpdf"], g["is_diffuse"])
    N = g["w"].shape[0]
    resp = torch.empty((N, K), device=gpu)
    mix.posterior(ds, resp)
    got = resp.cpu().numpy()
    # the golden responsibilities (fp32 oracle) and the GPU's, both judged by
    # the fp64 evaluation of the same float parameters with the fixture's
    # heuristic mix on its diffuse rows (test_gpu_parity._check_resp)
    exact, q, c = posterior_f64(p, g["x"], g["hpdf"], g["is_diffuse"], return_qc=True)
    live_g, live_got = g["resp"].sum(1) > 0, got.sum(1) > 0
    # a row the fixture explains is explained here and vice versa: no row is
    # live on one side and all-zero on the other (and the fixture has live
    # rows to compare: 25 % at K = 16, most at K = 128)
    assert not np.any(live_g != live_got), int(np.sum(live_g != live_got))
    assert live_g.sum() >= 200
    live = live_g
    eg = np.abs(got[live] - exact[live]).max()
    eo = np.abs(g["resp"][live] - exact[live]).max()
    plog("golden_resp_abs_err_vs_fp64", eg, 4 * eo + 1e-5, golden_fp32_err=eo)
    # the flat 2e-5 bound on the explained, well-conditioned rows, against the
    # fp64 evaluation and against the committed fixture
    check_explained(got, g["resp"], exact, q, c, plog, tag=f"golden_K{K}")
    # and against the committed fixture itself: 1e-4 absolute (both evaluate the
    # same float parameters in fp32; where the fp64 evaluation departs from both
    # -- different FTZ flush points of tiny densities -- they still agree)
    dg = np.abs(got[live] - g["resp"][live]).max()
    plog("golden_resp_abs_diff_vs_golden", dg, 1e-4)
    assert eg <= 4 * eo + 1e-5
    assert dg <= 1e-4
    st = torch.zeros(pkg.stats_len(K), dtype=torch.float64, device=gpu)
    mix.estep_stats(ds, st)
    s = st.cpu().numpy()
    ex = g["stats_exact"]
    W, Wx = s[2:2 + K], ex[2:2 + K]
    ew = np.abs(W - Wx).max() / ex[1]
    plog("golden_stats_W_rel_err_vs_exact", ew, 1e-6,
         golden_fp32_err=np.abs(g["stats_faithful"][2:2 + K] - Wx).max() / ex[1])
    assert ew <= 1e-6
    np.testing.assert_allclose(s[1], ex[1], rtol=1e-6)


def test_gpu_guide_vs_golden(pkg, gpu):
    import torch
    g = _load("golden_em_K16.npz")
    K = 16
    mix = pkg.SDMM(K)
    mix.set_params(g["em_exact_weights"], g["em_exact_mean"], g["em_exact_cov"])
    p = mix.get_params()
    np.testing.assert_array_equal(p["weights"], g["q2_weights"])
    c = [torch.from_numpy(g["q_c"][i].copy()).to(gpu) for i in range(3)]
    u = [torch.from_numpy(g["q_u"][i].copy()).to(gpu) for i in range(3)]
    d, pdf, comp = mix.guide(c, u)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(comp.cpu().numpy(), g["q2_comp"])     # bit-exact selection
    dg = np.stack([t.cpu().numpy() for t in d], 1)
    np.testing.assert_allclose(dg, g["q2_dir"], atol=1e-5)
    np.testing.assert_allclose(pdf.cpu().numpy(), g["q2_pdf"], rtol=1e-4, atol=1e-7)
