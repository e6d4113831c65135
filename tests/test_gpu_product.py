"""GPU: product sampling with a learned BSDF (sdmm_guide_product_batch /
sdmm_pdf_product_batch, guide.hip guide_product_kernel) against the oracle's
restatement of jmm MixtureModel::multiply (oracle/sdmm_oracle_product.inc):

  * heuristicConditionalWeight per query (0.3 product / 0.5 conditional /
    1 BSDF only, sdmm_proc.cpp:383-392): equal;
  * the sampled index (k * M + j for product samples, the joint index for
    plain-conditional samples): BIT-EXACT;
  * product samples and their pdfs: the kernel follows the oracle op for op
    with the oracle's correctly rounded transcendentals -> 1e-6 abs / 1e-5 rel
    (plain-conditional samples keep the guide's 1e-5 / 1e-4 tolerances);
  * pdf of given directions: 1e-5 rel (product) / 1e-4 rel (conditional).
Parity against sdmm-lib is unpinned (absent); tests/test_product.py pins the
oracle with analytic KATs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _model(pkg, oracle, synth, K, iters, N=8192):
    b = synth.em_batch(N, 128)
    pos, nrm = synth.model_seed_points(b, K)
    mix = pkg.SDMM(K)
    mix.init_hemisphere(pos[:K // 8], nrm[:K // 8], synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, synth.SEED_MODEL)
    ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"])
    for _ in range(iters):
        mix.optimize(ds)
    p = mix.get_params()
    m = oracle.Mixture(K)
    m.copy_params_from(p)
    m.valid[:] = p["valid"]
    return b, mix, m


@pytest.mark.parametrize("K,iters,B,M,cap,nq", [(16, 3, 3, 4, 40, 3000), (128, 4, 2, 6, 40, 3000),
                                                (64, 2, 1, 1, 40, 3000),
                                                # the Kitchen config: K=512 x 8 materials x 8 lobes
                                                (512, 2, 8, 8, 64, 2000), (512, 2, 8, 8, 40, 2000),
                                                # candidate capacity 0: every query through the
                                                # full-K fallback kernel of the product path
                                                (128, 4, 2, 6, 0, 1500), (512, 2, 8, 8, 0, 1000)])
def test_product_matches_oracle(pkg, oracle, synth, gpu, plog, K, iters, B, M, cap, nq):
    import torch
    b, mix, om = _model(pkg, oracle, synth, K, iters)
    mix.set_guide_capacity(cap)
    bw, bmean, bcov = synth.bsdf_table(B, M, seed=K)
    c, u = synth.sample_queries_near(b, nq * 2 // 3)
    c2, u2 = synth.queries(nq - nq * 2 // 3)
    c = np.concatenate([c, c2], 1)
    u = np.concatenate([u, u2], 1)
    F = synth.shading_frames(nq, seed=K + 1)
    mat = ((np.arange(nq) % (B + 1)) - 1).astype(np.int32)          # -1: no learned BSDF
    tt = lambda a: [torch.from_numpy(np.ascontiguousarray(a[i])).to(gpu) for i in range(a.shape[0])]
    ct, ut, Ft = tt(c), tt(u), tt(F.T)
    matt = torch.from_numpy(mat).to(gpu)
    table = pkg.BsdfTable(bw, bmean, bcov, device=gpu)
    d, pdf, comp, h = mix.guide_product(ct, ut, table, matt, Ft)
    torch.cuda.synchronize()
    dg = np.stack([x.cpu().numpy() for x in d], 1)
    pg, cg, hg = pdf.cpu().numpy(), comp.cpu().numpy(), h.cpu().numpy()
    dr, pr, cr, hr = oracle.guide_product_batch(om, c.T, u.T, mat, F, bw, bmean, bcov)
    prod = hr == np.float32(0.3)
    cond = hr == np.float32(0.5)
    plog("product_heuristic_mismatches", int((hg != hr).sum()), 0)
    plog("product_index_mismatches", int((cg != cr).sum()), 0, product_frac=float(prod.mean()))
    if prod.any():
        plog("product_dir_abs_err", np.abs(dg[prod] - dr[prod]).max(), 1e-6)
        plog("product_pdf_err_over_tol(1e-5 rel + 1e-8 abs)",
             (np.abs(pg[prod] - pr[prod]) / (1e-8 + 1e-5 * np.abs(pr[prod]))).max(), 1.0)
    np.testing.assert_array_equal(hg, hr)
    np.testing.assert_array_equal(cg, cr)                 # bit-exact index selection
    assert prod.mean() > 0.3 and cond.sum() > 0
    np.testing.assert_allclose(dg[prod], dr[prod], atol=1e-6)
    np.testing.assert_allclose(pg[prod], pr[prod], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(dg[cond], dr[cond], atol=1e-5)
    np.testing.assert_allclose(pg[cond], pr[cond], rtol=1e-4, atol=1e-7)
    bsdf_only = hr == 1.0
    assert (cg[bsdf_only] == -1).all() and (pg[bsdf_only] == 0).all()
    # pdfSurface with the product: pdf of given directions
    rng = np.random.default_rng(K)
    dd = rng.normal(size=(nq, 3)).astype(np.float32)
    dd /= np.linalg.norm(dd, axis=1, keepdims=True)
    dd[::3] = dr[::3]                                       # and the sampled directions themselves
    pq, hq = mix.pdf_product(ct, tt(dd.T), table, matt, Ft)
    torch.cuda.synchronize()
    _, prq, _, hrq = oracle.guide_product_batch(om, c.T, u.T, mat, F, bw, bmean, bcov, dgiven=dd)
    np.testing.assert_array_equal(hq.cpu().numpy(), hrq)
    pq = pq.cpu().numpy()
    np.testing.assert_allclose(pq[prod], prq[prod], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(pq[cond], prq[cond], rtol=1e-4, atol=1e-7)


def test_product_argument_errors(pkg, synth, gpu):
    import torch
    mix = pkg.SDMM(16)
    b = synth.em_batch(512, 128)
    pos, nrm = synth.model_seed_points(b, 16)
    mix.init_hemisphere(pos[:2], nrm[:2], synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, 1)
    bw, bmean, bcov = synth.bsdf_table(1, 65)
    table = pkg.BsdfTable(bw, bmean, bcov, device=gpu)
    z = [torch.zeros(4, device=gpu) for _ in range(9)]
    with pytest.raises(pkg.SDMMError):
        mix.guide_product(z[:3], z[:3], table, torch.zeros(4, dtype=torch.int32, device=gpu), z)
