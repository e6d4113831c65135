"""Product sampling over the spatial tree's leaves (sdmm_guide_product_wavefront
/ sdmm_pdf_product_wavefront): sampleSurface / pdfSurface with sampleProduct
for a wavefront of bounces (sdmm_proc.cpp:309-392, :474-502) -- find the
query's leaf (:314), multiply that leaf's conditional by the query material's
learned-BSDF lobes (:327-381), sample / evaluate the product (h = 0.3), the
plain conditional (h = 0.5) or BSDF only (h = 1).

Parity against the oracle (oracle/sdmm_oracle_product.inc) on each query's own
leaf (node ids from the oracle's tree find): heuristic weights equal, sampled
indices BIT-EXACT (k * M + j for product samples), product directions / pdfs
within 1e-6 abs / 1e-5 rel and plain-conditional ones within 1e-5 / 1e-4 rel
(the tolerances of test_gpu_product.py); queries without a trained leaf are
BSDF only.  Also: the mixed bounce (choice + dgiven, a pdf query where
choice <= h) against the oracle's mixed mode, diffuse materials (the plugin's
slice-0 rule), K = 16 and the Kitchen's K = 512 x 8 materials x 8 lobes, at
candidate capacity 40 and 0 (every query through the full-K wave kernel)."""
import numpy as np
import pytest

from test_gpu_wavefront import _queries, _tree_and_leaf_mixtures

pytestmark = pytest.mark.gpu


def _check(plog, tag, hg, hr, cg, cr, dg, dr, pg, pr):
    prod = hr == np.float32(0.3)
    cond = hr == np.float32(0.5)
    plog(f"{tag}_heuristic_mismatches", int((hg != hr).sum()), 0)
    plog(f"{tag}_index_mismatches", int((cg != cr).sum()), 0, product_frac=float(prod.mean()))
    np.testing.assert_array_equal(hg, hr)
    np.testing.assert_array_equal(cg, cr)
    if prod.any():
        plog(f"{tag}_product_dir_abs_err", float(np.abs(dg[prod] - dr[prod]).max()), 1e-6)
    np.testing.assert_allclose(dg[prod], dr[prod], atol=1e-6)
    np.testing.assert_allclose(pg[prod], pr[prod], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(dg[cond], dr[cond], atol=1e-5)
    np.testing.assert_allclose(pg[cond], pr[cond], rtol=1e-4, atol=1e-7)
    only = hr == 1.0
    assert (cg[only] == -1).all() and (pg[only] == 0).all()
    return prod, cond


@pytest.mark.parametrize("K,B,M,cap,nq", [(16, 4, 3, 40, 1 << 14), (16, 4, 3, 0, 3000),
                                          (512, 8, 8, 64, 2000), (512, 8, 8, 40, 2000),
                                          (512, 8, 8, 0, 1000)])
def test_product_wavefront_matches_oracle(pkg, oracle, synth, gpu, plog, K, B, M, cap, nq):
    import torch
    b, t, mixes, leaves = _tree_and_leaf_mixtures(pkg, synth, K, iters=2 if K <= 64 else 1)
    for m in mixes:
        if m is not None:
            m.set_guide_capacity(cap)
    c, u, d, ct, ut, dt = _queries(gpu, nq, 21, 0.0, 1.0)
    bw, bmean, bcov = synth.bsdf_table(B, M, seed=K + 3)
    diffuse = (np.arange(B) % 3 == 1).astype(np.uint8)            # some diffuse materials
    F = synth.shading_frames(nq, seed=K + 5)
    mat = ((np.arange(nq) % (B + 1)) - 1).astype(np.int32)          # -1: no learned BSDF
    tt = lambda a: [torch.from_numpy(np.ascontiguousarray(a[i])).to(gpu) for i in range(a.shape[0])]
    Ft = tt(F.T)
    matt = torch.from_numpy(mat).to(gpu)
    table = pkg.BsdfTable(bw, bmean, bcov, device=gpu, diffuse=diffuse)
    node = torch.empty(nq, dtype=torch.int32, device=gpu)
    dw, pw, cw, hw = t.guide_product(mixes, ct, ut, table, matt, Ft, node_out=node)
    # the mixed bounce: BSDF-sampled directions d, choices
    choice = np.random.default_rng(K).uniform(0, 1, nq).astype(np.float32)
    chw = torch.from_numpy(choice).to(gpu)
    dmw, pmw, cmw, hmw = t.guide_product(mixes, ct, ut, table, matt, Ft, choice=chw, dgiven=dt)
    pdw, hpw = t.pdf_product(mixes, ct, dt, table, matt, Ft)
    torch.cuda.synchronize()
    node = node.cpu().numpy()
    aabb, child, _ = t.nodes()
    np.testing.assert_array_equal(node, oracle.stree_find(aabb, child, c.T.copy()))
    np_ = lambda x: x.cpu().numpy()
    dw, dmw = np.stack([np_(x) for x in dw], 1), np.stack([np_(x) for x in dmw], 1)
    pw, cw, hw, pmw, cmw, hmw, pdw, hpw = map(np_, (pw, cw, hw, pmw, cmw, hmw, pdw, hpw))
    has = np.array([(v >= 0 and mixes[v] is not None) for v in node])
    assert has.sum() > nq // 2 and (~has).sum() > 0
    for arr_c, arr_h, arr_p in ((cw, hw, pw), (cmw, hmw, pmw)):
        assert (arr_c[~has] == -1).all() and (arr_h[~has] == 1).all() and (arr_p[~has] == 0).all()
    assert (pdw[~has] == 0).all() and (hpw[~has] == 1).all()
    nprod = nmix = 0
    for v in np.unique(node[has]):
        sel = np.nonzero(node == v)[0]
        p = mixes[v].get_params()
        om = oracle.Mixture(mixes[v].K)
        om.copy_params_from(p)
        om.valid[:] = p["valid"]
        args = (om, c[:, sel].T.copy(), u[:, sel].T.copy(), mat[sel], F[sel], bw, bmean, bcov)
        dr, pr, cr, hr = oracle.guide_product_batch(*args, diffuse=diffuse)
        prod, _ = _check(plog, "product_wavefront", hw[sel], hr, cw[sel], cr, dw[sel], dr, pw[sel], pr)
        nprod += int(prod.sum())
        dsel = d[:, sel].T.copy()
        dr, pr, cr, hr = oracle.guide_product_batch(*args, dgiven=dsel, diffuse=diffuse, choice=choice[sel])
        _check(plog, "product_wavefront_mixed", hmw[sel], hr, cmw[sel], cr, dmw[sel], dr, pmw[sel], pr)
        nmix += int((cr == -2).sum())
        _, pr, _, hr = oracle.guide_product_batch(*args, dgiven=dsel, diffuse=diffuse)
        np.testing.assert_array_equal(hpw[sel], hr)
        pp = hr == np.float32(0.3)
        np.testing.assert_allclose(pdw[sel][pp], pr[pp], rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(pdw[sel][~pp], pr[~pp], rtol=1e-4, atol=1e-7)
    assert nprod > has.sum() // 4 and nmix > 0


def test_product_wavefront_equals_per_leaf_batch(pkg, synth, gpu):
    """Every query's outputs are BITWISE those of sdmm_guide_product_batch
    against its own leaf's mixture."""
    import torch
    b, t, mixes, leaves = _tree_and_leaf_mixtures(pkg, synth, 16)
    nq = 1 << 14
    c, u, d, ct, ut, dt = _queries(gpu, nq, 23, 0.0, 1.0)
    B, M = 3, 4
    bw, bmean, bcov = synth.bsdf_table(B, M, seed=7)
    F = synth.shading_frames(nq, seed=8)
    mat = ((np.arange(nq) % (B + 1)) - 1).astype(np.int32)
    Ft = [torch.from_numpy(np.ascontiguousarray(F.T[i])).to(gpu) for i in range(9)]
    matt = torch.from_numpy(mat).to(gpu)
    table = pkg.BsdfTable(bw, bmean, bcov, device=gpu)
    node = torch.empty(nq, dtype=torch.int32, device=gpu)
    dw, pw, cw, hw = t.guide_product(mixes, ct, ut, table, matt, Ft, node_out=node)
    torch.cuda.synchronize()
    node = node.cpu().numpy()
    for v in np.unique(node):
        if v < 0 or mixes[v] is None:
            continue
        idx = torch.from_numpy(np.nonzero(node == v)[0]).to(gpu)
        dr, pr, cr, hr = mixes[v].guide_product([x[idx] for x in ct], [x[idx] for x in ut], table, matt[idx],
                                                [x[idx] for x in Ft])
        torch.cuda.synchronize()
        for a, r in ((cw[idx], cr), (pw[idx], pr), (hw[idx], hr)):
            np.testing.assert_array_equal(a.cpu().numpy(), r.cpu().numpy())
        for a, r in zip(dw, dr):
            np.testing.assert_array_equal(a[idx].cpu().numpy(), r.cpu().numpy())
