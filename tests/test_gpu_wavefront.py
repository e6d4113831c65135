"""Guided wavefront over the spatial tree's leaves (sdmm_guide_wavefront /
sdmm_pdf_wavefront): SDMMRenderer::sampleSurface / pdfSurface for a batch of
bounces (sdmm_proc.cpp:309-421, :510-590) -- find the query's leaf
(STree.find, :314), guide against that leaf's mixture, BSDF-only when the
leaf has none (:316-323).

Parity: every query's outputs are BITWISE those of sdmm_guide_batch /
sdmm_pdf_batch against its own leaf's mixture, node ids equal
sdmm_stree_find's, and queries without a mixture give comp -1, pdf 0; and,
directly against the oracle, the node ids equal or_stree_find's and every
query's component index is the oracle's (or_conditional_create + sample on
its leaf's parameters), direction within 1e-5 and pdf within 1e-4 rel."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _tree_and_leaf_mixtures(pkg, synth, K, n=60000, threshold=6000, skip_every=5, iters=2):
    import torch
    b = synth.em_batch(n, 128)
    t = pkg.STree(np.float32([0, 0, 0]), np.float32([1, 1, 1]))
    t.split_to_depth(1)
    t.split(b["x"][0:3].copy(), threshold)
    ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"])
    out, seg = t.route(ds)
    nn = len(seg) - 1
    xs = np.stack([x.cpu().numpy() for x in out.x])
    npos = max(K // 8, 1)
    mixes = [None] * nn
    leaves = []
    for v in range(nn):
        a, e = int(seg[v]), int(seg[v + 1])
        if e - a < 4 * npos:
            continue
        leaves.append(v)
        if len(leaves) % skip_every == 0:
            continue                                   # an untrained leaf: BSDF only
        m = pkg.SDMM(K)
        m.init_hemisphere(xs[0:3, a:a + npos].T.copy(), xs[3:6, a:a + npos].T.copy(), synth.DEPTH_PRIOR,
                          synth.SPATIAL_DISTANCE, 11 + v)
        for _ in range(iters):
            m.optimize(pkg.DeviceSamples([x[a:e] for x in out.x], out.w[a:e]))
        mixes[v] = m
    torch.cuda.synchronize()
    return b, t, mixes, leaves


def _queries(gpu, nq, seed, lo=-0.05, hi=1.05):
    import torch
    rng = np.random.default_rng(seed)
    c = rng.uniform(lo, hi, size=(3, nq)).astype(np.float32)   # some queries fall outside the tree
    u = rng.uniform(0, 1, size=(3, nq)).astype(np.float32)
    d = rng.normal(size=(3, nq)).astype(np.float32)
    d /= np.linalg.norm(d, axis=0, keepdims=True)
    tt = lambda a: [torch.from_numpy(a[i].copy()).to(gpu) for i in range(3)]
    return c, u, d, tt(c), tt(u), tt(d)


def _oracle_check(oracle, t, mixes, c, u, d, node, has, cw, dw, pw, pdw, plog):
    """The wavefront's outputs against the C oracle: node ids from the
    oracle's tree find, per leaf the oracle's guide / pdf batch on that leaf's
    parameters."""
    aabb, child, _ = t.nodes()
    np.testing.assert_array_equal(node, oracle.stree_find(aabb, child, c.T.copy()))
    mism, derr, perr = 0, 0.0, 0.0
    for v in np.unique(node[has]):
        sel = np.nonzero(node == v)[0]
        p = mixes[v].get_params()
        om = oracle.Mixture(mixes[v].K)
        om.copy_params_from(p)
        om.valid[:] = p["valid"]
        dr, pr, cr, _ = oracle.guide_batch(om, c[:, sel].T.copy(), u[:, sel].T.copy())
        mism += int((cw[sel] != cr).sum())
        np.testing.assert_array_equal(cw[sel], cr)
        np.testing.assert_allclose(dw[:, sel].T, dr, atol=1e-5)
        np.testing.assert_allclose(pw[sel], pr, rtol=1e-4, atol=1e-7)
        pdr = oracle.pdf_batch(om, c[:, sel].T.copy(), d[:, sel].T.copy())
        np.testing.assert_allclose(pdw[sel], pdr, rtol=1e-4, atol=1e-7)
        derr = max(derr, float(np.abs(dw[:, sel].T - dr).max()))
        perr = max(perr, float((np.abs(pw[sel] - pr) / (1e-7 + 1e-4 * np.abs(pr))).max()))
    plog("wavefront_vs_oracle_index_mismatches", mism, 0)
    plog("wavefront_vs_oracle_dir_abs_err", derr, 1e-5)
    plog("wavefront_vs_oracle_pdf_err_over_tol", perr, 1.0)


@pytest.mark.parametrize("K,nq,cap", [(16, 1 << 15, 40), (16, 3000, 40), (64, 1 << 14, 40),
                                      (128, 1 << 14, 64), (128, 1 << 14, 40), (128, 1 << 14, 4), (128, 1 << 14, 0)])
def test_wavefront_equals_per_leaf_guide(pkg, oracle, synth, gpu, plog, K, nq, cap):
    """K = 128 is configs[2]'s leaf size: the tree kernels' candidate pass
    (capacity 40), the 16-lane group fallback most queries take at capacity 4,
    and every query on the full-K path at capacity 0 -- indices bit-exact
    against the oracle per leaf (sdmm_proc.cpp:275-590 at K = 128 leaves)."""
    import torch
    b, t, mixes, leaves = _tree_and_leaf_mixtures(pkg, synth, K)
    assert sum(m is not None for m in mixes) >= 4 and sum(mixes[v] is None for v in leaves) >= 1
    for m in mixes:
        if m is not None:
            m.set_guide_capacity(cap)
    c, u, d, ct, ut, dt = _queries(gpu, nq, 5)
    node = torch.empty(nq, dtype=torch.int32, device=gpu)
    dw, pw, cw = t.guide(mixes, ct, ut, node_out=node)
    pdw = t.pdf(mixes, ct, dt)
    ref_node = t.find(ct)
    torch.cuda.synchronize()
    node, ref_node = node.cpu().numpy(), ref_node.cpu().numpy()
    np.testing.assert_array_equal(node, ref_node)
    dw = np.stack([x.cpu().numpy() for x in dw])
    pw, cw, pdw = pw.cpu().numpy(), cw.cpu().numpy(), pdw.cpu().numpy()
    has = np.array([(v >= 0 and mixes[v] is not None) for v in node])
    assert (~has).sum() > 0 and has.sum() > nq // 2
    # no mixture (outside the tree, inner/untrained leaf): BSDF only
    assert (cw[~has] == -1).all() and (pw[~has] == 0).all() and (pdw[~has] == 0).all()
    assert (dw[:, ~has] == 0).all()
    _oracle_check(oracle, t, mixes, c, u, d, node, has, cw, dw, pw, pdw, plog)
    served = 0
    for v in np.unique(node[has]):
        sel = np.nonzero(node == v)[0]
        cs = [x[torch.from_numpy(sel).to(gpu)] for x in ct]
        us = [x[torch.from_numpy(sel).to(gpu)] for x in ut]
        ds_ = [x[torch.from_numpy(sel).to(gpu)] for x in dt]
        dr, pr, cr = mixes[v].guide(cs, us)
        pdr = mixes[v].pdf(cs, ds_)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(cw[sel], cr.cpu().numpy())
        np.testing.assert_array_equal(pw[sel], pr.cpu().numpy())
        np.testing.assert_array_equal(dw[:, sel], np.stack([x.cpu().numpy() for x in dr]))
        np.testing.assert_array_equal(pdw[sel], pdr.cpu().numpy())
        served += len(sel)
    assert served == has.sum()
    assert (cw[has] >= 0).mean() > 0.5


def test_wavefront_mixed_K_and_fallback(pkg, synth, gpu):
    """Leaves with different K in one wavefront (16 and 512: the fallback runs
    32-wide for the largest K), and capacity-0-equivalent queries far from
    every component; still bitwise per leaf."""
    import torch
    b, t, m16, leaves = _tree_and_leaf_mixtures(pkg, synth, 16, skip_every=1000)
    _, _, m512, _ = _tree_and_leaf_mixtures(pkg, synth, 512, threshold=6000, skip_every=1000, iters=1)
    mixes = [m512[v] if (i % 3 == 0 and m512[v] is not None) else m16[v] for i, v in enumerate(range(len(m16)))]
    assert any(m is not None and m.K == 512 for m in mixes)
    nq = 1 << 14
    c, u, d, ct, ut, dt = _queries(gpu, nq, 9, 0.0, 1.0)
    node = torch.empty(nq, dtype=torch.int32, device=gpu)
    dw, pw, cw = t.guide(mixes, ct, ut, node_out=node)
    torch.cuda.synchronize()
    node = node.cpu().numpy()
    dw = np.stack([x.cpu().numpy() for x in dw])
    pw, cw = pw.cpu().numpy(), cw.cpu().numpy()
    for v in np.unique(node):
        sel = np.nonzero(node == v)[0]
        if mixes[v] is None:
            assert (cw[sel] == -1).all()
            continue
        idx = torch.from_numpy(sel).to(gpu)
        dr, pr, cr = mixes[v].guide([x[idx] for x in ct], [x[idx] for x in ut])
        torch.cuda.synchronize()
        np.testing.assert_array_equal(cw[sel], cr.cpu().numpy())
        np.testing.assert_array_equal(pw[sel], pr.cpu().numpy())
        np.testing.assert_array_equal(dw[:, sel], np.stack([x.cpu().numpy() for x in dr]))


def test_wavefront_table_update_and_stream(pkg, synth, gpu):
    """The per-node table is re-uploaded when a leaf's mixture changes, and
    the wavefront runs on a caller stream shared with the mixtures."""
    import torch
    b, t, mixes, leaves = _tree_and_leaf_mixtures(pkg, synth, 16)
    nq = 4096
    c, u, d, ct, ut, dt = _queries(gpu, nq, 13, 0.0, 1.0)
    s = torch.cuda.Stream()
    t.set_stream(s)
    for m in mixes:
        if m is not None:
            m.set_stream(s)
    _, p1, c1 = t.guide(mixes, ct, ut)
    none = [None] * len(mixes)
    _, p2, c2 = t.guide(none, ct, ut)
    _, p3, c3 = t.guide(mixes, ct, ut)
    s.synchronize()
    assert (c2.cpu().numpy() == -1).all() and (p2.cpu().numpy() == 0).all()
    np.testing.assert_array_equal(c1.cpu().numpy(), c3.cpu().numpy())
    np.testing.assert_array_equal(p1.cpu().numpy(), p3.cpu().numpy())
    with pytest.raises(ValueError):
        t.guide(mixes[:-1], ct, ut)
    # bound table: the same bits as passing the table per call
    t.bind(mixes)
    _, p4, c4 = t.guide(None, ct, ut)
    s.synchronize()
    np.testing.assert_array_equal(c1.cpu().numpy(), c4.cpu().numpy())
    np.testing.assert_array_equal(p1.cpu().numpy(), p4.cpu().numpy())
    # a tree changed by a split has no bound table any more
    t.split_to_depth(2)
    with pytest.raises(pkg.SDMMError):
        t.guide(None, ct, ut)
    t.set_stream(None)


def test_wavefront_orders_after_em_on_other_streams(pkg, synth, gpu):
    """the leaf mixtures step on their own stream, the tree guides on
    torch's stream, with NO synchronisation in between -- the wavefront waits for
    the EM (events on the mixtures' streams), so its outputs equal those of a
    run with a device synchronisation between the two."""
    import torch
    b = synth.em_batch(200000, 128)
    ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"])
    side = torch.cuda.Stream()

    def run(sync):
        t = pkg.STree(np.float32([0, 0, 0]), np.float32([1, 1, 1]))
        t.split_to_depth(1)
        out, seg = t.route(ds)
        torch.cuda.synchronize()
        xs = np.stack([x.cpu().numpy() for x in out.x])
        mixes = [None] * (len(seg) - 1)
        for v in range(len(seg) - 1):
            a, e = int(seg[v]), int(seg[v + 1])
            if e - a < 64:
                continue
            m = pkg.SDMM(128, stream=side)
            m.init_hemisphere(xs[0:3, a:a + 16].T.copy(), xs[3:6, a:a + 16].T.copy(), synth.DEPTH_PRIOR,
                              synth.SPATIAL_DISTANCE, 3 + v)
            mixes[v] = (m, pkg.DeviceSamples([x[a:e] for x in out.x], out.w[a:e]))
        side.synchronize()
        t.bind([None if x is None else x[0] for x in mixes])
        for x in mixes:                              # enqueued on `side`, not waited for
            if x is not None:
                x[0].optimize(x[1], 3)
        if sync:
            torch.cuda.synchronize()
        c, u, d, ct, ut, dt = _queries(gpu, 1 << 16, 9)
        dd, pdf, comp = t.guide(None, ct, ut)
        torch.cuda.current_stream().synchronize()
        return np.stack([x.cpu().numpy() for x in dd]), pdf.cpu().numpy(), comp.cpu().numpy()

    a, r = run(False), run(True)
    for x, y in zip(a, r):
        np.testing.assert_array_equal(x, y)
