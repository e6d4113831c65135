"""Guide contexts (sdmm_guide_ctx_*, sdmm_stree_publish): the reference's
render workers call create_conditional / sample / pdf concurrently, each with
thread_local scratch (sdmm_proc.cpp:1086-1106).  Here each host thread owns a
context (its own stream and scratch) on one published tree and serves its
tiles' bounces with no lock.

Parity: every query's outputs from many threads at once are BITWISE those of
one sdmm_guide_pdf_wavefront / sdmm_guide_product_wavefront call over the
whole batch (whose per-leaf parity against the oracle is
test_gpu_wavefront.py / test_gpu_product_wavefront.py)."""
import threading

import numpy as np
import pytest

from test_gpu_wavefront import _queries, _tree_and_leaf_mixtures

pytestmark = pytest.mark.gpu


def _run_threads(n_threads, tiles, work):
    """work(ctx_index, tile) on n_threads threads, tiles dealt round robin;
    re-raises the first exception."""
    errors = []

    def body(i):
        try:
            for k in range(i, len(tiles), n_threads):
                work(i, tiles[k])
        except Exception as e:   # noqa: BLE001 -- reported by the main thread
            errors.append(e)

    th = [threading.Thread(target=body, args=(i,)) for i in range(n_threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errors:
        raise errors[0]


@pytest.mark.parametrize("K,tile", [(16, 1 << 15), (128, 20000), (128, 3000)])
def test_ctx_threads_equal_one_wavefront(pkg, synth, gpu, K, tile):
    """8 threads x tiles of `tile` queries (>= 16 K: each tile served in
    Morton order; 3000: as given) == one call over the whole batch."""
    import torch
    b, t, mixes, leaves = _tree_and_leaf_mixtures(pkg, synth, K)
    nq = 8 * tile + 123
    c, u, d, ct, ut, dt = _queries(gpu, nq, 31, 0.0, 1.0)
    mode = torch.from_numpy((np.random.default_rng(3).uniform(size=nq) < 0.4).astype(np.uint8)).to(gpu)
    t.bind(mixes)
    dr, pr, cr = t.guide_pdf(None, ct, ut, dt, mode)
    torch.cuda.synchronize()
    with pytest.raises(pkg.SDMMError):       # not published yet
        ctx = pkg.GuideContext(t)
        ctx.guide_pdf(ct, ut, dt, mode)
    t.publish()
    n_threads = 8
    ctxs = [pkg.GuideContext(t) for _ in range(n_threads)]
    d_out = [torch.full((nq,), -7.0, device=gpu) for _ in range(3)]
    p_out = torch.full((nq,), -7.0, device=gpu)
    c_out = torch.full((nq,), -7, dtype=torch.int32, device=gpu)
    torch.cuda.synchronize()
    tiles = [(a, min(a + tile, nq)) for a in range(0, nq, tile)]

    def work(i, ab):
        a, e = ab
        off = lambda x: x.data_ptr() + 4 * a
        ctxs[i].guide_pdf_into(e - a, [off(x) for x in ct], [off(x) for x in ut], [off(x) for x in dt],
                               mode.data_ptr() + a, [off(x) for x in d_out], off(p_out), off(c_out))
        ctxs[i].synchronize()

    _run_threads(n_threads, tiles, work)
    np.testing.assert_array_equal(c_out.cpu().numpy(), cr.cpu().numpy())
    np.testing.assert_array_equal(p_out.cpu().numpy(), pr.cpu().numpy())
    for x, y in zip(d_out, dr):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
    assert (cr.cpu().numpy() >= 0).mean() > 0.3 and (cr.cpu().numpy() == -2).mean() > 0.2
    for x in ctxs:
        x.close()


def test_ctx_product_threads_equal_one_wavefront(pkg, synth, gpu):
    """sampleProduct (the mixed bounce, choice + dgiven) from 6 threads ==
    one sdmm_guide_product_wavefront call."""
    import torch
    b, t, mixes, leaves = _tree_and_leaf_mixtures(pkg, synth, 16)
    tile = 4096
    nq = 6 * 3 * tile
    c, u, d, ct, ut, dt = _queries(gpu, nq, 37, 0.0, 1.0)
    B, M = 4, 3
    bw, bmean, bcov = synth.bsdf_table(B, M, seed=9)
    F = synth.shading_frames(nq, seed=10)
    mat = ((np.arange(nq) % (B + 1)) - 1).astype(np.int32)
    Ft = [torch.from_numpy(np.ascontiguousarray(F.T[i])).to(gpu) for i in range(9)]
    matt = torch.from_numpy(mat).to(gpu)
    table = pkg.BsdfTable(bw, bmean, bcov, device=gpu, diffuse=(np.arange(B) % 2).astype(np.uint8))
    choice = torch.from_numpy(np.random.default_rng(4).uniform(size=nq).astype(np.float32)).to(gpu)
    t.bind(mixes)
    dr, pr, cr, hr = t.guide_product(None, ct, ut, table, matt, Ft, choice=choice, dgiven=dt)
    torch.cuda.synchronize()
    t.publish()
    ctxs = [pkg.GuideContext(t) for _ in range(6)]
    outs = [None] * (nq // tile)
    tiles = list(range(nq // tile))

    def work(i, k):
        sl = slice(k * tile, (k + 1) * tile)
        outs[k] = ctxs[i].guide_product([x[sl] for x in ct], [x[sl] for x in ut], table, matt[sl],
                                        [x[sl] for x in Ft], choice=choice[sl], dgiven=[x[sl] for x in dt])
        ctxs[i].synchronize()

    _run_threads(6, tiles, work)
    cat = lambda j: torch.cat([o[j] for o in outs]).cpu().numpy()
    np.testing.assert_array_equal(cat(2), cr.cpu().numpy())
    np.testing.assert_array_equal(cat(1), pr.cpu().numpy())
    np.testing.assert_array_equal(cat(3), hr.cpu().numpy())
    for a in range(3):
        np.testing.assert_array_equal(torch.cat([o[0][a] for o in outs]).cpu().numpy(), dr[a].cpu().numpy())
    assert (cr.cpu().numpy() == -2).any() and (hr.cpu().numpy() == np.float32(0.3)).any()


def test_ctx_unpublished_after_change(pkg, synth, gpu):
    """A split or a new binding un-publishes the tree: context calls fail with
    SDMM_E_STATE until sdmm_stree_publish runs again."""
    import torch
    b, t, mixes, leaves = _tree_and_leaf_mixtures(pkg, synth, 16)
    nq = 2048
    c, u, d, ct, ut, dt = _queries(gpu, nq, 41, 0.0, 1.0)
    mode = torch.zeros(nq, dtype=torch.uint8, device=gpu)
    t.publish(mixes)
    ctx = pkg.GuideContext(t)
    _, p1, c1 = ctx.guide_pdf(ct, ut, dt, mode)
    ctx.synchronize()
    t.bind([None] * len(mixes))                  # a different table
    with pytest.raises(pkg.SDMMError):
        ctx.guide_pdf(ct, ut, dt, mode)
    t.publish(mixes)
    _, p2, c2 = ctx.guide_pdf(ct, ut, dt, mode)
    ctx.synchronize()
    np.testing.assert_array_equal(c1.cpu().numpy(), c2.cpu().numpy())
    np.testing.assert_array_equal(p1.cpu().numpy(), p2.cpu().numpy())
    t.split_to_depth(3)
    with pytest.raises(pkg.SDMMError):
        ctx.guide_pdf(ct, ut, dt, mode)
    ctx.close()


def test_ctx_host_batch_equals_one_wavefront(pkg, synth, gpu):
    """sdmm_ctx_guide_pdf_host_batch: several requests' pinned host planes
    (strides larger than their sizes, one empty request, ragged sizes) served
    as one wavefront == one device call over the concatenated queries,
    bitwise; pageable host buffers are refused (SDMM_E_INVALID)."""
    import torch
    b, t, mixes, leaves = _tree_and_leaf_mixtures(pkg, synth, 128)
    sizes = [5000, 0, 12345, 77, 30000]
    nq = sum(sizes)
    c, u, d, ct, ut, dt = _queries(gpu, nq, 41, 0.0, 1.0)
    mode_np = (np.random.default_rng(9).uniform(size=nq) < 0.5).astype(np.uint8)
    mode = torch.from_numpy(mode_np).to(gpu)
    t.bind(mixes)
    dr, pr, cr = t.guide_pdf(None, ct, ut, dt, mode)
    torch.cuda.synchronize()
    t.publish()
    ctx = pkg.GuideContext(t)
    planes = np.concatenate([c, u, d]).astype(np.float32)          # (9, nq)
    reqs, outs, off = [], [], 0
    for n in sizes:
        stride = n + 64
        inp = torch.zeros((9, stride), dtype=torch.float32).pin_memory()
        inp[:, :n] = torch.from_numpy(planes[:, off:off + n])
        md = torch.from_numpy(mode_np[off:off + n].copy()).pin_memory()
        out = torch.full((4, stride + 3), -7.0, dtype=torch.float32).pin_memory()
        cp = torch.full((n,), -9, dtype=torch.int32).pin_memory()
        reqs.append((inp, md, out, cp))
        outs.append((off, n, out, cp))
        off += n
    ctx.guide_pdf_host(reqs)
    for off, n, out, cp in outs:
        for k in range(3):
            np.testing.assert_array_equal(out[k, :n].numpy(), dr[k][off:off + n].cpu().numpy())
        np.testing.assert_array_equal(out[3, :n].numpy(), pr[off:off + n].cpu().numpy())
        np.testing.assert_array_equal(cp.numpy(), cr[off:off + n].cpu().numpy())
        assert (out[:, n:].numpy() == -7.0).all()                  # nothing past the request
    inp, md, out, cp = reqs[0]
    with pytest.raises(pkg.SDMMError):
        ctx.guide_pdf_host([(inp.clone(), md, out, cp)])           # pageable input planes
    ctx.close()
