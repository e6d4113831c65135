"""Spatial tree (jmm SNTree restatement, sntree.h:93-299): the library's
host-built tree against the C oracle's (CPU, bitwise), device find / route
against the oracle's find (GPU, bit-exact node ids), and the routed batch
driving the per-leaf EM (GPU)."""
import numpy as np
import pytest


def _points(synth, n, seed=4):
    b = synth.em_batch(n, 128)
    return b, b["x"][0:3].copy()


@pytest.mark.parametrize("depth,threshold,n", [(0, 4000, 60000), (1, 3000, 60000), (2, 20000, 60000),
                                               (3, 50000, 60000), (0, 2000, 400000)])
def test_tree_matches_oracle(pkg, oracle, synth, depth, threshold, n):
    """split_to_depth + split(threshold) -> identical node arrays (ids, boxes,
    children, axes) from the library and from the oracle.  n = 400000: the
    host split recurses into both children of a large node on two threads
    (> 2^15 samples each) and must still number the nodes in creation order."""
    b, p = _points(synth, n)
    lo, hi = np.float32([0.0, 0.0, 0.0]), np.float32([1.0, 0.95, 0.9])
    t = pkg.STree(lo, hi)
    t.split_to_depth(depth)
    t.split(p, threshold)
    aabb, child, axis = t.nodes()
    oa, oc, ox = oracle.stree_build(lo, hi, depth, p, threshold)
    np.testing.assert_array_equal(child, oc)
    np.testing.assert_array_equal(aabb, oa)
    np.testing.assert_array_equal(axis, ox)
    leaves = child[:, 0] < 0
    assert leaves.sum() == (len(child) + 1) // 2
    # root is the cube over the AABB (SNTree ctor)
    np.testing.assert_array_equal(aabb[0], np.float32([0, 0, 0, 1, 1, 1]))
    # children of a data split: child 0 is the upper part along the split axis
    inner = np.nonzero(~leaves)[0]
    for i in inner[:50]:
        a = axis[i]
        c0, c1 = child[i]
        assert aabb[c0, a] >= aabb[c1, a] and aabb[c0, 3 + a] == aabb[i, 3 + a]
    # every leaf holds <= threshold points unless it could not be split
    ids = oracle.stree_find(aabb, child, p.T[:5000])
    assert (ids >= 0).all() and leaves[ids].all()


@pytest.mark.gpu
def test_device_find_and_route(pkg, oracle, synth, gpu):
    import torch
    b, p = _points(synth, 200000)
    lo, hi = np.float32([0, 0, 0]), np.float32([1, 1, 1])
    t = pkg.STree(lo, hi)
    t.split_to_depth(2)
    t.split(p, 6000)
    aabb, child, axis = t.nodes()
    # queries: samples, exact split-plane coordinates, box corners, outside points, NaN
    rng = np.random.default_rng(3)
    q = p[:, :20000].copy()
    inner = np.nonzero(child[:, 0] >= 0)[0]
    for j, i in enumerate(inner[:2000]):
        c0 = child[i, 0]
        q[axis[i], j] = aabb[c0, axis[i]]                  # on the plane: child 0 (upper) wins
    q[:, 2000:2008] = np.float32([[0, 1, 0, 1, 0, 1, 0, 1], [0, 0, 1, 1, 0, 0, 1, 1], [0, 0, 0, 0, 1, 1, 1, 1]])
    q[:, 2008:2100] = rng.uniform(-0.5, 1.5, size=(3, 92)).astype(np.float32)
    q[0, 2100] = np.nan
    qt = [torch.from_numpy(q[i].copy()).to(gpu) for i in range(3)]
    got = t.find(qt).cpu().numpy()
    ref = oracle.stree_find(aabb, child, q.T)
    np.testing.assert_array_equal(got, ref)
    # route: leaf-contiguous, stable inside a leaf, seg = per-node counts
    ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"], b["hpdf"], b["is_diffuse"])
    out, seg = t.route(ds)
    torch.cuda.synchronize()
    ids = oracle.stree_find(aabb, child, p.T)
    order = np.argsort(np.where(ids < 0, len(child), ids), kind="stable")
    for i in range(6):
        np.testing.assert_array_equal(out.x[i].cpu().numpy(), b["x"][i][order])
    np.testing.assert_array_equal(out.w.cpu().numpy(), b["w"][order])
    counts = np.bincount(ids[ids >= 0], minlength=len(child))
    np.testing.assert_array_equal(np.diff(seg), counts)


@pytest.mark.gpu
def test_routed_leaves_batched_em(pkg, synth, gpu):
    """route -> one mixture per tree node -> ONE sdmm_em_step_batched over the
    routed planes with the route's own seg equals each node's own em_step
    (inner nodes own no samples and stay untouched): the plugin's optimise
    loop over the tree (volpath_sdmm.cpp:287-311)."""
    import torch
    b, p = _points(synth, 60000)
    t = pkg.STree(np.float32([0, 0, 0]), np.float32([1, 1, 1]))
    t.split_to_depth(1)
    t.split(p, 8000)
    ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"])
    out, seg = t.route(ds)
    nn = len(seg) - 1
    K = 16
    xs = np.stack([x.cpu().numpy() for x in out.x])

    def mixes():
        ms = []
        for v in range(nn):
            a = int(seg[v]) if seg[v + 1] - seg[v] >= 2 else 0
            m = pkg.SDMM(K)
            m.init_hemisphere(xs[0:3, a:a + 2].T.copy(), xs[3:6, a:a + 2].T.copy(), synth.DEPTH_PRIOR,
                              synth.SPATIAL_DISTANCE, 7 + v)
            ms.append(m)
        return ms
    A, B = mixes(), mixes()
    inside = pkg.DeviceSamples([x[:int(seg[nn])] for x in out.x], out.w[:int(seg[nn])])
    pkg.em_step_batched(A, inside, seg, 1)
    for m, v in zip(B, range(nn)):
        a, e = int(seg[v]), int(seg[v + 1])
        if e > a:
            m.optimize(pkg.DeviceSamples([x[a:e] for x in out.x], out.w[a:e]))
    torch.cuda.synchronize()
    assert (np.diff(seg) > 0).sum() >= 8
    for ma, mb in zip(A, B):
        pa, pb = ma.get_params(), mb.get_params()
        for k in ("weights", "mean", "cov"):
            np.testing.assert_array_equal(pa[k], pb[k])


def _gap_tree(pkg):
    """Root [0,1]^3 split on x at 0.5; its upper child split on y with an
    ulp-scale GAP (y in (0.59, 0.6) belongs to neither grandchild), the lower
    child split on y at 0.5.  Node ids in creation order."""
    aabb = np.float32([
        [0, 0, 0, 1, 1, 1],            # 0 root
        [0.5, 0, 0, 1, 1, 1],          # 1 upper x (child 0)
        [0, 0, 0, 0.5, 1, 1],          # 2 lower x (child 1)
        [0.5, 0.6, 0, 1, 1, 1],        # 3 child 0 of 1
        [0.5, 0, 0, 1, 0.59, 1],       # 4 child 1 of 1 (gap below 0.6)
        [0, 0.5, 0, 0.5, 1, 1],        # 5 child 0 of 2
        [0, 0, 0, 0.5, 0.5, 1]])       # 6 child 1 of 2
    child = np.int32([[1, 2], [3, 4], [5, 6], [-1, -1], [-1, -1], [-1, -1], [-1, -1]])
    axis = np.int32([0, 1, 1, 2, 2, 2, 2])
    t = pkg.STree(np.float32([0, 0, 0]), np.float32([1, 1, 1]))
    t.set_nodes(aabb, child, axis)
    return t, aabb, child


def _gap_queries():
    # on the root's plane x = 0.5 (in both children) inside the upper child's
    # y gap: the depth-first search leaves node 1 empty-handed and finds node 5
    q = np.float32([[0.5, 0.595, 0.5], [0.5, 0.59, 0.5], [0.5, 0.6, 0.5], [0.75, 0.595, 0.5],
                    [0.25, 0.595, 0.5], [0.5, 0.3, 0.2], [0.5, 0.595, 1.0]])
    expect = np.int32([5, 4, 3, -1, 5, 4, 5])
    return q, expect


def test_find_backtracks_like_sntree(pkg, oracle):
    """SNTreeNode::find (jmm/sntree.h:62-83) backtracks out of a subtree whose
    children miss the point; the oracle restates it."""
    t, aabb, child = _gap_tree(pkg)
    q, expect = _gap_queries()
    np.testing.assert_array_equal(oracle.stree_find(aabb, child, q), expect)


def test_split_leaves_plugin_block(pkg, oracle, synth):
    """sdmm_stree_split_leaves: the built plugin's splitting block
    (volpath_sdmm.cpp:253-260) -- split_to_depth(2), then split_leaf_recurse(i,
    4000) over the nodes while leaf_nodes() <= 2048; == the oracle's split, and
    nothing happens above the leaf cap."""
    b, p = _points(synth, 120000)
    lo, hi = np.float32([0, 0, 0]), np.float32([1, 1, 1])
    t = pkg.STree(lo, hi)
    t.split_to_depth(2)
    assert t.leaf_nodes == 64
    t.split_leaves(p, 4000, 2048)
    aabb, child, axis = t.nodes()
    oa, oc, ox = oracle.stree_build(lo, hi, 2, p, 4000)
    np.testing.assert_array_equal(child, oc)
    np.testing.assert_array_equal(aabb, oa)
    assert t.leaf_nodes == int((child[:, 0] < 0).sum()) > 64
    u = pkg.STree(lo, hi)
    u.split_to_depth(2)
    u.split_leaves(p, 4000, 10)                      # 64 leaves > cap: no split
    assert u.num_nodes == 127 and u.leaf_nodes == 64
    # split_leaf_recurse on one leaf with that leaf's samples == split() of a
    # one-leaf tree
    v = pkg.STree(lo, hi)
    v.split_leaf_recurse(0, p, 4000)
    w = pkg.STree(lo, hi)
    w.split(p, 4000)
    for x, y in zip(v.nodes(), w.nodes()):
        np.testing.assert_array_equal(x, y)
    v.split_leaf_recurse(0, p, 10)                   # an inner node now: no-op
    np.testing.assert_array_equal(v.nodes()[1], w.nodes()[1])


@pytest.mark.gpu
def test_device_find_backtracks(pkg, oracle, gpu):
    import torch
    t, aabb, child = _gap_tree(pkg)
    q, expect = _gap_queries()
    got = t.find([torch.from_numpy(q[:, i].copy()).to(gpu) for i in range(3)]).cpu().numpy()
    np.testing.assert_array_equal(got, expect)


@pytest.mark.gpu
@pytest.mark.parametrize("n,threshold,grid,tight", [(400000, 2000, 0, False), (120000, 3000, 64, False),
                                                    (60000, 500, 0, False), (120000, 3000, 64, True),
                                                    (60000, 800, 16, True)])
def test_device_split_equals_host_split(pkg, oracle, synth, gpu, monkeypatch, n, threshold, grid, tight):
    """sdmm_stree_split_leaf_recurse_device (the split on device-resident
    positions, level by level) builds node arrays IDENTICAL to the host
    split_leaf_recurse_many and to the oracle's recursion, for several leaves
    at once; grid > 0 snaps the points to a lattice so many lie exactly on
    split planes (they go to both children).  tight: SDMM_SPLIT_TIGHT=1
    sizes the level scratch without headroom, so the duplicated plane samples
    take the regrowth branch (split_grow re-layout)."""
    import torch
    if tight:
        monkeypatch.setenv("SDMM_SPLIT_TIGHT", "1")
    b, p = _points(synth, n)
    if grid:
        p = np.floor(p * grid) / grid
    lo, hi = np.float32([0, 0, 0]), np.float32([1, 1, 1])
    th, td = pkg.STree(lo, hi), pkg.STree(lo, hi)
    for t in (th, td):
        t.split_to_depth(1)
    aabb, child, _ = th.nodes()
    ids = oracle.stree_find(aabb, child, p.T)
    leaves = [v for v in range(len(child)) if child[v, 0] < 0 and (ids == v).sum() > threshold]
    per = [p[:, ids == v] for v in leaves]
    th.split_leaf_recurse_many(leaves, per, threshold)
    cat = np.concatenate(per, axis=1)
    counts = np.array([x.shape[1] for x in per], np.int64)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
    planes = [torch.from_numpy(np.ascontiguousarray(cat[i])).to(gpu) for i in range(3)]
    td.split_leaf_recurse_device(leaves, planes, starts, counts, threshold)
    for a, c in zip(th.nodes(), td.nodes()):
        np.testing.assert_array_equal(a, c)
    assert td.num_nodes > len(child) + 10
    # and the oracle's sequential recursion from the same leaves
    oa, oc, ox = oracle.stree_build(lo, hi, 1, p, threshold)
    np.testing.assert_array_equal(td.nodes()[1], oc)
    np.testing.assert_array_equal(td.nodes()[0], oa)
