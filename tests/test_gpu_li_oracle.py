"""GPU: the device Li (sdmm_li_render, csrc/render.hip) against its CPU
restatement (oracle/sdmm_oracle_li.inc) on the same scene, tree, seed and
leaf parameters -- configs[0]'s Cornell Box.

  * unguided (BSDF sampling only): the saved-vertex records (what the EM
    trains on), the vertex counts and the image BIT-EXACT;
  * guided (trained K = 16 leaves) and guided with sampleProduct: the guide is
    the oracle's conditional / product on each leaf's parameters; its
    directions come from correctly rounded transcendentals (the kernel's
    within 1e-5, tests/test_gpu_parity.py), so a path's later vertices may
    drift by rounding.  Paths whose vertex counts agree and whose records all
    agree within 1e-3 relative (1e-5 absolute) must be >= 99 % of all paths,
    and every vertex's guided-or-not outcome (the oracle's per-bounce
    component index) is reported; the images agree in the mean within 0.5 %.
"""
import numpy as np
import pytest

from test_gpu_li import _scene, _train, _tree

pytestmark = pytest.mark.gpu
SPP, SEED = 4, 12345


def _oracle_mixes(oracle, node_mix):
    out = []
    for m in node_mix:
        if m is None:
            out.append(None)
            continue
        p = m.get_params()
        om = oracle.Mixture(m.K)
        om.copy_params_from(p)
        om.valid[:] = p["valid"]
        out.append(om)
    return out


def _device(sc, tree, node_mix, guided, table=None, spp=SPP, seed=SEED):
    import torch
    img, verts, st = sc.render(tree, node_mix, spp=spp, guided=guided, seed=seed, learned_bsdf=table)
    rec, nv = verts.to_numpy()
    torch.cuda.synchronize()
    return img.cpu().numpy(), rec.reshape(16, verts.s.max_vertices, -1), nv, st


def test_unguided_li_bitwise(pkg, oracle, scenes, gpu, plog):
    desc = scenes.cornell_box(128, 72)
    sc = pkg.Scene(desc)
    tree = _tree(pkg, sc)
    img, rec, nv, _ = _device(sc, tree, None, False)
    aabb, child, _ = tree.nodes()
    r = oracle.li_render(desc, aabb, child, spp=SPP, seed=SEED, threads=8)
    plog("li_unguided_nv_mismatch", int((nv != r["nv"]).sum()), 0)
    np.testing.assert_array_equal(nv, r["nv"])
    sel = np.arange(rec.shape[1])[:, None] < nv[None, :]
    diff = np.abs(rec - r["rec"])[:, sel]
    plog("li_unguided_rec_max_abs_diff", float(diff.max()), 0.0)
    np.testing.assert_array_equal(rec[:, sel], r["rec"][:, sel])
    plog("li_unguided_image_max_abs_diff", float(np.abs(img - r["image"]).max()), 0.0)
    np.testing.assert_array_equal(img, r["image"])


def _compare_guided(oracle, plog, tag, img, rec, nv, r):
    P = nv.shape[0]
    same_n = nv == r["nv"]
    V = rec.shape[1]
    sel = np.arange(V)[:, None] < nv[None, :]
    rel = np.abs(rec - r["rec"]) / (1e-5 + 1e-3 * np.abs(r["rec"]))
    rel = np.where(sel[None], rel, 0.0).max(axis=(0, 1))
    match = same_n & (rel <= 1.0)
    comps = r["comps"]
    guided = (comps >= 0).sum()
    plog(f"{tag}_matching_path_frac", float(match.mean()), 0.99, lower=True, paths=P,
         oracle_guided_samples=int(guided), oracle_bsdf_chosen=int((comps == -2).sum()))
    assert match.mean() >= 0.99, (match.mean(), (~same_n).sum())
    assert guided > P // 4
    m1, m2 = float(img.mean()), float(r["image"].mean())
    plog(f"{tag}_image_mean_rel_diff", abs(m1 - m2) / m2, 5e-3)
    assert abs(m1 - m2) <= 5e-3 * m2


@pytest.mark.parametrize("K", [16, 128])
def test_guided_li_matches_oracle(pkg, oracle, scenes, gpu, plog, K):
    """K = 128: configs[2]'s leaf size (the Torus meshes are LFS pointers; the
    Cornell Box stands in), through the tree wavefront's K = 128 kernels."""
    desc = scenes.cornell_box(128, 72)
    sc = pkg.Scene(desc)
    tree = _tree(pkg, sc)
    node_mix = _train(pkg, sc, tree, 4, 8, K=K)
    assert any(m is not None and m.K == K for m in node_mix)
    img, rec, nv, _ = _device(sc, tree, node_mix, True)
    aabb, child, _ = tree.nodes()
    r = oracle.li_render(desc, aabb, child, node_mix=_oracle_mixes(oracle, node_mix), guided=True, spp=SPP,
                         seed=SEED, threads=16)
    _compare_guided(oracle, plog, f"li_guided_K{K}", img, rec, nv, r)


def test_product_li_matches_oracle(pkg, oracle, scenes, gpu, plog):
    desc = scenes.cornell_box(128, 72)
    sc = pkg.Scene(desc)
    tree = _tree(pkg, sc)
    node_mix = _train(pkg, sc, tree, 4, 8)
    learned = scenes.diffuse_learned_bsdf(len(desc["reflectance"]) // 3)
    table = pkg.BsdfTable(*learned[:3], device=gpu, diffuse=learned[3])
    img, rec, nv, _ = _device(sc, tree, node_mix, True, table=table)
    aabb, child, _ = tree.nodes()
    r = oracle.li_render(desc, aabb, child, node_mix=_oracle_mixes(oracle, node_mix), guided=True, spp=SPP,
                         seed=SEED, learned=learned, threads=16)
    _compare_guided(oracle, plog, "li_product", img, rec, nv, r)


PLASTIC = ("TallBox", "ShortBox", "Floor")


def test_black_base_plastic_unguided_bitwise(pkg, oracle, scenes, gpu, plog):
    """A smooth plastic with a black diffuse base (specular sampling weight
    exactly 1: sdmm_scene_create accepts the closed end of [0, 1]) on the
    floor: the device Li equals the CPU Li bit for bit, unguided."""
    desc = scenes.cornell_box(128, 72, plastic=("Floor",))
    names = list(scenes._BSDFS)
    f = names.index("Floor")
    bp = desc["bsdf_params"].reshape(-1, 8).copy()
    bp[f] = scenes.plastic_params((0.0, 0.0, 0.0))
    assert bp[f, 7] == 1.0
    desc["bsdf_params"] = bp.reshape(-1)
    refl = desc["reflectance"].reshape(-1, 3).copy()
    refl[f] = 0.0
    desc["reflectance"] = refl.reshape(-1)
    sc = pkg.Scene(desc)
    tree = _tree(pkg, sc)
    img, rec, nv, _ = _device(sc, tree, None, False)
    aabb, child, _ = tree.nodes()
    r = oracle.li_render(desc, aabb, child, spp=SPP, seed=SEED, threads=8)
    np.testing.assert_array_equal(nv, r["nv"])
    sel = np.arange(rec.shape[1])[:, None] < nv[None, :]
    np.testing.assert_array_equal(rec[:, sel], r["rec"][:, sel])
    np.testing.assert_array_equal(img, r["image"])


def test_plastic_li_matches_oracle(pkg, oracle, scenes, gpu, plog):
    """A delta + smooth BSDF (smooth plastic on the boxes and the floor, the
    Kitchen's `plastic`) through the device Li and the CPU Li: unguided
    bitwise (records, vertex counts -- a delta bounce saves none -- image);
    guided with trained K = 16 leaves >= 99 % of the paths (the guide is
    queried on every plastic bounce, a BSDF-chosen delta lobe returns
    weight / h with pdf * h: sdmm_proc.cpp:297, :383-409)."""
    desc = scenes.cornell_box(128, 72, plastic=PLASTIC)
    sc = pkg.Scene(desc)
    tree = _tree(pkg, sc)
    img, rec, nv, st = _device(sc, tree, None, False)
    aabb, child, _ = tree.nodes()
    r = oracle.li_render(desc, aabb, child, spp=SPP, seed=SEED, threads=8)
    np.testing.assert_array_equal(nv, r["nv"])
    sel = np.arange(rec.shape[1])[:, None] < nv[None, :]
    plog("li_plastic_unguided_rec_max_abs_diff", float(np.abs(rec - r["rec"])[:, sel].max()), 0.0)
    np.testing.assert_array_equal(rec[:, sel], r["rec"][:, sel])
    np.testing.assert_array_equal(img, r["image"])
    # delta bounces trace a ray but save no vertex
    assert st["segments"] > int(nv.sum())
    node_mix = _train(pkg, sc, tree, 4, 8)
    img, rec, nv, _ = _device(sc, tree, node_mix, True)
    aabb, child, _ = tree.nodes()
    r = oracle.li_render(desc, aabb, child, node_mix=_oracle_mixes(oracle, node_mix), guided=True, spp=SPP,
                         seed=SEED, threads=16)
    _compare_guided(oracle, plog, "li_plastic_guided", img, rec, nv, r)


GLOSSY = ("TallBox", "Floor")


def test_conductor_li_unguided_bitwise(pkg, oracle, scenes, gpu, plog):
    """Rough conductors (Beckmann, roughconductor.cpp) on the tall box and the
    floor: the device Li equals the CPU Li bit for bit, unguided -- records,
    vertex counts, image -- at two roughnesses."""
    for alpha in (0.2, 0.05):
        desc = scenes.cornell_box(128, 72, conductor=GLOSSY, alpha=alpha)
        sc = pkg.Scene(desc)
        tree = _tree(pkg, sc)
        img, rec, nv, _ = _device(sc, tree, None, False)
        aabb, child, _ = tree.nodes()
        r = oracle.li_render(desc, aabb, child, spp=SPP, seed=SEED, threads=8)
        np.testing.assert_array_equal(nv, r["nv"])
        sel = np.arange(rec.shape[1])[:, None] < nv[None, :]
        plog(f"li_conductor_a{alpha}_unguided_rec_max_abs_diff", float(np.abs(rec - r["rec"])[:, sel].max()), 0.0)
        np.testing.assert_array_equal(rec[:, sel], r["rec"][:, sel])
        np.testing.assert_array_equal(img, r["image"])


@pytest.mark.parametrize("K", [16, 512])
def test_glossy_product_li_matches_oracle(pkg, oracle, scenes, gpu, plog, K):
    """sampleProduct with a NON-diffuse learned BSDF inside the render: each
    rough-conductor bounce conditions the material's learned SDMM4 on
    (theta_i, alpha) and prunes it to 2 lobes (getDMM, roughconductor.cpp:
    182-194; learned_bsdf.h), rotates them to wi (rotate_to_wo) and takes
    them to world through the shading frame (sdmm_proc.cpp:340-355) -- the
    product's non-diffuse branch, the Kitchen's (configs[4], K = 512) glossy
    materials -- beside the diffuse materials' slice-0 rule.  >= 99 % of the
    paths match the CPU Li, whose conditional is the oracle's restatement."""
    desc = scenes.cornell_box(128, 72, conductor=GLOSSY)
    assert desc["learned_models"][list(scenes._BSDFS).index("Floor")] is not None
    sc = pkg.Scene(desc)
    tree = _tree(pkg, sc)
    node_mix = _train(pkg, sc, tree, 4, 8, K=K)
    assert any(m is not None and m.K == K for m in node_mix)
    learned = scenes.diffuse_learned_bsdf(len(desc["reflectance"]) // 3)
    table = pkg.BsdfTable(*learned[:3], device=gpu, diffuse=learned[3])
    img, rec, nv, _ = _device(sc, tree, node_mix, True, table=table)
    aabb, child, _ = tree.nodes()
    r = oracle.li_render(desc, aabb, child, node_mix=_oracle_mixes(oracle, node_mix), guided=True, spp=SPP,
                         seed=SEED, learned=learned, threads=16)
    _compare_guided(oracle, plog, f"li_glossy_product_K{K}", img, rec, nv, r)
    # the conductor's bounces used the product (k * max(M, 2) + j indices of
    # its own rows; the diffuse rows hold one lobe): some guided samples come
    # from the conditioned model's second lobe
    comps = r["comps"]
    assert ((comps >= 0) & (comps % 2 != 0)).sum() > 0


def test_conductor_without_learned_model_plain_conditional(pkg, oracle, scenes, gpu, plog):
    """A rough conductor with no learned model (m_sdmm == nullptr: getDMM
    returns false, roughconductor.cpp:182-184): its product bounces fall back
    to the plain conditional with h 0.5 (sdmm_proc.cpp:383) -- device == CPU
    Li."""
    desc = scenes.cornell_box(128, 72, conductor=GLOSSY, learned=None)
    assert "learned_models" not in desc
    sc = pkg.Scene(desc)
    tree = _tree(pkg, sc)
    node_mix = _train(pkg, sc, tree, 4, 8)
    learned = scenes.diffuse_learned_bsdf(len(desc["reflectance"]) // 3)
    table = pkg.BsdfTable(*learned[:3], device=gpu, diffuse=learned[3])
    img, rec, nv, _ = _device(sc, tree, node_mix, True, table=table)
    aabb, child, _ = tree.nodes()
    r = oracle.li_render(desc, aabb, child, node_mix=_oracle_mixes(oracle, node_mix), guided=True, spp=SPP,
                         seed=SEED, learned=learned, threads=16)
    _compare_guided(oracle, plog, "li_conductor_no_model", img, rec, nv, r)
