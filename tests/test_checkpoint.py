"""Checkpoints (.asdmm JSON) -- the accelerator save of
saveCheckpoint() -> sdmm::save_json(m_accelerator, path)
(volpath_sdmm.cpp:117-126) and jmm MixtureModel::save/load
(mixture_model.h:315-326).  sdmm-lib's own schema is absent from the snapshot
(parity unpinned for the file format); what is pinned is the round trip: a
reloaded tree has the saved node table and finds the same leaves, a reloaded
mixture has bitwise the saved canonical + derived arrays and stepwise state,
and guides / steps bitwise like the original (GPU tests).

CPU tests cover the tree-only checkpoint and the rejection of malformed files
(no device objects are created for them)."""
import json

import numpy as np
import pytest


def _tree(pkg, synth, depth=2, threshold=3000, n=40000):
    b = synth.em_batch(n, 128)
    t = pkg.STree(np.float32([0, 0, 0]), np.float32([1, 0.9, 0.8]))
    t.split_to_depth(depth)
    t.split(b["x"][0:3].copy(), threshold)
    return b, t


def test_tree_checkpoint_round_trip(pkg, synth, oracle, tmp_path):
    b, t = _tree(pkg, synth)
    path = tmp_path / "model_00000.asdmm"
    t.save_json(path)
    doc = json.loads(path.read_text())
    assert doc["format"] == "sdmm-amd.asdmm" and doc["version"] == 1
    assert doc["num_nodes"] == t.num_nodes and doc["mixtures"] == []
    t2, mixes = pkg.STree.load_json(path)
    assert mixes == [None] * t.num_nodes
    for a, e in zip(t.nodes(), t2.nodes()):
        np.testing.assert_array_equal(a, e)
    # the reloaded table routes points like the oracle's find on the saved one
    aabb, child, _ = t2.nodes()
    p = b["x"][0:3].T[:3000].copy()
    np.testing.assert_array_equal(oracle.stree_find(aabb, child, p), oracle.stree_find(*t.nodes()[:2], p))


def test_set_nodes_validates_the_table(pkg, synth):
    _, t = _tree(pkg, synth, depth=1, threshold=100000)
    aabb, child, axis = t.nodes()
    t.set_nodes(aabb, child, axis)                      # identity
    bad = child.copy()
    bad[0, 0] = 0                                       # a cycle: root is its own child
    with pytest.raises(pkg.SDMMError, match="malformed"):
        t.set_nodes(aabb, bad, axis)
    bad = child.copy()
    bad[0, 1] = -1                                      # half a split
    with pytest.raises(pkg.SDMMError, match="malformed"):
        t.set_nodes(aabb, bad, axis)
    ax = axis.copy()
    ax[0] = 3
    with pytest.raises(pkg.SDMMError, match="malformed"):
        t.set_nodes(aabb, child, ax)
    # the failed calls left the table unchanged
    for a, e in zip((aabb, child, axis), t.nodes()):
        np.testing.assert_array_equal(a, e)


@pytest.mark.parametrize("mutate,msg", [
    (lambda d: d.update(format="other"), "format"),
    (lambda d: d.update(version=2), "format"),
    (lambda d: d.update(num_nodes=0), "num_nodes"),
    (lambda d: d["nodes"]["aabb"].pop(), "node table"),
    (lambda d: d["nodes"]["child"].__setitem__(0, 0), "malformed"),
    (lambda d: d["mixtures"].append({"node": 0, "mixture": {"K": 16}}), "em_params"),
    (lambda d: d["mixtures"].append({"node": 10 ** 6, "mixture": {}}), "node id"),
])
def test_malformed_checkpoints_are_rejected(pkg, synth, tmp_path, mutate, msg):
    _, t = _tree(pkg, synth, depth=1, threshold=100000)
    path = tmp_path / "m.asdmm"
    t.save_json(path)
    doc = json.loads(path.read_text())
    mutate(doc)
    path.write_text(json.dumps(doc))
    with pytest.raises(pkg.SDMMError, match=msg):
        pkg.STree.load_json(path)


def test_truncated_and_missing_files(pkg, synth, tmp_path):
    _, t = _tree(pkg, synth, depth=1, threshold=100000)
    path = tmp_path / "m.asdmm"
    t.save_json(path)
    text = path.read_text()
    path.write_text(text[: len(text) // 2])
    with pytest.raises(pkg.SDMMError, match="parse"):
        pkg.STree.load_json(path)
    with pytest.raises(pkg.SDMMError, match="cannot open"):
        pkg.STree.load_json(tmp_path / "absent.asdmm")


# ---------------------------------------------------------------- GPU -------
def _fitted(pkg, synth, K, n=1 << 15, iters=3, seed=7):
    b = synth.em_batch(n, 128)
    pos, nrm = synth.model_seed_points(b, K)
    m = pkg.SDMM(K)
    m.init_hemisphere(pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, seed)
    ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"])
    for _ in range(iters):
        m.optimize(ds)
    return b, m, ds


def _assert_same_mixture(a, e):
    pa, pe = a.get_params(), e.get_params()
    for k in pa:
        np.testing.assert_array_equal(np.asarray(pa[k]), np.asarray(pe[k]), err_msg=k)
    sa, se = a.get_state(), e.get_state()
    for k in sa:
        np.testing.assert_array_equal(sa[k], se[k], err_msg=k)
    assert a.em_params() == e.em_params()


@pytest.mark.gpu
@pytest.mark.parametrize("K", [16, 128])
def test_mixture_checkpoint_is_bitwise(pkg, synth, gpu, tmp_path, K):
    """save -> load gives the same arrays and state; the next EM step and a
    guided batch from the reloaded mixture are bitwise the original's."""
    import torch
    b, m, ds = _fitted(pkg, synth, K)
    path = tmp_path / "mix.json"
    m.save_json(path)
    m2 = pkg.SDMM.load_json(path)
    assert m2.K == K
    _assert_same_mixture(m, m2)
    m.optimize(ds)
    m2.optimize(ds)
    torch.cuda.synchronize()
    _assert_same_mixture(m, m2)
    c, u = synth.sample_queries_near(b, 4096, seed=3)
    ct = [torch.from_numpy(c[i].copy()).to(gpu) for i in range(3)]
    ut = [torch.from_numpy(u[i].copy()).to(gpu) for i in range(3)]
    d1, p1, k1 = m.guide(ct, ut)
    d2, p2, k2 = m2.guide(ct, ut)
    torch.cuda.synchronize()
    assert torch.equal(k1, k2) and torch.equal(p1, p2)
    for x, y in zip(d1, d2):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_accelerator_checkpoint_guides_bitwise(pkg, synth, gpu, tmp_path):
    """The whole accelerator (tree + per-leaf mixtures, some leaves untrained):
    the reloaded one serves a guided wavefront bitwise like the saved one."""
    import torch
    from tests.test_gpu_wavefront import _queries, _tree_and_leaf_mixtures
    b, t, mixes, leaves = _tree_and_leaf_mixtures(pkg, synth, 16)
    path = tmp_path / "model_00003.asdmm"
    t.save_json(path, mixes)
    t2, mixes2 = pkg.STree.load_json(path)
    assert [m is None for m in mixes] == [m is None for m in mixes2]
    for a, e in zip(mixes, mixes2):
        if a is not None:
            _assert_same_mixture(a, e)
    _, _, _, c, u, _ = _queries(gpu, 1 << 14, seed=5)
    r1 = t.guide(mixes, c, u)
    r2 = t2.guide(mixes2, c, u)
    torch.cuda.synchronize()
    for x, y in zip(r1[0] + [r1[1], r1[2]], r2[0] + [r2[1], r2[2]]):
        assert torch.equal(x, y)


def test_cpp_mirror_run_outputs(pkg, tmp_path):
    """The C++ mirror writes the integrator's run outputs (scene_norm.json,
    stats.json, checkpoints/model_%05i.asdmm) in the layout the reference's
    scripts read (combine_renders.py:100-105, run_tests.py:74-78), and reloads
    the checkpoint -- CPU only (tree without mixtures)."""
    import subprocess
    src = tmp_path / "w.cpp"
    src.write_text(r'''
#include "sdmm_amd.hpp"
#include <cstdio>
int main(int argc, char** argv) {
    const std::string dir = argv[1];
    const float lo[3] = {-1.5f, 0.f, 2.f}, hi[3] = {1.5f, 2.f, 3.f};
    sdmm_amd::write_scene_norm(dir + "/scene_norm.json", lo, 3.0f);
    sdmm_amd::SpatialTree t(lo, hi);
    t.split_to_depth(3);
    sdmm_amd::RunStats st;
    double total = 0;
    for (int it = 0; it < 3; ++it) {
        total += 0.5 * (it + 1);
        st.push(it, 0.5 * (it + 1), total, 3.25, 4 << it, (4 << (it + 1)) - 4);
        sdmm_amd::save_checkpoint(dir + "/run", it, t, {});
    }
    st.write(dir + "/stats.json");
    std::vector<std::unique_ptr<sdmm_amd::Mixture>> mixes;
    auto t2 = sdmm_amd::SpatialTree::load_json(dir + "/run/checkpoints/model_00002.asdmm", 0, mixes);
    std::printf("%d %d %zu\n", t.nodes(), t2->nodes(), mixes.size());
    return t.nodes() == t2->nodes() && (int)mixes.size() == t.nodes() ? 0 : 1;
}
''')
    lib = pkg.LIB_PATH.parent
    exe = tmp_path / "w"
    root = pkg.REPO
    subprocess.run(["g++", "-std=c++17", f"-I{root / 'sdmm-mitsuba_amd' / 'host'}", f"-I{root / 'include'}",
                    str(src), f"-L{lib}", "-lsdmm_amd", f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.split() == ["1023", "1023", "1023"]   # split_to_depth(3): 3 axis splits per level, 2^9 leaves
    norm = json.loads((tmp_path / "scene_norm.json").read_text())
    assert norm == {"scene_min": [-1.5, 0.0, 2.0], "spatial_norm": 3.0}
    stats = json.loads((tmp_path / "stats.json").read_text())
    assert [s["iteration"] for s in stats] == [0, 1, 2]
    assert stats[-1]["total_elapsed_seconds"] == 3.0 and stats[-1]["spp"] == 16
    assert set(stats[0]) == {"iteration", "elapsed_seconds", "total_elapsed_seconds", "mean_path_length",
                             "spp", "total_spp"}
    assert sorted(p.name for p in (tmp_path / "run" / "checkpoints").iterdir()) == \
        ["model_00000.asdmm", "model_00001.asdmm", "model_00002.asdmm"]


def test_write_exr_round_trip(pkg, tmp_path):
    """iteration%05i.exr (SDMMWorkResult::dumpIndividual, sdmm_wr.cpp:115-146):
    a float RGB OpenEXR with the spp / iteration / time attributes, read back
    bit for bit by an independent minimal reader."""
    from helpers import read_exr
    rng = np.random.default_rng(3)
    rgb = rng.standard_normal((3, 7, 11)).astype(np.float32) * 100
    rgb[1, 2, 3] = np.inf
    path = tmp_path / "iteration00003.exr"
    pkg.write_exr(path, rgb, spp=8, iteration=3, time=1.25)
    back, attrs = read_exr(path)
    np.testing.assert_array_equal(back, rgb)
    assert attrs["spp"] == 8 and attrs["iteration"] == 3 and attrs["time"] == 1.25
    assert [c for c, _ in attrs["channels"]] == ["B", "G", "R"]
