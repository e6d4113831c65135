"""GPU: the C++ mirror header (sdmm-mitsuba_amd/host/sdmm_amd.hpp) driven in
the plugin's pattern -- per-leaf mixtures on concurrent host threads, host
training data staged through sdmm_em_step_host -- gives bitwise the same
mixtures as the device-resident Python path, and both match the oracle."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _build(tmp_path):
    exe = tmp_path / "plugin_harness"
    lib = ROOT / "sdmm-mitsuba_amd" / "lib"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT / 'sdmm-mitsuba_amd' / 'host'}",
                    f"-I{ROOT / 'include'}", str(ROOT / "tests" / "cpp" / "plugin_harness.cpp"),
                    f"-L{lib}", "-lsdmm_amd", f"-Wl,-rpath,{lib}", "-pthread", "-o", str(exe)],
                   check=True)
    return exe


def test_plugin_pattern_harness(pkg, oracle, synth, gpu, tmp_path):
    import torch
    K, L, N = 16, 4, 4 * 3000
    b = synth.em_batch(N, 128)
    w = b["w"].copy()
    with open(tmp_path / "in.bin", "wb") as f:
        np.array([N], np.int64).tofile(f)
        np.array([K, L], np.int32).tofile(f)
        b["x"].astype(np.float32).tofile(f)
        w.astype(np.float32).tofile(f)
        b["normals"].astype(np.float32).tofile(f)
    exe = _build(tmp_path)
    subprocess.run([str(exe), str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], check=True, timeout=120)
    out = np.fromfile(tmp_path / "out.bin", np.float32).reshape(L, -1)
    for l in range(L):
        a, e = N * l // L, N * (l + 1) // L
        # TrainingData::push_back drops zero weights (samples.h:281-283)
        keep = w[a:e] != 0
        x = b["x"][:, a:e][:, keep]
        ww = w[a:e][keep]
        nrm = b["normals"][a:e][keep]
        mix = pkg.SDMM(K)
        mix.init_hemisphere(x[0:3, :K // 8].T, nrm[:K // 8], 0.01, 0.1, 0x1A17 + l)
        ds = pkg.DeviceSamples.from_numpy(x, ww)
        for _ in range(5):                       # 3 plugin calls: 2 + 2 + 1 EM steps
            mix.optimize(ds)
        p = mix.get_params()
        got = out[l]
        np.testing.assert_array_equal(got[:K], p["weights"])
        np.testing.assert_array_equal(got[K:7 * K].reshape(K, 6), p["mean"])
        np.testing.assert_array_equal(got[7 * K:].reshape(K, 25), p["cov"])
        # and the exact-E-step oracle agrees to the EM tolerance of
        # test_gpu_parity.py: 1e-4 relative, flat (the north-star bound)
        s = oracle.Samples(x, ww)
        runs = {}
        for mode in ("exact", "accurate"):
            m, st = oracle.hemisphere_init(K // 8, x[0:3, :K // 8].T, nrm[:K // 8], 0.01, 0.1, 0x1A17 + l)
            for _ in range(5):
                oracle.optimize(m, st, s, accurate=mode)
            runs[mode] = np.asarray(m.weights)
        ex = runs["exact"]
        rel = lambda a: float(np.max(np.abs(a - ex) / np.maximum(np.abs(ex), 1e-7)))
        assert rel(p["weights"]) <= 1e-4, (rel(p["weights"]), rel(runs["accurate"]))


@pytest.mark.parametrize("L,debug", [(6, 0), (16, 0), (6, 1)])
def test_plugin_pattern_batched_equals_threaded(pkg, synth, gpu, tmp_path, L, debug):
    """The harness in batched mode (one sdmm_em_step_batched_host per plugin
    call over all leaves, sdmm_amd::em_step_leaves) gives bitwise the same
    per-leaf mixtures as the thread-per-leaf sdmm_em_step_host pattern (L
    host threads at once, each creating, initialising, stepping and
    destroying its own handle).  debug: SDMM_AMD_DEBUG_SYNC=1, every mixture
    call checked by a stream synchronisation (a fault names its call and
    thread)."""
    import os
    env = dict(os.environ, SDMM_AMD_DEBUG_SYNC=str(debug))
    K, N = 16, L * 2500
    b = synth.em_batch(N, 128)
    with open(tmp_path / "in.bin", "wb") as f:
        np.array([N], np.int64).tofile(f)
        np.array([K, L], np.int32).tofile(f)
        b["x"].astype(np.float32).tofile(f)
        b["w"].astype(np.float32).tofile(f)
        b["normals"].astype(np.float32).tofile(f)
    exe = _build(tmp_path)
    subprocess.run([str(exe), str(tmp_path / "in.bin"), str(tmp_path / "threads.bin")], check=True, timeout=120,
                   env=env)
    subprocess.run([str(exe), str(tmp_path / "in.bin"), str(tmp_path / "batched.bin"), "batched"], check=True,
                   timeout=120, env=env)
    a = np.fromfile(tmp_path / "threads.bin", np.float32)
    c = np.fromfile(tmp_path / "batched.bin", np.float32)
    assert a.size == L * K * 32
    np.testing.assert_array_equal(a, c)


@pytest.mark.parametrize("async_", [0, 1])
def test_guiding_model_cpp_driver_equals_python(pkg, gpu, tmp_path, async_):
    """The plugin's render() loop driven from C++ (tests/cpp/guiding_harness.cpp
    through sdmm_amd::Scene / GuidingModel) == the same loop from Python
    (pkg.Guiding), bitwise: every pass's image and the trained-leaf counts;
    optimizeAsync off and on."""
    import importlib
    import torch
    scenes = importlib.import_module("sdmm_mitsuba_amd.scenes")
    W, H, spp_total, spp_it = 96, 54, 32, 8
    d = scenes.cornell_box(W, H)
    nq = d["quads"].size // 9
    with open(tmp_path / "scene.bin", "wb") as f:
        np.array([nq, d["reflectance"].size // 3, d["radiance"].size // 3, W, H, spp_total, spp_it],
                 np.int32).tofile(f)
        d["quads"].astype(np.float32).tofile(f)
        for k in ("flip_normals", "bsdf", "emitter"):
            d[k].astype(np.int32).tofile(f)
        d["reflectance"].astype(np.float32).tofile(f)
        d["radiance"].astype(np.float32).tofile(f)
        np.asarray(d["camera_to_world"], np.float32).tofile(f)
        np.array([d["fov_x_deg"]], np.float32).tofile(f)
    exe = tmp_path / "guiding_harness"
    lib = ROOT / "sdmm-mitsuba_amd" / "lib"
    subprocess.run(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    f"-I{ROOT / 'sdmm-mitsuba_amd' / 'host'}", f"-I{ROOT / 'include'}",
                    str(ROOT / "tests" / "cpp" / "guiding_harness.cpp"), f"-L{lib}", "-lsdmm_amd",
                    "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{lib}", "-Wl,-rpath,/opt/rocm/lib", "-pthread",
                    "-o", str(exe)], check=True)
    subprocess.run([str(exe), str(tmp_path / "scene.bin"), str(tmp_path / "out.bin"), str(tmp_path / "exr")]
                   + (["async"] if async_ else []), check=True, timeout=300)
    out = np.fromfile(tmp_path / "out.bin", np.uint8)
    rec = 12 + 4 * 3 * W * H
    passes = spp_total // spp_it
    assert out.size == passes * rec
    sc = pkg.Scene(d)
    _, _, tmin, tmax = sc.normalization()
    g = pkg.Guiding(tmin, tmax, optimize_async=async_)
    for it in range(passes):
        train = it * spp_it < spp_total // 4
        img, _, st = g.iteration(sc, spp_it, seed=1 + it, push_seed=1001 + it, train=train)
        torch.cuda.synchronize()
        chunk = out[it * rec:(it + 1) * rec]
        head = chunk[:12].view(np.int32)
        assert head[0] == g.trained, (it, head, g.trained)
        if train:
            assert head[1] == st["leaves"] and head[2] == st["optimized"]
        np.testing.assert_array_equal(chunk[12:].view(np.float32).reshape(3, H, W), img.cpu().numpy(),
                                      err_msg=f"pass {it}")
        # the pass's dumps (sdmm_wr.cpp:144-145): the image, and the mean of squares >= its square
        from helpers import read_exr
        exr, attrs = read_exr(tmp_path / "exr" / f"iteration{it:05d}.exr")
        np.testing.assert_array_equal(exr, img.cpu().numpy())
        assert attrs["iteration"] == it and attrs["spp"] == spp_it
        sqr, _ = read_exr(tmp_path / "exr" / f"iteration_sqr{it:05d}.exr")
        assert np.all(sqr >= exr * exr * (1 - 1e-5) - 1e-30)
    assert g.trained > 0


def _build_guide_pattern(tmp_path):
    exe = tmp_path / "guide_pattern_harness"
    lib = ROOT / "sdmm-mitsuba_amd" / "lib"
    subprocess.run(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    f"-I{ROOT / 'include'}", f"-I{ROOT / 'sdmm-mitsuba_amd' / 'host'}",
                    str(ROOT / "tests" / "cpp" / "guide_pattern_harness.cpp"),
                    f"-L{lib}", "-lsdmm_amd", "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{lib}",
                    "-Wl,-rpath,/opt/rocm/lib", "-pthread", "-o", str(exe)], check=True)
    return exe


def write_guide_queries(path, c, u, dg, mode):
    with open(path, "wb") as f:
        np.array([c.shape[1]], np.int64).tofile(f)
        for a in (c, u, dg):
            a.astype(np.float32).tofile(f)
        mode.astype(np.uint8).tofile(f)


@pytest.mark.parametrize("K", [16, 128])
def test_guide_pattern_threads_equal_single_thread(pkg, synth, gpu, tmp_path, K):
    """The plugin's guided bounce from C++ worker threads, each with its own
    guide context on the published tree (tests/cpp/guide_pattern_harness.cpp,
    the pattern of plugin/volpath_sdmm_amd.cpp guideWavefront): 8 threads x
    4096-query tiles == 1 thread, bitwise, and both == one
    sdmm_guide_pdf_wavefront over the whole batch on the original mixtures
    (the harness guides on the checkpoint's restored ones)."""
    import torch
    from test_gpu_wavefront import _queries, _tree_and_leaf_mixtures
    b, t, mixes, leaves = _tree_and_leaf_mixtures(pkg, synth, K)
    nq = 40000
    c, u, d, ct, ut, dt = _queries(gpu, nq, 51, 0.0, 1.0)
    mode = (np.random.default_rng(6).uniform(size=nq) < 0.5).astype(np.uint8)
    dr, pr, cr = t.guide_pdf(mixes, ct, ut, dt, torch.from_numpy(mode).to(gpu))
    torch.cuda.synchronize()
    t.save_json(tmp_path / "model.asdmm", mixes)
    write_guide_queries(tmp_path / "q.bin", c, u, d, mode)
    exe = _build_guide_pattern(tmp_path)
    outs = []
    # one thread; 8 threads on their own contexts; 8 threads gathered by
    # sdmm_amd::GuideBatcher (batches of up to 12 K queries, 2 in flight: the
    # 4096-query tiles straddle batch boundaries and a ragged last tile)
    for i, (threads, extra) in enumerate(((1, []), (8, []), (8, ["2", "batch:12288:300"]))):
        r = subprocess.run([str(exe), str(tmp_path / "model.asdmm"), str(tmp_path / "q.bin"),
                            str(tmp_path / f"o{i}.bin"), str(threads), "4096", "2"] + extra,
                           check=True, timeout=120, capture_output=True, text=True)
        assert '"queries_per_s"' in r.stdout
        outs.append(np.fromfile(tmp_path / f"o{i}.bin", np.uint8))
    np.testing.assert_array_equal(outs[0], outs[1])
    np.testing.assert_array_equal(outs[0], outs[2])
    o = outs[1]
    dd = o[:12 * nq].view(np.float32).reshape(3, nq)
    pp = o[12 * nq:16 * nq].view(np.float32)
    cc = o[16 * nq:].view(np.int32)
    np.testing.assert_array_equal(cc, cr.cpu().numpy())
    np.testing.assert_array_equal(pp, pr.cpu().numpy())
    np.testing.assert_array_equal(dd, np.stack([x.cpu().numpy() for x in dr]))
