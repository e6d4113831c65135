"""Batched per-leaf EM (sdmm_em_step_batched) -- SURVEY.md 8(f) rank 1.

The plugin optimises every tree leaf's own mixture with sdmm::em_step on a
thread pool (volpath_sdmm.cpp:287-311; leaves with >= 16 samples, :140-149).
The batched entry point runs all leaves in one launch sequence.  Parity:
  * bitwise equal to calling sdmm_em_step on each leaf one by one (same work
    split, same partial rows, same fp64 reduction order, same M-step);
  * each leaf against the CPU oracle's StepwiseTangentEM (through the existing
    single-mixture tolerance, 1e-4 relative on the mixture parameters);
  * edge cases: empty leaves, a 1-sample leaf, leaves with non-finite weights,
    leaves of the tile-kernel size class (K = 128), duplicate handles refused.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PARAM_KEYS = ("weights", "mean", "cov", "cdf", "cholLInv", "detInv")


def _leaves(synth, sizes, K, seed=3):
    """Leaf sample sets drawn from the synthetic generator, stored back to back;
    each leaf's seed points are its own first samples (initializeDMMContext
    seeds a leaf from its data, volpath_sdmm.cpp:132-138)."""
    total = int(sum(sizes))
    b = synth.em_batch(max(total, 16), 128)
    rng = np.random.default_rng(seed)
    perm = rng.permutation(b["x"].shape[1])[:total]
    x, w = b["x"][:, perm], b["w"][perm]
    nrm = b["normals"][perm]
    seg = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    return x, w, nrm, seg


def _make_mixes(pkg, synth, x, nrm, seg, K, gpu):
    n_pos = K // 8
    mixes = []
    for i in range(len(seg) - 1):
        a = seg[i]
        # seed positions: the leaf's first samples (or batch samples if the leaf is tiny)
        src = np.arange(a, a + n_pos) if seg[i + 1] - a >= n_pos else np.arange(n_pos)
        m = pkg.SDMM(K, device=gpu.index)
        m.init_hemisphere(x[0:3, src].T.copy(), nrm[src].copy(), synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE,
                          synth.SEED_MODEL + i)
        mixes.append(m)
    return mixes


def _device_samples(pkg, x, w):
    return pkg.DeviceSamples.from_numpy(x, w)


@pytest.mark.parametrize("K,sizes,iters", [
    (16, [4000, 0, 1, 17, 2500, 16, 700, 4096], 2),
    (16, [64] * 40 + [3000] * 3, 1),
    (32, [1000, 1500, 0, 2200], 2),
    (128, [5000, 300, 9000], 2),
    (512, [3000, 40, 7000], 1),
])
def test_batched_equals_sequential_bitwise(pkg, synth, gpu, K, sizes, iters):
    import torch
    x, w, nrm, seg = _leaves(synth, sizes, K)
    w = w.copy()
    if len(w) > 100:
        w[5] = np.inf          # non-finite and zero weights exercise the guards
        w[7] = np.nan
        w[11] = 0.0
    ds = _device_samples(pkg, x, w)
    batched = _make_mixes(pkg, synth, x, nrm, seg, K, gpu)
    single = _make_mixes(pkg, synth, x, nrm, seg, K, gpu)
    pkg.em_step_batched(batched, ds, seg, iters)
    for i, m in enumerate(single):
        a, b = int(seg[i]), int(seg[i + 1])
        leaf = pkg.DeviceSamples([t[a:b] for t in ds.x], ds.w[a:b])
        if b > a:
            m.optimize(leaf, iters)
    torch.cuda.synchronize()
    for i in range(len(sizes)):
        pb, ps = batched[i].get_params(), single[i].get_params()
        for k in PARAM_KEYS + ("valid",):
            np.testing.assert_array_equal(pb[k], ps[k], err_msg=f"leaf {i} ({sizes[i]} samples) {k}")
        sb, ss = batched[i].get_state(), single[i].get_state()
        for k in sb:
            np.testing.assert_array_equal(sb[k], ss[k], err_msg=f"leaf {i} state {k}")


def test_batched_leaves_match_oracle(pkg, oracle, synth, gpu):
    """Each leaf of a batched step against the oracle run on that leaf alone,
    with the bound of test_em_matches_oracle: distance to the exact (fp64
    E-step) EM <= max(1e-4, 2 x the fp32-E oracle's own distance)."""
    import torch
    from test_gpu_parity import RTOL_PARAMS, _exact_em, _param_err
    K, sizes, iters = 16, [3000, 5000, 2000], 2
    x, w, nrm, seg = _leaves(synth, sizes, K, seed=9)
    ds = _device_samples(pkg, x, w)
    mixes = _make_mixes(pkg, synth, x, nrm, seg, K, gpu)
    pkg.em_step_batched(mixes, ds, seg, iters)
    torch.cuda.synchronize()
    n_pos = K // 8
    for i in range(len(sizes)):
        a, b = int(seg[i]), int(seg[i + 1])
        src = np.arange(a, a + n_pos)
        args = (n_pos, x[0:3, src].T.copy(), nrm[src].copy(), synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE,
                synth.SEED_MODEL + i)
        om, ost = oracle.hemisphere_init(*args, mode=1)
        xm, xst = oracle.hemisphere_init(*args, mode=1)
        os_ = oracle.Samples(x[:, a:b], w[a:b])
        leaf = {"x": x[:, a:b], "w": w[a:b], "hpdf": None, "is_diffuse": None}
        for _ in range(iters):
            assert oracle.optimize(om, ost, os_, accurate=True) == 1
            _exact_em(oracle, xm, xst, leaf, 1)
        p = mixes[i].get_params()
        o = {k: getattr(om, k) for k in ("weights", "mean", "cov")}
        xx = {k: getattr(xm, k) for k in ("weights", "mean", "cov")}
        eg, eo = _param_err(p, xx), _param_err(o, xx)
        assert eg <= max(RTOL_PARAMS, 2 * eo), f"leaf {i}: gpu {eg:.2e} vs oracle-fp32-E {eo:.2e}"


def test_batched_rejects_bad_arguments(pkg, synth, gpu):
    x, w, nrm, seg = _leaves(synth, [100, 100], 16)
    ds = _device_samples(pkg, x, w)
    mixes = _make_mixes(pkg, synth, x, nrm, seg, 16, gpu)
    with pytest.raises(pkg.SDMMError):
        pkg.em_step_batched([mixes[0], mixes[0]], ds, seg, 1)          # duplicate handle
    with pytest.raises(pkg.SDMMError):
        pkg.em_step_batched(mixes, ds, np.array([0, 150, 100]), 1)    # decreasing offsets
    with pytest.raises(pkg.SDMMError):
        pkg.em_step_batched(mixes, ds, np.array([0, 100, 10 ** 6]), 1)  # past the batch
    other = pkg.SDMM(32, device=gpu.index)
    other.init_hemisphere(x[0:3, :4].T.copy(), nrm[:4].copy(), synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, 1)
    with pytest.raises(pkg.SDMMError):
        pkg.em_step_batched([mixes[0], other], ds, seg, 1)            # K differs


@pytest.mark.parametrize("fail_at", [1, 3])
def test_create_many_failure_cleanup(pkg, gpu, monkeypatch, fail_at):
    """A stream-ordered slab whose member fail_at (> 0) fails to be created:
    the members already carved are destroyed, the slab is freed exactly once
    (no use after free), the call reports the error, and the next creation
    from a fresh slab succeeds (create_many's cleanup path)."""
    import ctypes as C
    import torch
    lib = pkg.lib()
    st = torch.cuda.Stream(gpu)
    out = (C.c_void_p * 5)()
    monkeypatch.setenv("SDMM_TEST_FAIL_MEMBER", str(fail_at))
    rc = lib.sdmm_create_many_on_stream(16, None, gpu.index, C.c_void_p(st.cuda_stream), 5, out)
    assert rc == 0, "the injection must need the explicit debug switch"
    for v in out:
        lib.sdmm_destroy(C.c_void_p(v))
    monkeypatch.setenv("SDMM_DEBUG_FAULT_INJECTION", "1")
    rc = lib.sdmm_create_many_on_stream(16, None, gpu.index, C.c_void_p(st.cuda_stream), 5, out)
    assert rc != 0
    assert all(v is None for v in out), "failed creation left handles behind"
    monkeypatch.delenv("SDMM_TEST_FAIL_MEMBER")
    rc = lib.sdmm_create_many_on_stream(16, None, gpu.index, C.c_void_p(st.cuda_stream), 5, out)
    assert rc == 0
    for v in out:
        lib.sdmm_destroy(C.c_void_p(v))
    torch.cuda.synchronize()


def test_iterations_run_concurrent_threads(pkg, synth, gpu):
    """sdmm_iterations_run with >= 64 mixtures from 4 host threads at once --
    the plugin's per-leaf worker threads (volpath_sdmm.cpp:287-311) calling it
    beside each other's mixture creation / EM steps / destruction (hipMalloc /
    hipFree) -- completes and returns every mixture's count.  (Round 2's
    version with stream-ordered pool allocations and pageable copies hung in
    this pattern; DESIGN.md, training passes.)"""
    import ctypes as C
    import threading
    import torch
    lib = pkg.lib()
    b = synth.em_batch(4096, 128)
    pos, nrm = synth.model_seed_points(b, 16)
    ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"])
    errors, counts = [], {}

    def worker(t):
        try:
            mixes = [pkg.SDMM(16, device=gpu.index) for _ in range(64 + 8 * t)]
            for m in mixes:
                m.init_hemisphere(pos[:2], nrm[:2], synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, 3 + t)
            for j in range(t + 1):
                mixes[j].optimize(ds, 1 + j % 3)
            tab = (C.c_void_p * len(mixes))(*[m.h.value for m in mixes])
            out = (C.c_int * len(mixes))()
            for rep in range(20):
                assert lib.sdmm_iterations_run(tab, len(mixes), out) == 0
                extra = pkg.SDMM(16, device=gpu.index)      # a creation + destruction beside it
                del extra
            counts[t] = list(out)
        except Exception as e:   # surfaced below
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=90)
    assert not any(th.is_alive() for th in ths), "sdmm_iterations_run did not complete"
    assert not errors, errors
    torch.cuda.synchronize()
    for t in range(4):
        expect = [1 + j % 3 for j in range(t + 1)] + [0] * (64 + 8 * t - t - 1)
        assert counts[t] == expect, (t, counts[t][:8])
