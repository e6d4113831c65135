"""The headline configuration (BASELINE configs[1]) at FULL size: N = 2^20
synthetic samples, K = 128, the model after 5 warm EM iterations -- the exact
workload bench.py times.  The oracle cannot evaluate 2^20 x 128 pairs in test
time, so the full batch is checked through size-independent properties and a
strided subsample against the oracle:

  * every responsibility is finite; every live row sums to 1 (|sum - 1| <=
    1e-5), dead rows (all components flushed or the sample rejected) are the
    ones the oracle also rejects on the subsample;
  * a strided 4096-row subsample is held to the bound of
    test_gpu_parity._check_resp (4 x the fp32 oracle's distance to the fp64
    evaluation + 1e-5);
  * the full-batch statistics: weightSum equals the fp64 sum of the finite
    weights (rel 1e-6), and the split-phase statistics of two half shards add
    up to the whole batch's (linearity, rel 1e-6 of the total weight).
"""
import numpy as np
import pytest

from test_gpu_parity import _check_resp

pytestmark = pytest.mark.gpu


def test_headline_full_size(pkg, oracle, synth, gpu, plog):
    import torch
    N, K = 1 << 20, 128
    b = synth.em_batch(N, 128)
    pos, nrm = synth.model_seed_points(b, K)
    mix = pkg.SDMM(K)
    mix.init_hemisphere(pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, synth.SEED_MODEL)
    ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"], b["hpdf"], b["is_diffuse"], device=gpu)
    for _ in range(5):
        mix.optimize(ds)
    resp = torch.empty((N, K), device=gpu)
    mix.posterior(ds, resp)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(resp).all())
    rs = resp.sum(1, dtype=torch.float64)
    live = rs > 0
    rs_err = float((rs[live] - 1.0).abs().max())
    plog("full_size_rowsum_abs_err", rs_err, 1e-5, live_rows=int(live.sum()))
    assert rs_err <= 1e-5
    # strided subsample against the oracle
    sub = np.arange(0, N, N // 4096)
    got = resp[torch.from_numpy(sub).to(gpu)].cpu().numpy()
    p = mix.get_params()
    m = oracle.Mixture(K)
    m.copy_params_from(p)
    m.valid[:] = p["valid"]
    ref = oracle.responsibilities(m, oracle.Samples(b["x"][:, sub], b["w"][sub]))
    _check_resp(got, ref, p, b["x"][:, sub], plog)
    np.testing.assert_array_equal(live.cpu().numpy()[sub], ref.sum(1) > 0)
    del resp

    # statistics over the whole batch: weightSum and shard linearity
    L = pkg.stats_len(K)
    full = torch.zeros(L, dtype=torch.float64, device=gpu)
    mix.estep_stats(ds, full)
    halves = torch.zeros(L, dtype=torch.float64, device=gpu)
    part = torch.zeros(L, dtype=torch.float64, device=gpu)
    for r in range(2):
        mix.estep_stats(ds.shard(r, 2), part)
        mix.synchronize()
        halves += part
    torch.cuda.synchronize()
    w = b["w"].astype(np.float64)
    ws = w[np.isfinite(w)].sum()
    full = full.cpu().numpy()
    halves = halves.cpu().numpy()
    e_ws = abs(full[1] - ws) / ws
    e_lin = float(np.abs(full - halves).max() / abs(full[1]))
    plog("full_size_weightsum_rel_err", e_ws, 1e-6)
    plog("full_size_shard_linearity_rel_err", e_lin, 1e-6)
    assert e_ws <= 1e-6
    assert e_lin <= 1e-6
