#!/usr/bin/env python3
"""Would an exact cull of flushed (sample, component) pairs pay for the
headline responsibility E-step?    CPU measurement at the
bench's state: the synthetic 2^20-sample batch, the K = 128 model after the
bench's 5 warm EM iterations (oracle, accurate mode), then on the first 2^16
samples:

  * live fraction: pairs whose fp32 responsibility is non-zero (the FTZ
    flush of NORM5 exp(-q/2) detInv J pi, mixture_model.h:146-192);
  * spatially live: pairs whose spatial lower bound q_sp = |L_sp (p - mu)|^2
    (the first three rows of L^-1 touch only the position, so q >= q_sp) does
    NOT prove the flush (NORM5 exp(-q_sp / 2) >= 2^-126): the most an exact
    cull could skip without evaluating the directional part;
  * for the kernel's lane = component-pair mapping, the per-lane count of
    spatially live samples in a block of B consecutive samples and its max
    over the 64 lanes (a wave's trip count if each lane walked only its own
    live samples).

usage: python tools/cull_measure.py   (~3 min, 8 threads)"""
import importlib
import importlib.util
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
spec = importlib.util.spec_from_file_location("sdmm_mitsuba_amd", ROOT / "sdmm-mitsuba_amd" / "__init__.py",
                                              submodule_search_locations=[str(ROOT / "sdmm-mitsuba_amd")])
mod = importlib.util.module_from_spec(spec)
sys.modules["sdmm_mitsuba_amd"] = mod
spec.loader.exec_module(mod)
synth = importlib.import_module("sdmm_mitsuba_amd.synth")
from oracle import oracle as orc  # noqa: E402  (test infrastructure: the checker)

N, K, NS = 1 << 20, 128, 1 << 16
b = synth.em_batch(N, 128)
pos, nrm = synth.model_seed_points(b, K)
m, st = orc.hemisphere_init(K // 8, pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, synth.SEED_MODEL, mode=1)
s = orc.Samples(b["x"], b["w"], b["hpdf"], b["is_diffuse"])
for _ in range(5):
    orc.optimize(m, st, s, accurate=True)
sub = orc.Samples(b["x"][:, :NS].copy(), b["w"][:NS].copy())
live = orc.responsibilities(m, sub) != 0
mean = np.asarray(m.mean, np.float64).reshape(-1, 6)
Li = np.asarray(m.cholLInv, np.float64).reshape(-1, 5, 5)[:, :3, :3]
p = b["x"][0:3, :NS].T.astype(np.float64)
u = np.einsum("kij,nkj->nki", Li, p[:, None, :] - mean[None, :, :3])
qsp = (u * u).sum(-1)
thr = 2 * (np.log(float(np.float32(0.39894228040143267794) ** 5)) + 126 * np.log(2))
slive = qsp < thr
print(f"live pairs {live.mean():.3f} ({live.sum(1).mean():.1f} of {K} per sample); "
      f"spatially live {slive.mean():.3f} ({slive.sum(1).mean():.1f} per sample)")
for B in (64, 16):
    lanes = slive.reshape(NS // B, B, K // 2, 2).any(-1).sum(1) / B
    print(f"block {B}: lane live fraction mean {lanes.mean():.3f}, max over the wave's lanes mean "
          f"{lanes.max(1).mean():.3f}")
