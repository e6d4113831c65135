#!/usr/bin/env python3
"""Guided-query microbenchmark (A/B of guide-kernel variants).

The bench's guide line in isolation: a K=128 mixture after 5 EM steps on the
2^20-sample synthetic batch, Q = 2^20 queries near the samples, device time
per guide call from one HIP-event pair on the mixture's stream; plus the tree
wavefront (K=16 leaves) with events on the tree's own stream.  Prints one JSON
line.  SDMM_AMD_LIB selects an alternative build of the library (variant .so
files built with extra -D flags), e.g. SDMM_AMD_LIB=build_ab/noscreen.so."""
import importlib.util
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def load_pkg():
    spec = importlib.util.spec_from_file_location("sdmm_mitsuba_amd", ROOT / "sdmm-mitsuba_amd" / "__init__.py",
                                                  submodule_search_locations=[str(ROOT / "sdmm-mitsuba_amd")])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["sdmm_mitsuba_amd"] = mod
    spec.loader.exec_module(mod)
    if os.environ.get("SDMM_AMD_LIB"):
        mod.LIB_PATH = Path(os.environ["SDMM_AMD_LIB"]).resolve()
    return mod


def timed(torch, fn, stream, steps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    ev[0].record(stream)
    for _ in range(steps):
        fn()
    ev[1].record(stream)
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1e3 / steps   # us


def digest(a):
    return int(np.bitwise_xor.reduce((a.astype(np.int64) * 2654435761 + np.arange(a.size)) % (1 << 31)))


def main():
    import torch
    pkg = load_pkg()
    import importlib
    synth = importlib.import_module("sdmm_mitsuba_amd.synth")
    dev = torch.device("cuda:0")
    N, K, Q = 1 << 20, 128, 1 << 20
    b = synth.em_batch(N, 128)
    pos, nrm = synth.model_seed_points(b, K)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"], device=dev)
        m = pkg.SDMM(K, stream=stream)
        m.init_hemisphere(pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, synth.SEED_MODEL)
        for _ in range(int(os.environ.get("GUIDE_EM_ITERS", "15"))):   # bench.py: 5 warm + 10 timed EM steps
            m.optimize(ds)
        if os.environ.get("GUIDE_CAP"):
            m.set_guide_capacity(int(os.environ["GUIDE_CAP"]))
        c, u = synth.sample_queries_near(b, Q)
        ct = [torch.from_numpy(c[i].copy()).to(dev) for i in range(3)]
        ut = [torch.from_numpy(u[i].copy()).to(dev) for i in range(3)]
        out = m.guide(ct, ut)
        torch.cuda.synchronize()
        g_us = timed(torch, lambda: m.guide(ct, ut, out), stream, 10)
        res = {"guide_us": g_us, "guide_Gq_per_s": Q / g_us * 1e-3, "comp_digest": digest(out[2].cpu().numpy()),
               "pdf_sum": float(out[1].cpu().numpy().astype(np.float64).sum())}
        # tree wavefront: K=16 leaves fitted on their routed samples
        tree = pkg.STree(np.float32([0, 0, 0]), np.float32([1, 1, 1]))
        tree.split_to_depth(3)
        tree.split(b["x"][0:3], 16000)
        tree.set_stream(stream)
        routed, seg = tree.route(ds)
        xs = np.stack([x.cpu().numpy() for x in routed.x])
        mixes = [None] * tree.num_nodes
        for v in range(tree.num_nodes):
            a, e = int(seg[v]), int(seg[v + 1])
            if e - a < 64:
                continue
            mm = pkg.SDMM(16, stream=stream)
            mm.init_hemisphere(xs[0:3, a:a + 2].T.copy(), xs[3:6, a:a + 2].T.copy(), synth.DEPTH_PRIOR,
                               synth.SPATIAL_DISTANCE, synth.SEED_MODEL + v)
            leaf = pkg.DeviceSamples([x[a:e] for x in routed.x], routed.w[a:e])
            mm.optimize(leaf)
            mm.optimize(leaf)
            mixes[v] = mm
        tree.bind(mixes)
        tout = tree.guide(None, ct, ut)
        torch.cuda.synchronize()
        tstream = torch.cuda.ExternalStream(int(pkg.lib().sdmm_stree_get_stream(tree.h) or 0))
        res["wavefront_us"] = timed(torch, lambda: tree.guide(None, ct, ut, tout), tstream, 10)
        res["wavefront_Gq_per_s"] = Q / res["wavefront_us"] * 1e-3
        res["wavefront_comp_digest"] = digest(tout[2].cpu().numpy())
    res["lib"] = pkg.LIB_PATH.name
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
