#!/usr/bin/env python3
"""Launch each hot kernel a few times on the bench workload, for rocprofv3
PMC passes (tools/gpu_pmc.sh).  No timing here: the counters are the output.

    python tools/prof_kernels.py [--K 128] [--N 1048576] [--reps 5] [--what resp,stats,guide]
"""
import argparse
import importlib
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--N", type=int, default=1 << 20)
    ap.add_argument("--Q", type=int, default=1 << 18)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--em-warm", type=int, default=5)
    ap.add_argument("--what", default="resp,stats,guide")
    a = ap.parse_args()
    import torch
    from conftest import load_pkg
    pkg = load_pkg()
    synth = importlib.import_module("sdmm_mitsuba_amd.synth")
    dev = torch.device("cuda:0")
    b = synth.em_batch(a.N, 128)
    pos, nrm = synth.model_seed_points(b, a.K)
    mix = pkg.SDMM(a.K)
    mix.init_hemisphere(pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, synth.SEED_MODEL)
    ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"], b["hpdf"], b["is_diffuse"], device=dev)
    for _ in range(a.em_warm):
        mix.optimize(ds)
    what = a.what.split(",")
    if "resp" in what:
        resp = torch.empty((a.N, a.K), device=dev)
        for _ in range(a.reps):
            mix.posterior(ds, resp)
    if "stats" in what:
        st = torch.zeros(pkg.stats_len(a.K), dtype=torch.float64, device=dev)
        for _ in range(a.reps):
            mix.estep_stats(ds, st)
    if "guide" in what:
        c, u = synth.queries(a.Q)
        ct = [torch.from_numpy(c[i].copy()).to(dev) for i in range(3)]
        ut = [torch.from_numpy(u[i].copy()).to(dev) for i in range(3)]
        for _ in range(a.reps):
            mix.guide(ct, ut)
    torch.cuda.synchronize()
    print("prof_kernels done")


if __name__ == "__main__":
    main()
