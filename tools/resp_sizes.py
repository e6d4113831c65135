#!/usr/bin/env python3
"""Responsibility E-step time per launch at the strong-scaling shard sizes
(N = 2^20 / world for world = 1, 2, 4, 8) with the kernel SDMM_RESP_KERNEL
selects (default: the library's choice).

    python tools/resp_sizes.py [--K 128]
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
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import torch
    from conftest import load_pkg
    pkg = load_pkg()
    synth = importlib.import_module("sdmm_mitsuba_amd.synth")
    dev = torch.device("cuda:0")
    N = 1 << 20
    b = synth.em_batch(N, 128)
    pos, nrm = synth.model_seed_points(b, a.K)
    mix = pkg.SDMM(a.K)
    mix.init_hemisphere(pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, synth.SEED_MODEL)
    ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"], b["hpdf"], b["is_diffuse"], device=dev)
    for _ in range(5):
        mix.optimize(ds)
    for world in (1, 2, 4, 8):
        n = N // world
        part = pkg.DeviceSamples.from_numpy(b["x"][:, :n].copy(), b["w"][:n].copy(), b["hpdf"][:n].copy(),
                                            b["is_diffuse"][:n].copy(), device=dev)
        resp = torch.empty((n, a.K), device=dev)
        for _ in range(5):
            mix.posterior(part, resp)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            mix.posterior(part, resp)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / a.reps
        print(f"{mix.kernel_name('resp'):36s} world {world}  n {n:8d}  {us:8.1f} us/launch  "
              f"{n / us / 1e3:6.2f} G samples/s", flush=True)


if __name__ == "__main__":
    main()
