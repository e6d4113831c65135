#!/usr/bin/env python3
"""Guided-query throughput vs query order: the bench's queries (sample
positions, random order) as given, and the same queries pre-sorted along a
Morton curve of the condition position (what a coherent wavefront looks like).

    python tools/guide_coherence.py [--Q 1048576] [--K 128]
"""
import argparse
import importlib
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def morton3(c, bits=10):
    q = np.clip((c * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1)
    key = np.zeros(c.shape[1], np.int64)
    for b in range(bits):
        for a in range(3):
            key |= ((q[a] >> b) & 1) << (3 * b + a)
    return key


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--Q", type=int, default=1 << 20)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from conftest import load_pkg
    pkg = load_pkg()
    synth = importlib.import_module("sdmm_mitsuba_amd.synth")
    dev = torch.device("cuda:0")
    b = synth.em_batch(1 << 20, 128)
    pos, nrm = synth.model_seed_points(b, a.K)
    mix = pkg.SDMM(a.K)
    mix.init_hemisphere(pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, synth.SEED_MODEL)
    ds = pkg.DeviceSamples.from_numpy(b["x"], b["w"], device=dev)
    for _ in range(5):
        mix.optimize(ds)
    c, u = synth.sample_queries_near(b, a.Q)
    order = np.argsort(morton3(c), kind="stable")
    for name, cc, uu in (("random", c, u), ("morton-sorted", c[:, order], u[:, order])):
        ct = [torch.from_numpy(np.ascontiguousarray(cc[i])).to(dev) for i in range(3)]
        ut = [torch.from_numpy(np.ascontiguousarray(uu[i])).to(dev) for i in range(3)]
        out = mix.guide(ct, ut)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            mix.guide(ct, ut, out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        print(f"{name:14s} {ms:.3f} ms  {a.Q / ms / 1e3:.1f} M queries/s", flush=True)


if __name__ == "__main__":
    main()
