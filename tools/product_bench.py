"""Kitchen product bench in isolation (bench.py large_k's guide_product_K512
workload): K=512 model after 6 EM steps on the 2^20-sample batch, 2^18
queries, 8 materials x 8 lobes.  Prints per-call time and the number of
queries that took the full-K fallback, per candidate capacity."""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from bench import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=512)
    ap.add_argument("--em", type=int, default=6)
    ap.add_argument("--Q", type=int, default=1 << 18)
    ap.add_argument("--caps", default="40")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dump", help="save the fitted mixture's parameters and the queries (npz)")
    a = ap.parse_args()
    import torch
    import importlib
    pkg = load_pkg()
    synth = importlib.import_module("sdmm_mitsuba_amd.synth")
    dev = torch.device("cuda:0")
    batch = synth.em_batch(1 << 20, 128)
    ds = pkg.DeviceSamples.from_numpy(batch["x"], batch["w"], batch["hpdf"], batch["is_diffuse"], device=dev)
    pos, nrm = synth.model_seed_points(batch, a.K)
    m = pkg.SDMM(a.K)
    m.init_hemisphere(pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, synth.SEED_MODEL)
    for _ in range(a.em):
        m.optimize(ds)
    q = a.Q
    c, u = synth.sample_queries_near(batch, q, seed=synth.SEED_QUERIES + 7)
    B, M = 8, 8
    bw, bmean, bcov = synth.bsdf_table(B, M)
    F = synth.shading_frames(q)
    mat = (np.arange(q) % B).astype(np.int32)
    tt = lambda x: [torch.from_numpy(np.ascontiguousarray(x[i])).to(dev) for i in range(x.shape[0])]
    ct, ut, Ft = tt(c), tt(u), tt(F.T)
    matt = torch.from_numpy(mat).to(dev)
    table = pkg.BsdfTable(bw, bmean, bcov, device=dev)
    if a.dump:
        np.savez_compressed(a.dump, c=c, u=u, F=F, mat=mat, **m.get_params())
    for cap in [int(x) for x in a.caps.split(",")]:
        m.set_guide_capacity(cap)
        m.guide_product(ct, ut, table, matt, Ft)
        fb = m.guide_fallback_count()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            m.guide_product(ct, ut, table, matt, Ft)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.reps
        print(f"K={a.K} cap={cap}: {dt * 1e3:.2f} ms/call, {q / dt / 1e6:.2f} M queries/s, "
              f"fallback queries {fb} ({fb / q:.2%})", flush=True)


if __name__ == "__main__":
    main()
