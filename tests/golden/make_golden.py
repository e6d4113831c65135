#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.npz) with the CPU oracle.

The reference ships no golden vectors for this path, so these
fixtures are regression vectors of the oracle (itself pinned by the analytic
KATs in tests/test_oracle.py).  Every fixture stores its inputs, so it does not
depend on the synthetic generator staying unchanged.

    python tests/golden/make_golden.py
"""
import importlib
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_pkg  # noqa: E402

OUT = Path(__file__).resolve().parent


def mixture_arrays(m):
    from oracle.oracle import MIX_FIELDS
    d = {f: np.array(getattr(m, f)) for f in MIX_FIELDS}
    d["valid"] = m.valid.copy()
    d["normalization"] = np.float32(m.s.normalization)
    return d


def main():
    load_pkg()
    synth = importlib.import_module("sdmm_mitsuba_amd.synth")
    from oracle import oracle as o
    o.build()

    # --- init + responsibilities + statistics (K=16 and K=128) -------------
    for K, N in ((16, 1024), (128, 512)):
        b = synth.em_batch(N, 128, heuristic=True)
        pos, nrm = synth.model_seed_points(b, K)
        m, st = o.hemisphere_init(K // 8, pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE,
                                  synth.SEED_MODEL, mode=1)
        s = o.Samples(b["x"], b["w"], b["hpdf"], b["is_diffuse"])
        resp = o.responsibilities(m, s)
        out = {"x": b["x"], "w": b["w"], "hpdf": b["hpdf"], "is_diffuse": b["is_diffuse"],
               "seed_pos": pos, "seed_nrm": nrm, "resp": resp,
               "stats_faithful": o.calculate_stats(m, s, accurate="faithful"),
               "stats_accurate": o.calculate_stats(m, s, accurate="accurate"),
               "stats_exact": o.calculate_stats(m, s, accurate="exact")}
        out.update({"init_" + k: v for k, v in mixture_arrays(m).items()})
        np.savez_compressed(OUT / f"golden_estep_K{K}.npz", **out)

    # --- 3 EM iterations (exact and faithful) + guided queries, K=16 ---------
    K, N = 16, 2048
    b = synth.em_batch(N, 16, guards=True)
    pos, nrm = synth.model_seed_points(b, K)
    s = o.Samples(b["x"], b["w"])
    out = {"x": b["x"], "w": b["w"], "seed_pos": pos, "seed_nrm": nrm}
    for mode, acc in (("exact", "exact"), ("faithful", "faithful")):
        m, st = o.hemisphere_init(K // 8, pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE,
                                  synth.SEED_MODEL, mode=0 if mode == "faithful" else 1)
        for _ in range(3):
            assert o.optimize(m, st, s, accurate=acc) == 1
        out.update({f"em_{mode}_" + k: v for k, v in mixture_arrays(m).items()})
        if mode == "exact":
            c, u = synth.sample_queries_near(b, 64)
            d, pdf, comp, slot = o.guide_batch(m, c.T, u.T)
            out.update({"q_c": c, "q_u": u, "q_dir": d, "q_pdf": pdf, "q_comp": comp, "q_slot": slot,
                        "pdf_at_dir": o.pdf_batch(m, c.T, d)})
            # the same mixture re-loaded through set(mean, cov) + configure()
            # (what sdmm_set_params does): guided outputs for the GPU fixture test
            r = o.Mixture(K)
            for k in range(K):
                r.set_component(k, m.mean[k].astype(np.float64), m.cov[k].astype(np.float64), mode=1)
            r.weights[:] = m.weights
            r.configure()
            d2, pdf2, comp2, slot2 = o.guide_batch(r, c.T, u.T)
            out.update({"q2_dir": d2, "q2_pdf": pdf2, "q2_comp": comp2,
                        "q2_weights": np.array(r.weights)})
    np.savez_compressed(OUT / "golden_em_K16.npz", **out)
    for f in sorted(OUT.glob("*.npz")):
        print(f.name, f.stat().st_size, "bytes")


if __name__ == "__main__":
    main()
