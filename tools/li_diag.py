"""Diagnostics of the device Li's guiding on the Cornell Box (GPU).

Trains with the test's host loop for T iterations and reports, per T: trained
leaves, the fraction of saved vertices whose bounce ray hit the light (the
direct-hit rate -- guiding towards the light raises it), and the per-pixel MSE
of guided / unguided renders against a high-spp unguided reference.
"""
import argparse
import importlib
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", default="2,4,8")
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--res", default="160x90")
    ap.add_argument("--K", type=int, default=16)
    args = ap.parse_args()
    import torch
    from conftest import load_pkg
    pkg = load_pkg()
    scenes = importlib.import_module("sdmm_mitsuba_amd.scenes")
    t = importlib.import_module("test_gpu_li")
    w, h = (int(x) for x in args.res.split("x"))
    sc = pkg.Scene(scenes.cornell_box(w, h))
    ref_tree = t._tree(pkg, sc)
    ref = sc.render(ref_tree, None, spp=2048, seed=99991)[0].cpu().numpy().mean(0)
    lum = lambda im: im.cpu().numpy().mean(0)
    for T in [int(x) for x in args.iters.split(",")]:
        tree = t._tree(pkg, sc)
        node_mix = t._train(pkg, sc, tree, T, args.spp, K=args.K)
        trained = sum(m is not None for m in node_mix)
        res = {}
        for guided in (False, True):
            img, verts, st = sc.render(tree, node_mix if guided else None, spp=64, guided=guided, seed=5 + guided)
            rec, nv = verts.to_numpy()
            V = verts.s.max_vertices
            r = rec.reshape(16, V, -1)
            sel = np.arange(V)[:, None] < nv[None, :]
            wsum = r[0][sel] + r[1][sel] + r[2][sel]
            first = r[0][0][nv > 0] + r[1][0][nv > 0] + r[2][0][nv > 0]
            mse = float(np.mean((lum(img) - ref) ** 2))
            res[guided] = (mse, float(np.mean(wsum > 0)), float(np.mean(first > 0)), float(lum(img).mean()))
        print(f"T={T} leaves={tree.leaf_nodes} trained={trained} "
              f"unguided mse={res[False][0]:.4g} hit={res[False][1]:.4f} first={res[False][2]:.4f} mean={res[False][3]:.4f} | "
              f"guided mse={res[True][0]:.4g} hit={res[True][1]:.4f} first={res[True][2]:.4f} mean={res[True][3]:.4f} "
              f"ratio={res[True][0] / res[False][0]:.3f}", flush=True)
    print(f"reference mean {ref.mean():.4f}")


if __name__ == "__main__":
    main()
