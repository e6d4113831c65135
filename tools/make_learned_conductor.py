#!/usr/bin/env python3
"""Write the synthetic learned rough-conductor BSDF the glossy Cornell scene
uses (sdmm-mitsuba_amd/data/conductor_beckmann_4c.sdmm4.json).

The reference conditions each glossy material's learned SDMM4 (BSDF::SDMM4,
include/mitsuba/render/bsdf.h:310-314: (theta_i, alpha) x direction) per
bounce (roughconductor.cpp:182-194); its files (test-suite/scenes/*/
conductor_*_4c.sdmm) are Git-LFS pointers in the snapshot, so a synthetic
4-component model with the same structure stands in.  It is built as a joint
Gaussian per component rather than fitted: component k sits at a condition
(theta_k, alpha_k) of a 2 x 2 grid; its direction is the mirror direction of
an incident direction at elevation theta_k, azimuth 0 (the canonical frame of
getDMM, rotated onto wi's azimuth by rotate_to_wo afterwards); and its tangent
coordinates t = v (theta - theta_k) + n, with v the mirror direction's
derivative in theta expressed in the component's Coordinates frame and n an
isotropic lobe of standard deviation 2 alpha_k (a Beckmann lobe's reflected
spread).  So the joint covariance is PD by construction, S_dc is non-zero (the
conditional mean follows theta_i) and pruning to 2 keeps the two components
nearest the condition.

    python tools/make_learned_conductor.py [out.json]
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "sdmm-mitsuba_amd" / "data" / "conductor_beckmann_4c.sdmm4.json"


def coordinates(n):
    """jmm Coordinates (utils.h:32-48): rows t1, t2, n (float32 arithmetic)."""
    n = np.asarray(n, np.float32)
    sign = np.float32(np.copysign(1.0, n[2]))
    a = np.float32(-1.0) / (sign + n[2])
    b = n[0] * n[1] * a
    return np.array([[1 + sign * n[0] * n[0] * a, sign * b, -sign * n[0]],
                     [b, sign + n[1] * n[1] * a, -n[1]], n], np.float32)


def model():
    thetas, alphas = (0.35, 1.05), (0.1, 0.35)
    s_theta, s_alpha = 0.35, 0.12
    w, means, covs = [], [], []
    for th in thetas:
        for al in alphas:
            mu = np.array([-np.sin(th), 0.0, np.cos(th)])
            mu = (mu / np.linalg.norm(mu)).astype(np.float32)
            T = coordinates(mu).astype(np.float64)
            dmu = np.array([-np.cos(th), 0.0, -np.sin(th)])     # d(mirror direction) / d(theta)
            v = T[:2] @ dmu
            # x = (theta, alpha, t1, t2) = A z, z ~ N(0, I): theta = s_theta z0,
            # alpha = s_alpha z1, t = v s_theta z0 + 2 alpha z2..3
            A = np.zeros((4, 4))
            A[0, 0] = s_theta
            A[1, 1] = s_alpha
            A[2:, 0] = v * s_theta
            A[2, 2] = A[3, 3] = 2.0 * al
            cov = A @ A.T
            w.append(0.25)
            means.append([th, al, *mu.tolist()])
            covs.append(cov.reshape(-1).tolist())
    return np.float32(w), np.float32(means), np.float32(covs)


def main():
    out = Path(sys.argv[1]) if len(sys.argv) > 1 else OUT
    w, mu, cv = model()
    f9 = lambda a: [float(f"{float(x):.9g}") for x in np.asarray(a, np.float32).reshape(-1)]
    doc = {"format": "sdmm-amd.sdmm4", "version": 1, "M": int(len(w)), "weights": f9(w), "means": f9(mu),
           "covs": f9(cv)}
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(doc) + "\n")
    print(out)


if __name__ == "__main__":
    main()
