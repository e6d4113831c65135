"""Synthetic EM / guiding workloads of BASELINE.md section 2 and SURVEY.md 8(d).

Not part of the hot path: this builds deterministic input batches (numpy,
seeded) for the bench, the smoke test and the parity tests.

  * generator mixture: K_gen components from uniformHemisphereInit
    (mixture_model_init.h:79-242) at n_pos = K_gen/8 spatial centres uniform in
    [0.1, 0.9]^3 with random unit normals (seed 0x5D3D), spatial distance 0.1;
  * samples: component ~ pi, tangent ~ N(0, Sigma_k) (MVTN::sample,
    multivariate_tangent_normal.h:321-339), exp map to a position in [0,1]^3-ish
    and a unit direction (seed 0xE11);
  * weights ~ LogNormal(0, 1) (seed 0xBEEF) with 0.1 % zeros and 0.01 %
    non-finite values to exercise the guards of stepwise_tangent.h:288-293;
  * isDiffuse all 0 (or 50 % with hpdf = 1/(4 pi) for the heuristic variant);
  * the model under fit: a fresh uniformHemisphereInit with K components whose
    seed positions/normals are the first K/8 samples (the kMeansPlusPlus=false
    branch, mixture_model_init.h:139-141), jitter seed 0x1A17.
"""
from __future__ import annotations

import numpy as np

SEED_CENTRES = 0x5D3D
SEED_SAMPLES = 0xE11
SEED_WEIGHTS = 0xBEEF
SEED_MODEL = 0x1A17
SEED_QUERIES = 0x6A1D
DEPTH_PRIOR = 0.01
SPATIAL_DISTANCE = 0.1


def coordinates(n: np.ndarray) -> np.ndarray:
    """Coordinates(n).to for a batch of unit vectors n (..., 3) -> (..., 3, 3)."""
    n = np.asarray(n, np.float64)
    sign = np.copysign(1.0, n[..., 2])
    a = -1.0 / (sign + n[..., 2])
    b = n[..., 0] * n[..., 1] * a
    to = np.zeros(n.shape[:-1] + (3, 3))
    to[..., 0, 0] = 1.0 + sign * n[..., 0] * n[..., 0] * a
    to[..., 0, 1] = sign * b
    to[..., 0, 2] = -sign * n[..., 0]
    to[..., 1, 0] = b
    to[..., 1, 1] = sign + n[..., 1] * n[..., 1] * a
    to[..., 1, 2] = -n[..., 1]
    to[..., 2, :] = n
    return to


def random_unit(rng, n):
    v = rng.normal(size=(n, 3))
    return v / np.linalg.norm(v, axis=1, keepdims=True)


def generator_mixture(K_gen: int = 128):
    from . import hemisphere_init_host
    rng = np.random.default_rng(SEED_CENTRES)
    n_pos = K_gen // 8
    pos = rng.uniform(0.1, 0.9, size=(n_pos, 3)).astype(np.float32)
    nrm = random_unit(rng, n_pos).astype(np.float32)
    g = hemisphere_init_host(pos, nrm, DEPTH_PRIOR, SPATIAL_DISTANCE, SEED_CENTRES)
    g["positions"], g["normals"] = pos, nrm
    return g


def sample_mixture(g: dict, n: int, rng) -> tuple[np.ndarray, np.ndarray]:
    """Draw n samples of the 6-D embedding; also return the generator normal."""
    K = g["weights"].shape[0]
    comp = rng.choice(K, size=n, p=g["weights"].astype(np.float64) / g["weights"].sum())
    L = np.linalg.cholesky(g["cov"].astype(np.float64))          # (K, 5, 5)
    mean = g["mean"].astype(np.float64)
    to = coordinates(mean[:, 3:6])                                  # (K, 3, 3)
    out = np.zeros((6, n))
    todo = np.arange(n)
    while todo.size:
        z = rng.normal(size=(todo.size, 5))
        v = np.einsum("nij,nj->ni", L[comp[todo]], z)
        t = v[:, 3:5]
        length = np.linalg.norm(t, axis=1)
        ok = length < np.pi
        sinc = np.where(length > 1e-8, np.sin(length) / np.maximum(length, 1e-30), 1.0)
        rel = np.stack([t[:, 0] * sinc, t[:, 1] * sinc, np.cos(length)], axis=1)
        d = np.einsum("nji,nj->ni", to[comp[todo]], rel)             # m_rotation = to^T
        idx = todo[ok]
        out[0:3, idx] = (mean[comp[idx], 0:3] + v[ok, 0:3]).T
        out[3:6, idx] = (d[ok] / np.linalg.norm(d[ok], axis=1, keepdims=True)).T
        todo = todo[~ok]
    normals = g["normals"][comp // 8]
    return out.astype(np.float32), normals.astype(np.float32)


def em_batch(n: int, K_gen: int = 128, heuristic: bool = False, guards: bool = True, part: int = 0):
    """Synthetic EM batch: dict with x (6,n), w, hpdf, is_diffuse, normals.
    part p > 0: an independent batch of the same distribution (rank p's share
    of a weak-scaled global batch; part 0 is the single-GPU batch)."""
    g = generator_mixture(K_gen)
    rng = np.random.default_rng(SEED_SAMPLES + 7919 * part)
    x, normals = sample_mixture(g, n, rng)
    wr = np.random.default_rng(SEED_WEIGHTS + 7919 * part)
    w = wr.lognormal(0.0, 1.0, size=n).astype(np.float32)
    if guards and n >= 16:
        zi = wr.choice(n, size=max(1, n // 1000), replace=False)
        w[zi] = 0.0
        bi = wr.choice(n, size=max(1, n // 10000), replace=False)
        w[bi[0::2]] = np.inf
        w[bi[1::2]] = np.nan
    if heuristic:
        isd = (wr.random(n) < 0.5).astype(np.uint8)
        hpdf = np.full(n, 1.0 / (4.0 * np.pi), np.float32)
    else:
        isd = np.zeros(n, np.uint8)
        hpdf = np.zeros(n, np.float32)
    return {"x": x, "w": w, "hpdf": hpdf, "is_diffuse": isd, "normals": normals, "generator": g}


def model_seed_points(batch: dict, K: int):
    """Seed positions/normals of the model under fit (first K/8 samples)."""
    n_pos = K // 8
    pos = batch["x"][0:3, :n_pos].T.copy()
    nrm = batch["normals"][:n_pos].copy()
    return pos, nrm


def queries(nq: int, seed: int = SEED_QUERIES):
    """Guided-query batch: condition c in [0,1]^3 and three uniforms."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(0.0, 1.0, size=(3, nq)).astype(np.float32)
    u = rng.uniform(0.0, 1.0, size=(3, nq)).astype(np.float32)
    u = np.minimum(u, np.float32(0.99999994))
    return c, u


def sample_queries_near(batch: dict, nq: int, seed: int = SEED_QUERIES):
    """Queries whose conditions are sample positions (where guiding happens)."""
    rng = np.random.default_rng(seed)
    idx = rng.choice(batch["x"].shape[1], size=nq)
    c = batch["x"][0:3, idx].copy()
    u = rng.uniform(0.0, 1.0, size=(3, nq)).astype(np.float32)
    u = np.minimum(u, np.float32(0.99999994))
    return c, u


SEED_BSDF = 0xB5DF


def bsdf_table(B: int, M: int, seed: int = SEED_BSDF):
    """Synthetic learned-BSDF lobes (the plugin's `.sdmm` files are LFS
    pointers): B materials x M directional tangent normals in
    the local shading frame -- weights (B, M) summing to 1, unit means (B, M, 3)
    in the upper hemisphere (z >= 0.3), SPD 2x2 covariances (B, M, 4) with
    standard deviations in [0.05, 0.6]."""
    rng = np.random.default_rng(seed)
    w = rng.uniform(0.2, 1.0, size=(B, M))
    w /= w.sum(1, keepdims=True)
    m = rng.normal(size=(B, M, 3))
    m[..., 2] = np.abs(m[..., 2]) + 0.6
    m /= np.linalg.norm(m, axis=-1, keepdims=True)
    sd = rng.uniform(0.05, 0.6, size=(B, M, 2))
    ang = rng.uniform(0, np.pi, size=(B, M))
    c, s = np.cos(ang), np.sin(ang)
    cov = np.zeros((B, M, 4))
    cov[..., 0] = c * c * sd[..., 0] ** 2 + s * s * sd[..., 1] ** 2
    cov[..., 3] = s * s * sd[..., 0] ** 2 + c * c * sd[..., 1] ** 2
    cov[..., 1] = cov[..., 2] = c * s * (sd[..., 0] ** 2 - sd[..., 1] ** 2)
    return w.astype(np.float32), m.astype(np.float32), cov.astype(np.float32)


def shading_frames(nq: int, seed: int = SEED_BSDF + 1):
    """Per-query to-world frames F = [s t n] (row-major 3x3, columns s, t, n)
    with n uniform on the sphere: (nq, 9) float32."""
    rng = np.random.default_rng(seed)
    n = random_unit(rng, nq).astype(np.float64)
    to = coordinates(n)                      # rows s, t, n of Coordinates(n)
    F = np.transpose(to, (0, 2, 1))          # columns s, t, n
    return F.reshape(nq, 9).astype(np.float32)
