"""Shared numerics for the parity tests (numpy, fp64)."""
import numpy as np

NORM5 = float(np.float32(np.float32(0.3989422804014327) ** 5))


def posterior_f64(mix_params: dict, x: np.ndarray) -> np.ndarray:
    """posteriorAndLog (mixture_model.h:146-192) in float64 from the float
    mixture parameters: the 'exact' reference both fp32 paths are judged by."""
    w = np.asarray(mix_params["weights"], np.float64)
    mean = np.asarray(mix_params["mean"], np.float64).reshape(-1, 6)
    to = np.asarray(mix_params["to"], np.float64).reshape(-1, 3, 3)
    Li = np.asarray(mix_params["cholLInv"], np.float64).reshape(-1, 5, 5)
    di = np.asarray(mix_params["detInv"], np.float64)
    x = np.asarray(x, np.float64)
    p, d = x[0:3].T, x[3:6].T                               # (N,3)
    r = np.einsum("kij,nj->nki", to, d)                     # (N,K,3)
    c = r[..., 2]
    bad = (c <= -1) | (np.abs(d).sum(1) == 0)[:, None]
    cc = np.minimum(c, 1.0)
    th = np.arccos(np.clip(cc, -1, 1))
    s = np.sqrt(np.maximum(1 - cc * cc, 0))
    a = np.where(s < 1e-3, 1.0, th / np.where(s > 0, s, 1))
    tau = np.concatenate([p[:, None, :] - mean[None, :, :3], (r[..., :2] * a[..., None])], -1)
    u = np.einsum("kij,nkj->nki", Li, tau)
    q = (u * u).sum(-1)
    pdf = NORM5 * np.exp(-0.5 * q) * di[None] * a
    pdf[bad] = 0
    post = w[None] * pdf
    S = post.sum(1, keepdims=True)
    with np.errstate(invalid="ignore", divide="ignore"):
        out = np.where(S > 0, post / S, 0.0)
    return out
