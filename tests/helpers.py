"""Shared numerics for the parity tests (numpy, fp64)."""
import numpy as np

NORM5 = float(np.float32(np.float32(0.3989422804014327) ** 5))
FLT_MIN = float(np.finfo(np.float32).tiny)


def _ftz(a):
    """Flush the values an fp32 FTZ/DAZ evaluation would flush (the plugin's
    flushDenormals=true, volpath_sdmm.cpp:88-90)."""
    return np.where(np.abs(a) < FLT_MIN, 0.0, a)


def _pdf_ftz(q, di, a, w):
    """pi_k * NORM5 * exp(-q/2) * detInv * J with the fp32 flush points."""
    p1 = _ftz(NORM5 * np.exp(-0.5 * q))
    p2 = _ftz(p1 * _ftz(di * a))
    return _ftz(w * p2)


def posterior_f64(mix_params: dict, x: np.ndarray, hpdf=None, is_diffuse=None, h=0.5, return_qc=False):
    """posteriorAndLog (mixture_model.h:146-192) in float64 from the float
    mixture parameters: the 'exact' reference both fp32 paths are judged by.
    With is_diffuse: the heuristic mix S' = (1-h) S + h hpdf on those rows,
    gamma_k = (1-h) q_k / S' (:170-181).  return_qc: also the (N, K)
    Mahalanobis distances q and cosines c = cos(theta) of each pair."""
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
    post = _pdf_ftz(q, di[None], a, w[None])
    post[bad] = 0
    S = post.sum(1, keepdims=True)
    if return_qc:
        return posterior_f64(mix_params, x, hpdf, is_diffuse, h), q, c
    if is_diffuse is None:
        with np.errstate(invalid="ignore", divide="ignore"):
            return np.where(S > 0, post / S, 0.0)
    dif = (np.asarray(is_diffuse) != 0)[:, None]
    hp = np.asarray(hpdf, np.float64)[:, None]
    S2 = np.where(dif, (1.0 - h) * S + h * hp, S)
    with np.errstate(invalid="ignore", divide="ignore"):
        inv = 1.0 / S2
        scale = np.where(dif, (1.0 - h) * inv, inv)
        return np.where(np.isfinite(inv) & (S2 > 0), post * scale, 0.0)


def explained_rows(post, q, c, qmax=100.0, cmin=1e-2, pmin=1e-7):
    """Rows the mixture explains with well-conditioned fp32 arithmetic: the
    fp64 max posterior sits at q < qmax, and no component with posterior
    > pmin is near-antipodal (1 + c < cmin: there theta/sin(theta) amplifies
    the fp32 rounding of c, and both fp32 paths -- the reference's and the
    GPU's -- carry up to ~4e-3 of absolute error in such rows)."""
    n = post.shape[0]
    qm = q[np.arange(n), post.argmax(1)]
    cond = ~((post > pmin) & (1.0 + c < cmin)).any(1)
    return (qm < qmax) & (post.sum(1) > 0) & cond


def estep_f64(mix_params: dict, x, w, hpdf=None, is_diffuse=None, h=0.5, chunk=2048):
    """calculateStats + sumWeights (stepwise_tangent.h:270-353, :462-475) in
    float64 from the float mixture parameters.  Returns the oracle stats
    layout [H, weightSum, W(K), M(5K), C(25K)]."""
    wt = np.asarray(mix_params["weights"], np.float64)
    mean = np.asarray(mix_params["mean"], np.float64).reshape(-1, 6)
    to = np.asarray(mix_params["to"], np.float64).reshape(-1, 3, 3)
    Li = np.asarray(mix_params["cholLInv"], np.float64).reshape(-1, 5, 5)
    di = np.asarray(mix_params["detInv"], np.float64)
    K = wt.shape[0]
    x = np.asarray(x, np.float64)
    w = np.asarray(w, np.float64)
    N = w.shape[0]
    hp = np.zeros(N) if hpdf is None else np.asarray(hpdf, np.float64)
    isd = np.zeros(N, bool) if is_diffuse is None else np.asarray(is_diffuse) != 0
    fin = np.isfinite(w)
    wsum = w[fin].sum()
    H = 0.0
    W = np.zeros(K)
    M = np.zeros((K, 5))
    C = np.zeros((K, 5, 5))
    for a in range(0, N, chunk):
        sl = slice(a, min(N, a + chunk))
        ww = w[sl]
        use = np.isfinite(ww) & (ww != 0)
        p, d = x[0:3, sl].T, x[3:6, sl].T
        r = np.einsum("kij,nj->nki", to, d)
        c = r[..., 2]
        bad = (c <= -1) | (np.abs(d).sum(1) == 0)[:, None]
        cc = np.minimum(c, 1.0)
        th = np.arccos(np.clip(cc, -1, 1))
        s = np.sqrt(np.maximum(1 - cc * cc, 0))
        aa = np.where(s < 1e-3, 1.0, th / np.where(s > 0, s, 1))
        tdir = r[..., :2] * aa[..., None]
        tau_rel = np.concatenate([p[:, None, :] - mean[None, :, :3], tdir], -1)
        u = np.einsum("kij,nkj->nki", Li, tau_rel)
        q = (u * u).sum(-1)
        post = _pdf_ftz(q, di[None], aa, wt[None])
        post[bad] = 0
        S = post.sum(1)
        dd = isd[sl]
        S2 = np.where(dd, (1 - h) * S + h * hp[sl], S)
        with np.errstate(divide="ignore", invalid="ignore"):
            inv = 1.0 / S2
        ok = np.isfinite(inv)
        g = np.where(ok, np.where(dd, inv * (1 - h), inv), 0.0)
        gam = post * g[:, None]
        with np.errstate(invalid="ignore"):
            hpost = np.where(ok & dd, h * hp[sl] * inv, 0.0)
        H += (np.where(use, ww, 0) * hpost).sum()
        with np.errstate(invalid="ignore"):
            v = np.where((gam >= 1e-10) & use[:, None], ww[:, None] * gam, 0.0)
        tau = np.concatenate([np.broadcast_to(p[:, None, :], tdir.shape[:2] + (3,)), tdir], -1)
        tau = np.where(bad[..., None], 0.0, tau)
        W += v.sum(0)
        M += np.einsum("nk,nki->ki", v, tau)
        C += np.einsum("nk,nki,nkj->kij", v, tau, tau)
    return np.concatenate([[H, wsum], W, M.reshape(-1), C.reshape(-1)])


def read_exr(path):
    """Minimal reader for the uncompressed scanline float OpenEXR files
    sdmm_write_exr writes: (rgb (3, H, W) float32, attributes dict)."""
    import struct
    data = open(path, "rb").read()
    assert struct.unpack_from("<I", data, 0)[0] == 20000630, "not an OpenEXR file"
    pos, attrs = 8, {}
    while data[pos] != 0:
        e = data.index(b"\0", pos); name = data[pos:e].decode(); pos = e + 1
        e = data.index(b"\0", pos); typ = data[pos:e].decode(); pos = e + 1
        size = struct.unpack_from("<i", data, pos)[0]; pos += 4
        val = data[pos:pos + size]; pos += size
        if typ == "int":
            attrs[name] = struct.unpack("<i", val)[0]
        elif typ == "float":
            attrs[name] = struct.unpack("<f", val)[0]
        elif typ == "box2i":
            attrs[name] = struct.unpack("<4i", val)
        elif typ == "compression":
            attrs[name] = val[0]
        elif typ == "chlist":
            chans, q = [], 0
            while val[q] != 0:
                e = val.index(b"\0", q); cname = val[q:e].decode(); q = e + 1
                ptype = struct.unpack_from("<i", val, q)[0]; q += 16
                chans.append((cname, ptype))
            attrs[name] = chans
        else:
            attrs[name] = val
    pos += 1
    x0, y0, x1, y1 = attrs["dataWindow"]
    W, H = x1 - x0 + 1, y1 - y0 + 1
    assert attrs["compression"] == 0 and all(p == 2 for _, p in attrs["channels"])
    offsets = struct.unpack_from(f"<{H}Q", data, pos)
    names = [c for c, _ in attrs["channels"]]
    img = {c: np.zeros((H, W), np.float32) for c in names}
    for off in offsets:
        y, size = struct.unpack_from("<ii", data, off)
        row = np.frombuffer(data, np.float32, count=len(names) * W, offset=off + 8).reshape(len(names), W)
        for k, c in enumerate(names):
            img[c][y - y0] = row[k]
    return np.stack([img["R"], img["G"], img["B"]]), attrs
