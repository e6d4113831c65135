"""CPU: the Li restatement (oracle/sdmm_oracle_li.inc, SDMMRenderer::Li of
sdmm_proc.cpp:592-871) pinned by an analytic known answer -- the white
furnace: a closed box whose every wall is a one-sided area emitter (Le facing
inward) with diffuse reflectance rho.  With no NEE every bounce's BSDF sample
has weight f cos / pdf = rho and hits an emitting wall, so a path that is
never terminated by roulette (rrDepth >= maxDepth) carries exactly
Le (1 + rho + ... + rho^(maxDepth-1)) -- the same in every pixel -- and each
saved vertex's weight is Le / clampedPdf (its own emitter hit) plus the
recorded radiance of the later hits.  Also the image-side bookkeeping: the
mean of squares, vertex counts and the ordering of the counter RNG."""
import numpy as np
import pytest


def _furnace(rho, le, w=24, h=16):
    # unit cube [-1, 1]^3 as six quads with INWARD normals, every face an emitter
    faces = []
    for axis in range(3):
        for sgn in (-1.0, 1.0):
            u, v = (axis + 1) % 3, (axis + 2) % 3
            p0 = np.zeros(3); p0[axis] = sgn; p0[u] = -1; p0[v] = -1
            e1 = np.zeros(3); e1[u] = 2
            e2 = np.zeros(3); e2[v] = 2
            if sgn > 0:               # e1 x e2 = +axis: flip to point inward (-axis)
                faces.append((p0, e1, e2, 1))
            else:
                faces.append((p0, e1, e2, 0))
    quads = np.concatenate([np.concatenate([a, b, c]) for a, b, c, _ in faces]).astype(np.float32)
    cam = np.eye(4, dtype=np.float32)
    cam[0:3, 3] = [0.1, -0.05, 0.2]
    return {
        "quads": quads, "flip_normals": np.array([f[3] for f in faces], np.int32),
        "bsdf": np.zeros(6, np.int32), "reflectance": np.float32([rho] * 3),
        "emitter": np.zeros(6, np.int32), "radiance": np.float32([le] * 3),
        "camera_to_world": cam.reshape(-1), "fov_x_deg": 70.0, "near_clip": 1e-2, "width": w, "height": h,
    }


@pytest.mark.parametrize("rho,le,max_depth", [(0.5, 1.0, 4), (0.8, 2.0, 10), (0.25, 1.5, 6)])
def test_furnace_known_answer(oracle, rho, le, max_depth):
    d = _furnace(rho, le)
    aabb = np.float32([[0, 0, 0, 1, 1, 1]])
    child = np.int32([[-1, -1]])
    V = max_depth - 1
    r = oracle.li_render(d, aabb, child, spp=3, max_depth=max_depth, rr_depth=max_depth, V=V, seed=7, threads=2)
    expect = le * sum(np.float64(rho) ** k for k in range(max_depth))
    np.testing.assert_allclose(r["image"], expect, rtol=2e-6)
    np.testing.assert_allclose(r["image_sqr"], expect * expect, rtol=4e-6)
    assert (r["nv"] == V).all()                     # every bounce saves a vertex, no path ends early
    # vertex k: throughput rho^(k+1), weight Le / clampedPdf + the later hits recorded
    # through it: sum_{j>k} rho^(j-k) Le / clampedPdf_k
    rec = r["rec"]
    for k in range(V):
        np.testing.assert_allclose(rec[3, k], rho ** (k + 1), rtol=2e-6)
        later = le * sum(rho ** j for j in range(V - k))
        np.testing.assert_allclose(rec[0, k] * rec[6, k], later, rtol=5e-6)
    # unit directions, conditions inside the normalised box
    dirs = rec[10:13]
    np.testing.assert_allclose(np.sqrt((dirs ** 2).sum(0)), 1.0, atol=2e-6)
    assert (rec[7:10] >= -1e-6).all() and (rec[7:10] <= 1 + 1e-6).all()


def test_threads_do_not_change_results(oracle):
    d = _furnace(0.6, 1.0)
    d["reflectance"] = np.float32([0.6, 0.3, 0.1])
    aabb = np.float32([[0, 0, 0, 1, 1, 1]])
    child = np.int32([[-1, -1]])
    a = oracle.li_render(d, aabb, child, spp=2, max_depth=10, rr_depth=3, V=9, seed=3, threads=1)
    b = oracle.li_render(d, aabb, child, spp=2, max_depth=10, rr_depth=3, V=9, seed=3, threads=5)
    for k in ("image", "image_sqr", "rec", "nv"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    # roulette after depth 3 ends some paths early
    assert (a["nv"] < 9).any() and (a["nv"] > 3).any()


def test_pixel_range_is_a_slice(oracle, scenes):
    d = scenes.cornell_box(32, 18)
    aabb = np.float32([[-1e-5, -1e-5, -1e-5, 1, 1, 1]])
    child = np.int32([[-1, -1]])
    full = oracle.li_render(d, aabb, child, spp=2, seed=11, threads=2)
    part = oracle.li_render(d, aabb, child, spp=2, seed=11, pixels=(100, 300), threads=2)
    np.testing.assert_array_equal(full["image"].reshape(3, -1)[:, 100:300], part["image"].reshape(3, -1)[:, 100:300])
    np.testing.assert_array_equal(full["rec"][:, :, 200:600], part["rec"])


def _plastic_albedo(cos_i, bp, rho):
    """Directional albedo of SmoothPlastic (plastic.cpp:250-290): Fi spec +
    (1 - Fi) invEta2 rho / (1 - fdrInt) * int (1 - F(cos_o)) cos_o / pi dw,
    the integral 1 - int_0^1 F(sqrt(xi)) dxi (fdrExt) by quadrature."""
    from scipy.integrate import quad
    import importlib
    scenes = importlib.import_module("sdmm_mitsuba_amd.scenes")
    eta, inv_eta2, fdr_int = float(bp[4]), float(bp[5]), float(bp[6])
    fdr_ext, _ = quad(lambda xi: scenes._fresnel_dielectric(np.sqrt(xi), eta), 0.0, 1.0, epsabs=1e-12, limit=200)
    fi = np.array([scenes._fresnel_dielectric(c, eta) for c in cos_i])
    return fi * float(bp[1]) + (1 - fi) * inv_eta2 * rho / (1 - fdr_int) * (1 - fdr_ext)


@pytest.mark.parametrize("rho", [0.6, 0.0])
def test_plastic_albedo_known_answer(oracle, scenes, rho):
    """The plastic bounce (delta specular lobe + Fresnel-weighted diffuse
    base) against its closed-form directional albedo: a box whose far face is
    plastic and whose other faces are black emitters (Le = 1); with one
    scatter (maxDepth 2) a pixel's expected radiance is the albedo at its
    camera ray's incidence angle -- both lobes are exercised (the delta lobe
    saves no vertex, the diffuse one does).  rho = 0: a black base, whose
    specular sampling weight sAvg / (0 + sAvg) is exactly 1 -- only the delta
    lobe is ever sampled and the albedo is Fi."""
    d = _furnace(0.0, 1.0, w=24, h=16)
    bp = scenes.plastic_params((rho, rho, rho))
    far = 5                                           # axis 2, sgn +1: the face the camera looks at
    d["bsdf"] = np.zeros(6, np.int32)
    d["bsdf"][far] = 1
    d["reflectance"] = np.float32([0.0, 0.0, 0.0, rho, rho, rho])
    d["bsdf_params"] = np.concatenate([np.zeros(8, np.float32), bp])
    d["emitter"] = np.zeros(6, np.int32)
    d["emitter"][far] = -1
    aabb = np.float32([[0, 0, 0, 1, 1, 1]])
    child = np.int32([[-1, -1]])
    spp = 256
    r = oracle.li_render(d, aabb, child, spp=spp, max_depth=2, rr_depth=2, V=1, seed=5, threads=4)
    # camera rays through the pixel centres: cos(theta_i) = d_z (the face normal is -z)
    W, H = d["width"], d["height"]
    tanx = np.tan(np.radians(35.0))
    sx = (np.arange(W) + 0.5) / W
    sy = (np.arange(H) + 0.5) / H
    lx = (1 - 2 * sx)[None, :] * tanx
    ly = (1 - 2 * sy)[:, None] * tanx / (W / H)
    cos_i = 1 / np.sqrt(lx ** 2 + ly ** 2 + 1)
    want = _plastic_albedo(cos_i.reshape(-1), bp, rho).reshape(H, W)
    img = r["image"][0]
    var = (r["image_sqr"][0] - img ** 2) / spp                         # per-pixel variance of the mean
    err = abs(img.mean() - want.mean())
    sig = np.sqrt(var.sum()) / img.size
    print("plastic albedo", img.mean(), want.mean(), sig)
    assert err <= 4 * sig + 2e-4, (img.mean(), want.mean(), sig)
    # both lobes taken: vertices saved for the diffuse lobe only
    if rho > 0:
        assert 0 < (r["nv"] == 1).mean() < 1
    else:
        assert bp[7] == 1.0 and (r["nv"] == 0).all()
