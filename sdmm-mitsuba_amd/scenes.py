"""Analytic scenes for the device Li (sdmm_scene_* in include/sdmm_gpu.h).

cornell_box(): the test suite's Cornell Box, test-suite/scenes/cornell-box/
cornell-box.xml -- film 640x360 (:26-28), perspective fov 35 along x with the
toWorld of :17-19, five rectangles (:75-116; flipNormals on the back, right
and left walls), two cubes (:118-132), the area light (:134-143) and the
diffuse reflectances of :36-73.  The integrator settings of the suite's
_integrators/sdmm.xml: maxDepth = rrDepth = 10.

Mitsuba shapes as parallelograms: a rectangle is [-1, 1]^2 x {0} under
toWorld (normal +z), a cube [-1, 1]^3 (outward normals), both transformed by
the 4x4 matrix of the XML (row major).

The emitter's spectrum "400:0, 500:1600, 600:3180, 700:3680" (piecewise
linear) is converted to linear sRGB here: integrated against the CIE 1931
2-degree observer (the analytic multi-lobe fit of Wyman, Sloan and Shirley,
JCGT 2013) over 360-830 nm, normalised by the integral of y-bar, then XYZ ->
linear sRGB (D65).  Mitsuba's own RGB-mode conversion is not reproducible
here (no Mitsuba); the image is therefore not compared with Mitsuba renders --
the device Li is checked for unbiasedness and its training batches for
parity with the host-routed reference instead (tests/test_gpu_li.py).
"""
import json
from pathlib import Path

import numpy as np

CORNELL_MAX_DEPTH = 10       # _integrators/sdmm.xml: maxDepth
CORNELL_RR_DEPTH = 10        # rrDepth = maxDepth

_RECTS = [
    # (matrix row major 3x4, bsdf, flipNormals)
    ("-4.37114e-008 1 4.37114e-008 0 0 -8.74228e-008 2 0 1 4.37114e-008 1.91069e-015 0", "Floor", False),
    ("-1 7.64274e-015 -1.74846e-007 0 8.74228e-008 8.74228e-008 -2 2 0 -1 -4.37114e-008 0", "Ceiling", False),
    ("1.91069e-015 1 1.31134e-007 0 1 3.82137e-015 -8.74228e-008 1 -4.37114e-008 1.31134e-007 -2 -1",
     "BackWall", True),
    ("4.37114e-008 -1.74846e-007 2 1 1 3.82137e-015 -8.74228e-008 1 3.82137e-015 1 2.18557e-007 0",
     "RightWall", True),
    ("-4.37114e-008 8.74228e-008 -2 -1 1 3.82137e-015 -8.74228e-008 1 0 -1 -4.37114e-008 0", "LeftWall", True),
]
_CUBES = [
    ("0.0851643 0.289542 1.31134e-008 0.328631 3.72265e-009 1.26563e-008 -0.3 0.3 "
     "-0.284951 0.0865363 5.73206e-016 0.374592", "ShortBox"),
    ("0.286776 0.098229 -2.29282e-015 -0.335439 -4.36233e-009 1.23382e-008 -0.6 0.6 "
     "-0.0997984 0.282266 2.62268e-008 -0.291415", "TallBox"),
]
_LIGHT = ("4.700000e-02 -3.322060e-09 -1.561370e-09 -5.000000e-03 -4.108880e-09 7.806860e-10 -1.786000e-02 "
          "1.980000e+00 4.108880e-09 3.800000e-02 1.661032e-09 -3.000000e-02")
_BSDFS = {
    "LeftWall": (0.63, 0.065, 0.05), "RightWall": (0.14, 0.45, 0.091), "Floor": (0.725, 0.71, 0.68),
    "Ceiling": (0.725, 0.71, 0.68), "BackWall": (0.725, 0.71, 0.68), "ShortBox": (0.725, 0.71, 0.68),
    "TallBox": (0.725, 0.71, 0.68), "Light": (0.0, 0.0, 0.0),
}
_LIGHT_SPD = [(400.0, 0.0), (500.0, 1600.0), (600.0, 3180.0), (700.0, 3680.0)]
_CAMERA = "-1 0 0 0 0 1 0 1 0 0 -1 6.8 0 0 0 1"


def _mat(s):
    return np.array([float(x) for x in s.split()], np.float64).reshape(3, 4)


def _cie_xyz(lam):
    """CIE 1931 colour matching functions, multi-lobe analytic fit (Wyman et al. 2013)."""
    def g(x, mu, s1, s2):
        s = np.where(x < mu, s1, s2)
        return np.exp(-0.5 * ((x - mu) / s) ** 2)
    x = 1.056 * g(lam, 599.8, 37.9, 31.0) + 0.362 * g(lam, 442.0, 16.0, 26.7) - 0.065 * g(lam, 501.1, 20.4, 26.2)
    y = 0.821 * g(lam, 568.8, 46.9, 40.5) + 0.286 * g(lam, 530.9, 16.3, 31.1)
    z = 1.217 * g(lam, 437.0, 11.8, 36.0) + 0.681 * g(lam, 459.0, 26.0, 13.8)
    return x, y, z


def spectrum_to_rgb(spd):
    """Piecewise-linear SPD (wavelength, value) -> linear sRGB (zero outside the samples)."""
    lam = np.arange(360.0, 831.0, 1.0)
    w, v = zip(*spd)
    s = np.interp(lam, w, v, left=0.0, right=0.0)
    xb, yb, zb = _cie_xyz(lam)
    X, Y, Z = (np.sum(s * xb), np.sum(s * yb), np.sum(s * zb))
    k = 1.0 / np.sum(yb)
    X, Y, Z = X * k, Y * k, Z * k
    m = np.array([[3.240479, -1.537150, -0.498535], [-0.969256, 1.875991, 0.041556],
                  [0.055648, -0.204043, 1.057311]])
    return np.maximum(m @ np.array([X, Y, Z]), 0.0)


def _rect(M):
    """Corner and edges with e1 x e2 along Mitsuba's normal (inverse transpose of +z)."""
    A, t = M[:, :3], M[:, 3]
    p0 = A @ np.array([-1.0, -1.0, 0.0]) + t
    e1, e2 = A @ np.array([2.0, 0.0, 0.0]), A @ np.array([0.0, 2.0, 0.0])
    return (p0, e2, e1) if np.linalg.det(A) < 0 else (p0, e1, e2)


def _cube_faces(M):
    A, t = M[:, :3], M[:, 3]
    flip = np.linalg.det(A) < 0
    faces = []
    for ax in range(3):
        b, c = (ax + 1) % 3, (ax + 2) % 3
        for s in (1.0, -1.0):
            u = np.zeros(3); u[b] = 2.0
            v = np.zeros(3); v[c] = 2.0
            if (s < 0) != flip:                 # u x v must point along s e_ax after the transform
                u, v = v, u
            corner = np.zeros(3); corner[ax] = s
            corner -= 0.5 * u + 0.5 * v
            faces.append((A @ corner + t, A @ u, A @ v))
    return faces


def _fresnel_dielectric(cos_i, eta):
    """fresnelDielectricExt (libcore/util.cpp:651-681), reflectance only (float64)."""
    if eta == 1.0:
        return 0.0
    scale = 1.0 / eta if cos_i > 0 else eta
    ct2 = 1.0 - (1.0 - cos_i * cos_i) * scale * scale
    if ct2 <= 0.0:
        return 1.0
    ci, ct = abs(cos_i), np.sqrt(ct2)
    rs = (ci - eta * ct) / (ci + eta * ct)
    rp = (eta * ci - ct) / (eta * ci + ct)
    return 0.5 * (rs * rs + rp * rp)


def plastic_params(diffuse_rgb, specular_rgb=(1.0, 1.0, 1.0), int_ior=1.49, ext_ior=1.000277):
    """The 8 bsdf_params floats of a smooth plastic (bsdfs/plastic.cpp:148-200;
    include/sdmm_gpu.h sdmm_scene_desc): kind 1, specularReflectance, eta =
    intIOR / extIOR (polypropylene / air, the plugin's defaults), 1 / eta^2,
    fdrInt = fresnelDiffuseReflectance(1 / eta) (the integral over xi of
    F(sqrt(xi)), here by adaptive quadrature in double where Mitsuba runs a
    Gauss-Lobatto rule: the constant may differ in its last float bits), and
    the specular sampling weight sAvg / (dAvg + sAvg) from the luminances."""
    from scipy.integrate import quad
    f32 = np.float32
    eta = f32(f32(int_ior) / f32(ext_ior))
    inv_eta2 = f32(f32(1.0) / f32(eta * eta))
    fdr_int, _ = quad(lambda xi: _fresnel_dielectric(np.sqrt(xi), 1.0 / float(eta)), 0.0, 1.0,
                      epsabs=1e-12, epsrel=1e-12, limit=200)

    def lum(c):
        c = [f32(x) for x in c]
        return f32(f32(f32(c[0] * f32(0.212671)) + f32(c[1] * f32(0.715160))) + f32(c[2] * f32(0.072169)))
    d_avg, s_avg = lum(diffuse_rgb), lum(specular_rgb)
    ssw = f32(s_avg / f32(d_avg + s_avg))
    return np.array([1.0, *specular_rgb, eta, inv_eta2, fdr_int, ssw], np.float32)


def conductor_params(specular_rgb=(1.0, 1.0, 1.0), eta=1.2, k=7.0, alpha=0.2):
    """The 8 bsdf_params floats of a rough conductor (bsdfs/roughconductor.cpp;
    include/sdmm_gpu.h sdmm_scene_desc): kind 2, specularReflectance, a gray
    eta / k (default: aluminium-like, |n + ik| of Al over the visible), the
    isotropic Beckmann alpha (sampleVisible = false)."""
    return np.array([2.0, *specular_rgb, eta, k, alpha, 0.0], np.float32)


LEARNED_CONDUCTOR = Path(__file__).resolve().parent / "data" / "conductor_beckmann_4c.sdmm4.json"


def load_learned(path=LEARNED_CONDUCTOR):
    """A learned BSDF file (sdmm-amd.sdmm4 JSON, include/sdmm_gpu.h
    sdmm_learned4_load_json) as (weights[M], means[M][5], covs[M][16])
    float32 -- the numbers are written with 9 digits, so they round-trip."""
    doc = json.loads(Path(path).read_text())
    if doc.get("format") != "sdmm-amd.sdmm4" or doc.get("version") != 1:
        raise ValueError(f"{path}: not an sdmm-amd.sdmm4 file")
    M = int(doc["M"])
    return (np.asarray(doc["weights"], np.float32).reshape(M), np.asarray(doc["means"], np.float32).reshape(M, 5),
            np.asarray(doc["covs"], np.float32).reshape(M, 16))


def cornell_box(width=640, height=360, plastic=(), conductor=(), alpha=0.2, learned=LEARNED_CONDUCTOR):
    """sdmm_scene_desc fields for the Cornell Box (numpy arrays).  plastic:
    names of BSDFs (e.g. "TallBox", "ShortBox", "Floor") rendered as smooth
    plastic over their diffuse reflectance (a delta specular lobe beside a
    smooth one, like the Kitchen's `plastic` materials, kitchen.xml);
    conductor: names rendered as rough conductors (the Kitchen's glossy
    `roughconductor` materials) tinted by their reflectance, Beckmann alpha,
    each with the learned BSDF `learned` (an sdmm4 file; None: no learned
    model, so product sampling falls back to the plain conditional there) --
    the synthetic stand-in of tools/make_learned_conductor.py by default."""
    names = list(_BSDFS)
    quads, bsdf, flip, emitter = [], [], [], []
    for m, name, fl in _RECTS:
        quads.append(np.concatenate(_rect(_mat(m))))
        bsdf.append(names.index(name)); flip.append(int(fl)); emitter.append(-1)
    for m, name in _CUBES:
        for f in _cube_faces(_mat(m)):
            quads.append(np.concatenate(f))
            bsdf.append(names.index(name)); flip.append(0); emitter.append(-1)
    quads.append(np.concatenate(_rect(_mat(_LIGHT))))
    bsdf.append(names.index("Light")); flip.append(0); emitter.append(0)
    cam = np.array([float(x) for x in _CAMERA.split()], np.float32)
    extra = {}
    if plastic or conductor:
        unknown = (set(plastic) | set(conductor)) - set(names)
        if unknown or set(plastic) & set(conductor):
            raise ValueError(f"unknown or doubly assigned BSDFs {sorted(unknown | (set(plastic) & set(conductor)))}")
        bp = np.zeros((len(names), 8), np.float32)
        for i, nm in enumerate(names):
            if nm in plastic:
                bp[i] = plastic_params(_BSDFS[nm])
            elif nm in conductor:
                bp[i] = conductor_params(tuple(min(1.0, 1.25 * c) for c in _BSDFS[nm]), alpha=alpha)
        extra["bsdf_params"] = bp.reshape(-1)
        if conductor and learned is not None:
            model = load_learned(learned)
            extra["learned_models"] = [model if nm in conductor else None for nm in names]
    return {**extra,
        "quads": np.asarray(quads, np.float32).reshape(-1),
        "flip_normals": np.asarray(flip, np.int32),
        "bsdf": np.asarray(bsdf, np.int32),
        "reflectance": np.asarray([_BSDFS[n] for n in names], np.float32).reshape(-1),
        "emitter": np.asarray(emitter, np.int32),
        "radiance": spectrum_to_rgb(_LIGHT_SPD).astype(np.float32),
        "camera_to_world": cam,
        "fov_x_deg": 35.0,
        "near_clip": 1e-2,
        "width": width,
        "height": height,
    }


def diffuse_learned_bsdf(n_bsdfs: int, sigma: float = 0.65):
    """Learned-BSDF tables for diffuse materials (the plugin's sampleProduct
    path; the suite's `diffuse.sdmm` files are LFS pointers, so the table is
    synthesised): per BSDF ONE directional lobe -- the plugin's diffuse case
    re-centres only slice 0 on the shading normal (sdmm_proc.cpp:335-339), so
    a diffuse learned BSDF is one lobe around the normal.  sigma: the lobe's
    tangent-space standard deviation (0.65 rad ~ the spread of a cosine lobe).
    Returns (weights (B, 1), local means (B, 1, 3), covs (B, 1, 4), diffuse (B,))."""
    B = int(n_bsdfs)
    w = np.ones((B, 1), np.float32)
    m = np.zeros((B, 1, 3), np.float32)
    m[..., 2] = 1.0
    cov = np.zeros((B, 1, 4), np.float32)
    cov[..., 0] = cov[..., 3] = sigma * sigma
    return w, m, cov, np.ones(B, np.uint8)
