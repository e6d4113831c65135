#!/usr/bin/env python3
"""Fit and validate the polynomial behind estep.hip angle_over_sin().

theta/sin(theta) for c = cos(theta) >= 0 is, with u = (1 - c)/2,
    h(u) = asin(sqrt u) / (sqrt u * sqrt(1 - u)),
analytic on [0, 1/2] (nearest singularity at u = 1).  h is fitted by relative
least squares on Chebyshev-distributed nodes and evaluated in float32
Horner/FMA emulation.  For c < 0 the kernel uses theta = pi - theta':
f(c) = pi / sqrt(1 - c^2) - h(u).  The whole construction, including the
reference quirk `sin < 1e-3 -> 1` (mvtn.h:163-164), is compared with float64.

    python tools/fit_angle_over_sin.py
"""
import numpy as np

np.seterr(divide="ignore", invalid="ignore")
f32 = np.float32


def h_exact(u):
    u = np.asarray(u, np.float64)
    s = np.sqrt(u)
    g = np.where(u > 0, np.arcsin(s) / np.where(s > 0, s, 1), 1.0)
    return g / np.sqrt(1 - u)


def fma(a, b, c):
    return (np.float64(a) * np.float64(b) + np.float64(c)).astype(np.float32)


def horner(cf, x):
    r = np.full_like(x, cf[-1], dtype=np.float32)
    for k in range(len(cf) - 2, -1, -1):
        r = fma(r, x, cf[k])
    return r


def fit(deg):
    x = 0.25 * (1 - np.cos(np.linspace(0, np.pi, 6000)))
    A = np.vander(x, deg + 1, increasing=True)
    y = h_exact(x)
    c, *_ = np.linalg.lstsq(A / y[:, None], np.ones_like(y), rcond=None)
    return c.astype(np.float32)


def angle_over_sin_kernel(c, cf):
    """float32 emulation of estep.hip angle_over_sin (v_rsq taken as exact)."""
    c = c.astype(np.float32)
    u = fma(f32(-0.5), np.abs(c), f32(0.5))
    h = horner(cf, u)
    s2 = fma(-c, c, f32(1.0))
    r = (1.0 / np.sqrt(s2.astype(np.float64))).astype(np.float32)
    fneg = fma(f32(np.pi), r, -h)
    f = np.where(c < 0, fneg, h)
    return np.where(s2 < f32(1e-6), f32(1.0), f)


def reference(c):
    c = c.astype(np.float64)
    s = np.sqrt(1 - c * c)
    return np.where(s < 1e-3, 1.0, np.arccos(c) / np.where(s > 0, s, 1))


def main():
    uu = np.linspace(0, 0.5, 400001).astype(np.float32)
    for deg in (7, 8, 9, 10):
        cf = fit(deg)
        err = np.abs(horner(cf, uu) / h_exact(uu.astype(np.float64)) - 1).max()
        print(f"degree {deg}: max rel err on [0, 1/2] {err:.3e}  coeffs {[float(x) for x in cf]}")
    cf = fit(9)
    c = np.concatenate([np.linspace(-1, 1, 2000001), 1 - np.logspace(-9, -1, 10000),
                        -1 + np.logspace(-6, -1, 10000)]).astype(np.float32)
    a, b = angle_over_sin_kernel(c, cf), reference(c)
    away = np.sqrt(1 - c.astype(np.float64) ** 2) > 1.001e-3     # off the quirk boundary
    print("kernel form (degree 9): max rel err vs float64 %.3e" % np.abs(a[away] / b[away] - 1).max())
    th = np.arccos(c.astype(np.float64)).astype(np.float32)
    s = np.sqrt(fma(-c, c, f32(1))).astype(np.float32)
    o32 = np.where(s < 1e-3, 1, (th / s).astype(np.float32))
    print("reference fp32 acos/sqrt form: max rel err vs float64 %.3e" % np.abs(o32[away] / b[away] - 1).max())


if __name__ == "__main__":
    main()
