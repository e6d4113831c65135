"""The guide kernels' Gaussian weight NORM exp(-q/2) (csrc/fastexp.h): a
table-driven double evaluation decided by a Ziv rounding test, else the
reference expression (float)((double)norm * exp(-0.5 * (double)q))
(multivariate_normal.h:126, multivariate_tangent_normal.h:359).

CPU: the host build of the same function against libm (math.exp) on random,
edge and crafted near-rounding-boundary arguments, bit for bit; the crafted
cases must take the slow path.  GPU: the device build against the host build
and libm on the same arrays, bit for bit.
"""
import math

import numpy as np
import pytest

NORM3 = np.float32(0.063493635934240969)   # (2 pi)^-3/2 as the kernels hold it
NORM2 = np.float32(0.15915494309189535)    # (2 pi)^-1


def _ref(q, norm):
    """(float)((double)norm * exp(-0.5 * (double)q)) with libm's exp."""
    n = float(norm)
    out = np.empty(q.shape, dtype=np.float32)
    for i, v in enumerate(q.tolist()):
        try:
            out[i] = np.float32(n * math.exp(-0.5 * v))
        except OverflowError:   # (q = -inf; never produced by a sum of squares)
            out[i] = np.float32(np.inf)
    return out


def _ftz(a):
    """The plugin's FTZ: a float result below FLT_MIN is 0 (every caller
    multiplies the weight next, which flushes a denormal input to 0)."""
    a = a.copy()
    a[np.abs(a) < np.finfo(np.float32).tiny] = 0.0
    return a


def _boundary_cases(norm, n_draw=1 << 22, width=2.0 ** -15, seed=7):
    """q whose float64 weight lies within `width` float ulps of a rounding
    midpoint (the fast path's margin is 2^-16 ulp plus its 2^-44 error)."""
    rng = np.random.default_rng(seed)
    q = rng.uniform(0.0, 168.0, n_draw).astype(np.float32)
    v = float(norm) * np.exp(-0.5 * q.astype(np.float64))
    f = v.astype(np.float32)
    e = np.frexp(f.astype(np.float64))[1]                 # f in [2^(e-1), 2^e)
    ulp = np.ldexp(1.0, e - 24)
    frac = (v - f.astype(np.float64)) / ulp               # in [-0.5, 0.5]
    sel = np.abs(np.abs(frac) - 0.5) < width
    return q[sel]


def _cases(norm):
    rng = np.random.default_rng(1)
    parts = [
        rng.uniform(0.0, 200.0, 200000).astype(np.float32),
        (rng.standard_normal(50000) ** 2 * 3).astype(np.float32),
        np.array([0.0, -0.0, 1e-30, 1e-8, 0.5, 1.0, 2.0, 168.0, 168.4, 168.5, 169.0, 170.0, 171.0,
                  174.0, 175.5, 176.0, 180.0, 300.0, 1e4, 1e30, 3.4e38, np.inf, np.nan], dtype=np.float32),
        # exact powers of two of the result: q = -2 ln(2^-m / norm)
        np.array([-2.0 * math.log(2.0 ** -m / float(norm)) for m in range(1, 126)], dtype=np.float32),
        # the FLT_MIN edge: v = FLT_MIN (1 + d)
        np.array([-2.0 * math.log(2.0 ** -126 * (1 + d) / float(norm))
                  for d in (-1e-3, -1e-6, -2e-7, 0.0, 2e-7, 1e-6, 1e-3)], dtype=np.float32),
    ]
    return np.concatenate(parts)


@pytest.mark.parametrize("norm", [NORM3, NORM2])
def test_host_norm_exp_matches_libm(pkg, norm):
    q = _cases(norm)
    got, fast = pkg.norm_exp(q, float(norm))
    ref = _ftz(_ref(q, norm))
    bad = ~((got == ref) | (np.isnan(got) & np.isnan(ref)))
    assert not bad.any(), (q[bad][:8], got[bad][:8], ref[bad][:8])
    # the fast path decides the common case
    fin = (q >= 0) & (q < 160)
    assert fast[fin].mean() > 0.999


@pytest.mark.parametrize("norm", [NORM3, NORM2])
def test_host_boundary_cases_take_the_slow_path(pkg, norm):
    q = _boundary_cases(norm)
    assert q.size > 50
    got, fast = pkg.norm_exp(q, float(norm))
    ref = _ftz(_ref(q, norm))
    np.testing.assert_array_equal(got, ref)
    # within 2^-17 ulp of a midpoint the fast path must decline
    tight = _boundary_cases(norm, width=2.0 ** -17)
    _, ft = pkg.norm_exp(tight, float(norm))
    assert tight.size > 5 and not ft.any()
    assert (fast == 0).sum() >= tight.size


@pytest.mark.gpu
@pytest.mark.parametrize("norm", [NORM3, NORM2])
def test_device_norm_exp_matches_host_and_libm(pkg, gpu, norm):
    import torch
    q = np.concatenate([_cases(norm), _boundary_cases(norm)])
    host, hfast = pkg.norm_exp(q, float(norm))
    dev, dfast = pkg.norm_exp(torch.from_numpy(q).to(gpu), float(norm), device=gpu)
    dev, dfast = dev.cpu().numpy(), dfast.cpu().numpy()
    same = (dev == host) | (np.isnan(dev) & np.isnan(host))
    assert same.all(), (q[~same][:8], dev[~same][:8], host[~same][:8])
    np.testing.assert_array_equal(dfast, hfast)   # the same decision on both sides
    ref = _ftz(_ref(q, norm))
    assert ((dev == ref) | (np.isnan(dev) & np.isnan(ref))).all()
    assert (dfast == 0).sum() > 50   # the crafted cases exercised the slow path on the device
