#!/usr/bin/env python3
"""Fit and validate the polynomial behind estep.hip angle_over_sin().

g(u) = asin(sqrt u)/sqrt u on u in [0, 1/2] (relative least squares on
Chebyshev-distributed nodes), evaluated in float32 Horner/FMA emulation; then
the whole theta/sin(theta) construction (incl. the c<0 reflection and the
reference quirk sin<1e-3 -> 1, mvtn.h:163-164) against float64.
"""
import numpy as np
np.seterr(divide="ignore", invalid="ignore")
# g(u) = asin(sqrt(u))/sqrt(u), u in [0, 0.5];  f(c) = theta/sin(theta) for c=cos(theta)>=0: f = g(u)/sqrt(1-u), u=(1-c)/2
def g(u):
    u = np.asarray(u, np.float64); s = np.sqrt(u)
    return np.where(u > 0, np.arcsin(s)/np.where(s>0, s, 1), 1.0)
for deg in (5,6,7,8):
    # least-squares on Chebyshev nodes, relative weighting
    x = 0.25*(1-np.cos(np.linspace(0,np.pi,4000)))*1.0  # [0,0.5]
    A = np.vander(x, deg+1, increasing=True)
    y = g(x)
    # minimise relative error: weight 1/y
    c, *_ = np.linalg.lstsq(A/ y[:,None], np.ones_like(y), rcond=None)
    xx = np.linspace(0, 0.5, 200001)
    # evaluate in float32 Horner with fma emulation via float64 then round each step
    cf = c.astype(np.float32)
    r = np.full_like(xx, cf[-1], dtype=np.float32); xf = xx.astype(np.float32)
    for k in range(deg-1, -1, -1):
        r = (r.astype(np.float64)*xf + cf[k]).astype(np.float32)
    err = np.abs(r/g(xx) - 1).max()
    print(deg, err, list(map(float, cf)))

f32 = np.float32
C = [1.0, 0.1666697859764099, 0.07487323880195618, 0.04657839611172676, 0.01616133376955986, 0.07724328339099884, -0.09260322898626328, 0.1111316829919815]
C = [f32(x) for x in C]
def fma(a,b,c): return (np.float64(a)*np.float64(b)+np.float64(c)).astype(np.float32)
def rsq(x): return (1.0/np.sqrt(np.float64(x))).astype(np.float32)   # ~1ulp hardware; emulate exact
def fast(c):
    c = c.astype(np.float32); ac = np.abs(c)
    u = fma(f32(-0.5), ac, f32(0.5))
    g = np.full_like(u, C[7])
    for k in range(6, -1, -1): g = fma(g, u, C[k])
    h = rsq(fma(f32(0.5), ac, f32(0.5)))
    fpos = (g*h).astype(np.float32)
    s2 = fma(-c, c, f32(1.0))
    r = rsq(s2)
    fneg = fma(f32(np.pi), r, -fpos)
    f = np.where(c < 0, fneg, fpos)
    return np.where(s2 < f32(1e-6), f32(1.0), f)
def ref(c):
    c = c.astype(np.float64); s = np.sqrt(1-c*c); th = np.arccos(c)
    return np.where(s < 1e-3, 1.0, th/np.where(s>0,s,1))
c = np.concatenate([np.linspace(-1,1,2000001), 1-np.logspace(-9,-1,10000), -1+np.logspace(-6,-1,10000)]).astype(np.float32)
a = fast(c); b = ref(c)
rel = np.abs(a/b - 1)
ok = np.sqrt(1-c.astype(np.float64)**2) > 1.001e-3
print("max rel err (away from quirk boundary):", rel[ok].max(), "at c=", c[ok][rel[ok].argmax()])
# compare with float acos path (what the oracle's fp32 does): (float)acos/ sqrtf
th32 = np.arccos(c.astype(np.float64)).astype(np.float32); s32 = np.sqrt(fma(-c,c,f32(1))).astype(np.float32)
o32 = np.where(s32 < 1e-3, 1, (th32/s32).astype(np.float32))
print("fp32 acos/sqrt path rel err:", np.abs(o32[ok]/b[ok]-1).max())
