"""Debug: the rare-angle responsibility case, split vs tile kernel."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch
from conftest import load_pkg
import importlib
pkg = load_pkg()
synth = importlib.import_module("sdmm_mitsuba_amd.synth")
from oracle import oracle
from test_gpu_parity import _setup
gpu = torch.device("cuda:0")
K = 128
N = 999
b, mix, om, ost, ds, os_ = _setup(pkg, oracle, synth, K, N)
print("kernel", mix.kernel_name("resp"))
x = b["x"].copy()
mu = mix.get_params()["mean"][:, 3:6].astype(np.float64)
rng = np.random.default_rng(7)
modes = np.full(N, -1)
for i in range(0, N, 5):
    k = rng.integers(K)
    d = mu[k] / np.linalg.norm(mu[k])
    mode = (i // 5) % 4
    modes[i] = mode
    if mode == 1:
        d = -d
    elif mode == 2:
        t = np.cross(d, [0.0, 0.0, 1.0] if abs(d[2]) < 0.9 else [1.0, 0.0, 0.0])
        t /= np.linalg.norm(t)
        d = -np.cos(4e-4) * d + np.sin(4e-4) * t
    elif mode == 3:
        d = mu[k]
    x[3:6, i] = d.astype(np.float32)
x[:, 1::97] = np.nan
xt = [torch.from_numpy(x[i].copy()).to(gpu) for i in range(6)]
d2 = pkg.DeviceSamples(xt, ds.w)
resp = torch.empty((N, K), device=gpu)
mix.posterior(d2, resp)
got = resp.cpu().numpy()
ref = oracle.responsibilities(om, oracle.Samples(x, b["w"]))
lg = got.sum(1) > 0
lr = ref.sum(1) > 0
bad = np.nonzero(lg != lr)[0]
print("mismatch rows", len(bad), "got-live-only", int((lg & ~lr).sum()), "ref-live-only", int((~lg & lr).sum()))
print("rows", bad[:40])
print("modes", modes[bad[:40]])
print("tiles", np.unique(bad // 16)[:40])
for r in bad[:6]:
    print(r, "got sum", got[r].sum(), "ref sum", ref[r].sum(), "nz got", np.count_nonzero(got[r]), "nz ref", np.count_nonzero(ref[r]), "nan", np.isnan(got[r]).sum())
print("tile0 got sums", np.round(got[:16].sum(1), 4))
print("tile0 ref sums", np.round(ref[:16].sum(1), 4))
