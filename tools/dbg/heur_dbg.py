"""Debug: heuristic row sums, split vs tile kernel."""
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
from helpers import posterior_f64
gpu = torch.device("cuda:0")
K, N = 128, 2048
b, mix, om, ost, ds, os_ = _setup(pkg, oracle, synth, K, N, heuristic=True)
resp = torch.empty((N, K), device=gpu)
mix.posterior(ds, resp)
got = resp.cpu().numpy()
ref = oracle.responsibilities(om, os_)
exact = posterior_f64(mix.get_params(), b["x"], b["hpdf"], b["is_diffuse"])
print("kernel", mix.kernel_name("resp"))
rs = np.abs(got.sum(1) - exact.sum(1))
o = np.argsort(-rs)[:8]
for r in o:
    print(r, "err", rs[r], "got", got[r].sum(), "exact", exact[r].sum(), "ref", ref[r].sum(), "dif", b["is_diffuse"][r],
          "maxrel", np.max(np.abs(got[r] - exact[r]) / np.maximum(exact[r], 1e-30)), "tile", r // 16, "col", r % 16)
