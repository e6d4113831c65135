"""The Cornell Box line of bench.py alone (configs[0] on the device)."""
import importlib.util
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
spec = importlib.util.spec_from_file_location("bench", ROOT / "bench.py")
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)

if __name__ == "__main__":
    import torch
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, nargs="+", default=[16])
    ap.add_argument("--modes", type=int, nargs="+", default=[0, 1])
    ap.add_argument("--product", action="store_true", help="sampleProduct (the learned diffuse lobes)")
    a = ap.parse_args()
    pkg = bench.load_pkg()
    for K in a.K:
      for mode in a.modes:
        out = bench.cornell_bench(pkg, torch.device("cuda", 0), None, 1, optimize_async=mode, K=K,
                                  product=a.product)
        print(json.dumps({k: v for k, v in out.items() if k != "iterations"}), flush=True)
        for it in out["iterations"]:
            print(json.dumps(it), flush=True)
