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
    pkg = bench.load_pkg()
    for mode in (0, 1):
        out = bench.cornell_bench(pkg, torch.device("cuda", 0), None, 1, optimize_async=mode)
        print(json.dumps({k: v for k, v in out.items() if k != "iterations"}))
        for it in out["iterations"]:
            print(json.dumps(it))
