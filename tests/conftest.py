"""Test configuration: markers, package loading and shared fixtures.

`-m "not gpu"` tests run on CPU (oracle KATs, golden fixtures, C-ABI symbol
table, host logic, gloo world_size-2 sharding).  `-m gpu` tests are the parity
tests proper: they call the HIP library through the C ABI and compare it with
the CPU oracle (oracle/) on the same seeded inputs.
"""
import importlib.util
import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def load_pkg():
    name = "sdmm_mitsuba_amd"
    if name in sys.modules:
        return sys.modules[name]
    pkg_dir = ROOT / "sdmm-mitsuba_amd"
    spec = importlib.util.spec_from_file_location(name, pkg_dir / "__init__.py",
                                                  submodule_search_locations=[str(pkg_dir)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built HIP library")


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.build()
    return o


@pytest.fixture(scope="session")
def synth(pkg):
    import importlib
    return importlib.import_module("sdmm_mitsuba_amd.synth")


@pytest.fixture(scope="session")
def scenes(pkg):
    import importlib
    return importlib.import_module("sdmm_mitsuba_amd.scenes")


@pytest.fixture
def plog(request):
    """record(quantity, realized, bound): append the realized max error of a
    parity check next to the bound it was held to, one JSON line per check, to
    $SDMM_PARITY_LOG (default gpurun_out/parity_errors.jsonl; the round's copy
    is committed under profiles/)."""
    path = Path(os.environ.get("SDMM_PARITY_LOG", ROOT / "gpurun_out" / "parity_errors.jsonl"))

    def record(quantity, realized, bound, lower=False, **extra):
        """lower=True: `bound` is a lower bound (ok when realized >= bound)."""
        path.parent.mkdir(parents=True, exist_ok=True)
        ok = float(realized) >= float(bound) if lower else float(realized) <= float(bound)
        row = {"test": request.node.nodeid, "quantity": quantity, "realized": float(realized),
               "bound": float(bound), "ok": bool(ok)}
        if lower:
            row["bound_kind"] = "lower"
        row.update({k: (v if isinstance(v, (int, float, str, bool)) else str(v)) for k, v in extra.items()})
        with open(path, "a") as f:
            f.write(json.dumps(row) + "\n")
        return realized

    return record


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")
