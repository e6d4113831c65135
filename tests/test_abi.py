"""CPU: the C-ABI library loads and exports every symbol include/sdmm_gpu.h
declares; host-side logic (initialisation, argument validation) without a GPU."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _declared():
    text = (ROOT / "include" / "sdmm_gpu.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sdmm_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(pkg):
    lib = C.CDLL(str(pkg.LIB_PATH))
    names = _declared()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"declared in sdmm_gpu.h but not exported: {missing}"
    assert sorted(pkg.EXPORTED_SYMBOLS) == names


def test_abi_constants(pkg):
    lib = pkg.lib()
    assert lib.sdmm_abi_version() == 1
    for K in (1, 16, 128, 512):
        assert lib.sdmm_stats_len(K) == 2 + 21 * K == pkg.stats_len(K)


def test_hemisphere_init_host_matches_oracle_bitwise(pkg, oracle, synth):
    b = synth.em_batch(512, 128)
    for K, seed in ((16, 1), (128, 0x1A17), (256, 99)):
        pos, nrm = synth.model_seed_points(b, K)
        h = pkg.hemisphere_init_host(pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, seed)
        m, st = oracle.hemisphere_init(K // 8, pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, seed)
        np.testing.assert_array_equal(h["mean"], m.mean)
        np.testing.assert_array_equal(h["cov"].reshape(K, 25), m.cov)
        np.testing.assert_array_equal(h["bpriors"].reshape(-1), st.bPriors)
        np.testing.assert_array_equal(h["bdepth"].reshape(-1), st.bDepth)
        np.testing.assert_allclose(h["weights"], 1.0 / K)


def test_invalid_arguments_are_reported_not_raised(pkg):
    lib = pkg.lib()
    rc = lib.sdmm_hemisphere_init_host(None, None, 0, 0.01, 0.1, 1, None, None, None, None, None)
    assert rc == -1
    assert b"invalid" in lib.sdmm_last_error()
    h = C.c_void_p()
    assert lib.sdmm_create(0, None, 0, C.byref(h)) == -1         # K out of range
    assert lib.sdmm_create(513, None, 0, C.byref(h)) == -1
    assert not h.value
    # null handles are reported, never dereferenced
    assert lib.sdmm_set_guide_capacity(None, 8) == -1
    ci = C.c_int()
    assert lib.sdmm_layout(None, C.byref(ci), None, None, None) == -1


def test_python_binding_fails_loudly_without_library(pkg, tmp_path, monkeypatch):
    monkeypatch.setattr(pkg, "LIB_PATH", tmp_path / "missing.so")
    monkeypatch.setattr(pkg, "_lib", None)
    with pytest.raises(pkg.SDMMError):
        pkg.lib()


def test_shard_ranges_partition_the_batch(pkg):
    for n in (0, 1, 7, 1 << 20, 1000003):
        for world in (1, 2, 3, 8):
            rs = [pkg.shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c and a <= b


def test_cpp_mirror_header_compiles(tmp_path):
    """The C++ host mirror (sdmm-mitsuba_amd/host/sdmm_amd.hpp) compiles and
    links against the C ABI without a GPU (the plugin-side include)."""
    import subprocess
    src = tmp_path / "m.cpp"
    src.write_text('#include "sdmm_amd.hpp"\nint main() { return sdmm_abi_version() == 1 ? 0 : 1; }\n')
    lib = ROOT / "sdmm-mitsuba_amd" / "lib"
    exe = tmp_path / "m"
    subprocess.run(["g++", "-std=c++17", f"-I{ROOT / 'sdmm-mitsuba_amd' / 'host'}", f"-I{ROOT / 'include'}",
                    str(src), f"-L{lib}", "-lsdmm_amd", f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True)


def test_comm_host_transport_without_gpu(pkg):
    """sdmm_comm_init_host validates its arguments and reports rank/size; the
    host transport needs no device until a collective runs."""
    lib = pkg.lib()
    h = C.c_void_p()
    assert lib.sdmm_comm_init_host(2, 0, 0, pkg._HOST_ALLREDUCE(), pkg._HOST_BCAST(), None, C.byref(h)) == -1
    assert lib.sdmm_comm_init_host(1, 1, 0, pkg._HOST_ALLREDUCE(), pkg._HOST_BCAST(), None, C.byref(h)) == -1
    comm = pkg.Comm.host(3, 2, lambda a: None, lambda a, root: None)
    assert comm.rank == 2 and comm.size == 3
    comm.close()
    assert lib.sdmm_comm_rank(None) == -1 and lib.sdmm_comm_size(None) == 0
