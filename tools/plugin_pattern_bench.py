#!/usr/bin/env python3
"""The drop-in plugin's per-tile guided bounce, timed.

plugin/volpath_sdmm_amd.cpp (guideWavefront) serves each render tile's
bounce with ONE guided-wavefront call: upload the tile's query planes from
pinned host staging (9 float planes + the mode byte, one copy), the call,
download 4 float planes + the component index (one copy), synchronise.
Round 5 ran it under a global mutex on the model's stream (back-to-back calls
of the tile size).  Round 6 runs it through guide contexts (stream + scratch)
on the published tree, leased from a pool by the render workers, so the
workers' calls overlap.  This tool trains the Cornell Box guiding model
(K = 128 leaves, as the bench's cornell_k128 line), takes real queries -- the
saved vertices of one guided render (condition c, the sampled world direction
as the BSDF direction), uniforms from a fixed generator, half of them pdf
queries -- and times:
  * one thread, per tile size: the plugin pattern (pinned H2D + wavefront +
    D2H + synchronise) and the wavefront alone on device-resident planes;
  * the "threads_*" rows: C++ worker threads (tests/cpp/guide_pattern_harness.cpp)
    sharing a pool of guide contexts -- or, "_batch" rows, gathered into large
    wavefronts by sdmm_amd::GuideBatcher -- aggregate queries/s, outputs
    checked bitwise against the one-thread run.

    python tools/plugin_pattern_bench.py [--reps 20]
"""
import argparse
import importlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--keep", default=None, help="write the model / queries / harness here and keep them")
    ap.add_argument("--rows", default=None, help="comma list of threaded-row indices to run (default: all)")
    ap.add_argument("--no-tiles", action="store_true", help="skip the one-thread Python tile rows")
    a = ap.parse_args()
    import torch
    from conftest import load_pkg
    pkg = load_pkg()
    scenes = importlib.import_module("sdmm_mitsuba_amd.scenes")
    dev = torch.device("cuda:0")
    desc = scenes.cornell_box(640, 360)
    sc = pkg.Scene(desc)
    _, _, tmin, tmax = sc.normalization()
    g = pkg.Guiding(tmin, tmax, device=0, K=128)
    img = torch.zeros(3, 360, 640, device=dev)
    for it in range(3):                       # train for 16 spp, then one guided pass
        g.iteration(sc, 8, seed=1 + it, push_seed=1001 + it, train=it < 2, image=img)
    tree = g.tree
    node_mix = g.node_mixtures()
    _, verts, _ = sc.render(tree, node_mix, spp=8, guided=True, seed=99)
    rec, nv = verts.to_numpy()
    V = verts.s.max_vertices
    r = rec.reshape(16, V, -1)
    sel = np.arange(V)[:, None] < nv[None, :]
    c = np.stack([r[7][sel], r[8][sel], r[9][sel]]).astype(np.float32)
    dg = np.stack([r[10][sel], r[11][sel], r[12][sel]]).astype(np.float32)
    n_all = c.shape[1]
    rng = np.random.default_rng(5)
    u = rng.uniform(0, 1, size=(3, n_all)).astype(np.float32)
    mode = (rng.uniform(0, 1, size=n_all) < 0.5).astype(np.uint8)
    tree.bind(node_mix)
    ts = torch.cuda.ExternalStream(tree.stream_ptr) if tree.stream_ptr else torch.cuda.current_stream()
    out = {"queries_available": int(n_all), "K": 128, "scene": "Cornell Box 640x360, trained 16 spp",
           "pattern": "pinned H2D of 9 planes + mode, sdmm_guide_pdf_wavefront, D2H of 4 planes + comp, sync"}
    for T in (4096, 32768, 262144, min(n_all, 1 << 21)):
        if T > n_all or a.no_tiles:
            continue
        h_in = torch.from_numpy(np.concatenate([c[:, :T], u[:, :T], dg[:, :T]]).copy()).pin_memory()
        h_mode = torch.from_numpy(mode[:T].copy()).pin_memory()
        d_in = torch.empty((9, T), device=dev)
        d_mode = torch.empty(T, dtype=torch.uint8, device=dev)
        h_out = torch.empty((4, T)).pin_memory()
        h_comp = torch.empty(T, dtype=torch.int32).pin_memory()

        def device_call():
            cc = [d_in[i] for i in range(3)]
            uu = [d_in[3 + i] for i in range(3)]
            gg = [d_in[6 + i] for i in range(3)]
            return tree.guide_pdf(None, cc, uu, gg, d_mode)

        def plugin_call():
            with torch.cuda.stream(ts):
                d_in.copy_(h_in, non_blocking=True)
                d_mode.copy_(h_mode, non_blocking=True)
                d, pdf, comp = device_call()
                h_out[0:3].copy_(torch.stack(d), non_blocking=True)
                h_out[3].copy_(pdf, non_blocking=True)
                h_comp.copy_(comp, non_blocking=True)
            ts.synchronize()

        with torch.cuda.stream(ts):
            d_in.copy_(h_in)
            d_mode.copy_(h_mode)
        torch.cuda.synchronize()
        for fn in (plugin_call, device_call):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            plugin_call()
        tp = (time.perf_counter() - t) / a.reps
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            device_call()
        torch.cuda.synchronize()
        td = (time.perf_counter() - t) / a.reps
        out[f"tile_{T}"] = {"plugin_pattern_ms": tp * 1e3, "plugin_pattern_queries_per_s": T / tp,
                            "device_resident_ms": td * 1e3, "device_resident_queries_per_s": T / td,
                            "transfer_bytes_per_call": T * (9 * 4 + 1 + 4 * 4 + 4)}
        print(json.dumps({f"tile_{T}": out[f"tile_{T}"]}), flush=True)
    # the reference's threading (sdmm_proc.cpp:1086-1106) through guide
    # contexts: C++ worker threads, each its own context / stream / pinned
    # staging on the published tree (tests/cpp/guide_pattern_harness.cpp)
    import subprocess
    import tempfile
    from test_gpu_harness import write_guide_queries
    tmp = Path(a.keep) if a.keep else Path(tempfile.mkdtemp(prefix="gpb_"))
    tmp.mkdir(parents=True, exist_ok=True)
    tree.save_json(tmp / "model.asdmm", node_mix)
    n_mt = min(n_all, 1 << 21)
    write_guide_queries(tmp / "q.bin", c[:, :n_mt], u[:, :n_mt], dg[:, :n_mt], mode[:n_mt])
    exe = tmp / "guide_pattern_harness"
    lib = ROOT / "sdmm-mitsuba_amd" / "lib"
    subprocess.run(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    f"-I{ROOT / 'include'}", f"-I{ROOT / 'sdmm-mitsuba_amd' / 'host'}",
                    str(ROOT / "tests" / "cpp" / "guide_pattern_harness.cpp"),
                    f"-L{lib}", "-lsdmm_amd", "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{lib}",
                    "-Wl,-rpath,/opt/rocm/lib", "-pthread", "-o", str(exe)], check=True)
    ref = None
    import os
    # (threads, tile, contexts (0: one per thread), mode ("", "resident", "batch[:T:W]"), extra env)
    rows = [(1, 32768, 0, "", {}), (1, 32768, 0, "resident", {}), (4, 32768, 0, "", {}), (16, 32768, 4, "", {}),
            (16, 32768, 4, "resident", {}), (16, 32768, 2, "batch", {}), (16, 32768, 3, "batch", {}),
            (16, 32768, 4, "batch", {}), (16, 32768, 3, "batch:131072:200", {}), (16, 32768, 3, "batch:524288:400", {}),
            (16, 4096, 3, "batch", {}), (16, 262144, 3, "batch", {}), (16, 4096, 4, "", {}), (16, 262144, 4, "", {})]
    if a.rows:
        rows = [rows[int(i)] for i in a.rows.split(",")]
    for threads, T, nctx, mode, extra in rows:
        r = subprocess.run([str(exe), str(tmp / "model.asdmm"), str(tmp / "q.bin"), str(tmp / "o.bin"), str(threads),
                            str(T), str(max(2, a.reps // 4)), str(nctx)] + ([mode] if mode else []),
                           check=True, timeout=300, capture_output=True, text=True, env=dict(os.environ, **extra))
        row = json.loads(r.stdout.strip().splitlines()[-1])
        got = np.fromfile(tmp / "o.bin", np.uint8)
        if ref is None:
            ref = got
        row["bitwise_equal_to_1_thread"] = bool(np.array_equal(got, ref))
        key = f"threads_{threads}_ctx_{nctx or threads}_tile_{T}" + (f"_{mode}" if mode else "") + "".join(
            f"_{k}={v}" for k, v in extra.items())
        row["env"] = extra
        out[key] = row
        print(json.dumps({key: row}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
