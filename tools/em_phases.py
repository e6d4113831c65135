#!/usr/bin/env python3
"""EM-step phase breakdown at the strong-scaling shard sizes (VERDICT r3 item
6): per shard of N = 2^20 / world samples at K (default 128) -- the fused
E + statistics kernels (sdmm_estep_stats), the M-step alone (sdmm_mstep: the
fp64 M-step, MVTN::set, CDF and record packing), the full EM step
(sdmm_em_step) and, with a world-1 RCCL communicator, the sharded EM step
(stats + all-reduce + M-step) and the bare all-reduce of the 2 + 21 K + 1
doubles.  Device times from events on the library's stream.

    python tools/em_phases.py [--K 128] [--reps 50] [--no-rccl]
"""
import argparse
import importlib
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--no-rccl", action="store_true")
    ap.add_argument("--worlds", default="1,8", help="shard counts to time (comma list)")
    a = ap.parse_args()
    import torch
    from conftest import load_pkg
    pkg = load_pkg()
    synth = importlib.import_module("sdmm_mitsuba_amd.synth")
    dev = torch.device("cuda:0")
    N = 1 << 20
    b = synth.em_batch(N, 128)
    pos, nrm = synth.model_seed_points(b, a.K)
    comm = None
    if not a.no_rccl:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1)
        comm = pkg.Comm.from_torch(0)

    def timed(fn, reps):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1000 / reps

    out = []
    for world in [int(w) for w in a.worlds.split(",")]:
        n = N // world
        mix = pkg.SDMM(a.K)
        mix.init_hemisphere(pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, synth.SEED_MODEL)
        part = pkg.DeviceSamples.from_numpy(b["x"][:, :n].copy(), b["w"][:n].copy(), b["hpdf"][:n].copy(),
                                            b["is_diffuse"][:n].copy(), device=dev)
        for _ in range(5):
            mix.optimize(part)
        st = torch.zeros(pkg.stats_len(a.K) + 1, dtype=torch.float64, device=dev)
        r = {"world": world, "n": n, "K": a.K}
        r["estep_stats_us"] = timed(lambda: mix.estep_stats(part, st), a.reps)
        r["mstep_us"] = timed(lambda: mix.mstep(st, n), a.reps)
        r["em_step_us"] = timed(lambda: mix.optimize(part), a.reps)
        if comm is not None:
            r["em_step_sharded_rccl_world1_us"] = timed(lambda: mix.optimize_sharded(comm, part), a.reps)
            buf = torch.zeros(pkg.stats_len(a.K) + 1, dtype=torch.float64, device=dev)
            r["allreduce_bytes"] = buf.numel() * 8
            r["allreduce_rccl_world1_us"] = timed(lambda: comm.allreduce_f64(buf), a.reps)
        print(json.dumps(r), flush=True)
        out.append(r)
    if comm is not None:
        comm.close()


if __name__ == "__main__":
    main()
