"""CPU, world_size 2 over gloo: the sample-sharded EM protocol of the multi-GPU
path.  Each rank computes the sufficient statistics of its
contiguous shard, the ranks SUM them with an all-reduce, and every rank runs
the identical M-step with n_total = global sample count.  The result must equal
the single-process EM on the whole batch, and be identical on every rank
(no broadcast needed).  The statistics here come from the oracle; on the GPU
the same sequence is sdmm_estep_stats -> RCCL all_reduce -> sdmm_mstep
(bench.py em_step)."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, iters):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    from conftest import load_pkg
    pkg = load_pkg()
    import importlib
    synth = importlib.import_module("sdmm_mitsuba_amd.synth")
    from oracle import oracle as orc
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    K, N = 64, 6000
    b = synth.em_batch(N, 128, heuristic=True)
    pos, nrm = synth.model_seed_points(b, K)
    m, st = orc.hemisphere_init(K // 8, pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE,
                                synth.SEED_MODEL, mode=1)
    a, e = pkg.shard_range(N, rank, world)
    s = orc.Samples(b["x"][:, a:e], b["w"][a:e], b["hpdf"][a:e], b["is_diffuse"][a:e])
    for _ in range(iters):
        stats = torch.from_numpy(orc.calculate_stats(m, s, accurate="exact"))
        dist.all_reduce(stats)                       # SUM over ranks
        assert orc.mstep(m, st, stats.numpy(), N, accurate="exact") == 1
    np.savez(Path(out_dir) / f"rank{rank}.npz", weights=m.weights, mean=m.mean, cov=m.cov,
             sgC=st.d["sgC"], it=st.s.iterationsRun)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_em_equals_single_process(tmp_path, oracle, synth, pkg):
    import torch.multiprocessing as mp
    world, iters = 2, 3
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), iters), nprocs=world, join=True)
    r0 = np.load(tmp_path / "rank0.npz")
    r1 = np.load(tmp_path / "rank1.npz")
    for k in ("weights", "mean", "cov", "sgC"):
        np.testing.assert_array_equal(r0[k], r1[k])  # replicated M-step: bitwise identical
    # single-process reference
    K, N = 64, 6000
    b = synth.em_batch(N, 128, heuristic=True)
    pos, nrm = synth.model_seed_points(b, K)
    m, st = oracle.hemisphere_init(K // 8, pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE,
                                   synth.SEED_MODEL, mode=1)
    s = oracle.Samples(b["x"], b["w"], b["hpdf"], b["is_diffuse"])
    for _ in range(iters):
        oracle.optimize(m, st, s, accurate="exact")
    assert int(r0["it"]) == iters
    np.testing.assert_allclose(r0["weights"], m.weights, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(r0["mean"], m.mean, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(r0["cov"], m.cov, rtol=1e-5, atol=1e-9)
