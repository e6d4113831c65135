#!/usr/bin/env python3
"""Benchmark: EM samples/sec (N x K responsibilities) at K=128, N=2^20.

Headline step (BASELINE.json `metric`, configs[1]): one responsibility E-step
(MixtureModel::posteriorAndLog for every sample, mixture_model.h:146-192 --
the N x K hot loop of StepwiseTangentEM, stepwise_tangent.h:270-353) over a
synthetic batch of N = 2^20 samples against a K = 128 mixture that has been
through 5 warm EM iterations.  Inputs (SoA fp32 planes) are resident in HBM
before timing; the N x K fp32 responsibilities are written to HBM.

Multi-GPU (torchrun, one process per GPU): STRONG scaling (north_star, SURVEY
7/8e) -- the fixed N = 2^20 batch is sharded N/world contiguous samples per
rank (SURVEY 8e partitioning), no data-path collective for the E-step; EM
steps go through the library's own RCCL communicator (sdmm_comm_init_rccl,
sdmm_em_step_sharded: the fp64 sufficient statistics of the shards are
all-reduced over xGMI before each M-step).  value = N / max-over-ranks step
time.  An extra `weak` line times every rank on its own full N = 2^20 part of
an N x world batch.

Also reported (same JSON line): the full EM step (E-step + statistics +
all-reduce + M-step), guided queries/sec (conditional + sample + pdf, Q = 2^20,
replicas), the roofline of the dominant kernel (HIP events on the kernel's
stream) and the CPU baseline (the C oracle on the host cores, bounded sample).
"""
import argparse
import importlib.util
import json
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "sdmm-mitsuba_amd"
HBM_PEAK = 8.0e12            # B/s, MI355X spec (MI355X_MICROARCH.md)
FP32_PEAK = 157.3e12         # FLOP/s vector fp32 spec


def load_pkg():
    name = "sdmm_mitsuba_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_threads() -> int:
    """`nproc`: the CPUs this process may run on, capped by OMP_NUM_THREADS
    (GNU nproc honours it; the GPU box sets it to this job's CPU share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(batch, K, pos, nrm, synth, n_sample, threads, reps=20):
    """The CPU oracle (faithful fp32 restatement of jmm) on the host cores:
    (i) the responsibility E-step (the metric's step) and (ii) the full EM step
    (or_calculate_stats per thread on its sample shard, summed, then or_mstep --
    the reference's sample-sharded pattern, stepwise.h:248-396), each the MEDIAN
    of `reps` passes over a bounded sample, on `threads` = nproc host threads;
    plus single-thread passes (the reference EM's num_threads(1),
    stepwise_tangent.h:611)."""
    sys.path.insert(0, str(ROOT))
    from oracle import oracle as orc
    orc.build()

    def fresh():
        m, st = orc.hemisphere_init(K // 8, pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE,
                                    synth.SEED_MODEL, mode=0)
        return m, st

    m, st = fresh()

    def shards(n, nthreads):
        x, w = batch["x"][:, :n], batch["w"][:n]
        per = (n + nthreads - 1) // nthreads
        return [orc.Samples(x[:, t * per:min(n, (t + 1) * per)], w[t * per:min(n, (t + 1) * per)])
                for t in range(nthreads)]

    def parallel(fn, parts):
        ths = [threading.Thread(target=fn, args=(t, p)) for t, p in enumerate(parts)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        return time.perf_counter() - t0

    def estep_pass(parts):
        return parallel(lambda t, p: orc.responsibilities(m, p), parts)

    def em_pass(parts, mm, sst):
        acc = [None] * len(parts)

        def work(t, p):
            acc[t] = orc.calculate_stats(mm, p, accurate="faithful")
        t0 = time.perf_counter()
        parallel(work, parts)
        total = np.sum(acc, axis=0)
        orc.mstep(mm, sst, total, int(sum(p.s.n for p in parts)), accurate="faithful")
        return time.perf_counter() - t0

    n_e, n_em = n_sample, n_sample
    pe = shards(n_e, threads)
    te = sorted(estep_pass(pe) for _ in range(reps))
    pm = shards(n_em, threads)
    mm, sst = fresh()
    tm = sorted(em_pass(pm, mm, sst) for _ in range(reps))
    n1 = 1 << 16
    t1 = estep_pass(shards(n1, 1))
    m1, s1 = fresh()
    t1m = em_pass(shards(n1 // 2, 1), m1, s1)
    med = lambda v: v[len(v) // 2]
    return {"value": n_e / med(te), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"responsibility E-step, median of {reps} passes over the first {n_e} of the "
                      f"{batch['w'].shape[0]} samples, K={K}: oracle or_responsibilities (faithful fp32 jmm "
                      f"restatement) sample-sharded over {threads} host threads (nproc)",
            "seconds": float(sum(te)),
            "em_step": {"value": n_em / med(tm), "unit": "samples/s", "cores": threads,
                        "sample": f"full EM step (per-thread or_calculate_stats f32 + sum + or_mstep f32), "
                                  f"median of {reps} passes over {n_em} samples, K={K}",
                        "seconds": float(sum(tm))},
            "single_thread": {"value": n1 / t1, "cores": 1, "sample": f"E-step, {n1} samples, 1 pass",
                              "seconds": t1,
                              "em_step": {"value": (n1 // 2) / t1m, "sample": f"EM step, {n1 // 2} samples"}}}


def leaf_em_bench(pkg, synth, full, N, dev, stream, args, timed, world, rank, comm, K=16, leaf_samples=4096):
    """The plugin's per-leaf EM over N / leaf_samples leaves of K components
    (volpath_sdmm.cpp:287-311), leaf-sharded: rank r steps the
    leaves it owns (owner = leaf % world) in one batched call
    (sdmm_em_step_batched), then every leaf's parameters are broadcast from its
    owner (sdmm_mix_broadcast, one fused RCCL group) so every rank can guide
    with all of them.  Strong scaling (the leaves are fixed); also the same
    owned leaves stepped by per-leaf calls, for comparison."""
    n_leaves = N // leaf_samples
    seg = np.arange(n_leaves + 1, dtype=np.int64) * leaf_samples
    x = np.stack([t.cpu().numpy() for t in full.x])
    nrm = np.ascontiguousarray(x[3:6].T)    # seed "normals": any unit vectors (directions)
    n_pos = K // 8
    mixes = []
    for i in range(n_leaves):
        a = int(seg[i])
        m = pkg.SDMM(K, device=dev.index, stream=stream)
        m.init_hemisphere(x[0:3, a:a + n_pos].T.copy(), nrm[a:a + n_pos].copy(), synth.DEPTH_PRIOR,
                          synth.SPATIAL_DISTANCE, synth.SEED_MODEL + i)
        mixes.append(m)
    owner = (np.arange(n_leaves) % world).astype(np.int32)
    mine = [i for i in range(n_leaves) if owner[i] == rank]
    own_mixes = [mixes[i] for i in mine]
    import torch
    idx = torch.from_numpy(np.concatenate([np.arange(seg[i], seg[i + 1]) for i in mine])).to(dev)
    own = pkg.DeviceSamples([t[idx] for t in full.x], full.w[idx])
    own_seg = np.arange(len(mine) + 1, dtype=np.int64) * leaf_samples

    def step():
        pkg.em_step_batched(own_mixes, own, own_seg, 1)
        if comm is not None:
            pkg.mix_broadcast(mixes, owner, comm)
    step()                                          # warm-up (tables, partial rows)
    steps = max(3, args.steps // 4)
    b_wall, b_kern = timed(step, steps)
    leaves = [pkg.DeviceSamples([t[int(own_seg[j]):int(own_seg[j + 1])] for t in own.x],
                                own.w[int(own_seg[j]):int(own_seg[j + 1])]) for j in range(len(mine))]

    def sequential():
        for m, leaf in zip(own_mixes, leaves):
            m.optimize(leaf)
    sequential()
    s_wall, _ = timed(sequential, 2, events=False)
    return {"samples_per_s": n_leaves * leaf_samples / (b_wall / steps), "ms_per_step": b_wall / steps * 1e3,
            "device_ms_per_step": b_kern * 1e3, "leaves": n_leaves, "leaves_per_rank": len(mine), "K": K,
            "samples_per_leaf": leaf_samples,
            "scaling": "strong (leaves sharded over ranks, parameters broadcast from their owners)",
            "sequential_per_leaf_calls_ms": s_wall / 2 * 1e3}


def wavefront_bench(pkg, synth, batch, shard, tree, dev, stream, ct, ut, gout, timed, args, world, K=16):
    routed, seg = tree.route(shard)
    nn = len(seg) - 1
    x = np.stack([t.cpu().numpy() for t in routed.x[:6]])
    n_pos = K // 8
    mixes = [None] * nn
    for v in range(nn):
        a, e = int(seg[v]), int(seg[v + 1])
        if e - a < 64:
            continue
        m = pkg.SDMM(K, device=dev.index, stream=stream)
        m.init_hemisphere(x[0:3, a:a + n_pos].T.copy(), x[3:6, a:a + n_pos].T.copy(), synth.DEPTH_PRIOR,
                          synth.SPATIAL_DISTANCE, synth.SEED_MODEL + v)
        mixes[v] = m
    live = [v for v in range(nn) if mixes[v] is not None]
    sub = np.zeros(len(live) + 1, np.int64)
    parts_x = [[] for _ in range(6)]
    parts_w = []
    for i, v in enumerate(live):                   # the trained leaves' samples, contiguous
        a, e = int(seg[v]), int(seg[v + 1])
        for j in range(6):
            parts_x[j].append(routed.x[j][a:e])
        parts_w.append(routed.w[a:e])
        sub[i + 1] = sub[i] + (e - a)
    import torch
    leaf_samples = pkg.DeviceSamples([torch.cat(p) for p in parts_x], torch.cat(parts_w))
    pkg.em_step_batched([mixes[v] for v in live], leaf_samples, sub, 2)
    tree.set_stream(stream)
    tree.bind(mixes)                               # once per training iteration in the plugin
    tree.guide(None, ct, ut, gout)
    steps = max(3, args.steps // 4)
    # the tree runs on its own stream when handed torch's null stream (handle
    # 0): its device time is measured with events on THAT stream
    tree_stream = torch.cuda.ExternalStream(tree.stream_ptr) if tree.stream_ptr else stream
    w_wall, w_kern = timed(lambda: tree.guide(None, ct, ut, gout), steps, ev_stream=tree_stream)
    comp = gout[2].cpu().numpy()
    q = ct[0].numel()
    return {"queries_per_s": q * world / (w_wall / steps), "Q": q * world, "ms_per_step": w_wall / steps * 1e3,
            "kernel_us": w_kern * 1e6, "fp32_frac": q * 22.0 * K / w_kern / FP32_PEAK,
            "flops_per_query_lower_bound": 22 * K, "hbm_frac": q * 48.0 / w_kern / HBM_PEAK,
            "leaves_with_mixture": len(live), "nodes": nn, "K": K,
            "guided_frac": float((comp >= 0).mean()), "scaling": "weak (replicas: queries per rank)"}


def cornell_cpu_baseline(pkg, g, desc, spp, seed, threads, learned=None, budget_s=6.0, probe_px=512):
    """The CPU restatement of Li (oracle/sdmm_oracle_li.inc) rendering the same
    guided pass (the trained model's leaves as oracle mixtures, the same tree,
    seed and spp) over a bounded slice of the image on `threads` host threads:
    guided rays/s = bounce rays traced / wall time (the reference's CPU Li
    cannot run here: no Mitsuba)."""
    sys.path.insert(0, str(ROOT))
    from oracle import oracle as orc
    orc.build()
    mixes = []
    for m in g.node_mixtures():
        if m is None:
            mixes.append(None)
            continue
        p = m.get_params()
        om = orc.Mixture(m.K)
        om.copy_params_from(p)
        om.valid[:] = p["valid"]
        mixes.append(om)
    aabb, child, _ = g.tree.nodes()
    npix = desc["width"] * desc["height"]
    kw = dict(node_mix=mixes, guided=True, spp=spp, seed=seed, learned=learned, threads=threads)
    t = time.perf_counter()
    r = orc.li_render(desc, aabb, child, pixels=(0, probe_px), **kw)     # probe
    dt = time.perf_counter() - t
    n = int(min(npix, max(probe_px, probe_px * budget_s / max(dt, 1e-3))))
    t = time.perf_counter()
    r = orc.li_render(desc, aabb, child, pixels=(0, n), **kw)
    dt = time.perf_counter() - t
    rays = int(r["nv"].sum())
    return {"value": rays / dt, "unit": "rays/s", "cores": threads, "kind": "port",
            "sample": f"guided pass of the trained model, first {n} of {npix} pixels x {spp} spp "
                      f"({n * spp} paths, {rays} bounce rays): oracle or_li_render (CPU restatement of "
                      f"SDMMRenderer::Li with the oracle's conditional{' and product' if learned else ''}) "
                      f"on {threads} host threads",
            "seconds": dt}


def cornell_bench(pkg, dev, args, world, optimize_async=0, K=16, product=False, cpu=False, cpu_probe_px=512,
                  cpu_budget_s=6.0, glossy=()):
    """configs[0] on the device: the test suite's Cornell Box (640x360), K=16
    per leaf (K=128: the Torus line's K, configs[2], over the one scene whose
    geometry the snapshot holds), 64 spp rendered 8 spp per iteration, training (push + optimize)
    while samplesRendered < sampleCount / 4 (volpath_sdmm.cpp:411-507), the
    native guiding model (sdmm_guiding_iteration) with the device Li.  Replicas
    only (each rank renders the whole image; no exchange).  "guided rays/s" =
    bounce rays traced per second in the guided passes.  glossy: BSDFs made
    rough conductors (with product sampling: the non-diffuse learned-BSDF
    branch, per-bounce lobes rotated to wi)."""
    import torch
    scenes = importlib.import_module("sdmm_mitsuba_amd.scenes")
    desc = scenes.cornell_box(640, 360, conductor=glossy)
    sc = pkg.Scene(desc, device=dev.index)
    _, _, tmin, tmax = sc.normalization()
    table = learned = None
    if product:   # sampleProduct: every Cornell BSDF is diffuse, one learned lobe each
        learned = scenes.diffuse_learned_bsdf(len(desc["reflectance"]) // 3)
        table = pkg.BsdfTable(*learned[:3], device=dev, diffuse=learned[3])
    spp_total, spp_it = 64, 8
    img = torch.zeros(3, 360, 640, device=dev)
    acc = torch.zeros_like(img)
    its = []
    for rep in range(2):                          # the first run pages in code and scratch (untimed)
        g = pkg.Guiding(tmin, tmax, device=dev.index, optimize_async=optimize_async, K=K)
        acc.zero_()
        its = []
        torch.cuda.synchronize()
        t_all = time.perf_counter()
        for it, done in enumerate(range(0, spp_total, spp_it)):
            train = done < spp_total // 4
            t = time.perf_counter()
            _, ls, gs = g.iteration(sc, spp_it, seed=1 + it, push_seed=1001 + it, train=train, image=img,
                                    learned_bsdf=table)
            acc += img
            torch.cuda.synchronize()
            its.append({"ms": (time.perf_counter() - t) * 1e3, "train": train, "segments": ls["segments"],
                        "guided_queries": ls["guided_queries"], "fallback_queries": ls["fallback_queries"],
                        "paths": ls["paths"], "leaves": gs["leaves"] if train else None,
                        "optimized": gs["optimized"] if train else None, "trained": g.trained})
        total = time.perf_counter() - t_all
    guided = [x for x in its if not x["train"]]
    seg = sum(x["segments"] for x in guided)
    gms = sum(x["ms"] for x in guided)
    res = {"workload": f"Cornell Box 640x360{' with rough conductors ' + '/'.join(glossy) if glossy else ''}, "
                       f"K={K} per leaf, 64 spp (8 per iteration, training for the first 16)",
            "total_ms": total * 1e3, "guided_rays_per_s": seg / (gms * 1e-3),
            "guided_paths_per_s": sum(x["paths"] for x in guided) / (gms * 1e-3),
            "trained_leaves": its[-1]["trained"], "iterations": its,
            "image_mean": float((acc / len(its)).mean().item()), "replicas": world,
            "optimize_async": bool(optimize_async), "sample_product": bool(product)}
    if cpu:
        try:
            res["cpu_baseline"] = cornell_cpu_baseline(pkg, g, desc, spp_it, 1 + len(its) - 1, host_threads(),
                                                       learned, budget_s=cpu_budget_s, probe_px=cpu_probe_px)
        except Exception as e:  # reported, never required
            res["cpu_baseline"] = {"value": None, "error": repr(e)}
    return res


def large_k_bench(pkg, synth, batch, shard, dev, stream, timed, args, world, N, comm):
    """BASELINE configs[3] and [4] on one GPU: a full EM step at K=256 (Pool)
    and K=512 (Kitchen) on the same 2^20-sample batch (sample-sharded, RCCL
    all-reduce of the statistics when world > 1), and the Kitchen's guided
    bounce with learned-BSDF product sampling at K=512 (replicas: Q/world
    queries per rank; 8 materials x 8 lobes, every query with a material)."""
    import torch
    res = {}
    for K in (256, 512):
        pos, nrm = synth.model_seed_points(batch, K)
        m = pkg.SDMM(K, device=dev.index, stream=stream)
        m.init_hemisphere(pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, synth.SEED_MODEL)
        def em_step():
            if comm is not None:
                m.optimize_sharded(comm, shard)      # RCCL sum of the statistics (library)
            else:
                m.optimize(shard)
        for _ in range(3):
            em_step()
        steps = max(3, args.steps // 4)
        w, _ = timed(em_step, steps, events=False)
        res[f"em_step_K{K}"] = {"samples_per_s": N / (w / steps), "ms_per_step": w / steps * 1e3}
        if K == 512:
            q = (1 << 18) // world
            c, u = synth.sample_queries_near(batch, q, seed=synth.SEED_QUERIES + 7)
            B, M = 8, 8
            bw, bmean, bcov = synth.bsdf_table(B, M)
            F = synth.shading_frames(q)
            mat = (np.arange(q) % B).astype(np.int32)
            tt = lambda a: [torch.from_numpy(np.ascontiguousarray(a[i])).to(dev) for i in range(a.shape[0])]
            ct, ut, Ft = tt(c), tt(u), tt(F.T)
            matt = torch.from_numpy(mat).to(dev)
            table = pkg.BsdfTable(bw, bmean, bcov, device=dev)
            m.guide_product(ct, ut, table, matt, Ft)
            ps = max(3, args.steps // 4)
            pw, pk = timed(lambda: m.guide_product(ct, ut, table, matt, Ft), ps)
            res["guide_product_K512"] = {"queries_per_s": q * world / (pw / ps), "Q": q * world,
                                         "ms_per_step": pw / ps * 1e3, "kernel_us": pk * 1e6,
                                         "materials": B, "lobes": M}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # (the E-step's clock transient: per-launch times rise from ~163 to ~190 us
    # over launches 5-25 after the EM warm-up, fall to ~157-161 by launches
    # 50-100 and settle at ~149-155 from launch ~200 on
    # (profiles/round5_resp_series.json, profiles/round6_resp_series600.json:
    # 600 launches); the defaults time the sustained rate.  The driver's own
    # --warmup overrides --warmup, not --settle.)
    ap.add_argument("--warmup", type=int, default=60)
    # untimed E-step launches before the timed ones, at least: a driver run
    # with a small --warmup would otherwise time the clock transient; the
    # extra launches beyond --warmup are reported as "settle_launches"
    # (200 launches: ~32 ms)
    ap.add_argument("--settle", type=int, default=200)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--N", type=int, default=1 << 20)
    ap.add_argument("--Q", type=int, default=1 << 20)
    ap.add_argument("--em-warm", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="headline E-step only (profiling)")
    ap.add_argument("--no-large-k", action="store_true", help="skip the K=256/512 lines")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: nproc")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; SDMM_BENCH_REHEARSE=1 rehearses the N>1 path on a
    # box with fewer GPUs (ranks share devices, collectives over gloo) -- a
    # correctness rehearsal only, never a reported scaling number
    rehearse = os.environ.get("SDMM_BENCH_REHEARSE") == "1"
    gpu = local % torch.cuda.device_count() if rehearse else local
    if world > 1:
        torch.cuda.set_device(gpu)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    dev = torch.device("cuda", gpu if world > 1 else 0)
    torch.cuda.set_device(dev)

    pkg = load_pkg()
    synth = importlib.import_module("sdmm_mitsuba_amd.synth")
    K, N = args.K, args.N

    # strong scaling (the samples partition over ranks): every rank
    # builds the same N-sample batch (deterministic seeds) and owns the
    # contiguous shard [rank N/world, (rank+1) N/world); the E-step needs no
    # exchange, the EM step all-reduces the shards' statistics.  The model is
    # the same on every rank (the batch's own first samples seed it).
    t0 = time.perf_counter()
    batch = synth.em_batch(N, 128)
    pos, nrm = synth.model_seed_points(batch, K)
    log(f"[bench] rank {rank}/{world}: synthetic batch N={N} in {time.perf_counter() - t0:.1f}s")
    full = pkg.DeviceSamples.from_numpy(batch["x"], batch["w"], batch["hpdf"], batch["is_diffuse"],
                                        device=dev)
    shard = full.shard(rank, world) if world > 1 else full
    n_local = shard.n
    N_global = N

    stream = torch.cuda.current_stream(dev)
    mix = pkg.SDMM(K, device=dev.index, stream=stream)
    mix.init_hemisphere(pos, nrm, synth.DEPTH_PRIOR, synth.SPATIAL_DISTANCE, synth.SEED_MODEL)
    stats = torch.zeros(pkg.stats_len(K), dtype=torch.float64, device=dev)
    # the library's own communicator: RCCL over xGMI (the unique id travels
    # through torch.distributed); the rehearsal shares one GPU, where RCCL
    # refuses two ranks, so it uses the host transport over gloo
    comm = None
    if world > 1:
        comm = pkg.Comm.from_torch_gloo(dev.index) if rehearse else pkg.Comm.from_torch(dev.index)

    def em_step():
        if comm is not None:
            mix.optimize_sharded(comm, shard)      # stats -> RCCL all-reduce -> M-step (sdmm_em_step_sharded)
        else:
            mix.optimize(shard)

    for _ in range(args.em_warm):                  # 5 warm EM iterations
        em_step()
    torch.cuda.synchronize()

    resp = torch.empty((max(n_local, full.n if world > 1 else 0), K), dtype=torch.float32, device=dev)

    def estep():
        mix.posterior(shard, resp)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def timed(fn, steps, events=True, ev_stream=None):
        """Wall time of `steps` calls (barrier + synchronize on both sides, max
        over ranks) and, with events, the average device time per call from ONE
        pair of HIP events on the kernels' stream around the whole run (per-call
        event pairs would add their own marker cost to every launch)."""
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if events else None
        es = stream if ev_stream is None else ev_stream
        barrier()
        t = time.perf_counter()
        if events:
            ev[0].record(es)
        for _ in range(steps):
            fn()
        if events:
            ev[1].record(es)
        barrier()
        wall = time.perf_counter() - t
        wall_t = torch.tensor([wall], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(wall_t, op=dist.ReduceOp.MAX)
        kern = None
        if events:
            torch.cuda.synchronize()
            kern = ev[0].elapsed_time(ev[1]) * 1e-3 / steps
        return float(wall_t.item()), kern

    # ---- headline: responsibility E-step --------------------------------
    settle = max(0, args.settle - args.warmup)
    for _ in range(args.warmup + settle):
        estep()
    wall, kern = timed(estep, args.steps)
    ms_per_step = wall / args.steps * 1e3
    value = N_global / (wall / args.steps)
    bytes_per_launch = n_local * (28 + 4 * K)
    flops_per_launch = n_local * K * 66.0
    achieved = bytes_per_launch / kern
    log(f"[bench] E-step: {ms_per_step:.3f} ms/step wall, kernel {kern * 1e6:.1f} us, "
        f"{achieved / 1e12:.2f} TB/s")

    out = {
        "metric": "EM samples/sec (NxK resp) at K=128, N=2^20",
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_launches": settle,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (BASELINE.md 2: 2^20 samples from a K=128 uniformHemisphereInit "
                "generator, LogNormal weights with 0.1% zero / 0.01% non-finite; model after 5 EM steps)",
        "config": {"workload": "responsibility E-step, synthetic 5D sample batch (configs[1])",
                   "K": K, "N": N_global, "global_batch": N_global, "samples_per_gpu": n_local,
                   "parallelism": f"sample-sharded x{world} (strong: N fixed)",
                   "layout": "SoA fp32 in, [N][K] fp32 out"},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK, "traffic": None,
                     "kernel": mix.kernel_name("resp"),
                     "bytes_per_launch": bytes_per_launch, "kernel_us": kern * 1e6,
                     "fp32_frac": flops_per_launch / kern / FP32_PEAK},
    }
    # HBM traffic per launch from the committed rocprofv3 PMC summary of THIS
    # kernel (tools/gpu_pmc.sh + tools/pmc_summary.py), if it matches
    # (the newest round's summary that matches this kernel, K and N)
    for pmc in sorted((ROOT / "profiles").glob("round*_pmc_estep.json"), reverse=True):
        if world != 1:
            break
        try:
            pm = json.loads(pmc.read_text())
            same = pm.get("kernel", "").replace(" ", "") == mix.kernel_name("resp").replace(" ", "")
            if pm.get("K") == K and pm.get("N") == N and same:
                out["roofline"]["traffic"] = pm.get("hbm_bytes_per_launch")
                out["roofline"]["traffic_source"] = f"profiles/{pmc.name}"
                break
        except Exception:
            pass

    if not args.no_extra:
        # ---- full EM step (E-step stats + reduce + [all-reduce] + M-step) ----
        em_wall, _ = timed(em_step, max(5, args.steps // 2), events=False)
        em_steps = max(5, args.steps // 2)
        out["em_step"] = {"samples_per_s": N_global / (em_wall / em_steps),
                          "ms_per_step": em_wall / em_steps * 1e3}
        # ---- weak scaling (extra line): every rank its own full N-sample
        # part of an N x world batch (part 0 = the single-GPU batch) ----
        if world > 1:
            wb = synth.em_batch(N, 128, part=rank)
            wfull = pkg.DeviceSamples.from_numpy(wb["x"], wb["w"], wb["hpdf"], wb["is_diffuse"], device=dev)
            for _ in range(args.warmup):
                mix.posterior(wfull, resp)
            ww, wk = timed(lambda: mix.posterior(wfull, resp), args.steps)
            out["weak"] = {"metric": out["metric"], "samples_per_s": N * world / (ww / args.steps),
                           "ms_per_step": ww / args.steps * 1e3, "kernel_us": wk * 1e6,
                           "N": N * world, "samples_per_gpu": N, "scaling": "weak"}
            del wfull, wb
        # ---- fused stats kernel alone (per rank) ----
        st_wall, st_kern = timed(lambda: mix.estep_stats(shard, stats), args.steps)
        # the fused E-step + statistics is compute-bound: SURVEY 8(d)'s ~113
        # FP32 flops per (sample, component) pair (E-step 66 + rank-1 stats 47)
        out["estep_stats"] = {"ms_per_step": st_wall / args.steps * 1e3,
                              "samples_per_s": N_global / (st_wall / args.steps),
                              "kernel_us": st_kern * 1e6, "flops_per_pair": 113,
                              "fp32_frac": n_local * K * 113.0 / st_kern / FP32_PEAK}
        # ---- guided queries (replicas: each rank serves Q/world queries) ----
        # two query sets against the fitted K = 128 mixture: SURVEY 8(d)'s
        # stated workload (c uniform in [0,1]^3, 3 uniforms, seed 0x6A1D:
        # synth.queries) -- the primary line -- and queries at sample
        # positions, where guiding happens (the round-4 line, harder: the
        # fitted components are live there and the lists are longer)
        q_local = args.Q // world
        gout = ([torch.empty(q_local, device=dev) for _ in range(3)], torch.empty(q_local, device=dev),
                torch.empty(q_local, device=dev, dtype=torch.int32))
        g_steps = max(3, args.steps // 4)

        def guide_line(c, u):
            ct = [torch.from_numpy(c[i].copy()).to(dev) for i in range(3)]
            ut = [torch.from_numpy(u[i].copy()).to(dev) for i in range(3)]
            mix.guide(ct, ut, gout)
            g_wall, g_kern = timed(lambda: mix.guide(ct, ut, gout), g_steps)
            # FP32 fraction of the guided queries, counted from below: the K
            # marginal weights every query forms (3x3 triangular solve, squared
            # norm, scaling: ~22 flops per component; the exp and the kept
            # components' conditional / sample / pdf work not counted)
            return {"queries_per_s": q_local * world / (g_wall / g_steps), "Q": q_local * world,
                    "ms_per_step": g_wall / g_steps * 1e3, "bytes_per_query": 48,
                    "kernel_us": g_kern * 1e6, "flops_per_query_lower_bound": 22 * K,
                    "fp32_frac": q_local * 22.0 * K / g_kern / FP32_PEAK,
                    "hbm_frac": q_local * 48.0 / g_kern / HBM_PEAK,
                    "guided_frac": float((gout[2] >= 0).float().mean())}, ct, ut

        c, u = synth.queries(q_local, seed=synth.SEED_QUERIES + rank)
        out["guide"], _, _ = guide_line(c, u)
        out["guide"]["queries"] = "uniform c in [0,1]^3 (SURVEY 8(d), seed 0x6A1D)"
        c, u = synth.sample_queries_near(batch, q_local, seed=synth.SEED_QUERIES + rank)
        out["guide_near"], ct, ut = guide_line(c, u)
        out["guide_near"]["queries"] = "c at sample positions of the batch"
        # ---- batched per-leaf EM: the plugin's tree leaves,
        # each its own K=16 mixture over its own samples (volpath_sdmm.cpp:287-311);
        # leaves shard across ranks with no exchange (weak scaling per rank) ----
        out["leaf_em"] = leaf_em_bench(pkg, synth, full, N, dev, stream, args, timed, world, rank, comm)
        # ---- spatial tree (jmm SNTree restatement) as the built plugin sets it
        # up: split_to_depth(2) (sdmm/volpath_sdmm.cpp:398), then the splitting
        # block of optimize() -- split_leaf_recurse(i, 4000) over the nodes while
        # leaf_nodes() <= 2048 (:253-260, :528-529); device find over the batch
        # positions (STree.find, sdmm_proc.cpp:314) and the leaf routing ----
        tree = pkg.STree(np.float32([0, 0, 0]), np.float32([1, 1, 1]), device=dev.index)
        tree.split_to_depth(2)
        tree.split_leaves(batch["x"][0:3], 4000, 2048)
        node_ids = torch.empty(n_local, dtype=torch.int32, device=dev)
        pts = shard.x[0:3]
        tree.find(pts, node_ids)
        torch.cuda.synchronize()
        f_steps = max(5, args.steps)
        f_wall, _ = timed(lambda: (tree.find(pts, node_ids), torch.cuda.synchronize()), f_steps, events=False)
        r_wall, _ = timed(lambda: tree.route(shard), max(3, args.steps // 4), events=False)
        out["stree"] = {"nodes": tree.num_nodes, "leaves": tree.leaf_nodes,
                        "find_queries_per_s": n_local * world / (f_wall / f_steps),
                        "find_ms": f_wall / f_steps * 1e3,
                        "route_ms": r_wall / max(3, args.steps // 4) * 1e3,
                        "route_samples_per_s": n_local * world / (r_wall / max(3, args.steps // 4))}
        # ---- guided wavefront over the tree's leaves:
        # sampleSurface for Q bounces -- find the leaf, guide against its own
        # K=16 mixture (fitted by 2 batched EM steps on the routed samples) --
        # one sdmm_guide_wavefront call (replicas: Q/world queries per rank) ----
        out["guide_wavefront"] = wavefront_bench(pkg, synth, batch, shard, tree, dev, stream, ct, ut, gout,
                                                 timed, args, world)

    if not args.no_extra:
        cpu = rank == 0 and world == 1 and not args.no_cpu
        out["cornell"] = cornell_bench(pkg, dev, args, world, cpu=cpu)
        out["cornell_async"] = cornell_bench(pkg, dev, args, world, optimize_async=1)
        # configs[2]'s K (Torus, K=128 guided path tracing with Li/sampleSurface
        # on the device): the Torus meshes are LFS pointers in the snapshot, so
        # the same guided renderer runs over the Cornell Box with K=128 leaves
        out["cornell_k128"] = cornell_bench(pkg, dev, args, world, K=128, cpu=cpu)
        # ... with the reference's default optimizeAsync = true
        # (volpath_sdmm.cpp:65, :446-507): a training pass's EM runs beside
        # the next pass's render, which guides with the model it has
        out["cornell_k128_async"] = cornell_bench(pkg, dev, args, world, K=128, optimize_async=1)
        # sampleProduct (configs[4]'s learned-BSDF product sampling, sdmm_proc.cpp:327-392)
        # inside the full guided render: the Cornell BSDFs' synthesised diffuse lobes
        out["cornell_product"] = cornell_bench(pkg, dev, args, world, product=True, cpu=cpu)

    if not args.no_extra and not args.no_large_k:
        out["large_k"] = large_k_bench(pkg, synth, batch, shard, dev, stream, timed, args, world, N_global, comm)
        # configs[4] as a full guided render: K=512 leaves (the Kitchen's K) with
        # sampleProduct, over the Cornell Box (the Kitchen meshes are LFS
        # pointers; the device Li's BSDFs are diffuse, so the learned lobes are
        # the diffuse slice rule's).  CPU baseline on a bounded pixel slice (a
        # 16-pixel probe sizes a ~10 s sample: the CPU Li at K=512 x product is
        # slow per path)
        cpu = rank == 0 and world == 1 and not args.no_cpu
        out["cornell_k512_product"] = cornell_bench(pkg, dev, args, world, K=512, product=True, cpu=cpu,
                                                    cpu_probe_px=16, cpu_budget_s=10.0)
        # ... and with the Kitchen's glossy materials' branch: the tall box and
        # the floor rough conductors, whose per-bounce learned lobes take
        # rotate_to_wo + the shading frame into the product (sdmm_proc.cpp:340-355)
        out["cornell_k512_glossy_product"] = cornell_bench(pkg, dev, args, world, K=512, product=True, cpu=cpu,
                                                           cpu_probe_px=16, cpu_budget_s=10.0,
                                                           glossy=("TallBox", "Floor"))

    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(batch, K, pos, nrm, synth, min(args.cpu_sample, N),
                                               args.cpu_threads or host_threads())
        except Exception as e:  # the baseline is reported, never required
            out["cpu_baseline"] = {"value": None, "error": repr(e)}

    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
