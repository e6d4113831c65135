"""sdmm-mitsuba_amd -- MI355X-native SDMM path-guiding hot path.

Python binding (ctypes) of the C ABI in include/sdmm_gpu.h, used by the tests
and bench.py.  It mirrors the reference's jmm interface names (MixtureModel /
StepwiseTangentEM::optimize / posteriorAndLog / conditional+sample+pdf):

    mix = SDMM(K=128)                       # jmm::MixtureModel + StepwiseTangentEM
    mix.init_hemisphere(pos, nrm, ...)      # uniformHemisphereInit
    mix.optimize(samples)                   # StepwiseTangentEM::optimize (one EM step)
    mix.posterior(samples, out)             # posteriorAndLog over a batch
    d, pdf, comp = mix.guide(c, u)          # conditional + sample + pdf per query

Device buffers are torch tensors on the HIP device (torch is only the memory
and stream plumbing).  There is no CPU fallback: if lib/libsdmm_amd.so is
missing or the device is absent, every call fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
# SDMM_LIB_PATH: an A/B variant of the library (tools/build_variant.sh)
LIB_PATH = Path(os.environ.get("SDMM_LIB_PATH", PKG_DIR / "lib" / "libsdmm_amd.so"))
REPO = PKG_DIR.parent


class SDMMError(RuntimeError):
    pass


_lib = None


def build(arch: str = "gfx950", jobs: int = 4) -> Path:
    import subprocess
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", str(PKG_DIR), f"ARCH={arch}"], check=True)
    return LIB_PATH


# host-transport callbacks of sdmm_comm_init_host (include/sdmm_gpu.h)
_HOST_ALLREDUCE = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_size_t, C.c_void_p)
_HOST_BCAST = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p)


class _Samples(C.Structure):
    _fields_ = [("x", C.c_void_p * 6), ("w", C.c_void_p), ("hpdf", C.c_void_p),
                ("is_diffuse", C.c_void_p), ("n", C.c_int64)]


class _EmParams(C.Structure):
    _fields_ = [("alpha", C.c_float), ("bprior", C.c_float * 5), ("ni_prior_minus_one", C.c_float),
                ("epsilon", C.c_double), ("decrease_prior", C.c_int)]


PARAM_FIELDS = [("weights", 1), ("cdf", 1), ("mean", 6), ("cov", 25), ("to", 9), ("cholL", 25),
                ("cholLInv", 25), ("detInv", 1), ("muPremult", 6), ("condCov", 4), ("margL", 9),
                ("margDetInv", 1), ("condL", 4), ("condLInv", 4), ("condDetInv", 1)]


class _ParamsOut(C.Structure):
    _fields_ = [(n, C.c_void_p) for n, _ in PARAM_FIELDS] + [("valid", C.c_void_p),
                                                              ("normalization", C.c_void_p)]


def lib():
    """Load lib/libsdmm_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise SDMMError(f"{LIB_PATH} not found: run `make -C {PKG_DIR}` (or __graft_entry__.build())")
        # torch (the memory/stream plumbing) and this library share one HIP
        # runtime (same SONAME); let torch initialise it before our code object
        # registers, otherwise torch's later device discovery fails.
        try:
            import torch
            torch.cuda.is_available()
        except ImportError:
            pass
        L = C.CDLL(str(LIB_PATH))
        L.sdmm_last_error.restype = C.c_char_p
        L.sdmm_stats_len.restype = C.c_size_t
        L.sdmm_stats_len.argtypes = [C.c_int]
        L.sdmm_get_stream.restype = C.c_void_p
        L.sdmm_get_stream.argtypes = [C.c_void_p]
        L.sdmm_create.argtypes = [C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
        L.sdmm_destroy.argtypes = [C.c_void_p]
        L.sdmm_layout.argtypes = [C.c_void_p] + [C.POINTER(C.c_int)] * 4
        L.sdmm_kernel_name.argtypes = [C.c_void_p, C.c_int]
        L.sdmm_kernel_name.restype = C.c_char_p
        L.sdmm_set_guide_capacity.argtypes = [C.c_void_p, C.c_int]
        L.sdmm_guide_fallback_count.argtypes = [C.c_void_p, C.c_void_p]
        L.sdmm_set_stream.argtypes = [C.c_void_p, C.c_void_p]
        L.sdmm_synchronize.argtypes = [C.c_void_p]
        L.sdmm_init_hemisphere.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_float,
                                           C.c_float, C.c_uint64]
        L.sdmm_init_hemisphere_batched.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_float,
                                                   C.c_void_p, C.c_void_p]
        L.sdmm_hemisphere_init_host.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_float, C.c_float,
                                                C.c_uint64] + [C.c_void_p] * 5
        L.sdmm_em_step.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.sdmm_em_step_host.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.sdmm_estep_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.sdmm_mstep.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.sdmm_responsibilities.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.sdmm_guide_batch.argtypes = [C.c_void_p, C.c_int64, C.c_void_p * 3, C.c_void_p * 3,
                                       C.c_void_p * 3, C.c_void_p, C.c_void_p]
        L.sdmm_pdf_batch.argtypes = [C.c_void_p, C.c_int64, C.c_void_p * 3, C.c_void_p * 3, C.c_void_p]
        L.sdmm_sample_discrete_cdf.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int64,
                                               C.c_void_p]
        L.sdmm_get_params.argtypes = [C.c_void_p, C.c_void_p]
        L.sdmm_set_params.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.sdmm_get_state.argtypes = [C.c_void_p] + [C.c_void_p] * 7
        L.sdmm_set_state.argtypes = [C.c_void_p] + [C.c_void_p] * 7
        L.sdmm_em_params_default.argtypes = [C.c_void_p]
        L.sdmm_stree_set_stream.argtypes = [C.c_void_p, C.c_void_p]
        L.sdmm_stree_get_stream.restype = C.c_void_p
        L.sdmm_stree_get_stream.argtypes = [C.c_void_p]
        L.sdmm_guide_wavefront.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p * 3, C.c_void_p * 3,
                                           C.c_void_p * 3, C.c_void_p, C.c_void_p, C.c_void_p]
        L.sdmm_guide_product_batch.argtypes = [C.c_void_p, C.c_int64, C.c_void_p * 3, C.c_void_p * 3, C.c_void_p,
                                               C.c_void_p, C.c_void_p * 9, C.c_void_p * 3, C.c_void_p, C.c_void_p,
                                               C.c_void_p]
        L.sdmm_pdf_product_batch.argtypes = [C.c_void_p, C.c_int64, C.c_void_p * 3, C.c_void_p * 3, C.c_void_p,
                                             C.c_void_p, C.c_void_p * 9, C.c_void_p, C.c_void_p]
        L.sdmm_stree_bind_mixtures.argtypes = [C.c_void_p, C.c_void_p]
        L.sdmm_pdf_wavefront.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p * 3, C.c_void_p * 3,
                                         C.c_void_p]
        L.sdmm_save_json.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p]
        L.sdmm_load_json.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        L.sdmm_mix_save_json.argtypes = [C.c_void_p, C.c_char_p]
        L.sdmm_mix_load_json.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]
        L.sdmm_get_em_params.argtypes = [C.c_void_p, C.c_void_p]
        L.sdmm_restore_params.argtypes = [C.c_void_p, C.c_void_p]
        L.sdmm_stree_set_nodes.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.sdmm_comm_unique_id.argtypes = [C.c_void_p]
        L.sdmm_comm_init_rccl.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        L.sdmm_comm_init_host.argtypes = [C.c_int, C.c_int, C.c_int, _HOST_ALLREDUCE, _HOST_BCAST, C.c_void_p,
                                          C.POINTER(C.c_void_p)]
        L.sdmm_comm_destroy.argtypes = [C.c_void_p]
        L.sdmm_comm_rank.argtypes = [C.c_void_p]
        L.sdmm_comm_size.argtypes = [C.c_void_p]
        L.sdmm_comm_allreduce_f64.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.sdmm_em_step_sharded.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.sdmm_em_step_batched_sharded.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                                   C.c_void_p]
        L.sdmm_em_step_batched_iters.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.sdmm_mix_broadcast.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.sdmm_stree_leaf_nodes.argtypes = [C.c_void_p]
        L.sdmm_stree_split_leaf_recurse.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_int]
        L.sdmm_stree_split_leaves.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int]
        L.sdmm_guide_pdf_wavefront.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p * 3, C.c_void_p * 3,
                                               C.c_void_p * 3, C.c_void_p, C.c_void_p * 3, C.c_void_p, C.c_void_p,
                                               C.c_void_p]
        L.sdmm_clone.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
        L.sdmm_guiding_config_default.argtypes = [C.c_void_p]
        L.sdmm_guiding_create.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
        L.sdmm_guiding_destroy.argtypes = [C.c_void_p]
        L.sdmm_guiding_tree.argtypes = [C.c_void_p]
        L.sdmm_guiding_tree.restype = C.c_void_p
        L.sdmm_guiding_node_mixtures.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.sdmm_guiding_trained.argtypes = [C.c_void_p]
        L.sdmm_guiding_push.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.sdmm_guiding_optimize.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.sdmm_guiding_update.argtypes = [C.c_void_p]
        L.sdmm_guiding_iteration.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p,
                                             C.c_void_p, C.c_void_p, C.c_void_p]
        L.sdmm_scene_create.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
        L.sdmm_scene_destroy.argtypes = [C.c_void_p]
        L.sdmm_scene_normalization.argtypes = [C.c_void_p] + [C.c_void_p] * 4
        L.sdmm_li_render.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p]
        L.sdmm_write_exr.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_float]
        L.sdmm_push_training.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_uint64, C.c_void_p,
                                         C.POINTER(C.c_int64), C.c_void_p, C.POINTER(C.c_int64)]
        L.sdmm_kmeanspp_select.argtypes = [C.c_void_p, C.c_void_p * 3, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                           C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.sdmm_init_hemisphere_kmeanspp_batched.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p * 3,
                                                            C.c_void_p, C.c_float, C.c_void_p, C.c_void_p]
        L.sdmm_learned4_conditional.argtypes = [C.c_void_p, C.c_float, C.c_void_p, C.c_int, C.POINTER(C.c_int),
                                                C.c_void_p, C.c_void_p, C.c_void_p]
        L.sdmm_learned4_save_json.argtypes = [C.c_void_p, C.c_char_p]
        L.sdmm_learned4_conditional_device.argtypes = [C.c_void_p, C.c_float, C.c_int64, C.c_void_p * 3, C.c_int,
                                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.sdmm_learned4_load_json.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_int), C.c_void_p, C.c_void_p,
                                              C.c_void_p]
        L.sdmm_stree_publish.argtypes = [C.c_void_p, C.c_void_p]
        L.sdmm_guide_ctx_create.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]
        L.sdmm_guide_ctx_destroy.argtypes = [C.c_void_p]
        L.sdmm_guide_ctx_destroy.restype = None
        L.sdmm_guide_ctx_stream.argtypes = [C.c_void_p]
        L.sdmm_guide_ctx_stream.restype = C.c_void_p
        L.sdmm_ctx_guide_pdf_wavefront.argtypes = [C.c_void_p, C.c_int64, C.c_void_p * 3, C.c_void_p * 3,
                                                   C.c_void_p * 3, C.c_void_p, C.c_void_p * 3, C.c_void_p,
                                                   C.c_void_p, C.c_void_p]
        L.sdmm_ctx_guide_product_wavefront.argtypes = [C.c_void_p, C.c_int64, C.c_void_p * 3, C.c_void_p * 3,
                                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                       C.c_void_p * 9, C.c_void_p * 3, C.c_void_p, C.c_void_p,
                                                       C.c_void_p, C.c_void_p]
        L.sdmm_ctx_guide_pdf_host_batch.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        _lib = L
    return _lib


class _GuideHostReq(C.Structure):
    """sdmm_guide_host_req (include/sdmm_gpu.h)."""
    _fields_ = [("n", C.c_int64), ("inp", C.c_void_p), ("in_stride", C.c_int64), ("mode", C.c_void_p),
                ("out", C.c_void_p), ("out_stride", C.c_int64), ("comp", C.c_void_p)]


def _check(rc: int):
    if rc != 0:
        raise SDMMError(f"sdmm error {rc}: {lib().sdmm_last_error().decode()}")


def stats_len(K: int) -> int:
    return 2 + 21 * K


EXPORTED_SYMBOLS = [
    "sdmm_release_cached_scratch",
    "sdmm_em_params_default", "sdmm_create", "sdmm_destroy", "sdmm_num_components", "sdmm_layout",
    "sdmm_kernel_name",
    "sdmm_set_guide_capacity", "sdmm_set_guide_order", "sdmm_guide_fallback_count",
    "sdmm_set_stream", "sdmm_get_stream", "sdmm_synchronize", "sdmm_init_hemisphere",
    "sdmm_hemisphere_init_host", "sdmm_em_step", "sdmm_em_step_host", "sdmm_em_step_batched",
    "sdmm_em_step_batched_host",
    "sdmm_stats_len",
    "sdmm_estep_stats", "sdmm_mstep", "sdmm_responsibilities", "sdmm_guide_batch", "sdmm_pdf_batch",
    "sdmm_sample_discrete_cdf", "sdmm_get_params", "sdmm_set_params", "sdmm_get_state",
    "sdmm_set_state", "sdmm_last_error", "sdmm_abi_version",
    "sdmm_stree_create", "sdmm_stree_destroy", "sdmm_stree_split_to_depth", "sdmm_stree_split",
    "sdmm_stree_num_nodes", "sdmm_stree_get_nodes", "sdmm_stree_find", "sdmm_stree_route",
    "sdmm_stree_set_stream", "sdmm_stree_get_stream", "sdmm_guide_wavefront", "sdmm_pdf_wavefront",
    "sdmm_stree_bind_mixtures", "sdmm_guide_product_batch", "sdmm_pdf_product_batch",
    "sdmm_save_json", "sdmm_load_json", "sdmm_mix_save_json", "sdmm_mix_load_json", "sdmm_get_em_params",
    "sdmm_restore_params", "sdmm_stree_set_nodes",
    "sdmm_comm_unique_id", "sdmm_comm_init_rccl", "sdmm_comm_init_host", "sdmm_comm_destroy", "sdmm_comm_rank",
    "sdmm_comm_size", "sdmm_comm_allreduce_f64", "sdmm_em_step_sharded", "sdmm_em_step_batched_sharded",
    "sdmm_em_step_batched_iters", "sdmm_mix_broadcast",
    "sdmm_stree_leaf_nodes", "sdmm_stree_split_leaf_recurse", "sdmm_stree_split_leaves",
    "sdmm_guide_pdf_wavefront", "sdmm_scene_create", "sdmm_scene_destroy", "sdmm_scene_normalization",
    "sdmm_li_render", "sdmm_push_training", "sdmm_clone",
    "sdmm_guiding_config_default", "sdmm_guiding_create", "sdmm_guiding_destroy", "sdmm_guiding_tree",
    "sdmm_guiding_node_mixtures", "sdmm_guiding_trained", "sdmm_guiding_push", "sdmm_guiding_optimize",
    "sdmm_guiding_iteration", "sdmm_create_on_stream", "sdmm_create_many_on_stream", "sdmm_clone_many",
    "sdmm_init_hemisphere_batched", "sdmm_iterations_run", "sdmm_stree_split_leaf_recurse_many",
    "sdmm_em_step_batched_host_iters", "sdmm_write_exr", "sdmm_clone_many_on_stream", "sdmm_copy_many",
    "sdmm_guiding_update", "sdmm_kmeanspp_select", "sdmm_init_hemisphere_kmeanspp_batched",
    "sdmm_guide_product_wavefront", "sdmm_pdf_product_wavefront", "sdmm_stree_split_leaf_recurse_device",
    "sdmm_stree_publish", "sdmm_guide_ctx_create", "sdmm_guide_ctx_destroy", "sdmm_guide_ctx_stream",
    "sdmm_ctx_guide_pdf_wavefront", "sdmm_ctx_guide_product_wavefront", "sdmm_ctx_guide_pdf_host_batch",
    "sdmm_pinned_alloc", "sdmm_pinned_free",
    "sdmm_learned4_conditional", "sdmm_learned4_save_json", "sdmm_learned4_load_json",
    "sdmm_learned4_conditional_device",
]


def em_step_batched(mixes, samples, seg, iterations: int = 1):
    """Per-leaf EM of the plugin's optimisation loop (volpath_sdmm.cpp:287-311)
    as one batched launch: mixes[i] takes `iterations` EM steps over samples
    [seg[i], seg[i+1]) of `samples` (a DeviceSamples with the leaves stored
    back to back).  Bitwise the same as mixes[i].optimize(leaf i) one by one.
    Runs on mixes[0]'s stream."""
    seg = np.ascontiguousarray(seg, np.int64)
    n = len(mixes)
    assert seg.shape == (n + 1,), "seg needs len(mixes) + 1 offsets"
    hs = (C.c_void_p * max(n, 1))(*[m.h for m in mixes])
    _check(lib().sdmm_em_step_batched(hs, n, samples.ptr, seg.ctypes.data_as(C.POINTER(C.c_int64)),
                                      iterations))


def kmeanspp_select(samples, normals, seg, n_pos, uniforms, stream=None):
    """kMeansPPInit (mixture_model_init.h:244-330) for the leaves [seg[l],
    seg[l+1]) of `samples` (positions x[0..2], weights w) with device normal
    planes `normals`: (indices (n_leaves, n_pos) leaf-relative, positions
    (n_leaves, n_pos, 3), normals (n_leaves, n_pos, 3))."""
    import torch
    seg = np.ascontiguousarray(seg, np.int64)
    nl = seg.size - 1
    u = np.ascontiguousarray(uniforms, np.float32).reshape(-1)
    assert u.size == nl * n_pos
    nt = [t.contiguous() for t in normals]
    idx = np.zeros((nl, n_pos), np.int64)
    pos = np.zeros((nl, n_pos, 3), np.float32)
    nrm = np.zeros((nl, n_pos, 3), np.float32)
    dev = samples.w.device.index or 0
    st = stream if stream is not None else torch.cuda.current_stream(samples.w.device).cuda_stream
    _check(lib().sdmm_kmeanspp_select(samples.ptr, (C.c_void_p * 3)(*[t.data_ptr() for t in nt]), seg.ctypes.data,
                                      nl, n_pos, u.ctypes.data, dev, st, idx.ctypes.data, pos.ctypes.data,
                                      nrm.ctypes.data))
    return idx, pos, nrm


def init_hemisphere_batched(mixes, positions, normals, depth_prior, min_spatial_distance, seeds):
    """uniformHemisphereInit for many mixtures of one K (the guiding model's
    new leaves): mixture i from positions / normals [i] (K/8 x 3 each), its
    spatial distance and seed; the staging block is generated on the device."""
    n = len(mixes)
    K = mixes[0].K if n else 0
    pos = np.ascontiguousarray(positions, np.float32).reshape(n, K // 8, 3)
    nrm = np.ascontiguousarray(normals, np.float32).reshape(n, K // 8, 3)
    dist = np.ascontiguousarray(np.broadcast_to(np.asarray(min_spatial_distance, np.float32), (n,)))
    sd = np.ascontiguousarray(np.broadcast_to(np.asarray(seeds, np.uint64), (n,)))
    hs = (C.c_void_p * max(n, 1))(*[m.h for m in mixes])
    _check(lib().sdmm_init_hemisphere_batched(hs, n, pos.ctypes.data, nrm.ctypes.data, depth_prior,
                                              dist.ctypes.data, sd.ctypes.data))


def init_hemisphere_kmeanspp_batched(mixes, samples, normals, seg, depth_prior, min_spatial_distance, seeds):
    """uniformHemisphereInit with kMeansPlusPlus (mixture_model_init.h:130-138)
    for many mixtures of one K: mixture i over samples [seg[i], seg[i+1])."""
    seg = np.ascontiguousarray(seg, np.int64)
    n = len(mixes)
    assert seg.shape == (n + 1,)
    dist = np.ascontiguousarray(np.broadcast_to(np.asarray(min_spatial_distance, np.float32), (n,)))
    sd = np.ascontiguousarray(np.broadcast_to(np.asarray(seeds, np.uint64), (n,)))
    nt = [t.contiguous() for t in normals]
    hs = (C.c_void_p * max(n, 1))(*[m.h for m in mixes])
    _check(lib().sdmm_init_hemisphere_kmeanspp_batched(hs, n, samples.ptr, (C.c_void_p * 3)(*[t.data_ptr() for t in nt]),
                                                       seg.ctypes.data, depth_prior, dist.ctypes.data, sd.ctypes.data))


def _iters(n, iterations):
    it = np.full(n, iterations, np.int32) if np.isscalar(iterations) else np.ascontiguousarray(iterations, np.int32)
    assert it.shape == (n,), "one iteration count per mixture"
    return it


def em_step_batched_iters(mixes, samples, seg, iterations):
    """Batched per-leaf EM with per-leaf iteration counts (the plugin's 2 while
    em.iterations_run < 4, else 1; volpath_sdmm.cpp:299-305)."""
    seg = np.ascontiguousarray(seg, np.int64)
    n = len(mixes)
    it = _iters(n, iterations)
    hs = (C.c_void_p * max(n, 1))(*[m.h for m in mixes])
    _check(lib().sdmm_em_step_batched_iters(hs, n, samples.ptr, seg.ctypes.data, it.ctypes.data))


def em_step_batched_sharded(mixes, comm, samples, seg, iterations=1):
    """Per-leaf EM sample-sharded over the ranks of `comm`: this rank's samples
    of every leaf; one all-reduce of all leaves' statistics per round."""
    seg = np.ascontiguousarray(seg, np.int64)
    n = len(mixes)
    it = _iters(n, iterations)
    hs = (C.c_void_p * max(n, 1))(*[m.h for m in mixes])
    _check(lib().sdmm_em_step_batched_sharded(hs, n, comm.h, samples.ptr, seg.ctypes.data, it.ctypes.data))


def mix_broadcast(mixes, owner, comm):
    """Leaf-sharded EM: every mixture's parameters and EM state from its owner rank."""
    n = len(mixes)
    own = np.ascontiguousarray(owner, np.int32)
    assert own.shape == (n,)
    hs = (C.c_void_p * max(n, 1))(*[m.h for m in mixes])
    _check(lib().sdmm_mix_broadcast(hs, n, own.ctypes.data, comm.h))


class Comm:
    """A multi-GPU communicator (sdmm_comm).  Comm.rccl: RCCL over xGMI, one
    rank per GPU; Comm.host: the caller's own collective on host buffers (any
    backend -- e.g. torch.distributed gloo via Comm.from_torch_gloo)."""

    ID_BYTES = 128

    def __init__(self, h, keep=()):
        self.h = h
        self._keep = keep          # the host callbacks must outlive the communicator

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(Comm.ID_BYTES)
        _check(lib().sdmm_comm_unique_id(buf))
        return buf.raw

    @classmethod
    def rccl(cls, uid: bytes, nranks: int, rank: int, device: int = 0) -> "Comm":
        assert len(uid) == Comm.ID_BYTES
        h = C.c_void_p()
        _check(lib().sdmm_comm_init_rccl(C.create_string_buffer(uid, Comm.ID_BYTES), nranks, rank, device,
                                         C.byref(h)))
        return cls(h)

    @classmethod
    def from_torch(cls, device: int = 0, group=None) -> "Comm":
        """RCCL communicator over the ranks of a torch.distributed group (the
        unique id travels through it)."""
        import torch
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = Comm.unique_id() if rank == 0 else bytes(Comm.ID_BYTES)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        if dist.get_backend(group) == "nccl":
            t = t.to(torch.device("cuda", device))
        dist.broadcast(t, 0, group=group)
        return cls.rccl(bytes(t.cpu().tolist()), world, rank, device)

    @classmethod
    def host(cls, nranks: int, rank: int, allreduce, broadcast, device: int = 0) -> "Comm":
        """allreduce(np.ndarray float64) and broadcast(np.ndarray uint8, root)
        operate in place on host arrays."""
        def ar(ptr, count, _):
            try:
                allreduce(np.ctypeslib.as_array(ptr, shape=(count,)))
                return 0
            except Exception:
                return 1

        def bc(ptr, nbytes, root, _):
            try:
                broadcast(np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(nbytes,)), root)
                return 0
            except Exception:
                return 1
        fa, fb = _HOST_ALLREDUCE(ar), _HOST_BCAST(bc)
        h = C.c_void_p()
        _check(lib().sdmm_comm_init_host(nranks, rank, device, fa, fb, None, C.byref(h)))
        return cls(h, keep=(fa, fb))

    @classmethod
    def from_torch_gloo(cls, device: int = 0, group=None) -> "Comm":
        """Host transport over a torch.distributed CPU (gloo) group."""
        import torch
        import torch.distributed as dist

        def allreduce(a):
            dist.all_reduce(torch.from_numpy(a), group=group)

        def broadcast(a, root):
            dist.broadcast(torch.from_numpy(a), root, group=group)
        return cls.host(dist.get_world_size(group), dist.get_rank(group), allreduce, broadcast, device)

    @property
    def rank(self) -> int:
        return int(lib().sdmm_comm_rank(self.h))

    @property
    def size(self) -> int:
        return int(lib().sdmm_comm_size(self.h))

    def allreduce_f64(self, t, stream=None):
        """In-place SUM over ranks of a float64 device tensor."""
        import torch
        assert t.dtype == torch.float64 and t.is_cuda
        st = stream if stream is not None else torch.cuda.current_stream(t.device)
        _check(lib().sdmm_comm_allreduce_f64(self.h, t.data_ptr(), t.numel(),
                                             C.c_void_p(getattr(st, "cuda_stream", st) or 0)))

    def close(self):
        if getattr(self, "h", None):
            lib().sdmm_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """[a, b) of the contiguous sample shard owned by `rank` of `world`."""
    per = (n + world - 1) // world
    return min(n, rank * per), min(n, (rank + 1) * per)


def hemisphere_init_host(positions, normals, depth_prior, min_dist, seed):
    """uniformHemisphereInit on the host (no device needed): initial params."""
    pos = np.ascontiguousarray(positions, np.float32).reshape(-1, 3)
    nrm = np.ascontiguousarray(normals, np.float32).reshape(-1, 3)
    n_pos = pos.shape[0]
    K = 8 * n_pos
    out = {"weights": np.zeros(K, np.float32), "mean": np.zeros((K, 6), np.float32),
           "cov": np.zeros((K, 5, 5), np.float32), "bpriors": np.zeros((K, 5, 5), np.float32),
           "bdepth": np.zeros((K, 3, 3), np.float32)}
    _check(lib().sdmm_hemisphere_init_host(pos.ctypes.data, nrm.ctypes.data, n_pos, depth_prior,
                                           min_dist, seed, out["weights"].ctypes.data,
                                           out["mean"].ctypes.data, out["cov"].ctypes.data,
                                           out["bpriors"].ctypes.data, out["bdepth"].ctypes.data))
    return out


class DeviceSamples:
    """SoA sample planes resident in HBM (torch tensors on the HIP device)."""

    def __init__(self, x, w, hpdf=None, is_diffuse=None):
        import torch
        self.x = [t.contiguous() for t in x]
        self.w = w.contiguous()
        self.hpdf = None if hpdf is None else hpdf.contiguous()
        self.is_diffuse = None if is_diffuse is None else is_diffuse.to(torch.uint8).contiguous()
        assert len(self.x) == 6
        for t in self.x + [self.w]:
            assert t.dtype == torch.float32 and t.is_cuda, "sample planes must be fp32 device tensors"
        self.n = int(self.w.numel())
        self.s = _Samples()
        for i in range(6):
            self.s.x[i] = self.x[i].data_ptr()
        self.s.w = self.w.data_ptr()
        self.s.hpdf = self.hpdf.data_ptr() if self.hpdf is not None else None
        self.s.is_diffuse = self.is_diffuse.data_ptr() if self.is_diffuse is not None else None
        self.s.n = self.n

    @classmethod
    def from_numpy(cls, x, w, hpdf=None, is_diffuse=None, device="cuda"):
        import torch
        xt = [torch.from_numpy(np.ascontiguousarray(x[i], np.float32)).to(device) for i in range(6)]
        wt = torch.from_numpy(np.ascontiguousarray(w, np.float32)).to(device)
        ht = None if hpdf is None else torch.from_numpy(np.ascontiguousarray(hpdf, np.float32)).to(device)
        dt = None if is_diffuse is None else torch.from_numpy(np.ascontiguousarray(is_diffuse, np.uint8)).to(device)
        return cls(xt, wt, ht, dt)

    def shard(self, rank: int, world: int) -> "DeviceSamples":
        """Contiguous sample range of `rank` (SURVEY 8e partitioning)."""
        a, b = shard_range(self.n, rank, world)
        sl = lambda t: None if t is None else t[a:b]
        return DeviceSamples([t[a:b] for t in self.x], self.w[a:b], sl(self.hpdf), sl(self.is_diffuse))

    @property
    def ptr(self):
        return C.byref(self.s)


class SDMM:
    """One K-component SDMM + its stepwise EM state, resident on one GPU."""

    def __init__(self, K: int, device: int = 0, alpha=0.9, bprior=1e-5, ni_prior_minus_one=6e-5,
                 epsilon=1e-100, decrease_prior=True, stream=None):
        self.K = K
        p = _EmParams()
        p.alpha = alpha
        for i in range(5):
            p.bprior[i] = bprior
        p.ni_prior_minus_one = ni_prior_minus_one
        p.epsilon = epsilon
        p.decrease_prior = int(decrease_prior)
        h = C.c_void_p()
        _check(lib().sdmm_create(K, C.byref(p), device, C.byref(h)))
        self.h = h
        # Enqueue on the caller's stream so work is ordered with the torch ops
        # that allocate, fill and read the buffers (default: torch's current
        # stream; the C ABI's own default is a private non-blocking stream).
        if stream is None:
            import torch
            if torch.cuda.is_available():
                self.set_stream(torch.cuda.current_stream())
        else:
            self.set_stream(stream)

    def close(self):
        if getattr(self, "h", None):
            if getattr(self, "_owned", True):
                lib().sdmm_destroy(self.h)
            self.h = None

    @classmethod
    def _borrow(cls, h, owner) -> "SDMM":
        """A non-owning view of a handle that `owner` keeps alive (its stream untouched)."""
        self = cls.__new__(cls)
        self.h = C.c_void_p(h)
        self._owned = False
        self._owner = owner
        self.K = int(lib().sdmm_num_components(self.h))
        return self

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- streams ---------------------------------------------------------
    def set_stream(self, stream):
        """stream: a torch.cuda.Stream, a raw hipStream_t int, or None."""
        ptr = getattr(stream, "cuda_stream", stream)
        _check(lib().sdmm_set_stream(self.h, C.c_void_p(ptr or 0)))

    @property
    def stream_ptr(self) -> int:
        return lib().sdmm_get_stream(self.h) or 0

    def synchronize(self):
        _check(lib().sdmm_synchronize(self.h))

    # ---- init / params ---------------------------------------------------
    def init_hemisphere(self, positions, normals, depth_prior, min_spatial_distance, seed):
        pos = np.ascontiguousarray(positions, np.float32).reshape(-1, 3)
        nrm = np.ascontiguousarray(normals, np.float32).reshape(-1, 3)
        _check(lib().sdmm_init_hemisphere(self.h, pos.ctypes.data, nrm.ctypes.data, pos.shape[0],
                                          depth_prior, min_spatial_distance, seed))

    def set_params(self, weights, means, covs):
        w = np.ascontiguousarray(weights, np.float32)
        m = np.ascontiguousarray(means, np.float32)
        c = np.ascontiguousarray(covs, np.float32)
        _check(lib().sdmm_set_params(self.h, w.ctypes.data, m.ctypes.data, c.ctypes.data))

    def get_params(self) -> dict:
        K = self.K
        arrs = {n: np.zeros(K * w, np.float32) for n, w in PARAM_FIELDS}
        valid = np.zeros(K, np.int32)
        norm = np.zeros(1, np.float32)
        o = _ParamsOut()
        for n, _ in PARAM_FIELDS:
            setattr(o, n, arrs[n].ctypes.data)
        o.valid = valid.ctypes.data
        o.normalization = norm.ctypes.data
        _check(lib().sdmm_get_params(self.h, C.byref(o)))
        out = {n: (a if w == 1 else a.reshape(K, w)) for (n, w), a in zip(PARAM_FIELDS, arrs.values())}
        out["valid"] = valid
        out["normalization"] = float(norm[0])
        return out

    def get_state(self) -> dict:
        K = self.K
        st = {"scalars": np.zeros(9), "T": np.zeros(K), "sgW": np.zeros(K), "sgM": np.zeros(5 * K),
              "sgC": np.zeros(25 * K), "bpriors": np.zeros(25 * K, np.float32),
              "bdepth": np.zeros(9 * K, np.float32)}
        _check(lib().sdmm_get_state(self.h, *[st[k].ctypes.data for k in
                                              ("scalars", "T", "sgW", "sgM", "sgC", "bpriors", "bdepth")]))
        return st

    def set_state(self, st: dict):
        keys = ("scalars", "T", "sgW", "sgM", "sgC", "bpriors", "bdepth")
        arrs = []
        for k in keys:
            dt = np.float32 if k in ("bpriors", "bdepth") else np.float64
            arrs.append(np.ascontiguousarray(st[k], dt))
        _check(lib().sdmm_set_state(self.h, *[a.ctypes.data for a in arrs]))

    # ---- checkpoints (jmm MixtureModel::save/load, mixture_model.h:315-326) --
    def save_json(self, path):
        """Write this mixture (canonical + derived arrays + stepwise state) as JSON."""
        _check(lib().sdmm_mix_save_json(self.h, os.fsencode(path)))

    @classmethod
    def load_json(cls, path, device: int = 0, stream=None) -> "SDMM":
        """A new handle, bitwise the saved mixture (sdmm_mix_load_json)."""
        h = C.c_void_p()
        _check(lib().sdmm_mix_load_json(os.fsencode(path), device, C.byref(h)))
        return cls._adopt(h, stream)

    @classmethod
    def _adopt(cls, h, stream=None) -> "SDMM":
        self = cls.__new__(cls)
        self.h = h
        self.K = int(lib().sdmm_num_components(h))
        if stream is None:
            import torch
            if torch.cuda.is_available():
                self.set_stream(torch.cuda.current_stream())
        else:
            self.set_stream(stream)
        return self

    def clone(self) -> "SDMM":
        """A copy of this mixture and its stepwise EM state (sdmm_clone)."""
        h = C.c_void_p()
        _check(lib().sdmm_clone(self.h, C.byref(h)))
        return SDMM._adopt(h, self.stream_ptr or None)

    def em_params(self) -> dict:
        p = _EmParams()
        _check(lib().sdmm_get_em_params(self.h, C.byref(p)))
        return {"alpha": p.alpha, "bprior": list(p.bprior), "ni_prior_minus_one": p.ni_prior_minus_one,
                "epsilon": p.epsilon, "decrease_prior": p.decrease_prior}

    def restore_params(self, params: dict):
        """Exact inverse of get_params (every array, no MVTN::set re-derivation)."""
        K = self.K
        keep = {n: np.ascontiguousarray(params[n], np.float32).reshape(K * w) for n, w in PARAM_FIELDS}
        keep["valid"] = np.ascontiguousarray(params["valid"], np.int32).reshape(K)
        o = _ParamsOut()
        for n, _ in PARAM_FIELDS:
            setattr(o, n, keep[n].ctypes.data)
        o.valid = keep["valid"].ctypes.data
        _check(lib().sdmm_restore_params(self.h, C.byref(o)))

    def set_guide_capacity(self, cap: int):
        """Per-query candidate-list capacity of the guided-query kernel (0..64, default 40)."""
        _check(lib().sdmm_set_guide_capacity(self.h, cap))

    def guide_fallback_count(self) -> int:
        """Queries of the last guided call that took the full-K path (syncs)."""
        n = C.c_int(0)
        _check(lib().sdmm_guide_fallback_count(self.h, C.byref(n)))
        return int(n.value)

    def set_guide_order(self, coherent: bool):
        """Serve large guided batches in Morton order of c (default) or as given."""
        _check(lib().sdmm_set_guide_order(self.h, 1 if coherent else 0))

    def layout(self) -> dict:
        """E-step kernel layouts: (components per lane, lanes per sample)."""
        v = [C.c_int() for _ in range(4)]
        _check(lib().sdmm_layout(self.h, *[C.byref(x) for x in v]))
        return {"resp": (v[0].value, v[1].value), "stats": (v[2].value, v[3].value)}

    def kernel_name(self, which: str = "resp") -> str:
        """Name of the E-step kernel the handle launches ("resp" or "stats")."""
        return lib().sdmm_kernel_name(self.h, 0 if which == "resp" else 1).decode()

    # ---- EM --------------------------------------------------------------
    def optimize(self, samples: DeviceSamples, iterations: int = 1):
        """StepwiseTangentEM::optimize: `iterations` EM steps (enqueued, async)."""
        _check(lib().sdmm_em_step(self.h, samples.ptr, iterations))

    em_step = optimize

    def optimize_sharded(self, comm: "Comm", shard: DeviceSamples, iterations: int = 1):
        """Sample-sharded EM step(s): this rank's shard, statistics summed over
        the ranks of `comm` (sdmm_em_step_sharded)."""
        _check(lib().sdmm_em_step_sharded(self.h, comm.h, shard.ptr, iterations))

    def estep_stats(self, samples: DeviceSamples, stats):
        """Shard statistics into `stats` (fp64 device tensor of stats_len(K))."""
        assert stats.numel() >= stats_len(self.K) and stats.is_cuda
        _check(lib().sdmm_estep_stats(self.h, samples.ptr, stats.data_ptr()))

    def mstep(self, stats, n_total: int):
        _check(lib().sdmm_mstep(self.h, stats.data_ptr(), n_total))

    def posterior(self, samples: DeviceSamples, resp):
        """posteriorAndLog for every sample into resp (fp32 [N, K] device tensor)."""
        assert resp.numel() >= samples.n * self.K and resp.is_cuda
        _check(lib().sdmm_responsibilities(self.h, samples.ptr, resp.data_ptr()))

    responsibilities = posterior

    # ---- guiding ---------------------------------------------------------
    def guide(self, c, u, out=None):
        """conditional(c) -> sample(u) -> pdf: c, u are 3 device planes each."""
        import torch
        nq = c[0].numel()
        if out is None:
            dev = c[0].device
            out = ([torch.empty(nq, device=dev) for _ in range(3)], torch.empty(nq, device=dev),
                   torch.empty(nq, device=dev, dtype=torch.int32))
        d, pdf, comp = out
        cc = (C.c_void_p * 3)(*[t.data_ptr() for t in c])
        uu = (C.c_void_p * 3)(*[t.data_ptr() for t in u])
        dd = (C.c_void_p * 3)(*[t.data_ptr() for t in d])
        _check(lib().sdmm_guide_batch(self.h, nq, cc, uu, dd, pdf.data_ptr(), comp.data_ptr()))
        return d, pdf, comp

    def pdf(self, c, d, out=None):
        import torch
        nq = c[0].numel()
        if out is None:
            out = torch.empty(nq, device=c[0].device)
        cc = (C.c_void_p * 3)(*[t.data_ptr() for t in c])
        dd = (C.c_void_p * 3)(*[t.data_ptr() for t in d])
        _check(lib().sdmm_pdf_batch(self.h, nq, cc, dd, out.data_ptr()))
        return out

    def guide_product(self, c, u, bsdf, material, frame, out=None):
        """Product sampling with a learned BSDF (sdmm_guide_product_batch).
        bsdf: BsdfTable; material: int32 device tensor; frame: 9 device planes.
        Returns (d planes, pdf, comp, heuristic)."""
        import torch
        nq = c[0].numel()
        if out is None:
            dev = c[0].device
            out = ([torch.empty(nq, device=dev) for _ in range(3)], torch.empty(nq, device=dev),
                   torch.empty(nq, device=dev, dtype=torch.int32), torch.empty(nq, device=dev))
        d, pdf, comp, h = out
        cc = (C.c_void_p * 3)(*[t.data_ptr() for t in c])
        uu = (C.c_void_p * 3)(*[t.data_ptr() for t in u])
        dd = (C.c_void_p * 3)(*[t.data_ptr() for t in d])
        ff = (C.c_void_p * 9)(*[t.data_ptr() for t in frame])
        _check(lib().sdmm_guide_product_batch(self.h, nq, cc, uu, C.byref(bsdf.c), material.data_ptr(), ff, dd,
                                              pdf.data_ptr(), comp.data_ptr(), h.data_ptr()))
        return d, pdf, comp, h

    def pdf_product(self, c, d, bsdf, material, frame):
        import torch
        nq = c[0].numel()
        pdf = torch.empty(nq, device=c[0].device)
        h = torch.empty(nq, device=c[0].device)
        cc = (C.c_void_p * 3)(*[t.data_ptr() for t in c])
        dd = (C.c_void_p * 3)(*[t.data_ptr() for t in d])
        ff = (C.c_void_p * 9)(*[t.data_ptr() for t in frame])
        _check(lib().sdmm_pdf_product_batch(self.h, nq, cc, dd, C.byref(bsdf.c), material.data_ptr(), ff,
                                            pdf.data_ptr(), h.data_ptr()))
        return pdf, h

    def sample_discrete_cdf(self, cdf, u, out=None):
        import torch
        if out is None:
            out = torch.empty(u.numel(), device=u.device, dtype=torch.int32)
        _check(lib().sdmm_sample_discrete_cdf(self.h, cdf.data_ptr(), cdf.numel(), u.data_ptr(),
                                              u.numel(), out.data_ptr()))
        return out


class _BsdfTable(C.Structure):
    _fields_ = [("weights", C.c_void_p), ("means", C.c_void_p), ("covs", C.c_void_p), ("B", C.c_int),
                ("M", C.c_int), ("diffuse", C.c_void_p)]


class BsdfTable:
    """Learned-BSDF lobes on the device (sdmm_bsdf_table): weights (B, M),
    local unit means (B, M, 3), 2x2 covariances (B, M, 4); diffuse (B,)
    optional per-material flags (the plugin's diffuse case: slice 0 on the
    shading normal, sdmm_proc.cpp:335-339)."""

    def __init__(self, weights, means, covs, device="cuda", diffuse=None):
        import torch
        w = np.ascontiguousarray(weights, np.float32)
        self.B, self.M = w.shape
        self.w = torch.from_numpy(w.copy()).to(device)
        self.mean = torch.from_numpy(np.ascontiguousarray(means, np.float32).reshape(self.B, self.M, 3).copy()).to(device)
        self.cov = torch.from_numpy(np.ascontiguousarray(covs, np.float32).reshape(self.B, self.M, 4).copy()).to(device)
        self.diffuse = None
        if diffuse is not None:
            self.diffuse = torch.from_numpy(np.ascontiguousarray(diffuse, np.uint8).reshape(self.B).copy()).to(device)
        self.c = _BsdfTable(self.w.data_ptr(), self.mean.data_ptr(), self.cov.data_ptr(), self.B, self.M,
                            None if self.diffuse is None else self.diffuse.data_ptr())


class STree:
    """The guiding accelerator's spatial tree (jmm SNTree spatial part,
    sntree.h:93-299; the plugin's sdmm-lib DMMSTree is absent).  Built on the
    host; find / route run on the device (sdmm_stree_* in include/sdmm_gpu.h)."""

    def __init__(self, aabb_min, aabb_max, device: int = 0, stream=None):
        lo = np.ascontiguousarray(aabb_min, np.float32)
        hi = np.ascontiguousarray(aabb_max, np.float32)
        h = C.c_void_p()
        _check(lib().sdmm_stree_create(lo.ctypes.data_as(C.c_void_p), hi.ctypes.data_as(C.c_void_p),
                                       C.c_int(device), C.byref(h)))
        self.h = h
        # like SDMM: ordered with the torch ops that fill and read its buffers
        # (torch's current stream unless one is given)
        if stream is None:
            import torch
            if torch.cuda.is_available():
                self.set_stream(torch.cuda.current_stream(device))
        else:
            self.set_stream(stream)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None and getattr(self, "_owned", True):
            _lib.sdmm_stree_destroy(self.h)
        self.h = None

    def set_nodes(self, aabb, child, axis):
        """Replace the node table (the layout nodes() returns)."""
        a = np.ascontiguousarray(aabb, np.float32).reshape(-1, 6)
        c = np.ascontiguousarray(child, np.int32).reshape(-1, 2)
        x = np.ascontiguousarray(axis, np.int32).reshape(-1)
        _check(lib().sdmm_stree_set_nodes(self.h, C.c_int(a.shape[0]), a.ctypes.data_as(C.c_void_p),
                                          c.ctypes.data_as(C.c_void_p), x.ctypes.data_as(C.c_void_p)))

    def save_json(self, path, node_mix=None):
        """The accelerator checkpoint (.asdmm): sdmm::save_json(m_accelerator, path),
        volpath_sdmm.cpp:117-126 -- the node table plus every node's mixture
        (node_mix: one SDMM or None per node; None: tree only)."""
        tab = None if node_mix is None else self._node_table(node_mix)
        _check(lib().sdmm_save_json(self.h, tab, os.fsencode(path)))

    @classmethod
    def load_json(cls, path, device: int = 0, stream=None):
        """(tree, node_mix) from a checkpoint; node_mix[i] is a new SDMM or None."""
        n = C.c_int(0)
        _check(lib().sdmm_load_json(os.fsencode(path), device, None, None, 0, C.byref(n)))
        h = C.c_void_p()
        tab = (C.c_void_p * n.value)()
        _check(lib().sdmm_load_json(os.fsencode(path), device, C.byref(h), tab, n.value, C.byref(n)))
        tree = cls.__new__(cls)
        tree.h = h
        if stream is None:
            import torch
            if torch.cuda.is_available():
                tree.set_stream(torch.cuda.current_stream(device))
        else:
            tree.set_stream(stream)
        mixes = [None if tab[i] is None else SDMM._adopt(C.c_void_p(tab[i]), stream) for i in range(n.value)]
        return tree, mixes

    def split_to_depth(self, depth: int):
        _check(lib().sdmm_stree_split_to_depth(self.h, C.c_int(depth)))

    def split(self, positions, threshold: int):
        """split(threshold) over host positions (3, n)."""
        p = [np.ascontiguousarray(positions[i], np.float32) for i in range(3)]
        arr = (C.c_void_p * 3)(*[x.ctypes.data for x in p])
        _check(lib().sdmm_stree_split(self.h, arr, C.c_int64(p[0].shape[0]), C.c_int(threshold)))

    def split_leaf_recurse(self, node: int, positions, threshold: int):
        """split_leaf_recurse(node, threshold) with that node's positions (3, n)."""
        p = [np.ascontiguousarray(positions[i], np.float32) for i in range(3)]
        arr = (C.c_void_p * 3)(*[x.ctypes.data for x in p])
        _check(lib().sdmm_stree_split_leaf_recurse(self.h, int(node), arr, C.c_int64(p[0].shape[0]),
                                                   int(threshold)))

    def split_leaf_recurse_many(self, nodes, positions, threshold: int):
        """split_leaf_recurse for several leaves (increasing ids), leaf i with
        its own host positions positions[i] (3, n_i) (sdmm_stree_split_leaf_recurse_many)."""
        ps = [[np.ascontiguousarray(pp[i], np.float32) for i in range(3)] for pp in positions]
        arr = (C.c_void_p * (3 * len(ps)))(*[x.ctypes.data for pp in ps for x in pp])
        nd = np.ascontiguousarray(nodes, np.int32)
        cnt = np.array([pp[0].shape[0] for pp in ps], np.int64)
        _check(lib().sdmm_stree_split_leaf_recurse_many(self.h, len(ps), nd.ctypes.data_as(C.c_void_p), arr,
                                                        cnt.ctypes.data_as(C.c_void_p), int(threshold)))

    def split_leaf_recurse_device(self, nodes, planes, starts, counts, threshold: int):
        """The same on device planes (3 tensors): leaf i's positions are
        entries [starts[i], starts[i] + counts[i]) (sdmm_stree_split_leaf_recurse_device)."""
        nd = np.ascontiguousarray(nodes, np.int32)
        st = np.ascontiguousarray(starts, np.int64)
        cn = np.ascontiguousarray(counts, np.int64)
        arr = (C.c_void_p * 3)(*[t.data_ptr() for t in planes])
        _check(lib().sdmm_stree_split_leaf_recurse_device(self.h, len(nd), nd.ctypes.data_as(C.c_void_p), arr,
                                                          st.ctypes.data_as(C.c_void_p),
                                                          cn.ctypes.data_as(C.c_void_p), int(threshold)))

    def split_leaves(self, positions, threshold: int = 4000, max_leaf_nodes: int = 2048):
        """The built plugin's splitting block (volpath_sdmm.cpp:253-260)."""
        p = [np.ascontiguousarray(positions[i], np.float32) for i in range(3)]
        arr = (C.c_void_p * 3)(*[x.ctypes.data for x in p])
        _check(lib().sdmm_stree_split_leaves(self.h, arr, C.c_int64(p[0].shape[0]), int(threshold),
                                             int(max_leaf_nodes)))

    @property
    def leaf_nodes(self) -> int:
        return int(lib().sdmm_stree_leaf_nodes(self.h))

    @property
    def num_nodes(self) -> int:
        return int(lib().sdmm_stree_num_nodes(self.h))

    def nodes(self):
        n = self.num_nodes
        aabb = np.zeros((n, 6), np.float32)
        child = np.zeros((n, 2), np.int32)
        axis = np.zeros(n, np.int32)
        _check(lib().sdmm_stree_get_nodes(self.h, aabb.ctypes.data_as(C.c_void_p),
                                          child.ctypes.data_as(C.c_void_p), axis.ctypes.data_as(C.c_void_p)))
        return aabb, child, axis

    def find(self, p, out=None):
        """Node id per device point (3 device planes) -> int32 device tensor (-1: outside)."""
        import torch
        n = p[0].numel()
        if out is None:
            out = torch.empty(n, dtype=torch.int32, device=p[0].device)
        arr = (C.c_void_p * 3)(*[t.data_ptr() for t in p])
        _check(lib().sdmm_stree_find(self.h, C.c_int64(n), arr, C.c_void_p(out.data_ptr())))
        return out

    def route(self, samples: "DeviceSamples"):
        """Leaf-contiguous copy of `samples` and seg (num_nodes + 1 offsets)."""
        import torch
        x = [torch.empty_like(t) for t in samples.x]
        w = torch.empty_like(samples.w)
        hp = None if samples.hpdf is None else torch.empty_like(samples.hpdf)
        dd = None if samples.is_diffuse is None else torch.empty_like(samples.is_diffuse)
        out = DeviceSamples(x, w, hp, dd)
        seg = np.zeros(self.num_nodes + 1, np.int64)
        _check(lib().sdmm_stree_route(self.h, samples.ptr, out.ptr, seg.ctypes.data_as(C.c_void_p)))
        return out, seg

    # ---- guided wavefront over the leaves (sampleSurface, sdmm_proc.cpp:309-421)
    def _node_table(self, node_mix):
        if node_mix is None:
            return None                            # the bound table
        if len(node_mix) != self.num_nodes:
            raise ValueError(f"node_mix needs one entry per node ({self.num_nodes}), got {len(node_mix)}")
        return (C.c_void_p * len(node_mix))(*[(m.h.value if m is not None else None) for m in node_mix])

    def bind(self, node_mix):
        """Bind one mixture per node (None: no trained mixture) for
        guide/pdf calls made with node_mix=None."""
        _check(lib().sdmm_stree_bind_mixtures(self.h, self._node_table(node_mix)))

    def set_stream(self, stream):
        """Run on `stream` (a torch.cuda.Stream or a raw hipStream_t int; None /
        0 = the HIP null stream)."""
        ptr = None if stream is None else int(getattr(stream, "cuda_stream", stream))
        _check(lib().sdmm_stree_set_stream(self.h, C.c_void_p(ptr or None)))

    @property
    def stream_ptr(self) -> int:
        """The hipStream_t the tree's work runs on (0: the null stream)."""
        return int(lib().sdmm_stree_get_stream(self.h) or 0)

    def guide(self, node_mix, c, u, out=None, node_out=None):
        """Per query: leaf = find(c), then conditional/sample/pdf against
        node_mix[leaf] (None: no trained mixture -> comp -1, pdf 0)."""
        import torch
        nq = c[0].numel()
        tab = self._node_table(node_mix)
        if out is None:
            dev = c[0].device
            out = ([torch.empty(nq, device=dev) for _ in range(3)], torch.empty(nq, device=dev),
                   torch.empty(nq, device=dev, dtype=torch.int32))
        d, pdf, comp = out
        cc = (C.c_void_p * 3)(*[t.data_ptr() for t in c])
        uu = (C.c_void_p * 3)(*[t.data_ptr() for t in u])
        dd = (C.c_void_p * 3)(*[t.data_ptr() for t in d])
        _check(lib().sdmm_guide_wavefront(self.h, tab, nq, cc, uu, dd, pdf.data_ptr(), comp.data_ptr(),
                                          None if node_out is None else node_out.data_ptr()))
        return d, pdf, comp

    def pdf(self, node_mix, c, d, out=None):
        import torch
        nq = c[0].numel()
        tab = self._node_table(node_mix)
        if out is None:
            out = torch.empty(nq, device=c[0].device)
        cc = (C.c_void_p * 3)(*[t.data_ptr() for t in c])
        dd = (C.c_void_p * 3)(*[t.data_ptr() for t in d])
        _check(lib().sdmm_pdf_wavefront(self.h, tab, nq, cc, dd, out.data_ptr()))
        return out

    def guide_pdf(self, node_mix, c, u, dgiven, pdf_mode, node_out=None):
        """One mixed bounce (sdmm_guide_pdf_wavefront): query q samples its
        conditional (pdf_mode[q] == 0) or evaluates its gmmPdf at dgiven[q]."""
        import torch
        nq = c[0].numel()
        tab = self._node_table(node_mix)
        dev = c[0].device
        d = [torch.empty(nq, device=dev) for _ in range(3)]
        pdf = torch.empty(nq, device=dev)
        comp = torch.empty(nq, device=dev, dtype=torch.int32)
        cc = (C.c_void_p * 3)(*[t.data_ptr() for t in c])
        uu = (C.c_void_p * 3)(*[t.data_ptr() for t in u])
        gg = (C.c_void_p * 3)(*[t.data_ptr() for t in dgiven])
        dd = (C.c_void_p * 3)(*[t.data_ptr() for t in d])
        _check(lib().sdmm_guide_pdf_wavefront(self.h, tab, nq, cc, uu, gg, pdf_mode.data_ptr(), dd, pdf.data_ptr(),
                                              comp.data_ptr(), None if node_out is None else node_out.data_ptr()))
        return d, pdf, comp

    def publish(self, node_mix=None):
        """sdmm_stree_publish: nodes + mixture table (node_mix, or the bound
        one) uploaded and the mixtures' pending work done; GuideContext calls
        may then run from any thread until the tree or binding changes."""
        _check(lib().sdmm_stree_publish(self.h, self._node_table(node_mix)))

    def guide_product(self, node_mix, c, u, bsdf, material, frame, choice=None, dgiven=None, node_out=None):
        """Product sampling over the leaves (sdmm_guide_product_wavefront):
        per query the leaf's conditional times its material's learned-BSDF
        lobes; with choice + dgiven the mixed bounce (a pdf query at dgiven
        where choice <= h, comp -2).  Returns (d planes, pdf, comp, h)."""
        import torch
        nq = c[0].numel()
        tab = self._node_table(node_mix)
        dev = c[0].device
        d = [torch.empty(nq, device=dev) for _ in range(3)]
        pdf = torch.empty(nq, device=dev)
        comp = torch.empty(nq, device=dev, dtype=torch.int32)
        h = torch.empty(nq, device=dev)
        cc = (C.c_void_p * 3)(*[t.data_ptr() for t in c])
        uu = (C.c_void_p * 3)(*[t.data_ptr() for t in u])
        dd = (C.c_void_p * 3)(*[t.data_ptr() for t in d])
        ff = (C.c_void_p * 9)(*[t.data_ptr() for t in frame])
        gg = None if dgiven is None else (C.c_void_p * 3)(*[t.data_ptr() for t in dgiven])
        _check(lib().sdmm_guide_product_wavefront(
            self.h, tab, nq, cc, uu, None if choice is None else C.c_void_p(choice.data_ptr()), gg,
            C.byref(bsdf.c), C.c_void_p(material.data_ptr()), ff, dd, C.c_void_p(pdf.data_ptr()),
            C.c_void_p(comp.data_ptr()), C.c_void_p(h.data_ptr()),
            None if node_out is None else C.c_void_p(node_out.data_ptr())))
        return d, pdf, comp, h

    def pdf_product(self, node_mix, c, d, bsdf, material, frame):
        """pdfSurface with sampleProduct per query's leaf (sdmm_pdf_product_wavefront)."""
        import torch
        nq = c[0].numel()
        tab = self._node_table(node_mix)
        pdf = torch.empty(nq, device=c[0].device)
        h = torch.empty(nq, device=c[0].device)
        cc = (C.c_void_p * 3)(*[t.data_ptr() for t in c])
        dd = (C.c_void_p * 3)(*[t.data_ptr() for t in d])
        ff = (C.c_void_p * 9)(*[t.data_ptr() for t in frame])
        _check(lib().sdmm_pdf_product_wavefront(self.h, tab, nq, cc, dd, C.byref(bsdf.c),
                                                C.c_void_p(material.data_ptr()), ff, C.c_void_p(pdf.data_ptr()),
                                                C.c_void_p(h.data_ptr())))
        return pdf, h

    def push_training(self, vertices: "PathVertices", saved_per_path: int = 8, seed: int = 0):
        """Training records of Li's tail (sdmm_push_training): dict of device
        tensors x (6 planes), normal (3), w, stats, node, source; seg (host);
        lost (vertices outside the tree)."""
        import torch
        n = C.c_int64(0)
        lost = C.c_int64(0)
        _check(lib().sdmm_push_training(self.h, C.byref(vertices.s), int(saved_per_path), C.c_uint64(seed), None,
                                        C.byref(n), None, C.byref(lost)))
        m = n.value
        dev = torch.device("cuda", vertices.device)
        out = {"x": [torch.empty(m, device=dev) for _ in range(6)],
               "normal": [torch.empty(m, device=dev) for _ in range(3)],
               "w": torch.empty(m, device=dev), "stats": torch.empty(m, device=dev, dtype=torch.uint8),
               "node": torch.empty(m, device=dev, dtype=torch.int32),
               "source": torch.empty(m, device=dev, dtype=torch.int64)}
        o = _TrainingOut()
        for i in range(6):
            o.x[i] = out["x"][i].data_ptr()
        for i in range(3):
            o.normal[i] = out["normal"][i].data_ptr()
        o.w, o.stats = out["w"].data_ptr(), out["stats"].data_ptr()
        o.node, o.source, o.capacity = out["node"].data_ptr(), out["source"].data_ptr(), m
        seg = np.zeros(self.num_nodes + 1, np.int64)
        _check(lib().sdmm_push_training(self.h, C.byref(vertices.s), int(saved_per_path), C.c_uint64(seed),
                                        C.byref(o), C.byref(n), seg.ctypes.data_as(C.c_void_p), C.byref(lost)))
        out["seg"] = seg
        out["lost"] = lost.value
        return out


class _GuidingConfig(C.Structure):
    _fields_ = [("K", C.c_int), ("split_depth", C.c_int), ("split_threshold", C.c_int),
                ("max_leaf_nodes", C.c_int), ("saved_per_path", C.c_int), ("depth_prior", C.c_float),
                ("init_seed", C.c_uint64), ("optimize_async", C.c_int)]


class _GuidingStats(C.Structure):
    _fields_ = [("leaves", C.c_int), ("optimized", C.c_int), ("records", C.c_int64)]


class Guiding:
    """The plugin's guiding model on the device (sdmm_guiding_*): tree, per-leaf
    mixtures, training data and the render/optimize schedule."""

    def __init__(self, tree_min, tree_max, device: int = 0, **cfg):
        c = _GuidingConfig()
        lib().sdmm_guiding_config_default(C.byref(c))
        for k, v in cfg.items():
            setattr(c, k, v)
        lo = np.ascontiguousarray(tree_min, np.float32)
        hi = np.ascontiguousarray(tree_max, np.float32)
        h = C.c_void_p()
        _check(lib().sdmm_guiding_create(lo.ctypes.data_as(C.c_void_p), hi.ctypes.data_as(C.c_void_p), C.byref(c),
                                         int(device), C.byref(h)))
        self.h, self.device, self.cfg = h, device, c

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.sdmm_guiding_destroy(self.h)
            self.h = None

    @property
    def tree(self) -> "STree":
        t = STree.__new__(STree)
        t.h = C.c_void_p(lib().sdmm_guiding_tree(self.h))
        t._owned = False
        t._owner = self
        return t

    def node_mixtures(self):
        n = self.tree.num_nodes
        tab = (C.c_void_p * n)()
        _check(lib().sdmm_guiding_node_mixtures(self.h, tab, n))
        return [None if tab[i] is None else SDMM._borrow(tab[i], self) for i in range(n)]

    @property
    def trained(self) -> int:
        return int(lib().sdmm_guiding_trained(self.h))

    def push(self, vertices: "PathVertices", seed: int):
        _check(lib().sdmm_guiding_push(self.h, C.byref(vertices.s), C.c_uint64(seed)))

    def update(self):
        """async: wait for the running EM and refresh the conditioners (sdmm_guiding_update)."""
        _check(lib().sdmm_guiding_update(self.h))

    def optimize(self, spp: int) -> dict:
        st = _GuidingStats()
        _check(lib().sdmm_guiding_optimize(self.h, int(spp), C.byref(st)))
        return {"leaves": st.leaves, "optimized": st.optimized, "records": st.records}

    def iteration(self, scene: "Scene", spp: int, seed: int, push_seed: int, train: bool = True,
                  max_depth: int = 10, rr_depth: int = 10, bsdf_fraction: float = 0.5, saved_vertices: int = 9,
                  image=None, image_sqr=None, learned_bsdf: "BsdfTable" = None):
        """One pass of render()'s loop -> (image, li stats, optimize stats).
        learned_bsdf: sampleProduct with that table (rows = the scene's BSDFs)."""
        import torch
        if image is None:
            image = torch.zeros(3, scene.height, scene.width, device=torch.device("cuda", self.device))
        p = _LiParams()
        p.spp, p.max_depth, p.rr_depth, p.guided = int(spp), int(max_depth), int(rr_depth), 0
        p.bsdf_fraction, p.saved_vertices, p.seed = float(bsdf_fraction), int(saved_vertices), int(seed)
        p.pixel_begin, p.pixel_end = 0, scene.width * scene.height
        if learned_bsdf is not None:
            p.sample_product, p.learned_bsdf = 1, learned_bsdf.c
        ls = _LiStats()
        gs = _GuidingStats()
        _check(lib().sdmm_guiding_iteration(self.h, scene.h, C.byref(p), C.c_uint64(push_seed), int(train),
                                            C.c_void_p(image.data_ptr()),
                                            None if image_sqr is None else C.c_void_p(image_sqr.data_ptr()),
                                            C.byref(ls), C.byref(gs)))
        return image, {"paths": ls.paths, "segments": ls.segments, "guided_queries": ls.guided_queries,
                       "fallback_queries": ls.fallback_queries}, \
            {"leaves": gs.leaves, "optimized": gs.optimized, "records": gs.records}


def write_exr(path, rgb, spp: int = 0, iteration: int = 0, time: float = 0.0):
    """iteration%05i.exr / iteration_sqr%05i.exr (sdmm_write_exr): rgb is a
    (3, H, W) array (numpy or a tensor, copied to the host)."""
    a = rgb.detach().cpu().numpy() if hasattr(rgb, "detach") else rgb
    a = np.ascontiguousarray(a, np.float32)
    if a.ndim != 3 or a.shape[0] != 3:
        raise ValueError("rgb must be (3, H, W)")
    _check(lib().sdmm_write_exr(os.fsencode(path), a.shape[2], a.shape[1], a.ctypes.data, int(spp), int(iteration),
                                float(time)))


class _TrainingOut(C.Structure):
    _fields_ = [("x", C.c_void_p * 6), ("normal", C.c_void_p * 3), ("w", C.c_void_p), ("stats", C.c_void_p),
                ("node", C.c_void_p), ("source", C.c_void_p), ("capacity", C.c_int64)]


class _SceneDesc(C.Structure):
    _fields_ = [("n_quads", C.c_int), ("quads", C.c_void_p), ("flip_normals", C.c_void_p), ("bsdf", C.c_void_p),
                ("n_bsdfs", C.c_int), ("reflectance", C.c_void_p), ("emitter", C.c_void_p),
                ("n_emitters", C.c_int), ("radiance", C.c_void_p), ("camera_to_world", C.c_float * 16),
                ("fov_x_deg", C.c_float), ("near_clip", C.c_float), ("width", C.c_int), ("height", C.c_int),
                ("bsdf_params", C.c_void_p), ("learned_models", C.c_void_p)]


class _Learned4(C.Structure):
    _fields_ = [("M", C.c_int), ("weights", C.c_void_p), ("means", C.c_void_p), ("covs", C.c_void_p)]


class LearnedBSDF:
    """A glossy material's learned BSDF (sdmm_learned_bsdf4): the reference's
    BSDF::SDMM4 over (theta_i, alpha) x direction (bsdf.h:310-314) --
    weights[M], means[M][5] (theta, alpha, unit direction in the canonical
    local frame), covs[M][16] over the tangent (theta, alpha, t1, t2)."""

    def __init__(self, weights, means, covs):
        self.weights = np.ascontiguousarray(weights, np.float32).reshape(-1)
        M = self.weights.size
        self.means = np.ascontiguousarray(means, np.float32).reshape(M, 5)
        self.covs = np.ascontiguousarray(covs, np.float32).reshape(M, 16)
        self.c = _Learned4(M, self.weights.ctypes.data, self.means.ctypes.data, self.covs.ctypes.data)

    @property
    def M(self):
        return self.weights.size

    def arrays(self):
        return self.weights, self.means, self.covs

    def save_json(self, path):
        _check(lib().sdmm_learned4_save_json(C.byref(self.c), os.fsencode(path)))

    @classmethod
    def load_json(cls, path):
        M = C.c_int()
        _check(lib().sdmm_learned4_load_json(os.fsencode(path), 0, C.byref(M), None, None, None))
        w = np.zeros(M.value, np.float32)
        mu = np.zeros((M.value, 5), np.float32)
        cv = np.zeros((M.value, 16), np.float32)
        _check(lib().sdmm_learned4_load_json(os.fsencode(path), M.value, C.byref(M), w.ctypes.data, mu.ctypes.data,
                                             cv.ctypes.data))
        return cls(w, mu, cv)

    def conditional_device(self, alpha, wl, keep=2, stream=None):
        """sdmm_learned4_conditional_device over local directions wl (3
        device tensors): (weights (nq, keep), means (nq, keep, 3), covs (nq,
        keep, 4), n (nq,)) on the device."""
        import torch
        nq = wl[0].numel()
        dev = wl[0].device
        w = torch.empty((nq, keep), device=dev)
        m = torch.empty((nq, keep, 3), device=dev)
        c = torch.empty((nq, keep, 4), device=dev)
        n = torch.empty(nq, dtype=torch.int32, device=dev)
        st = torch.cuda.current_stream(dev) if stream is None else stream
        _check(lib().sdmm_learned4_conditional_device(
            C.byref(self.c), C.c_float(alpha), nq, (C.c_void_p * 3)(*[t.data_ptr() for t in wl]), keep,
            w.data_ptr(), m.data_ptr(), c.data_ptr(), n.data_ptr(), C.c_void_p(int(st.cuda_stream) or None)))
        return w, m, c, n

    def conditional(self, alpha, wi_local, keep=2):
        """getDMM + rotate_to_wo on the host (sdmm_learned4_conditional):
        (weights[n], means[n][3], covs[n][4]), n = 0 without a valid one."""
        wl = np.ascontiguousarray(wi_local, np.float32)
        n = C.c_int()
        w = np.zeros(8, np.float32)
        m = np.zeros((8, 3), np.float32)
        c = np.zeros((8, 4), np.float32)
        _check(lib().sdmm_learned4_conditional(C.byref(self.c), C.c_float(alpha), wl.ctypes.data, keep, C.byref(n),
                                               w.ctypes.data, m.ctypes.data, c.ctypes.data))
        return w[:n.value], m[:n.value], c[:n.value]


class _LiParams(C.Structure):
    _fields_ = [("spp", C.c_int), ("max_depth", C.c_int), ("rr_depth", C.c_int), ("guided", C.c_int),
                ("bsdf_fraction", C.c_float), ("saved_vertices", C.c_int), ("seed", C.c_uint64),
                ("pixel_begin", C.c_int64), ("pixel_end", C.c_int64), ("sample_product", C.c_int),
                ("learned_bsdf", _BsdfTable)]


class _PathVertices(C.Structure):
    _fields_ = [("n_paths", C.c_int64), ("max_vertices", C.c_int), ("path0", C.c_int64), ("rec", C.c_void_p),
                ("nv", C.c_void_p)]


class _LiStats(C.Structure):
    _fields_ = [("paths", C.c_int64), ("segments", C.c_int64), ("guided_queries", C.c_int64),
                ("fallback_queries", C.c_int64)]


def _hip():
    return C.CDLL("libamdhip64.so")


class GuideContext:
    """One render worker's guiding context on a published STree
    (sdmm_guide_ctx_*): its own HIP stream and scratch, so contexts run
    guided bounces from different host threads at once, as the reference's
    render workers call the conditional concurrently (sdmm_proc.cpp:1086-1106).
    Calls are asynchronous on the context's stream; the output planes are the
    caller's (device tensors) and valid after synchronize()."""

    def __init__(self, tree, stream=None):
        self.tree = tree
        h = C.c_void_p()
        ptr = None if stream is None else int(getattr(stream, "cuda_stream", stream))
        _check(lib().sdmm_guide_ctx_create(tree.h, C.c_void_p(ptr or None), C.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            lib().sdmm_guide_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream_ptr(self) -> int:
        return int(lib().sdmm_guide_ctx_stream(self.h) or 0)

    def synchronize(self):
        h = _hip()
        h.hipStreamSynchronize.argtypes = [C.c_void_p]
        assert h.hipStreamSynchronize(C.c_void_p(self.stream_ptr or None)) == 0

    def guide_pdf_into(self, nq, c, u, dgiven, pdf_mode, d, pdf, comp):
        """sdmm_ctx_guide_pdf_wavefront on raw device pointers (plane
        pointers as int sequences): the thread-friendly form (no tensor
        allocation; the GIL is released for the call)."""
        P3 = C.c_void_p * 3
        _check(lib().sdmm_ctx_guide_pdf_wavefront(self.h, nq, P3(*c), P3(*u), P3(*dgiven), C.c_void_p(pdf_mode),
                                                  P3(*d), C.c_void_p(pdf), C.c_void_p(comp), None))

    def guide_pdf(self, c, u, dgiven, pdf_mode):
        import torch
        nq = c[0].numel()
        dev = c[0].device
        d = [torch.empty(nq, device=dev) for _ in range(3)]
        pdf = torch.empty(nq, device=dev)
        comp = torch.empty(nq, device=dev, dtype=torch.int32)
        self.guide_pdf_into(nq, [t.data_ptr() for t in c], [t.data_ptr() for t in u], [t.data_ptr() for t in dgiven],
                            pdf_mode.data_ptr(), [t.data_ptr() for t in d], pdf.data_ptr(), comp.data_ptr())
        return d, pdf, comp

    def guide_pdf_host(self, reqs):
        """sdmm_ctx_guide_pdf_host_batch: reqs = [(inp, mode, out, comp)] host
        tensors (pinned: inp (9, n) float32, mode (n,) uint8, out (4, n)
        float32, comp (n,) int32), served as one wavefront; outputs written in
        place, synchronously."""
        arr = (_GuideHostReq * max(1, len(reqs)))()
        for i, (inp, mode, out, comp) in enumerate(reqs):
            n = int(mode.numel())
            arr[i] = _GuideHostReq(n, inp.data_ptr(), inp.stride(0), mode.data_ptr(), out.data_ptr(), out.stride(0),
                                   comp.data_ptr())
        _check(lib().sdmm_ctx_guide_pdf_host_batch(self.h, len(reqs), C.cast(arr, C.c_void_p)))

    def guide_product(self, c, u, bsdf, material, frame, choice=None, dgiven=None):
        """sdmm_ctx_guide_product_wavefront (see STree.guide_product)."""
        import torch
        nq = c[0].numel()
        dev = c[0].device
        d = [torch.empty(nq, device=dev) for _ in range(3)]
        pdf = torch.empty(nq, device=dev)
        comp = torch.empty(nq, device=dev, dtype=torch.int32)
        h = torch.empty(nq, device=dev)
        P3 = C.c_void_p * 3
        gg = None if dgiven is None else P3(*[t.data_ptr() for t in dgiven])   # kept alive over the call
        _check(lib().sdmm_ctx_guide_product_wavefront(
            self.h, nq, P3(*[t.data_ptr() for t in c]), P3(*[t.data_ptr() for t in u]),
            None if choice is None else C.c_void_p(choice.data_ptr()),
            None if gg is None else C.cast(gg, C.c_void_p),
            C.byref(bsdf.c), C.c_void_p(material.data_ptr()), (C.c_void_p * 9)(*[t.data_ptr() for t in frame]),
            P3(*[t.data_ptr() for t in d]), C.c_void_p(pdf.data_ptr()), C.c_void_p(comp.data_ptr()),
            C.c_void_p(h.data_ptr()), None))
        return d, pdf, comp, h


class PathVertices:
    """The saved vertices of the last Scene.render (scene-owned device memory,
    valid until the scene renders again)."""

    def __init__(self, s, scene, device):
        self.s, self.scene, self.device = s, scene, device

    def to_numpy(self):
        P, V = self.s.n_paths, self.s.max_vertices
        rec = np.empty(16 * V * P, np.float32)
        nv = np.empty(P, np.int32)
        import torch
        torch.cuda.synchronize(self.device)
        h = _hip()
        h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        assert h.hipMemcpy(rec.ctypes.data, self.s.rec, rec.nbytes, 2) == 0
        assert h.hipMemcpy(nv.ctypes.data, self.s.nv, nv.nbytes, 2) == 0
        return rec, nv


class Scene:
    """Analytic quad scene for the device Li (sdmm_scene_*); desc as
    scenes.cornell_box() returns it."""

    def __init__(self, desc: dict, device: int = 0):
        self._keep = {k: np.ascontiguousarray(v) for k, v in desc.items() if isinstance(v, np.ndarray)}
        d = _SceneDesc()
        d.n_quads = self._keep["quads"].size // 9
        d.quads = self._keep["quads"].ctypes.data
        d.flip_normals = self._keep["flip_normals"].ctypes.data if "flip_normals" in self._keep else None
        d.bsdf = self._keep["bsdf"].ctypes.data
        d.n_bsdfs = self._keep["reflectance"].size // 3
        d.reflectance = self._keep["reflectance"].ctypes.data
        if "emitter" in self._keep:
            d.emitter = self._keep["emitter"].ctypes.data
            d.n_emitters = self._keep["radiance"].size // 3
            d.radiance = self._keep["radiance"].ctypes.data
        for i, v in enumerate(np.asarray(desc["camera_to_world"], np.float32).reshape(-1)):
            d.camera_to_world[i] = float(v)
        d.fov_x_deg = float(desc["fov_x_deg"])
        d.near_clip = float(desc.get("near_clip", 1e-2))
        d.width, d.height = int(desc["width"]), int(desc["height"])
        if "bsdf_params" in self._keep:
            self._keep["bsdf_params"] = np.ascontiguousarray(self._keep["bsdf_params"], np.float32)
            d.bsdf_params = self._keep["bsdf_params"].ctypes.data
        if desc.get("learned_models"):
            # per BSDF: None or (weights, means, covs) / a LearnedBSDF
            self._models = [None if m is None else (m if isinstance(m, LearnedBSDF) else LearnedBSDF(*m))
                            for m in desc["learned_models"]]
            self._model_tab = (_Learned4 * d.n_bsdfs)()
            for b, m in enumerate(self._models):
                if m is not None:
                    self._model_tab[b] = m.c
            d.learned_models = C.cast(self._model_tab, C.c_void_p)
        self.width, self.height, self.device = d.width, d.height, device
        h = C.c_void_p()
        _check(lib().sdmm_scene_create(C.byref(d), int(device), C.byref(h)))
        self.h = h

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.sdmm_scene_destroy(self.h)
            self.h = None

    def normalization(self):
        """(scene_min, spatial_norm, tree_min, tree_max) -- render(), volpath_sdmm.cpp:375-393."""
        smin = np.zeros(3, np.float32)
        norm = np.zeros(1, np.float32)
        tmin = np.zeros(3, np.float32)
        tmax = np.zeros(3, np.float32)
        _check(lib().sdmm_scene_normalization(self.h, smin.ctypes.data, norm.ctypes.data, tmin.ctypes.data,
                                              tmax.ctypes.data))
        return smin, float(norm[0]), tmin, tmax

    def render(self, tree: "STree", node_mix=None, spp: int = 1, max_depth: int = 10, rr_depth: int = 10,
               guided: bool = False, bsdf_fraction: float = 0.5, saved_vertices: int = 9, seed: int = 0,
               pixels=None, image=None, image_sqr=None, learned_bsdf: "BsdfTable" = None):
        """One render pass (sdmm_li_render) -> (image (3, H, W) device tensor,
        PathVertices, stats dict).  learned_bsdf: sampleProduct with that
        learned-BSDF table (one row per scene BSDF)."""
        import torch
        if image is None:
            image = torch.zeros(3, self.height, self.width, device=torch.device("cuda", self.device))
        p = _LiParams()
        p.spp, p.max_depth, p.rr_depth, p.guided = int(spp), int(max_depth), int(rr_depth), int(guided)
        p.bsdf_fraction, p.saved_vertices, p.seed = float(bsdf_fraction), int(saved_vertices), int(seed)
        p.pixel_begin, p.pixel_end = (0, self.width * self.height) if pixels is None else pixels
        if learned_bsdf is not None:
            p.sample_product, p.learned_bsdf = 1, learned_bsdf.c
        v = _PathVertices()
        st = _LiStats()
        tab = None if not guided else tree._node_table(node_mix)
        _check(lib().sdmm_li_render(self.h, tree.h, tab, C.byref(p), C.c_void_p(image.data_ptr()),
                                    None if image_sqr is None else C.c_void_p(image_sqr.data_ptr()), C.byref(v),
                                    C.byref(st)))
        return image, PathVertices(v, self, self.device), {"paths": st.paths, "segments": st.segments,
                                                           "guided_queries": st.guided_queries,
                                                           "fallback_queries": st.fallback_queries}
