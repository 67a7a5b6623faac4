"""ctypes binding of libme_hip.so (the C ABI declared in include/me_hip.h).

The product path has no CPU fallback: if the HIP library is missing or no
device is present, every entry point raises ``MEError``.

torch is imported (when available) before the library is loaded so that the
process uses a single HIP runtime: libme_hip.so resolves ``libamdhip64.so.7``
to the copy torch already mapped.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_int32, c_long, c_size_t, c_uint8, c_uint32, c_void_p

import numpy as np

try:  # one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the ctypes path
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libme_hip.so")

ME_OK = 0
ME_HOST = 0
ME_DEVICE = 1
ERRORS = {
    -1: "ME_ERR_INVALID",
    -2: "ME_ERR_HIP",
    -3: "ME_ERR_NOMEM",
    -4: "ME_ERR_UNSUPPORTED",
    -5: "ME_ERR_STATE",
    -6: "ME_ERR_NO_DEVICE",
}

# kernel timing families (me_hip.h ME_KT_*)
KT = dict(MI=0, SCALE_RES=1, SCALE_NEQ=2, BA_LINEARIZE=3, BA_POINTS=4, BA_SCHUR=5, BA_SOLVE=6, BA_STEP=7,
          KLT=8, PYR=9, NMS=10)


class MEError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class ScaleStateC(ctypes.Structure):
    _fields_ = [
        ("n_left", c_int), ("n_right", c_int),
        ("X_left", POINTER(c_double)), ("X_right", POINTER(c_double)),
        ("tri_left", POINTER(c_uint8)), ("tri_right", POINTER(c_uint8)),
        ("last_left", POINTER(c_uint32)), ("last_right", POINTER(c_uint32)),
        ("lframe", c_uint32),
        ("K1", c_double * 9), ("K2", c_double * 9),
        ("q1", c_double * 4), ("t1", c_double * 3),
        ("q2", c_double * 4), ("t2", c_double * 3),
        ("scale", c_double), ("baseline", c_double),
        ("window_size", c_int),
        ("imgL", c_void_p), ("imgR", c_void_p),
        ("stride", c_int), ("cols", c_int), ("rows", c_int),
        ("bb_cols", c_int), ("bb_rows", c_int),
        ("mask", POINTER(c_uint8)), ("mask_len", c_int),
        ("img_mem", c_int), ("tracks_mem", c_int),
    ]


class OptimParamsC(ctypes.Structure):
    _fields_ = [
        ("type", c_int), ("minim", c_int), ("max_nb_iter", c_int),
        ("v", c_double), ("tau", c_double), ("mu", c_double), ("abs_tol", c_double), ("grad_tol", c_double),
        ("incr_tol", c_double), ("rel_tol", c_double), ("alpha", c_double),
        ("weighting", c_int),
    ]


class BAProblemC(ctypes.Structure):
    _fields_ = [
        ("n_cams", c_int), ("n_pts", c_int), ("n_obs", c_int),
        ("cams", POINTER(c_double)), ("pts", POINTER(c_double)), ("obs", POINTER(c_double)),
        ("cam_idx", POINTER(c_int32)), ("pt_idx", POINTER(c_int32)),
        ("K0", c_double * 9), ("K1", c_double * 9),
        ("baseline", c_double), ("feat_var", c_double),
        ("fixed_frames", c_int), ("mem", c_int),
        ("obs_dim", c_int), ("cam_id", POINTER(c_int32)),
    ]


class BAOptionsC(ctypes.Structure):
    _fields_ = [
        ("max_num_iterations", c_int),
        ("function_tolerance", c_double), ("gradient_tolerance", c_double), ("parameter_tolerance", c_double),
        ("initial_trust_region_radius", c_double), ("max_trust_region_radius", c_double),
        ("min_trust_region_radius", c_double),
        ("min_lm_diagonal", c_double), ("max_lm_diagonal", c_double), ("min_relative_decrease", c_double),
        ("max_num_consecutive_invalid_steps", c_int),
        ("jacobi_scaling", c_int),
    ]


class BASummaryC(ctypes.Structure):
    _fields_ = [
        ("status", c_int), ("termination", c_int), ("iterations", c_int), ("successful_steps", c_int),
        ("initial_cost", c_double), ("final_cost", c_double),
    ]


class VOChainArgsC(ctypes.Structure):
    """me_vo_chain_args (include/me_hip.h)."""
    _fields_ = [("pose", c_double * 6), ("R", c_double * 9), ("vel", c_double * 6), ("k1", c_int), ("k0", c_int),
                ("mode", c_int)]


class VOWindowC(ctypes.Structure):
    """me_vo_window (include/me_hip.h)."""
    _fields_ = [("stage", c_void_p), ("dev", c_void_p), ("stage_bytes", c_size_t), ("chain", c_int),
                ("cam_src", c_void_p), ("win_ids", c_void_p), ("prev_ids", c_void_p), ("n_prev", c_int),
                ("new_from", ctypes.c_int32), ("args", VOChainArgsC), ("frame", c_void_p), ("ids", c_void_p),
                ("first_frame", c_int)]


class VOLoopConfigC(ctypes.Structure):
    """me_vo_loop_config (include/me_hip.h)."""
    _fields_ = [("width", c_int), ("height", c_int), ("n_feats", c_int), ("window", c_int), ("ba_iters", c_int),
                ("scale_iters", c_int), ("fixed_frames", c_int), ("d_min", c_int), ("d_max", c_int),
                ("baseline", c_double), ("feat_var", c_double), ("K", c_double * 9), ("first_pose", c_double * 6),
                ("velocity", c_double * 6), ("has_velocity", c_int), ("log_events", c_int),
                ("async_enqueue", c_int)]


class VOFrameResultC(ctypes.Structure):
    """me_vo_frame_result (include/me_hip.h)."""
    _fields_ = [("t", c_int), ("n_tracked", c_int), ("n_new", c_int), ("n_active", c_int), ("n_window_pts", c_int),
                ("n_window_obs", c_int), ("scale", c_double), ("scale_stop", c_int), ("scale_iters", c_int),
                ("ba_iters", c_int), ("ba_cost", c_double), ("pose", c_double * 6)]


# me_vo_event as a numpy record (32 bytes: int kind, int t, int64 id, float feat[4])
VO_EVENT_DTYPE = np.dtype([("kind", np.int32), ("t", np.int32), ("id", np.int64), ("feat", np.float32, 4)])


class KLTParamsC(ctypes.Structure):
    _fields_ = [("win", c_int), ("max_level", c_int), ("max_iters", c_int), ("eps", c_double),
                ("min_eig", c_double)]


ALLREDUCE_FN = ctypes.CFUNCTYPE(c_int, POINTER(c_double), c_int, c_void_p)

# every symbol include/me_hip.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "me_abi_version", "me_range_push", "me_range_pop", "me_device_count", "me_create", "me_destroy", "me_last_error", "me_set_stream",
    "me_get_stream", "me_set_cu_mask", "me_stream_flags", "me_cu_count", "me_synchronize", "me_malloc", "me_free", "me_memcpy_h2d", "me_memcpy_d2h", "me_memcpy_d2d",
    "me_memcpy_async", "me_host_alloc", "me_host_free", "me_hbm_copy_gbs",
    "me_timing_enable", "me_timing_read", "me_timing_reset", "me_timing_sample",
    "me_mi_scores", "me_mutual_information", "me_entropy", "me_mi_epipolar_match", "me_mi_epipolar_match_count", "me_vo_new_cells", "me_compare_pc", "me_ccoeff_normed", "me_quantise",
    "me_optim_default_params", "me_scale_residuals", "me_scale_normal_equations", "me_scale_jacobian",
    "me_scale_optimise", "me_scale_last_counters", "me_scale_persistent", "me_scale_state_mi", "me_scale_inliers",
    "me_ba_default_options", "me_ba_solve", "me_ba_cost", "me_ba_evaluate", "me_ba_reduced_system",
    "me_ba_solve_sharded", "me_ba_covariance", "me_ba_solve_async", "me_ba_wait", "me_ba_wait_out", "me_ba_reserve", "me_ba_window_indices",
    "me_vo_ba_chain", "me_vo_window_submit",
    "me_comm_unique_id", "me_comm_create_rccl", "me_comm_create_callback", "me_comm_destroy", "me_comm_info",
    "me_comm_allreduce", "me_comm_calibrate", "me_comm_exchange_us", "me_ba_shard_worthwhile_comm", "me_ba_solve_comm", "me_ba_shard_worthwhile", "me_ba_shard_exchange_us",
    "me_klt_default_params", "me_klt_track",
    "me_nms_scanline3x3",
    "me_vo_default_params", "me_vo_srand", "me_vo_rand", "me_vo_process",
    "me_mono_default_params", "me_mono_vo_process",
    "me_vo_loop_default_config", "me_vo_loop_create", "me_vo_loop_destroy", "me_vo_loop_last_error",
    "me_vo_loop_process", "me_vo_loop_finish", "me_vo_loop_results", "me_vo_loop_events", "me_vo_loop_tracks",
    "me_vo_loop_poses", "me_vo_loop_frame_obs", "me_vo_loop_frames", "me_vo_loop_stats",
]

class MonoParamsC(ctypes.Structure):
    """me_mono_params (include/me_hip.h)."""
    _fields_ = [("fu", c_double), ("fv", c_double), ("cu", c_double), ("cv", c_double), ("prob", c_double),
                ("inlier_threshold", c_double), ("ransac", c_int)]


class VOParamsC(ctypes.Structure):
    """me_vo_params (include/me_hip.h)."""
    _fields_ = [
        ("method", c_int), ("step_size", c_double), ("eps", c_double),
        ("e1", c_double), ("e2", c_double), ("e3", c_double), ("e4", c_double),
        ("max_iter", c_int), ("nb_fixed_frames", c_int), ("ransac", c_int), ("n_ransac", c_int),
        ("inlier_threshold", c_double), ("baseline", c_double), ("weighting", c_int),
        ("fu1", c_double), ("fv1", c_double), ("fu2", c_double), ("fv2", c_double),
        ("cu1", c_double), ("cu2", c_double), ("cv1", c_double), ("cv2", c_double),
    ]


_lib = None


def load_library(path: str | None = None):
    """Load libme_hip.so and declare prototypes.  Raises MEError if missing.
    ME_LIB (environment) names another build of the same library (A/B timing,
    tools/gpu.sh ab); the default is the in-tree build."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("ME_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise MEError(-4, f"{path} not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    P = POINTER
    sig = {
        "me_abi_version": (c_int, []),
        "me_range_push": (c_int, [ctypes.c_char_p]),
        "me_range_pop": (c_int, []),
        "me_device_count": (c_int, [P(c_int)]),
        "me_create": (c_int, [P(c_void_p), c_int]),
        "me_destroy": (None, [c_void_p]),
        "me_last_error": (ctypes.c_char_p, [c_void_p]),
        "me_set_stream": (c_int, [c_void_p, c_void_p]),
        "me_get_stream": (c_void_p, [c_void_p]),
        "me_set_cu_mask": (c_int, [c_void_p, P(ctypes.c_uint32), c_int]),
        "me_synchronize": (c_int, [c_void_p]),
        "me_stream_flags": (c_int, [c_void_p, P(ctypes.c_uint)]),
        "me_malloc": (c_int, [c_void_p, P(c_void_p), c_size_t]),
        "me_free": (c_int, [c_void_p, c_void_p]),
        "me_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
        "me_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
        "me_memcpy_d2d": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
        "me_memcpy_async": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
        "me_host_alloc": (c_int, [c_void_p, P(c_void_p), c_size_t]),
        "me_host_free": (c_int, [c_void_p, c_void_p]),
        "me_timing_enable": (c_int, [c_void_p, c_int]),
        "me_timing_sample": (c_int, [c_void_p, c_int]),
        "me_timing_read": (c_int, [c_void_p, c_int, P(c_long), P(c_double)]),
        "me_timing_reset": (c_int, [c_void_p]),
        "me_hbm_copy_gbs": (c_int, [c_void_p, c_size_t, c_int, P(c_double)]),
        "me_mi_scores": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p,
                                 c_void_p, c_int, c_int, c_int, c_void_p]),
        "me_mutual_information": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                                          c_void_p]),
        "me_mi_epipolar_match": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_double, c_float,
                                         c_void_p, c_void_p]),
        "me_mi_epipolar_match_count": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                               c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_double,
                                               c_float, c_void_p, c_void_p]),
        "me_vo_new_cells": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_int, c_int,
                                    c_double, c_double, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
        "me_compare_pc": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
        "me_ccoeff_normed": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
        "me_quantise": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int]),
        "me_entropy": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p]),
        "me_optim_default_params": (None, [P(OptimParamsC)]),
        "me_scale_residuals": (c_int, [c_void_p, P(ScaleStateC), c_int, P(c_double), P(c_int)]),
        "me_scale_normal_equations": (c_int, [c_void_p, P(ScaleStateC), c_int, P(c_double), P(c_double),
                                              P(c_double)]),
        "me_scale_jacobian": (c_int, [c_void_p, P(ScaleStateC), c_int, P(c_double)]),
        "me_scale_optimise": (c_int, [c_void_p, P(ScaleStateC), P(OptimParamsC), c_int, P(c_int), P(c_int),
                                      P(c_double), c_int, P(c_long)]),
        "me_scale_last_counters": (c_int, [c_void_p, P(c_long), P(c_long), P(c_long), P(c_long)]),
        "me_scale_persistent": (c_int, [c_int, c_int]),
        "me_scale_state_mi": (c_int, [c_void_p, P(ScaleStateC), P(c_double), P(c_int)]),
        "me_scale_inliers": (c_int, [c_void_p, P(ScaleStateC), c_int, c_double, P(c_int), c_int, P(c_int)]),
        "me_ba_default_options": (None, [P(BAOptionsC)]),
        "me_ba_solve": (c_int, [c_void_p, P(BAProblemC), P(BAOptionsC), P(BASummaryC)]),
        "me_ba_solve_async": (c_int, [c_void_p, P(BAProblemC), P(BAOptionsC)]),
        "me_ba_wait": (c_int, [c_void_p, P(BASummaryC)]),
        "me_ba_wait_out": (c_int, [c_void_p, P(BASummaryC), c_void_p, c_void_p]),
        "me_ba_reserve": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int]),
        "me_vo_window_submit": (c_int, [c_void_p, P(VOWindowC), P(BAProblemC), P(BAOptionsC)]),
        "me_vo_ba_chain": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                   ctypes.c_int32, P(VOChainArgsC)]),
        "me_ba_cost": (c_int, [c_void_p, P(BAProblemC), P(c_double)]),
        "me_ba_window_indices": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p,
                                         c_void_p]),
        "me_ba_evaluate": (c_int, [c_void_p, P(BAProblemC), P(c_double), P(c_double), P(c_double)]),
        "me_ba_reduced_system": (c_int, [c_void_p, P(BAProblemC), c_double, P(c_double), P(c_double)]),
        "me_ba_covariance": (c_int, [c_void_p, P(BAProblemC), P(c_double), P(c_int)]),
        "me_ba_solve_sharded": (c_int, [c_void_p, P(BAProblemC), P(BAOptionsC), ALLREDUCE_FN, c_void_p,
                                        P(BASummaryC)]),
        "me_comm_unique_id": (c_int, [c_void_p, c_int]),
        "me_comm_create_rccl": (c_int, [c_void_p, c_int, c_int, c_void_p, P(c_void_p)]),
        "me_comm_create_callback": (c_int, [c_void_p, c_int, c_int, ALLREDUCE_FN, c_void_p, P(c_void_p)]),
        "me_comm_destroy": (None, [c_void_p]),
        "me_comm_info": (c_int, [c_void_p, P(c_int), P(c_int), P(c_int)]),
        "me_comm_allreduce": (c_int, [c_void_p, c_void_p, c_long, c_int]),
        "me_comm_calibrate": (c_int, [c_void_p, c_int]),
        "me_comm_exchange_us": (c_int, [c_void_p, P(c_double), P(c_double)]),
        "me_ba_shard_worthwhile_comm": (c_int, [c_void_p, c_long]),
        "me_ba_solve_comm": (c_int, [c_void_p, P(BAProblemC), P(BAOptionsC), c_void_p, P(BASummaryC)]),
        "me_ba_shard_worthwhile": (c_int, [c_long, c_int, c_double]),
        "me_ba_shard_exchange_us": (c_double, [c_int]),
        "me_cu_count": (c_int, [c_void_p, P(c_int)]),
        "me_vo_loop_default_config": (None, [P(VOLoopConfigC)]),
        "me_vo_loop_create": (c_int, [c_void_p, c_void_p, P(VOLoopConfigC), P(c_void_p)]),
        "me_vo_loop_destroy": (None, [c_void_p]),
        "me_vo_loop_last_error": (ctypes.c_char_p, [c_void_p]),
        "me_vo_loop_process": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int]),
        "me_vo_loop_finish": (c_int, [c_void_p]),
        "me_vo_loop_results": (c_int, [c_void_p, P(VOFrameResultC), c_int, P(c_int)]),
        "me_vo_loop_events": (c_int, [c_void_p, c_void_p, c_long, P(c_long)]),
        "me_vo_loop_tracks": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, P(c_int)]),
        "me_vo_loop_poses": (c_int, [c_void_p, c_void_p, c_void_p, c_int, P(c_int)]),
        "me_vo_loop_frame_obs": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, P(c_int)]),
        "me_vo_loop_frames": (c_int, [c_void_p, c_void_p, c_int, P(c_int)]),
        "me_vo_loop_stats": (c_int, [c_void_p, P(c_double), c_int]),
        "me_klt_default_params": (None, [P(KLTParamsC)]),
        "me_klt_track": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p, c_int, P(KLTParamsC)]),
        "me_nms_scanline3x3": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int,
                                       P(c_int)]),
        "me_vo_default_params": (None, [P(VOParamsC)]),
        "me_vo_srand": (c_int, [c_void_p, ctypes.c_uint]),
        "me_vo_rand": (c_int, [c_void_p, P(c_int)]),
        "me_vo_process": (c_int, [c_void_p, c_void_p, c_int, P(c_double), P(VOParamsC), c_int, P(c_double),
                                  P(c_double), P(c_double), P(c_int), P(c_int), P(c_int)]),
        "me_mono_default_params": (None, [P(MonoParamsC)]),
        "me_mono_vo_process": (c_int, [c_void_p, c_void_p, c_void_p, c_int, P(MonoParamsC), P(c_double),
                                       P(c_double), c_void_p, P(c_int), P(c_int)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def dptr(a: np.ndarray, ctype=c_double):
    """POINTER(ctype) to a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data_as(POINTER(ctype))


def vptr(a):
    if a is None:
        return None
    if isinstance(a, int):
        return c_void_p(a)
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return c_void_p(a.ctypes.data)


def cu_split(ncu: int, front_of_16: int, mode: str | None = None):
    """Disjoint CU sets (front, back) for two contexts, front_of_16 of every 16
    CUs to the front.  mode "xcd" (default; ME_CU_SPLIT overrides) gives each
    side whole XCDs: logical CU i sits on XCD i mod 8 (measured: the split by
    i mod 8 keeps the BA's L2 apart from the front end's, the split by
    i // 32 does not), so front = {i : i mod 8 < front_of_16 / 2}.  mode
    "interleaved": front = {i : i mod 16 < front_of_16}, every XCD shared."""
    mode = mode or os.environ.get("ME_CU_SPLIT", "xcd")
    if mode == "xcd" and front_of_16 % 2 == 0:
        front = [i for i in range(ncu) if i % 8 < front_of_16 // 2]
    else:
        front = [i for i in range(ncu) if i % 16 < front_of_16]
    fs = set(front)
    return front, [i for i in range(ncu) if i not in fs]


class Context:
    """One me_ctx (HIP device + stream + scratch).  One per host thread."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = c_void_p()
        rc = self.lib.me_create(ctypes.byref(h), device)
        if rc != ME_OK:
            raise MEError(rc, f"me_create(device={device}) failed: no usable HIP device "
                              "(the product path has no CPU fallback)")
        self.h = h
        self.device = device

    def check(self, rc: int, what: str = ""):
        if rc != ME_OK:
            msg = self.lib.me_last_error(self.h)
            raise MEError(rc, f"{what}: {msg.decode() if msg else ''}")

    def close(self):
        if getattr(self, "h", None):
            self.lib.me_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_stream(self, stream_handle: int | None):
        self.check(self.lib.me_set_stream(self.h, c_void_p(stream_handle) if stream_handle else None),
                   "me_set_stream")

    def set_cu_mask(self, cus):
        """Restrict the ctx-owned stream to the compute units in `cus` (an
        iterable of CU indices; None or empty: all CUs) -- me_set_cu_mask."""
        cus = sorted(set(cus or ()))
        nw = (cus[-1] // 32 + 1) if cus else 0
        words = (ctypes.c_uint32 * max(nw, 1))()
        for i in cus:
            words[i // 32] |= 1 << (i % 32)
        self.check(self.lib.me_set_cu_mask(self.h, words, nw), "me_set_cu_mask")

    def stream_ptr(self) -> int:
        """The context's HIP stream (me_get_stream) as an integer handle."""
        return int(self.lib.me_get_stream(self.h) or 0)

    def synchronize(self):
        self.check(self.lib.me_synchronize(self.h), "me_synchronize")

    # --- device memory on the ctx device (ctx stream) ---
    def malloc(self, nbytes: int) -> int:
        p = c_void_p()
        self.check(self.lib.me_malloc(self.h, ctypes.byref(p), int(nbytes)), "me_malloc")
        return p.value

    def free(self, ptr: int):
        self.check(self.lib.me_free(self.h, c_void_p(ptr)), "me_free")

    def h2d(self, dst: int, src: np.ndarray):
        src = np.ascontiguousarray(src)
        self.check(self.lib.me_memcpy_h2d(self.h, c_void_p(dst), src.ctypes.data, src.nbytes), "me_memcpy_h2d")

    def d2h(self, dst: np.ndarray, src: int):
        assert dst.flags.c_contiguous
        self.check(self.lib.me_memcpy_d2h(self.h, dst.ctypes.data, c_void_p(src), dst.nbytes), "me_memcpy_d2h")

    def d2d(self, dst: int, src: int, nbytes: int):
        self.check(self.lib.me_memcpy_d2d(self.h, c_void_p(dst), c_void_p(src), int(nbytes)), "me_memcpy_d2d")

    def copy_async(self, dst: int, src: int, nbytes: int):
        """hipMemcpyAsync (any direction) on the ctx stream."""
        self.check(self.lib.me_memcpy_async(self.h, c_void_p(dst), c_void_p(src), int(nbytes)), "me_memcpy_async")

    def host_alloc(self, nbytes: int) -> int:
        p = c_void_p()
        self.check(self.lib.me_host_alloc(self.h, ctypes.byref(p), int(nbytes)), "me_host_alloc")
        return p.value

    def host_free(self, ptr: int):
        self.check(self.lib.me_host_free(self.h, c_void_p(ptr)), "me_host_free")

    # --- kernel timing (HIP events on the ctx stream) ---
    def timing(self, on: bool = True, families=None):
        """Enable HIP-event timing of every kernel family, or only of `families` (names of KT)."""
        mask = 0
        if on:
            mask = 0xFFFF if families is None else sum(1 << KT[f] for f in families)
        self.check(self.lib.me_timing_enable(self.h, mask))

    def timing_sample(self, every: int):
        """Time every `every`-th launch of each timed family (me_timing_sample)."""
        self.check(self.lib.me_timing_sample(self.h, int(every)))

    def timing_reset(self):
        self.check(self.lib.me_timing_reset(self.h))

    def timing_read(self, family: str):
        n = c_long()
        ms = c_double()
        self.check(self.lib.me_timing_read(self.h, KT[family], ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value


class roctx_range:
    """roctx range around a block (rocprofv3 --marker-trace), through
    me_range_push / me_range_pop; a no-op unless `on`."""

    def __init__(self, name: str, on: bool = True):
        self.name, self.on = name.encode(), on

    def __enter__(self):
        if self.on:
            load_library().me_range_push(self.name)
        return self

    def __exit__(self, *a):
        if self.on:
            load_library().me_range_pop()


_default_ctx = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(int(os.environ.get("ME_DEVICE", os.environ.get("LOCAL_RANK", "0"))))
    return _default_ctx


def device_count() -> int:
    lib = load_library()
    n = c_int()
    lib.me_device_count(ctypes.byref(n))
    return n.value
