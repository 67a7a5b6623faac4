"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference path (oracle/*.cpp, parity
unpinned: see oracle/oracle.h).  Only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may use it, and only as the checker.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_float, c_int, c_int32, c_long, c_uint8, c_uint32, c_void_p

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")


class OScaleState(ctypes.Structure):
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
    ]


class OOptimParams(ctypes.Structure):
    _fields_ = [
        ("type", c_int), ("minim", c_int), ("max_nb_iter", c_int),
        ("v", c_double), ("tau", c_double), ("mu", c_double), ("abs_tol", c_double), ("grad_tol", c_double),
        ("incr_tol", c_double), ("rel_tol", c_double), ("alpha", c_double),
        ("weighting", c_int),
    ]


class OBAProblem(ctypes.Structure):
    _fields_ = [
        ("n_cams", c_int), ("n_pts", c_int), ("n_obs", c_int),
        ("cams", POINTER(c_double)), ("pts", POINTER(c_double)), ("obs", POINTER(c_double)),
        ("cam_idx", POINTER(c_int32)), ("pt_idx", POINTER(c_int32)),
        ("K0", c_double * 9), ("K1", c_double * 9),
        ("baseline", c_double), ("feat_var", c_double),
        ("fixed_frames", c_int),
        ("obs_dim", c_int), ("cam_id", POINTER(c_int32)),
    ]


class OBAOptions(ctypes.Structure):
    _fields_ = [
        ("max_num_iterations", c_int),
        ("function_tolerance", c_double), ("gradient_tolerance", c_double), ("parameter_tolerance", c_double),
        ("initial_trust_region_radius", c_double), ("max_trust_region_radius", c_double),
        ("min_trust_region_radius", c_double),
        ("min_lm_diagonal", c_double), ("max_lm_diagonal", c_double), ("min_relative_decrease", c_double),
        ("max_num_consecutive_invalid_steps", c_int),
        ("jacobi_scaling", c_int),
    ]


class OBASummary(ctypes.Structure):
    _fields_ = [
        ("status", c_int), ("termination", c_int), ("iterations", c_int), ("successful_steps", c_int),
        ("initial_cost", c_double), ("final_cost", c_double),
    ]


class OKLTParams(ctypes.Structure):
    _fields_ = [("win", c_int), ("max_level", c_int), ("max_iters", c_int), ("eps", c_double),
                ("min_eig", c_double)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        P = POINTER
        L.oracle_mutual_information.restype = c_float
        L.oracle_mutual_information.argtypes = [c_void_p, c_int, c_void_p, c_int, c_int, c_int]
        L.oracle_entropy.restype = c_float
        L.oracle_entropy.argtypes = [c_void_p, c_int, c_int, c_int]
        for f in (L.oracle_compare_pc, L.oracle_ccoeff_normed):
            f.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]
        L.oracle_quantise.argtypes = [c_void_p, c_int, c_int, c_int, c_int, c_int]
        L.oracle_pose_mul_cov.argtypes = [c_void_p] * 6 + [c_int] + [c_void_p] * 3
        L.oracle_pose_invert_cov.argtypes = [c_void_p] * 3
        L.oracle_pose_scale_cov.argtypes = [c_void_p, c_void_p, c_double, c_double]
        L.oracle_mi_histograms.argtypes = [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                           c_void_p]
        L.oracle_mi_scores.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                       c_void_p]
        L.oracle_log2f.restype = c_float
        L.oracle_log2f.argtypes = [c_float]
        L.oracle_log2f_mismatches.restype = c_long
        L.oracle_log2f_mismatches.argtypes = [c_uint32, c_uint32]
        L.oracle_optim_default_params.argtypes = [P(OOptimParams)]
        L.oracle_scale_residuals.argtypes = [P(OScaleState), c_int, P(c_double)]
        L.oracle_scale_normal_equations.argtypes = [P(OScaleState), c_int, P(c_double), P(c_double), P(c_double)]
        L.oracle_scale_jacobian.argtypes = [P(OScaleState), c_int, P(c_double)]
        L.oracle_scale_optimise.argtypes = [P(OScaleState), P(OOptimParams), c_int, P(c_int), P(c_double), c_int,
                                            P(c_long)]
        L.oracle_scale_inliers.argtypes = [P(OScaleState), c_double, P(c_int), c_int]
        L.oracle_scale_state_mi.argtypes = [P(OScaleState), P(c_double), P(c_int)]
        L.oracle_scale_counters.argtypes = [P(c_long)]
        L.oracle_ba_default_options.argtypes = [P(OBAOptions)]
        L.oracle_ba_evaluate.argtypes = [P(OBAProblem), P(c_double), P(c_double), P(c_double)]
        L.oracle_ba_cost.restype = c_double
        L.oracle_ba_cost.argtypes = [P(OBAProblem)]
        L.oracle_ba_solve.argtypes = [P(OBAProblem), P(OBAOptions), P(OBASummary), P(c_double), c_int]
        L.oracle_ba_reduced_system.argtypes = [P(OBAProblem), c_double, P(c_double), P(c_double)]
        L.oracle_ba_covariance.argtypes = [P(OBAProblem), P(c_double)]
        L.oracle_ba_reduced_system_ex.argtypes = [P(OBAProblem), c_double, c_int, P(c_double), P(c_double)]
        L.oracle_nms_scanline3x3.argtypes = [P(c_double), c_int, c_int, P(c_uint8), P(c_double), c_int]
        L.oracle_klt_track.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, P(c_float), P(c_float), P(c_uint8),
                                       c_int, P(OKLTParams)]
        L.oracle_pyr_down.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int]
        L.oracle_scharr.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]
        _lib = L
    return _lib


def _p(a, t=c_double):
    return None if a is None else a.ctypes.data_as(POINTER(t))


# ----------------------------------------------------------------- MI
def mutual_information(L: np.ndarray, R: np.ndarray) -> float:
    L = np.ascontiguousarray(L, np.uint8)
    R = np.ascontiguousarray(R, np.uint8)
    h, w = L.shape
    return float(np.float32(lib().oracle_mutual_information(L.ctypes.data, w, R.ctypes.data, w, w, h)))


def entropy(img: np.ndarray) -> float:
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    return float(np.float32(lib().oracle_entropy(img.ctypes.data, w, w, h)))


def _pairs(A, B):
    A = np.ascontiguousarray(A, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    if A.ndim == 2:
        A, B = A[None], B[None]
    return A, B


def compare_pc(A, B):
    A, B = _pairs(A, B)
    out = np.zeros(len(A), np.float32)
    lib().oracle_compare_pc(A.ctypes.data, B.ctypes.data, len(A), A.shape[1], A.shape[2], out.ctypes.data)
    return out


def ccoeff_normed(A, B):
    A, B = _pairs(A, B)
    out = np.zeros(len(A), np.float32)
    lib().oracle_ccoeff_normed(A.ctypes.data, B.ctypes.data, len(A), A.shape[1], A.shape[2], out.ctypes.data)
    return out


def quantise(img, lo, hi):
    img = np.array(img, np.uint8, copy=True, order="C")
    h, w = img.shape
    lib().oracle_quantise(img.ctypes.data, w, w, h, lo, hi)
    return img


def _d(a):
    return np.array(a, np.float64, copy=True, order="C")


def pose_mul_cov(q1, t1, c1, q2, t2, c2, reverse=False):
    """(q3, t3, cov3) of poseMultiplicationWithCovariance[Reverse] (feature_types.cpp:171-219)."""
    a = [_d(x) for x in (q1, t1, c1, q2, t2, c2)]
    q3, t3, c3 = np.zeros(4), np.zeros(3), np.zeros(36)
    lib().oracle_pose_mul_cov(*[x.ctypes.data for x in a], int(reverse), q3.ctypes.data, t3.ctypes.data,
                              c3.ctypes.data)
    return q3, t3, c3.reshape(6, 6)


def pose_invert_cov(q, t, c):
    q, t, c = _d(q), _d(t), _d(c)
    lib().oracle_pose_invert_cov(q.ctypes.data, t.ctypes.data, c.ctypes.data)
    return q, t, c.reshape(6, 6)


def pose_scale_cov(t, c, s, var):
    t, c = _d(t), _d(c)
    lib().oracle_pose_scale_cov(t.ctypes.data, c.ctypes.data, float(s), float(var))
    return t, c.reshape(6, 6)


def histograms(L, R):
    L = np.ascontiguousarray(L, np.uint8)
    R = np.ascontiguousarray(R, np.uint8)
    h, w = L.shape
    hl = np.zeros(20, np.int32)
    hr = np.zeros(20, np.int32)
    hj = np.zeros(400, np.int32)
    lib().oracle_mi_histograms(L.ctypes.data, w, R.ctypes.data, w, w, h, hl.ctypes.data, hr.ctypes.data,
                               hj.ctypes.data)
    return hl, hr, hj.reshape(20, 20)


def mi_scores(imgL, imgR, xyL, xyR, pw, ph):
    imgL = np.ascontiguousarray(imgL, np.uint8)
    imgR = np.ascontiguousarray(imgR, np.uint8)
    xyL = np.ascontiguousarray(xyL, np.int32)
    xyR = np.ascontiguousarray(xyR, np.int32)
    out = np.zeros(len(xyL), np.float32)
    lib().oracle_mi_scores(imgL.ctypes.data, imgL.shape[1], imgR.ctypes.data, imgR.shape[1], xyL.ctypes.data,
                           xyR.ctypes.data, len(xyL), pw, ph, out.ctypes.data)
    return out


def log2f_mismatches(lo: int, hi: int) -> int:
    return int(lib().oracle_log2f_mismatches(lo, hi))


# ----------------------------------------------------------------- ScaleState
def scale_state(sp, keep=None):
    """OScaleState from a synthetic.ScaleProblem (arrays kept alive in `keep`)."""
    if keep is None:
        keep = []
    s = OScaleState()
    s.n_left = len(sp.X_left)
    s.n_right = len(sp.X_right)
    for name in ("X_left", "X_right"):
        a = np.ascontiguousarray(getattr(sp, name), np.float64).reshape(-1)
        keep.append(a)
        setattr(s, name, _p(a))
    for name in ("tri_left", "tri_right"):
        a = np.ascontiguousarray(getattr(sp, name), np.uint8)
        keep.append(a)
        setattr(s, name, _p(a, c_uint8))
    for name in ("last_left", "last_right"):
        a = np.ascontiguousarray(getattr(sp, name), np.uint32)
        keep.append(a)
        setattr(s, name, _p(a, c_uint32))
    s.lframe = sp.lframe
    s.K1[:] = list(np.asarray(sp.K1, np.float64).ravel())
    s.K2[:] = list(np.asarray(sp.K2, np.float64).ravel())
    s.q1[:] = list(sp.q1)
    s.t1[:] = list(sp.t1)
    s.q2[:] = list(sp.q2)
    s.t2[:] = list(sp.t2)
    s.scale = sp.scale
    s.baseline = sp.baseline
    s.window_size = sp.window_size
    L = np.ascontiguousarray(sp.imgL, np.uint8)
    R = np.ascontiguousarray(sp.imgR, np.uint8)
    keep += [L, R]
    s.imgL = L.ctypes.data
    s.imgR = R.ctypes.data
    s.stride = L.shape[1]
    s.cols = L.shape[1]
    s.rows = L.shape[0]
    s.bb_cols = L.shape[1]
    s.bb_rows = L.shape[0]
    if sp.mask is not None:
        m = np.ascontiguousarray(sp.mask, np.uint8)
        keep.append(m)
        s.mask = _p(m, c_uint8)
        s.mask_len = len(m)
    return s, keep


def scale_residuals(sp, weighting=0):
    s, keep = scale_state(sp)
    res = np.zeros(len(sp.X_left) + len(sp.X_right) + 1)
    n = lib().oracle_scale_residuals(ctypes.byref(s), weighting, _p(res))
    if n < 0:
        raise RuntimeError(f"oracle_scale_residuals failed {n}")
    return res[:n]


def scale_normal_equations(sp, res, weighting=0):
    s, keep = scale_state(sp)
    res = np.ascontiguousarray(res, np.float64)
    JJ, e = c_double(), c_double()
    rc = lib().oracle_scale_normal_equations(ctypes.byref(s), weighting, _p(res), ctypes.byref(JJ), ctypes.byref(e))
    if rc < 0:
        raise RuntimeError(f"oracle_scale_normal_equations failed {rc}")
    return JJ.value, e.value


def scale_jacobian(sp, weighting=0):
    s, keep = scale_state(sp)
    JJ = c_double()
    rc = lib().oracle_scale_jacobian(ctypes.byref(s), weighting, ctypes.byref(JJ))
    if rc < 0:
        raise RuntimeError(f"oracle_scale_jacobian failed {rc}")
    return JJ.value


def optim_params(**kw):
    p = OOptimParams()
    lib().oracle_optim_default_params(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def scale_optimise(sp, test=0, **kw):
    s, keep = scale_state(sp)
    p = optim_params(**kw)
    it = c_int()
    trace = np.zeros(2 * 400)
    nmi = c_long()
    stop = lib().oracle_scale_optimise(ctypes.byref(s), ctypes.byref(p), test, ctypes.byref(it), _p(trace), 400,
                                       ctypes.byref(nmi))
    if stop < 0:
        raise RuntimeError(f"oracle_scale_optimise failed {stop}")
    cnt = (c_long * 3)()
    lib().oracle_scale_counters(cnt)
    return dict(stop=stop, scale=s.scale, iterations=it.value, trace=trace[:2 * min(it.value, 400)].reshape(-1, 2),
                mi_evals=nmi.value, res_evals=cnt[0], neq_evals=cnt[1], rejections=cnt[2])


def scale_state_mi(sp):
    """ScaleState::compute_residuals (optimisation.cpp:230-278), evident intent."""
    s, keep = scale_state(sp)
    out, n = c_double(), c_int()
    rc = lib().oracle_scale_state_mi(ctypes.byref(s), ctypes.byref(out), ctypes.byref(n))
    if rc < 0:
        raise RuntimeError(f"oracle_scale_state_mi failed {rc}")
    return out.value, n.value


def scale_inliers(sp, threshold):
    s, keep = scale_state(sp)
    idx = np.zeros(len(sp.X_left) + len(sp.X_right) + 1, np.int32)
    n = lib().oracle_scale_inliers(ctypes.byref(s), threshold, _p(idx, c_int), len(idx))
    return idx[:n]


# ----------------------------------------------------------------- BA
def ba_struct(bp, keep=None):
    if keep is None:
        keep = []
    p = OBAProblem()
    p.n_cams = len(bp.cams)
    p.n_pts = len(bp.pts)
    p.n_obs = len(bp.obs)
    cams = np.array(bp.cams, np.float64, order="C", copy=True)
    pts = np.array(bp.pts, np.float64, order="C", copy=True)
    obs = np.ascontiguousarray(bp.obs, np.float64)
    ci = np.ascontiguousarray(bp.cam_idx, np.int32)
    pi = np.ascontiguousarray(bp.pt_idx, np.int32)
    keep += [cams, pts, obs, ci, pi]
    p.cams, p.pts, p.obs = _p(cams), _p(pts), _p(obs)
    p.cam_idx, p.pt_idx = _p(ci, c_int32), _p(pi, c_int32)
    p.K0[:] = list(np.asarray(bp.K0, np.float64).ravel())
    p.K1[:] = list(np.asarray(bp.K1, np.float64).ravel())
    p.baseline = bp.baseline
    p.feat_var = bp.feat_var
    p.fixed_frames = bp.fixed_frames
    p.obs_dim = int(getattr(bp, "obs_dim", 4))
    if p.obs_dim == 2:
        cid = np.ascontiguousarray(bp.cam_id, np.int32)
        keep.append(cid)
        p.cam_id = _p(cid, c_int32)
    return p, keep, cams, pts


def ba_options(**kw):
    o = OBAOptions()
    lib().oracle_ba_default_options(ctypes.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def ba_evaluate(bp):
    p, keep, _, _ = ba_struct(bp)
    no, D = len(bp.obs), p.obs_dim
    r = np.zeros(D * no)
    Jc = np.zeros(6 * D * no)
    Jp = np.zeros(3 * D * no)
    lib().oracle_ba_evaluate(ctypes.byref(p), _p(r), _p(Jc), _p(Jp))
    return r.reshape(no, D), Jc.reshape(no, D, 6), Jp.reshape(no, D, 3)


def ba_covariance(bp):
    """Pose covariance blocks (n_cams, 6, 6) at the problem's parameters, or None (not PD)."""
    p, keep, _, _ = ba_struct(bp)
    cov = np.zeros(36 * len(bp.cams))
    ok = lib().oracle_ba_covariance(ctypes.byref(p), _p(cov))
    return cov.reshape(-1, 6, 6) if ok else None


def ba_cost(bp):
    p, keep, _, _ = ba_struct(bp)
    return lib().oracle_ba_cost(ctypes.byref(p))


def ba_solve(bp, **kw):
    p, keep, cams, pts = ba_struct(bp)
    o = ba_options(**kw)
    s = OBASummary()
    trace = np.zeros(200)
    lib().oracle_ba_solve(ctypes.byref(p), ctypes.byref(o), ctypes.byref(s), _p(trace), 200)
    return cams, pts, dict(status=s.status, termination=s.termination, iterations=s.iterations,
                           successful_steps=s.successful_steps, initial_cost=s.initial_cost,
                           final_cost=s.final_cost)


def ba_reduced_system(bp, radius=1e4):
    p, keep, _, _ = ba_struct(bp)
    m = len(bp.cams) - min(max(bp.fixed_frames, 0), len(bp.cams))
    n = 6 * m
    S = np.zeros(n * n)
    b = np.zeros(n)
    rc = lib().oracle_ba_reduced_system(ctypes.byref(p), radius, _p(S), _p(b))
    return S.reshape(n, n), b, rc


def ba_reduced_system_unscaled(bp, radius=1e300):
    """S, b without Jacobi scaling (additive over landmark shards)."""
    p, keep, _, _ = ba_struct(bp)
    m = len(bp.cams) - min(max(bp.fixed_frames, 0), len(bp.cams))
    n = 6 * m
    S = np.zeros(n * n)
    b = np.zeros(n)
    rc = lib().oracle_ba_reduced_system_ex(ctypes.byref(p), radius, 0, _p(S), _p(b))
    return S.reshape(n, n), b, rc


# ----------------------------------------------------------------- NMS / KLT
def nms(resp: np.ndarray):
    resp = np.ascontiguousarray(resp, np.float64)
    h, w = resp.shape
    mask = np.zeros((h, w), np.uint8)
    cap = h * w // 2 + 1
    mx = np.zeros(2 * cap)
    n = lib().oracle_nms_scanline3x3(_p(resp), w, h, _p(mask, c_uint8), _p(mx), cap)
    return mx[:2 * n].reshape(n, 2), mask


def klt_params(win=21, max_level=3, max_iters=30, eps=0.01, min_eig=1e-4):
    k = OKLTParams()
    k.win, k.max_level, k.max_iters, k.eps, k.min_eig = win, max_level, max_iters, eps, min_eig
    return k


def klt(prev, nxt, pts, **kw):
    prev = np.ascontiguousarray(prev, np.uint8)
    nxt = np.ascontiguousarray(nxt, np.uint8)
    pts = np.ascontiguousarray(pts, np.float32)
    h, w = prev.shape
    out = np.zeros_like(pts)
    st = np.zeros(len(pts), np.uint8)
    kp = klt_params(**kw)
    lib().oracle_klt_track(prev.ctypes.data, nxt.ctypes.data, w, h, w, _p(pts, c_float), _p(out, c_float),
                           _p(st, c_uint8), len(pts), ctypes.byref(kp))
    return out, st


def pyr_down(img):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    dh, dw = (h + 1) // 2, (w + 1) // 2
    out = np.zeros((dh, dw), np.uint8)
    lib().oracle_pyr_down(img.ctypes.data, w, h, w, out.ctypes.data, dw, dh, dw)
    return out


def scharr(img):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    dx = np.zeros((h, w), np.int16)
    dy = np.zeros((h, w), np.int16)
    lib().oracle_scharr(img.ctypes.data, w, h, w, dx.ctypes.data, dy.ctypes.data)
    return dx, dy


# ----------------------------------------------------------------- stereo VO
class OVOParams(ctypes.Structure):
    _fields_ = [("method", c_int), ("e1", c_double), ("e2", c_double), ("e3", c_double), ("e4", c_double),
                ("max_iter", c_int), ("ransac", c_int), ("n_ransac", c_int), ("inlier_threshold", c_double),
                ("baseline", c_double), ("fu1", c_double), ("fv1", c_double), ("fu2", c_double), ("fv2", c_double),
                ("cu1", c_double), ("cu2", c_double), ("cv1", c_double), ("cv2", c_double)]


def libc_rand_seq(seed: int, count: int) -> np.ndarray:
    """`count` values of glibc rand() after srand(seed) (the reference's sampler, :150)."""
    libc = ctypes.CDLL("libc.so.6")
    libc.rand.restype = c_int
    libc.srand(ctypes.c_uint(seed))
    return np.array([libc.rand() for _ in range(count)], np.int32)


def vo_process(matches, params: dict, rand_seq=None, init=None, max_outer=10000):
    """oracle_vo_process: returns (rc, motion (4,4), inliers).  rc 1/0 = process()
    result, -2 = the reference would never leave optimize(), -3 = rand_seq too short."""
    L = lib()
    if not getattr(L, "_vo_decl", False):
        L.oracle_vo_process.argtypes = [c_void_p, c_int, c_void_p, POINTER(OVOParams), c_void_p, c_int, c_void_p,
                                        c_void_p, POINTER(c_int), c_int]
        L.oracle_vo_process.restype = c_int
        L._vo_decl = True
    d = dict(method=0, e1=1e-3, e2=1e-12, e3=1e-12, e4=1e-15, max_iter=100, ransac=1, n_ransac=200,
             inlier_threshold=2.0, baseline=1.0, fu1=1.0, fv1=1.0, fu2=1.0, fv2=1.0, cu1=0.0, cu2=0.0, cv1=0.0,
             cv2=0.0)
    d.update({k: v for k, v in params.items() if k in d})
    p = OVOParams(**{k: (int(v) if isinstance(v, bool) else v) for k, v in d.items()})
    m = np.ascontiguousarray(matches, np.float32).reshape(-1, 8)
    if rand_seq is None:
        rand_seq = libc_rand_seq(1, 8 * d["n_ransac"] + 64)
    rs = np.ascontiguousarray(rand_seq, np.int32)
    ini = None if init is None else np.ascontiguousarray(init, np.float64)
    motion = np.zeros(16)
    inl = np.zeros(max(len(m), 1), np.int32)
    nin = c_int(0)
    rc = L.oracle_vo_process(m.ctypes.data, len(m), None if ini is None else ini.ctypes.data, ctypes.byref(p),
                             rs.ctypes.data, len(rs), motion.ctypes.data, inl.ctypes.data, ctypes.byref(nin),
                             max_outer)
    return rc, motion.reshape(4, 4), inl[:nin.value].copy()


# ------------------------------------------------------------------ Mono VO (oracle/mono.cpp)
class OMonoParams(ctypes.Structure):
    _fields_ = [("fu", c_double), ("fv", c_double), ("cu", c_double), ("cv", c_double), ("prob", c_double),
                ("inlier_threshold", c_double), ("ransac", c_int)]


def _mono_decl(L):
    if getattr(L, "_mono_decl", False):
        return
    L.oracle_mono_vo_process.argtypes = [c_void_p, c_void_p, c_int, POINTER(OMonoParams), c_void_p, c_void_p,
                                         c_void_p, POINTER(c_int), c_void_p]
    L.oracle_mono_vo_process.restype = c_int
    L.oracle_five_point.argtypes = [c_void_p, c_void_p, c_void_p]
    L.oracle_five_point.restype = c_int
    L.oracle_sampson.argtypes = [c_void_p, c_void_p, c_void_p]
    L.oracle_sampson.restype = c_float
    L.oracle_cv_rng_subsets.argtypes = [c_int, c_int, c_void_p]
    L.oracle_cv_rng_subsets.restype = c_int
    L._mono_decl = True


def mono_params(**kw) -> OMonoParams:
    d = dict(fu=1.0, fv=1.0, cu=0.0, cv=0.0, prob=0.99, inlier_threshold=2.0, ransac=1)
    d.update(kw)
    return OMonoParams(**{k: (int(v) if k == "ransac" else float(v)) for k, v in d.items()})


def mono_vo_process(f1, f2, **params):
    """oracle_mono_vo_process: (ok, Rt (4,4), E (3,3), inlier indices, stats (iters, best count, pose branch))."""
    L = lib()
    _mono_decl(L)
    a = np.ascontiguousarray(f1, np.float32).reshape(-1, 2)
    b = np.ascontiguousarray(f2, np.float32).reshape(-1, 2)
    n = len(a)
    Rt, E = np.zeros(16), np.zeros(9)
    inl = np.zeros(max(n, 1), np.int32)
    ni = c_int(0)
    st = np.zeros(3, np.int32)
    p = mono_params(**params)
    ok = L.oracle_mono_vo_process(a.ctypes.data, b.ctypes.data, n, ctypes.byref(p), Rt.ctypes.data, E.ctypes.data,
                                  inl.ctypes.data, ctypes.byref(ni), st.ctypes.data)
    return ok, Rt.reshape(4, 4), E.reshape(3, 3), inl[:ni.value].copy(), st


def five_point(x1, x2):
    L = lib()
    _mono_decl(L)
    a = np.ascontiguousarray(x1, np.float64).reshape(5, 2)
    b = np.ascontiguousarray(x2, np.float64).reshape(5, 2)
    E = np.zeros(90)
    n = L.oracle_five_point(a.ctypes.data, b.ctypes.data, E.ctypes.data)
    return E[:9 * n].reshape(n, 3, 3)


def cv_rng_subsets(count: int, n_sets: int) -> np.ndarray:
    L = lib()
    _mono_decl(L)
    idx = np.zeros(5 * n_sets, np.int32)
    k = L.oracle_cv_rng_subsets(count, n_sets, idx.ctypes.data)
    return idx[:5 * k].reshape(k, 5)
