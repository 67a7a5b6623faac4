"""Optimisers mirroring include/MotionEstimation/optimisation/{optimisation,BundleAdjuster}.h.

* ``Optimiser`` — Optimiser<ScaleState, vector<pair<Mat,Mat>>> (optimisation.h:100-125,
  src/optimisation/optimisation.cpp:29-747): the MI stereo-scale LM.  Residual /
  normal-equation evaluations run in scale.hip; the scalar LM control is the
  reference's, in libme_hip.so's host code.
* ``BundleAdjuster`` — BundleAdjuster<4> (BundleAdjuster.h:182-476): windowed
  stereo BA; the whole Ceres-style LM runs on the device (ba.hip).
* Array-level helpers (``scale_*``, ``ba_*``) take the flattened problems of
  synthetic.py and are what the parity tests and bench.py call.
"""
from __future__ import annotations

import copy

import ctypes
from ctypes import POINTER, byref, c_double, c_int, c_int32, c_long, c_uint8, c_uint32
from dataclasses import dataclass, field
from enum import Enum, IntEnum

import numpy as np

from ._lib import (ALLREDUCE_FN, BAOptionsC, BAProblemC, BASummaryC, ME_DEVICE, ME_HOST, Context, OptimParamsC,
                   ScaleStateC, default_context)
from .feature_types import CamPose, WBA_Point
from .rotation_utils import Quat, StopCondition, exp_map_Quat, log_map_Quat


def _p(a, t=c_double):
    return None if a is None else a.ctypes.data_as(POINTER(t))


# ============================================================ ScaleState LM
class OptimType(IntEnum):
    GN = 0
    LM = 1


@dataclass
class OptimisationParams:
    """OptimisationParams (optimisation.h:22-32) with the same defaults."""
    type: OptimType = OptimType.LM
    minim: bool = True
    MAX_NB_ITER: int = 20
    v: float = 2.0
    tau: float = 1e-3
    mu: float = 1e-20
    abs_tol: float = 1e-4
    grad_tol: float = 1e-4
    incr_tol: float = 1e-3
    rel_tol: float = 1e-4
    alpha: float = 1.0
    weighting: bool = False

    @staticmethod
    def fixed_iterations(n: int = 10) -> "OptimisationParams":
        """The bench frame's scale LM (10 iterations, no time or
        tolerance stop): LM, MAX_NB_ITER = n, abs/grad/incr/rel tolerances 0.
        The reference loop still ends early by SMALL_INCREMENT once mu has
        grown until the step is exactly 0 (optimisation.cpp:694-697)."""
        return OptimisationParams(MAX_NB_ITER=n, abs_tol=0.0, grad_tol=0.0, incr_tol=0.0, rel_tol=0.0)

    def oracle_kw(self) -> dict:
        """The same parameters as keyword arguments of tests/oracle.py's optim_params."""
        return dict(type=int(self.type), minim=int(self.minim), max_nb_iter=int(self.MAX_NB_ITER), v=self.v,
                    tau=self.tau, mu=self.mu, abs_tol=self.abs_tol, grad_tol=self.grad_tol, incr_tol=self.incr_tol,
                    rel_tol=self.rel_tol, alpha=self.alpha, weighting=int(self.weighting))

    def to_c(self) -> OptimParamsC:
        p = OptimParamsC()
        p.type, p.minim, p.max_nb_iter = int(self.type), int(self.minim), int(self.MAX_NB_ITER)
        p.v, p.tau, p.mu = self.v, self.tau, self.mu
        p.abs_tol, p.grad_tol, p.incr_tol, p.rel_tol = self.abs_tol, self.grad_tol, self.incr_tol, self.rel_tol
        p.alpha, p.weighting = self.alpha, int(self.weighting)
        return p


def scale_struct(sp, keep: list, img_mem: int = ME_HOST, dev_imgs=None, dev_tracks: dict | None = None) -> ScaleStateC:
    """ScaleStateC from a flattened problem (synthetic.ScaleProblem or ScaleState.flatten()).
    dev_tracks: device pointers {X_left, X_right, tri_left, tri_right, last_left, last_right}
    for a window already resident in HBM (tracks_mem = ME_DEVICE)."""
    s = ScaleStateC()
    s.n_left, s.n_right = len(sp.X_left), len(sp.X_right)
    s.tracks_mem = ME_DEVICE if dev_tracks else ME_HOST
    if dev_tracks:
        for name, t in (("X_left", c_double), ("X_right", c_double), ("tri_left", c_uint8), ("tri_right", c_uint8),
                        ("last_left", c_uint32), ("last_right", c_uint32)):
            setattr(s, name, ctypes.cast(dev_tracks[name], POINTER(t)))
    for name in (() if dev_tracks else ("X_left", "X_right")):
        a = np.ascontiguousarray(getattr(sp, name), np.float64).reshape(-1)
        keep.append(a)
        setattr(s, name, _p(a))
    for name in (() if dev_tracks else ("tri_left", "tri_right")):
        a = np.ascontiguousarray(getattr(sp, name), np.uint8)
        keep.append(a)
        setattr(s, name, _p(a, c_uint8))
    for name in (() if dev_tracks else ("last_left", "last_right")):
        a = np.ascontiguousarray(getattr(sp, name), np.uint32)
        keep.append(a)
        setattr(s, name, _p(a, c_uint32))
    s.lframe = int(sp.lframe)
    s.K1[:] = [float(x) for x in np.asarray(sp.K1).ravel()]
    s.K2[:] = [float(x) for x in np.asarray(sp.K2).ravel()]
    s.q1[:] = [float(x) for x in sp.q1]
    s.t1[:] = [float(x) for x in sp.t1]
    s.q2[:] = [float(x) for x in sp.q2]
    s.t2[:] = [float(x) for x in sp.t2]
    s.scale, s.baseline, s.window_size = float(sp.scale), float(sp.baseline), int(sp.window_size)
    h, w = sp.imgL.shape
    if img_mem == ME_DEVICE:
        s.imgL, s.imgR = dev_imgs
    else:
        L = np.ascontiguousarray(sp.imgL, np.uint8)
        R = np.ascontiguousarray(sp.imgR, np.uint8)
        keep += [L, R]
        s.imgL, s.imgR = L.ctypes.data, R.ctypes.data
    s.stride, s.cols, s.rows = w, w, h
    s.bb_cols = getattr(sp, "bb_cols", None) or w
    s.bb_rows = getattr(sp, "bb_rows", None) or h
    mask = getattr(sp, "mask", None)
    if mask is not None:
        m = np.ascontiguousarray(mask, np.uint8)
        keep.append(m)
        s.mask, s.mask_len = _p(m, c_uint8), len(m)
    s.img_mem = img_mem
    return s


def scale_residuals(sp, weighting=False, ctx: Context | None = None) -> np.ndarray:
    ctx = ctx or default_context()
    keep = []
    s = scale_struct(sp, keep)
    res = np.zeros(len(sp.X_left) + len(sp.X_right) + 1)
    n = c_int()
    ctx.check(ctx.lib.me_scale_residuals(ctx.h, byref(s), int(weighting), _p(res), byref(n)), "me_scale_residuals")
    return res[:n.value]


def scale_normal_equations(sp, residuals, weighting=False, ctx: Context | None = None):
    ctx = ctx or default_context()
    keep = []
    s = scale_struct(sp, keep)
    r = np.ascontiguousarray(residuals, np.float64)
    JJ, e = c_double(), c_double()
    ctx.check(ctx.lib.me_scale_normal_equations(ctx.h, byref(s), int(weighting), _p(r), byref(JJ), byref(e)),
              "me_scale_normal_equations")
    return JJ.value, e.value


def scale_jacobian(sp, weighting=False, ctx: Context | None = None) -> float:
    ctx = ctx or default_context()
    keep = []
    s = scale_struct(sp, keep)
    JJ = c_double()
    ctx.check(ctx.lib.me_scale_jacobian(ctx.h, byref(s), int(weighting), byref(JJ)), "me_scale_jacobian")
    return JJ.value


class ScaleCall:
    """One me_scale_optimise call in three parts: the arguments built here,
    run() -- the C calls only, so a worker thread running it holds the GIL
    for a few bytecodes (ctypes releases it inside) -- and result()."""

    def __init__(self, sp, params: OptimisationParams | None = None, test=False, ctx: Context | None = None,
                 img_mem: int = ME_HOST, dev_imgs=None, dev_tracks: dict | None = None):
        self.ctx = ctx or default_context()
        self.keep = []
        self.s = scale_struct(sp, self.keep, img_mem, dev_imgs, dev_tracks)
        self.p = (params or OptimisationParams()).to_c()
        self.test = int(test)
        self.stop, self.it, self.nmi = c_int(), c_int(), c_long()
        self.trace = np.zeros(2 * 400)
        self.cnt = (c_long(), c_long(), c_long(), c_long())

    def run(self):
        c = self.ctx
        c.check(c.lib.me_scale_optimise(c.h, byref(self.s), byref(self.p), self.test, byref(self.stop),
                                        byref(self.it), _p(self.trace), 400, byref(self.nmi)), "me_scale_optimise")
        c.check(c.lib.me_scale_last_counters(c.h, *(byref(x) for x in self.cnt)), "me_scale_last_counters")

    def result(self) -> dict:
        n = min(self.it.value, 400)
        nres, nneq, nrej, nexe = (x.value for x in self.cnt)
        return dict(stop=StopCondition(self.stop.value), scale=self.s.scale, iterations=self.it.value,
                    trace=self.trace[:2 * n].reshape(-1, 2), track_evals=self.nmi.value, res_evals=nres,
                    neq_evals=nneq, rejections=nrej, executed_evals=nexe)


def scale_optimise(sp, params: OptimisationParams | None = None, test=False, ctx: Context | None = None,
                   img_mem: int = ME_HOST, dev_imgs=None, dev_tracks: dict | None = None) -> dict:
    call = ScaleCall(sp, params, test, ctx, img_mem, dev_imgs, dev_tracks)
    call.run()
    return call.result()


def scale_state_mi(sp, ctx: Context | None = None):
    """ScaleState::compute_residuals(m_obs) (optimisation.cpp:230-278): the MI
    of the stacked left-track patch pairs (the evident intent; the reference's
    stacking copies nothing, see include/me_hip.h).  Returns (mi, n_patches)."""
    ctx = ctx or default_context()
    keep = []
    s = scale_struct(sp, keep)
    mi, n = c_double(), c_int()
    ctx.check(ctx.lib.me_scale_state_mi(ctx.h, byref(s), byref(mi), byref(n)), "me_scale_state_mi")
    return mi.value, n.value


def scale_inliers(sp, threshold: float, weighting=False, ctx: Context | None = None) -> np.ndarray:
    ctx = ctx or default_context()
    keep = []
    s = scale_struct(sp, keep)
    cap = len(sp.X_left) + len(sp.X_right) + 1
    idx = np.zeros(cap, np.int32)
    n = c_int()
    ctx.check(ctx.lib.me_scale_inliers(ctx.h, byref(s), int(weighting), threshold, _p(idx, c_int), cap, byref(n)),
              "me_scale_inliers")
    return idx[:n.value]


class DeviceScaleTracks:
    """The track arrays of a ScaleState window resident in HBM (tracks_mem = ME_DEVICE)."""

    def __init__(self, sp, ctx: Context | None = None):
        self.ctx = ctx or default_context()
        self.d = {}
        for name, dt in (("X_left", np.float64), ("X_right", np.float64), ("tri_left", np.uint8),
                         ("tri_right", np.uint8), ("last_left", np.uint32), ("last_right", np.uint32)):
            a = np.ascontiguousarray(getattr(sp, name), dt)
            self.d[name] = self.ctx.malloc(max(a.nbytes, 16))
            if a.nbytes:
                self.ctx.h2d(self.d[name], a)

    def close(self):
        for v in self.d.values():
            self.ctx.free(v)
        self.d = {}


@dataclass
class ScaleState:
    """ScaleState (optimisation.h:76-98)."""
    pts: tuple = field(default_factory=lambda: ([], []))          # (vector<WBA_Ptf>, vector<WBA_Ptf>)
    K: tuple = field(default_factory=lambda: (np.eye(3), np.eye(3)))
    poses: tuple = field(default_factory=lambda: ([], []))        # (vector<CamPose_qd>, vector<CamPose_qd>)
    scale: float = 1.0
    baseline: float = 0.0
    window_size: int = 5
    nb_params: int = 1

    def update(self, dX):
        self.scale += float(np.asarray(dX).ravel()[0])


@dataclass
class _Flat:
    X_left: np.ndarray
    X_right: np.ndarray
    tri_left: np.ndarray
    tri_right: np.ndarray
    last_left: np.ndarray
    last_right: np.ndarray
    lframe: int
    K1: np.ndarray
    K2: np.ndarray
    q1: np.ndarray
    t1: np.ndarray
    q2: np.ndarray
    t2: np.ndarray
    scale: float
    baseline: float
    window_size: int
    imgL: np.ndarray
    imgR: np.ndarray
    bb_cols: int
    bb_rows: int
    mask: np.ndarray | None = None


class Optimiser:
    """Optimiser<ScaleState, std::vector<std::pair<cv::Mat,cv::Mat>>> (optimisation.h:100-125)."""

    def __init__(self, observations, params: OptimisationParams | None = None, ctx: Context | None = None):
        self.m_obs = [(np.ascontiguousarray(L, np.uint8), np.ascontiguousarray(R, np.uint8)) for L, R in observations]
        self.m_params = params or OptimisationParams()
        self.m_state: ScaleState | None = None
        self.m_mask = None
        self.ctx = ctx or default_context()

    def _flatten(self, st: ScaleState, use_mask=True) -> _Flat:
        def arr(tracks):
            X = np.array([t.get3DLocation() for t in tracks], np.float64).reshape(-1, 4)
            tri = np.array([t.isTriangulated() for t in tracks], np.uint8)
            last = np.array([t.getLastFrameIdx() for t in tracks], np.uint32)
            return X, tri, last

        XL, tl, ll = arr(st.pts[0])
        XR, tr, lr = arr(st.pts[1])
        f_idx = len(st.poses[0]) - 1
        L, R = self.m_obs[f_idx]
        pl, pr = st.poses[0][-1], st.poses[1][-1]
        return _Flat(XL, XR, tl, tr, ll, lr, st.poses[0][0].ID + len(st.poses[0]) - 1,
                     np.asarray(st.K[0], np.float64), np.asarray(st.K[1], np.float64),
                     pl.orientation.coeffs(), np.asarray(pl.position, np.float64),
                     pr.orientation.coeffs(), np.asarray(pr.position, np.float64),
                     st.scale, st.baseline, st.window_size, L, R,
                     self.m_obs[0][0].shape[1], self.m_obs[1][0].shape[0] if len(self.m_obs) > 1 else L.shape[0],
                     (np.asarray(self.m_mask, np.uint8) if (use_mask and self.m_mask is not None and
                                                            len(self.m_mask)) else None))

    def optimise(self, state: ScaleState, test: bool = False, mask=None) -> StopCondition:
        self.m_state = state
        self.m_mask = mask
        r = scale_optimise(self._flatten(state), self.m_params, test, self.ctx)
        state.scale = r["scale"]
        self.last_result = r
        return r["stop"]

    def compute_residuals(self, state: ScaleState) -> np.ndarray:
        return scale_residuals(self._flatten(state), self.m_params.weighting, self.ctx).reshape(-1, 1)

    def getJacobian(self) -> np.ndarray:
        return np.array([[scale_jacobian(self._flatten(self.m_state), self.m_params.weighting, self.ctx)]])

    def compute_inliers(self, threshold: float) -> list:
        return list(scale_inliers(self._flatten(self.m_state, use_mask=False), threshold, self.m_params.weighting,
                                  self.ctx))


# ============================================================ Bundle adjustment
class Status(Enum):
    UNINITIALISED = 0
    INITIALISED = 1
    SUCCESSFUL = 2
    FAILED = 3


@dataclass
class CalibrationParameters:
    """CalibrationParameters (BundleAdjuster.h:35-45)."""
    K: list
    feat_var: float
    baseline: float = 0.0
    compute_cov: bool = False


@dataclass
class SolverOptions:
    """The Ceres options BundleAdjuster<4>::optimise sets (BundleAdjuster.h:463-466) + Ceres defaults.

    max_solver_time_in_seconds = 1.0 is replaced by max_num_iterations (deterministic)."""
    max_num_iterations: int = 50
    function_tolerance: float = 1e-3
    gradient_tolerance: float = 1e-10
    parameter_tolerance: float = 1e-8
    initial_trust_region_radius: float = 1e4
    max_trust_region_radius: float = 1e16
    min_trust_region_radius: float = 1e-32
    min_lm_diagonal: float = 1e-6
    max_lm_diagonal: float = 1e32
    min_relative_decrease: float = 1e-3
    max_num_consecutive_invalid_steps: int = 5
    jacobi_scaling: bool = True

    def to_c(self) -> BAOptionsC:
        o = BAOptionsC()
        for k, v in self.__dict__.items():
            setattr(o, k, int(v) if isinstance(v, bool) else v)
        return o

    @staticmethod
    def fixed_iterations(n: int) -> "SolverOptions":
        """Fixed work per solve (bench): tolerances off, exactly n LM iterations."""
        return SolverOptions(max_num_iterations=n, function_tolerance=0.0, gradient_tolerance=0.0,
                             parameter_tolerance=0.0)


def ba_struct(bp, keep: list):
    p = BAProblemC()
    p.n_cams, p.n_pts, p.n_obs = len(bp.cams), len(bp.pts), len(bp.obs)
    cams = np.ascontiguousarray(bp.cams, np.float64).copy()
    pts = np.ascontiguousarray(bp.pts, np.float64).copy()
    obs = np.ascontiguousarray(bp.obs, np.float64)
    ci = np.ascontiguousarray(bp.cam_idx, np.int32)
    pi = np.ascontiguousarray(bp.pt_idx, np.int32)
    keep += [cams, pts, obs, ci, pi]
    p.cams, p.pts, p.obs = _p(cams), _p(pts), _p(obs)
    p.cam_idx, p.pt_idx = _p(ci, c_int32), _p(pi, c_int32)
    p.K0[:] = [float(x) for x in np.asarray(bp.K0).ravel()]
    p.K1[:] = [float(x) for x in np.asarray(bp.K1).ravel()]
    p.baseline, p.feat_var, p.fixed_frames = float(bp.baseline), float(bp.feat_var), int(bp.fixed_frames)
    p.obs_dim = int(getattr(bp, "obs_dim", 4))
    if p.obs_dim == 2:  # BundleAdjuster<2>: Observation<2> + camID
        cid = np.ascontiguousarray(bp.cam_id, np.int32)
        keep.append(cid)
        p.cam_id = _p(cid, c_int32)
    return p, cams, pts


def _summary(s: BASummaryC) -> dict:
    return dict(status=s.status, termination=s.termination, iterations=s.iterations,
                successful_steps=s.successful_steps, initial_cost=s.initial_cost, final_cost=s.final_cost)


def ba_solve(bp, options: SolverOptions | None = None, ctx: Context | None = None):
    """Returns (cams, pts, summary) after the device LM solve."""
    ctx = ctx or default_context()
    keep = []
    p, cams, pts = ba_struct(bp, keep)
    o = (options or SolverOptions()).to_c()
    s = BASummaryC()
    ctx.check(ctx.lib.me_ba_solve(ctx.h, byref(p), byref(o), byref(s)), "me_ba_solve")
    return cams, pts, _summary(s)


class Comm:
    """me_comm: the communicator of the landmark-sharded BA, one
    per rank.  ``Comm.rccl`` joins the ranks with native RCCL (all-reduces
    enqueued on the ctx stream, no host round trip); ``Comm.callback`` wraps
    an ``allreduce(dev_ptr, n)`` callable (n > 0 sum, n < 0 max), e.g. a
    host-staged gloo exchange or threads driving several contexts."""

    def __init__(self, ctx: Context, handle, keep=None):
        self.ctx, self.h, self._keep = ctx, handle, keep

    @staticmethod
    def unique_id() -> bytes:
        from ._lib import load_library
        buf = ctypes.create_string_buffer(128)
        rc = load_library().me_comm_unique_id(buf, 128)
        if rc != 0:
            from ._lib import MEError
            raise MEError(rc, "me_comm_unique_id (ncclGetUniqueId) failed")
        return buf.raw

    @classmethod
    def rccl(cls, ctx: Context, world: int, rank: int, uid: bytes) -> "Comm":
        h = ctypes.c_void_p()
        idb = ctypes.create_string_buffer(bytes(uid), 128)
        ctx.check(ctx.lib.me_comm_create_rccl(ctx.h, int(world), int(rank), idb, byref(h)), "me_comm_create_rccl")
        return cls(ctx, h)

    @classmethod
    def callback(cls, ctx: Context, world: int, rank: int, allreduce) -> "Comm":
        def _cb(ptr, n, user):
            try:
                allreduce(ctypes.cast(ptr, ctypes.c_void_p).value, int(n))
                return 0
            except Exception:  # pragma: no cover
                import traceback
                traceback.print_exc()
                return -1

        cb = ALLREDUCE_FN(_cb)
        h = ctypes.c_void_p()
        ctx.check(ctx.lib.me_comm_create_callback(ctx.h, int(world), int(rank), cb, None, byref(h)),
                  "me_comm_create_callback")
        return cls(ctx, h, keep=cb)

    def info(self) -> dict:
        w, r, nat = c_int(), c_int(), c_int()
        self.ctx.check(self.ctx.lib.me_comm_info(self.h, byref(w), byref(r), byref(nat)), "me_comm_info")
        return dict(world=w.value, rank=r.value, native=bool(nat.value))

    def exchange_us(self) -> dict:
        """The communicator's calibrated exchange costs (me_comm_exchange_us:
        measured at creation, max over the ranks), microseconds per all-reduce
        of the packed camera system and of the step scalars."""
        a, b = c_double(), c_double()
        self.ctx.check(self.ctx.lib.me_comm_exchange_us(self.h, byref(a), byref(b)), "me_comm_exchange_us")
        return {"system": a.value, "scalars": b.value}

    def calibrate(self, reps: int = 10) -> dict:
        """Re-measure the exchange costs (collective: every rank calls it)."""
        self.ctx.check(self.ctx.lib.me_comm_calibrate(self.h, int(reps)), "me_comm_calibrate")
        return self.exchange_us()

    def shard_worthwhile(self, n_obs: int) -> bool:
        """The landmark-count gate at this communicator's world and calibrated
        costs (me_ba_shard_worthwhile_comm): the same answer on every rank."""
        return bool(self.ctx.lib.me_ba_shard_worthwhile_comm(self.h, int(n_obs)))

    def allreduce(self, dev_ptr: int, n: int, op: str = "sum"):
        self.ctx.check(self.ctx.lib.me_comm_allreduce(self.h, ctypes.c_void_p(dev_ptr), int(n),
                                                      0 if op == "sum" else 1), "me_comm_allreduce")

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.me_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ba_solve_comm(bp_local, comm: "Comm", options: SolverOptions | None = None, ctx: Context | None = None):
    """Landmark-sharded solve of this rank's shard over a communicator (me_ba_solve_comm)."""
    ctx = ctx or comm.ctx
    keep = []
    p, cams, pts = ba_struct(bp_local, keep)
    o = (options or SolverOptions()).to_c()
    s = BASummaryC()
    ctx.check(ctx.lib.me_ba_solve_comm(ctx.h, byref(p), byref(o), comm.h, byref(s)), "me_ba_solve_comm")
    return cams, pts, _summary(s)


def ba_solve_sharded(bp_local, allreduce, options: SolverOptions | None = None, ctx: Context | None = None):
    """Landmark-sharded solve; ``allreduce(dev_ptr, n)`` sums n doubles in place (n < 0: max over |n|)."""
    ctx = ctx or default_context()
    keep = []
    p, cams, pts = ba_struct(bp_local, keep)
    o = (options or SolverOptions()).to_c()
    s = BASummaryC()

    def _cb(ptr, n, user):
        try:
            allreduce(ctypes.cast(ptr, ctypes.c_void_p).value, int(n))
            return 0
        except Exception:  # pragma: no cover
            import traceback
            traceback.print_exc()
            return -1

    cb = ALLREDUCE_FN(_cb)
    keep.append(cb)
    ctx.check(ctx.lib.me_ba_solve_sharded(ctx.h, byref(p), byref(o), cb, None, byref(s)), "me_ba_solve_sharded")
    return cams, pts, _summary(s)


class DeviceBAProblem:
    """A BA window resident in HBM (me_ba_problem.mem == ME_DEVICE): the five
    input arrays live on the ctx device; solves update cams/pts in place on
    the device.  `reset()` restores the starting parameters (device copy)."""

    def __init__(self, bp, ctx: Context | None = None):
        self.ctx = ctx or default_context()
        self.bp = bp
        arrays = dict(cams=np.ascontiguousarray(bp.cams, np.float64), pts=np.ascontiguousarray(bp.pts, np.float64),
                      obs=np.ascontiguousarray(bp.obs, np.float64),
                      cam_idx=np.ascontiguousarray(bp.cam_idx, np.int32),
                      pt_idx=np.ascontiguousarray(bp.pt_idx, np.int32))
        self.obs_dim = int(getattr(bp, "obs_dim", 4))
        names = ["obs", "cam_idx", "pt_idx"]
        if self.obs_dim == 2:
            arrays["cam_id"] = np.ascontiguousarray(bp.cam_id, np.int32)
            names.append("cam_id")
        self.nbytes = {k: v.nbytes for k, v in arrays.items()}
        self.d = {}
        self._blocks = []
        for k in names:
            self.d[k] = self.ctx.malloc(max(arrays[k].nbytes, 16))
            self._blocks.append(self.d[k])
            self.ctx.h2d(self.d[k], arrays[k])
        # cams | pts (solved in place) and cams0 | pts0 (the starting point) are
        # each one block, so reset() is a single device copy
        self._poff = (self.nbytes["cams"] + 255) & ~255
        self._pspan = self._poff + self.nbytes["pts"]
        for sfx in ("", "0"):
            base = self.ctx.malloc(max(self._pspan, 16))
            self._blocks.append(base)
            self.d["cams" + sfx], self.d["pts" + sfx] = base, base + self._poff
            self.ctx.h2d(self.d["cams" + sfx], arrays["cams"])
            self.ctx.h2d(self.d["pts" + sfx], arrays["pts"])
        self.n_cams, self.n_pts, self.n_obs = len(bp.cams), len(bp.pts), len(bp.obs)

    def reset(self):
        self.ctx.d2d(self.d["cams"], self.d["cams0"], self._pspan)

    def struct(self) -> BAProblemC:
        p = BAProblemC()
        p.n_cams, p.n_pts, p.n_obs = self.n_cams, self.n_pts, self.n_obs
        p.cams = ctypes.cast(self.d["cams"], POINTER(c_double))
        p.pts = ctypes.cast(self.d["pts"], POINTER(c_double))
        p.obs = ctypes.cast(self.d["obs"], POINTER(c_double))
        p.cam_idx = ctypes.cast(self.d["cam_idx"], POINTER(c_int32))
        p.pt_idx = ctypes.cast(self.d["pt_idx"], POINTER(c_int32))
        p.K0[:] = [float(x) for x in np.asarray(self.bp.K0).ravel()]
        p.K1[:] = [float(x) for x in np.asarray(self.bp.K1).ravel()]
        p.baseline, p.feat_var = float(self.bp.baseline), float(self.bp.feat_var)
        p.fixed_frames, p.mem = int(self.bp.fixed_frames), ME_DEVICE
        p.obs_dim = self.obs_dim
        if self.obs_dim == 2:
            p.cam_id = ctypes.cast(self.d["cam_id"], POINTER(c_int32))
        return p

    def solve(self, options: SolverOptions | None = None) -> dict:
        p = self.struct()
        o = (options or SolverOptions()).to_c()
        s = BASummaryC()
        self.ctx.check(self.ctx.lib.me_ba_solve(self.ctx.h, byref(p), byref(o), byref(s)), "me_ba_solve")
        return _summary(s)

    def solve_sharded(self, allreduce, options: SolverOptions | None = None) -> dict:
        """me_ba_solve_sharded on this device-resident shard (a rank's landmark
        range, see shard_landmarks): ``allreduce(dev_ptr, n)`` sums n doubles
        across ranks in place (n < 0: max)."""
        p = self.struct()
        o = (options or SolverOptions()).to_c()
        s = BASummaryC()

        def _cb(ptr, n, user):
            try:
                allreduce(ctypes.cast(ptr, ctypes.c_void_p).value, int(n))
                return 0
            except Exception:  # pragma: no cover
                import traceback
                traceback.print_exc()
                return -1

        cb = ALLREDUCE_FN(_cb)
        self.ctx.check(self.ctx.lib.me_ba_solve_sharded(self.ctx.h, byref(p), byref(o), cb, None, byref(s)),
                       "me_ba_solve_sharded")
        return _summary(s)

    def solve_comm(self, comm: "Comm", options: SolverOptions | None = None) -> dict:
        """me_ba_solve_comm on this device-resident shard."""
        p = self.struct()
        o = (options or SolverOptions()).to_c()
        s = BASummaryC()
        self.ctx.check(self.ctx.lib.me_ba_solve_comm(self.ctx.h, byref(p), byref(o), comm.h, byref(s)),
                       "me_ba_solve_comm")
        return _summary(s)

    def solve_async(self, options: SolverOptions | None = None) -> None:
        """Queue the whole solve on the ctx stream and return (me_ba_solve_async);
        wait() blocks on it and returns the summary."""
        self._async = (self.struct(), (options or SolverOptions()).to_c())
        p, o = self._async
        self.ctx.check(self.ctx.lib.me_ba_solve_async(self.ctx.h, byref(p), byref(o)), "me_ba_solve_async")

    def wait(self) -> dict:
        s = BASummaryC()
        self.ctx.check(self.ctx.lib.me_ba_wait(self.ctx.h, byref(s)), "me_ba_wait")
        self._async = None
        return _summary(s)

    def download(self):
        cams = np.zeros((self.n_cams, 6))
        pts = np.zeros((self.n_pts, 3))
        self.ctx.d2h(cams, self.d["cams"])
        self.ctx.d2h(pts, self.d["pts"])
        return cams, pts

    def close(self):
        for v in self._blocks:
            self.ctx.free(v)
        self.d = {}
        self._blocks = []


def shard_landmarks(bp, rank: int, world: int):
    """Contiguous landmark range of `rank`, balanced by observation count
    (SURVEY §8e).  Returns (local problem, (first, last+1) landmark range).
    Cameras are replicated; observations follow their landmark."""
    npt = len(bp.pts)
    pidx = np.asarray(bp.pt_idx)
    cum = np.concatenate([[0], np.cumsum(np.bincount(pidx, minlength=npt))])
    total = cum[-1]
    cuts = [0] + [int(np.searchsorted(cum, total * k / world, side="left")) for k in range(1, world)] + [npt]
    cuts = np.maximum.accumulate(np.clip(cuts, 0, npt))
    lo, hi = int(cuts[rank]), int(cuts[rank + 1])
    sel = (pidx >= lo) & (pidx < hi)
    local = copy.copy(bp)
    local.cams = np.array(bp.cams, np.float64, copy=True)
    local.pts = np.array(bp.pts[lo:hi], np.float64, copy=True)
    local.obs = np.ascontiguousarray(np.asarray(bp.obs)[sel])
    local.cam_idx = np.ascontiguousarray(np.asarray(bp.cam_idx)[sel], dtype=np.int32)
    local.pt_idx = np.ascontiguousarray(pidx[sel] - lo, dtype=np.int32)
    if getattr(bp, "obs_dim", 4) == 2:
        local.cam_id = np.ascontiguousarray(np.asarray(bp.cam_id)[sel], dtype=np.int32)
    return local, (lo, hi)


class ThreadAllReduce:
    """Exchange between contexts driven by threads of one process (several
    contexts on one device, or one per device without a process group):
    device buffer -> host, summed (or max) over the ranks at a barrier, -> device."""

    def __init__(self, world: int):
        import threading

        self.world = world
        self.barrier = threading.Barrier(world)
        self.bufs = [None] * world

    def callback(self, rank: int, ctx: Context):
        def _ar(ptr, n):
            ctx.synchronize()
            a = np.zeros(abs(n))
            ctx.check(ctx.lib.me_memcpy_d2h(ctx.h, a.ctypes.data, ptr, 8 * abs(n)))
            self.bufs[rank] = a
            self.barrier.wait()
            tot = np.max(self.bufs, axis=0) if n < 0 else np.sum(self.bufs, axis=0)
            self.barrier.wait()
            ctx.check(ctx.lib.me_memcpy_h2d(ctx.h, ptr, np.ascontiguousarray(tot).ctypes.data, 8 * abs(n)))
            ctx.synchronize()

        return _ar


class _DeviceDoubles:
    """Zero-copy view of a device buffer for torch.as_tensor (CUDA array interface)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (ptr, False), "version": 2,
                                         "strides": None}


def torch_allreduce(group=None):
    """all-reduce callback over torch.distributed on device buffers (RCCL on
    MI355X): sums n doubles in place, or takes the max for n < 0."""
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device())

    def _ar(ptr: int, n: int):
        t = torch.as_tensor(_DeviceDoubles(ptr, abs(n)), device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM if n > 0 else dist.ReduceOp.MAX, group=group)

    return _ar


def host_staged_allreduce(group=None):
    """all-reduce callback for a CPU backend (gloo): device buffer -> host,
    dist.all_reduce, -> device, ordered on torch's current stream (the
    solver's stream inside ba_solve_distributed)."""
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device())

    def _ar(ptr: int, n: int):
        t = torch.as_tensor(_DeviceDoubles(ptr, abs(n)), device=dev)
        h = t.cpu()  # synchronises the stream the solver enqueued on
        dist.all_reduce(h, op=dist.ReduceOp.SUM if n > 0 else dist.ReduceOp.MAX, group=group)
        t.copy_(h)

    return _ar


def rccl_comm(ctx: Context, group=None, key: str = "me_rccl_uid") -> "Comm":
    """A native RCCL me_comm over the ranks of a torch.distributed group: rank
    0 draws the id (ncclGetUniqueId), the others read it from the group's
    store; every rank then joins on its ctx device (one process per GPU)."""
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    store = dist.distributed_c10d._get_default_store()
    k = f"{key}/{getattr(rccl_comm, '_n', 0)}"
    rccl_comm._n = getattr(rccl_comm, "_n", 0) + 1
    if rank == 0:
        uid = Comm.unique_id()
        store.set(k, uid)
    else:
        uid = store.get(k)
    return Comm.rccl(ctx, world, rank, uid)


_GROUP_COMMS = {}


def group_comm(ctx: Context, group=None) -> "Comm":
    """The library communicator of a torch.distributed group on this ctx,
    created (collectively, calibrated) on first use and kept: native RCCL for
    the nccl backend, a host-staged callback for gloo."""
    import torch.distributed as dist

    key = (id(ctx), id(group))
    comm = _GROUP_COMMS.get(key)
    if comm is None or comm.ctx is not ctx:
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        if dist.get_backend(group) == "gloo":
            comm = Comm.callback(ctx, world, rank, host_staged_allreduce(group))
        else:
            comm = rccl_comm(ctx, group)
        _GROUP_COMMS[key] = comm
    return comm


def shard_worthwhile(n_obs: int, world: int, xch_us: float = 0.0) -> bool:
    """The landmark-count gate of the sharded solve (me_ba_shard_worthwhile,
    include/me_hip.h): True when splitting n_obs observations over `world`
    ranks is predicted to save more landmark-kernel time per LM iteration
    than its two all-reduces cost (xch_us per exchange; <= 0: the built-in
    estimate).  Host only."""
    from ._lib import load_library

    return bool(load_library().me_ba_shard_worthwhile(int(n_obs), int(world), float(xch_us)))


def ba_solve_distributed(bp, options: SolverOptions | None = None, ctx: Context | None = None, group=None,
                         allreduce=None, comm: "Comm | None" = None, shard="auto", xch_us: float = 0.0):
    """Landmark-sharded BA over torch.distributed: each rank holds
    the cameras and a contiguous, observation-balanced landmark range; the
    packed reduced camera system (S, b, gradient, LM scalars) is summed across
    ranks once per LM iteration after the Schur pass and the step scalars once
    after the point step; every rank solves the same camera step and updates
    its own landmarks.  The exchange is the library's native RCCL communicator
    for the nccl backend (``comm``, or one created here), host-staged through
    the group for gloo, or the given ``allreduce(dev_ptr, n)`` callback.

    ``shard``: "auto" applies the landmark-count gate (Comm.shard_worthwhile
    on the window's observation count, priced at the exchange costs the
    group's communicator measured when it was created -- the max over the
    ranks, so the same decision on every rank; the communicator is created
    once per group and kept, ``xch_us`` > 0 overrides the measurement) --
    but only when the caller passes neither ``comm`` nor ``allreduce``: an
    explicit exchange means "shard" (a caller's communicator is
    never silently ignored).  Below the gate -- or with shard=False -- every
    rank solves the whole window on its own GPU (replicated, no collective;
    the same deterministic solve on every rank) and returns its landmark range
    of the result.  True always shards.  Returns (cams, local pts, (lo, hi),
    summary); summary["sharded"] says which ran.  (Round 4 changed the
    default from True to "auto"; a caller that wants the old behaviour below
    the gate passes shard=True.)"""
    import torch
    import torch.distributed as dist

    ctx = ctx or default_context()
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    local, rng = shard_landmarks(bp, rank, world)
    own = False
    if shard == "auto":
        if comm is not None or allreduce is not None:
            shard = True
        elif xch_us > 0.0:
            shard = shard_worthwhile(len(bp.obs), world, xch_us)
        elif world <= 1:
            shard = False
        else:  # the group's calibrated communicator prices the exchanges
            comm = group_comm(ctx, group)
            shard = comm.shard_worthwhile(len(bp.obs))
    if not shard:
        cams, pts, summ = ba_solve(bp.copy(), options, ctx)
        summ = dict(summ, sharded=False)
        return cams, pts[rng[0]:rng[1]], rng, summ
    if comm is None:
        if allreduce is None and dist.get_backend(group) != "gloo":
            comm, own = rccl_comm(ctx, group), True
        else:
            comm = Comm.callback(ctx, world, rank, allreduce or host_staged_allreduce(group))
            own = True
    try:
        if comm.info()["native"]:
            cams, pts, summ = ba_solve_comm(local, comm, options, ctx)
        else:
            # host-staged: kernels and the exchange ordered on one torch stream
            # (the default stream's handle is 0, which me_set_stream reads as
            # "the ctx-owned stream", and that one is not ordered with torch's)
            stream = torch.cuda.Stream()
            with torch.cuda.stream(stream):
                ctx.set_stream(stream.cuda_stream)
                try:
                    cams, pts, summ = ba_solve_comm(local, comm, options, ctx)
                finally:
                    ctx.set_stream(None)
    finally:
        if own:
            comm.close()
    return cams, pts, rng, dict(summ, sharded=True)


def ba_cost(bp, ctx: Context | None = None) -> float:
    ctx = ctx or default_context()
    keep = []
    p, _, _ = ba_struct(bp, keep)
    c = c_double()
    ctx.check(ctx.lib.me_ba_cost(ctx.h, byref(p), byref(c)), "me_ba_cost")
    return c.value


def ba_evaluate(bp, ctx: Context | None = None):
    ctx = ctx or default_context()
    keep = []
    p, _, _ = ba_struct(bp, keep)
    no, D = len(bp.obs), p.obs_dim
    r = np.zeros(D * no)
    Jc = np.zeros(6 * D * no)
    Jp = np.zeros(3 * D * no)
    ctx.check(ctx.lib.me_ba_evaluate(ctx.h, byref(p), _p(r), _p(Jc), _p(Jp)), "me_ba_evaluate")
    return r.reshape(no, D), Jc.reshape(no, D, 6), Jp.reshape(no, D, 3)


def ba_covariance(bp, ctx: Context | None = None):
    """Pose covariance blocks (n_cams, 6, 6) at the problem's current parameters
    (BundleAdjuster<M>::extract_covariance, BundleAdjuster.h:478-528), or None
    when J^T J is not positive definite (Ceres: rank-deficient Jacobian)."""
    ctx = ctx or default_context()
    keep = []
    p, _, _ = ba_struct(bp, keep)
    cov = np.zeros(36 * len(bp.cams))
    ok = c_int(0)
    ctx.check(ctx.lib.me_ba_covariance(ctx.h, byref(p), _p(cov), byref(ok)), "me_ba_covariance")
    return cov.reshape(-1, 6, 6) if ok.value else None


def ba_reduced_system(bp, radius: float = 1e4, ctx: Context | None = None):
    ctx = ctx or default_context()
    keep = []
    p, _, _ = ba_struct(bp, keep)
    m = len(bp.cams) - min(max(bp.fixed_frames, 0), len(bp.cams))
    S = np.zeros((6 * m) * (6 * m))
    b = np.zeros(6 * m)
    ctx.check(ctx.lib.me_ba_reduced_system(ctx.h, byref(p), radius, _p(S), _p(b)), "me_ba_reduced_system")
    return S.reshape(6 * m, 6 * m), b


@dataclass
class _BAArrays:
    cams: np.ndarray
    pts: np.ndarray
    obs: np.ndarray
    cam_idx: np.ndarray
    pt_idx: np.ndarray
    K0: np.ndarray
    K1: np.ndarray
    baseline: float
    feat_var: float
    fixed_frames: int
    obs_dim: int = 4
    cam_id: np.ndarray = None


class BundleAdjuster:
    """BundleAdjuster<M> (windowed BA, BundleAdjuster.h:182-528): M = 4 stereo
    tracks (StereoReprojectionError), M = 2 mono tracks (Standard/StereoRight
    error by the track's camera ID).  ``M`` defaults from the track features."""

    def __init__(self, params: CalibrationParameters, cams: list, obs: list, ctx: Context | None = None,
                 options: SolverOptions | None = None, M: int | None = None):
        if M is None:
            M = 4
            if obs:
                f = obs[0].getFeat(0) if obs[0].getNbFeatures() else None
                M = 2 if f is not None and not hasattr(f[0], "__len__") else 4
        if M not in (2, 4):
            raise ValueError("BundleAdjuster<M>: M is 2 (mono) or 4 (stereo)")
        self.M = M
        self.m_camera_covs = []
        self.calib_params = params
        self.m_status = Status.UNINITIALISED
        self.m_camera_params = []
        self.m_point_params = []
        self.m_observations = []
        self.options = options or SolverOptions()
        self.ctx = ctx or default_context()
        self.initialiseParameters(cams)
        self.initialiseObservations(obs, cams[0].ID if cams else 0)

    def initialiseParameters(self, cams, pts=None):
        if self.m_status != Status.UNINITIALISED:
            print("[Bundle Adjuster] system should be uninitialised!")
            return
        self.m_point_params = [] if pts is None else [np.asarray(p, np.float64) for p in pts]
        self.m_camera_params = []
        for pose in cams:  # BundleAdjuster.h:306-309
            rv = log_map_Quat(pose.orientation)
            self.m_camera_params.append(np.array([pose.position[0], pose.position[1], pose.position[2],
                                                  rv[0], rv[1], rv[2]], np.float64))

    def initialiseObservations(self, observations, first_frame: int):
        if self.m_status != Status.UNINITIALISED or not self.m_camera_params:
            print("[Bundle Adjuster] system should be uninitialised and cameras not empty!")
            return
        init_points = not self.m_point_params
        self.m_observations = []
        for pt_idx, track in enumerate(observations):  # BundleAdjuster.h:359-374
            if init_points:
                p = track.get3DLocation()
                self.m_point_params.append(np.array([p[0] / p[3], p[1] / p[3], p[2] / p[3]]))
            for i in range(track.getNbFeatures()):  # <2>: BundleAdjuster.h:322-344
                fi = track.getFrameIdx(i)
                if fi - first_frame >= 0:
                    if self.M == 4:
                        (xl, yl), (xr, yr) = track.getFeat(i)
                        data = (xl, yl, xr, yr)
                    else:
                        x, y = track.getFeat(i)
                        data = (x, y)
                    self.m_observations.append((data, fi - first_frame, pt_idx, track.getCameraID()))
        self.m_status = Status.INITIALISED

    def _arrays(self, fixed: int) -> _BAArrays:
        K = self.calib_params.K
        K0 = np.asarray(K[0], np.float64)
        if self.M == 4 and len(K) < 2:
            raise ValueError("StereoReprojectionError reads K[1] (BundleAdjuster.h:163): give two intrinsics")
        K1 = np.asarray(K[1] if len(K) > 1 else K[0], np.float64)  # <2> uses K[0] only
        obs = np.array([o[0] for o in self.m_observations], np.float64).reshape(-1, self.M)
        ci = np.array([o[1] for o in self.m_observations], np.int32)
        pi = np.array([o[2] for o in self.m_observations], np.int32)
        cid = np.array([o[3] for o in self.m_observations], np.int32)
        if self.M == 2 and self.calib_params.baseline == 0:  # BundleAdjuster.h:389-390 (mutates calib)
            self.calib_params.baseline = 0.5
        return _BAArrays(np.array(self.m_camera_params).reshape(-1, 6), np.array(self.m_point_params).reshape(-1, 3),
                         obs, ci, pi, K0, K1, self.calib_params.baseline, self.calib_params.feat_var, fixed,
                         self.M, cid)

    def optimise(self, fixedFrames: int) -> Status:
        if self.m_status != Status.INITIALISED:
            print("[Bundle Adjuster] system should be initiliased to perform optimisation!")
            return self.m_status
        arrays = self._arrays(fixedFrames)
        cams, pts, summ = ba_solve(arrays, self.options, self.ctx)
        self.m_camera_params = [c.copy() for c in cams]
        self.m_point_params = [p.copy() for p in pts]
        self.summary = summ
        if self.calib_params.compute_cov:  # BundleAdjuster.h:424-425,471-472
            arrays.cams, arrays.pts = cams, pts
            cov = ba_covariance(arrays, self.ctx)
            if cov is None:
                print("[Bundle Adjuster] error computing the covariance matrix")
            else:
                self.m_camera_covs = [c.copy() for c in cov]
        self.m_status = Status.SUCCESSFUL if summ["status"] == 2 else Status.FAILED
        return self.m_status

    def getPosesCovariance(self):
        return [c.copy() for c in self.m_camera_covs]

    def getPointsCovariance(self):  # never filled by the reference (BundleAdjuster.h:505-506,519-526)
        return []

    def getPoints(self):
        return [p.copy() for p in self.m_point_params]

    def getCameraPoses(self):
        out = []
        for idx, c in enumerate(self.m_camera_params):  # IDs renumbered 0..W-1 (BundleAdjuster.h:231-236)
            out.append(CamPose(idx, Quat(*exp_map_Quat(c[3:]).coeffs()), np.array(c[:3])))
        return out

    def getNbPoints(self):
        return len(self.m_point_params)

    def getNbCameras(self):
        return len(self.m_camera_params)

    def getNbObservations(self):
        return len(self.m_observations)

    def getStatus(self):
        return self.m_status
