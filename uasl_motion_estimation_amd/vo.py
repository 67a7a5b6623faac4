"""Frame-to-frame stereo visual odometry on MI355X (vo.hip).

Mirror of me::StereoVisualOdometry (include/MotionEstimation/vo/StereoVisualOdometry.h:18-95,
src/vo/StereoVisualOdometry.cpp:34-342) and me::VisualOdometry::parameters
(include/MotionEstimation/vo/VisualOdometry.h:19-33).  process() hands the
quad matches to me_vo_process: every RANSAC hypothesis is optimised on its own
GPU lane, inliers are counted per hypothesis by a workgroup, the best one's
inlier list is compacted and the final GN/LM runs in one workgroup.  The
RANSAC triples come from the context's glibc-compatible rand() stream (the
reference calls the unseeded rand(), :150), so a fresh context samples
exactly what a fresh reference process does; ``srand`` reseeds it.

Host-side behaviour kept from the reference: fewer than 6 matches returns
False and leaves the previous state and inliers untouched (:41-42); an init
that is not 6 values becomes zeros (:37-38).  The reference's loop-exit quirk
(:277) can make optimize() spin forever; such a run raises MEError
(ME_ERR_STATE) after ``max_outer`` passes instead of hanging.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, fields

import numpy as np

from ._lib import Context, VOParamsC, default_context, vptr


class Method:
    """VisualOdometry::Method (VisualOdometry.h:16)."""
    GN = 0
    LM = 1


@dataclass
class Parameters:
    """StereoVisualOdometry::parameters with the VisualOdometry::parameters base
    (StereoVisualOdometry.h:24-33, VisualOdometry.h:19-33); same defaults."""
    method: int = Method.GN
    step_size: float = 1.0
    eps: float = 1e-9
    e1: float = 1e-3
    e2: float = 1e-12
    e3: float = 1e-12
    e4: float = 1e-15
    max_iter: int = 100
    nb_fixed_frames: int = 2
    ransac: bool = True
    n_ransac: int = 200
    inlier_threshold: float = 2.0
    baseline: float = 1.0
    weighting: bool = False
    fu1: float = 1.0
    fv1: float = 1.0
    fu2: float = 1.0
    fv2: float = 1.0
    cu1: float = 0.0
    cu2: float = 0.0
    cv1: float = 0.0
    cv2: float = 0.0

    def to_c(self) -> VOParamsC:
        c = VOParamsC()
        for f in fields(self):
            v = getattr(self, f.name)
            setattr(c, f.name, int(v) if isinstance(v, bool) else v)
        return c


def matches_array(matches) -> np.ndarray:
    """(n, 8) float32 {f1, f2, f3, f4} from StereoOdoMatches objects or an array."""
    if isinstance(matches, np.ndarray):
        return np.ascontiguousarray(matches, np.float32).reshape(-1, 8)
    out = np.zeros((len(matches), 8), np.float32)
    for i, m in enumerate(matches):
        out[i] = (m.f1[0], m.f1[1], m.f2[0], m.f2[1], m.f3[0], m.f3[1], m.f4[0], m.f4[1])
    return out


def euler_motion(state) -> np.ndarray:
    """getMotion() (:331-342) of a 6-value state: [R4(state)^T | t]."""
    r, p, y = state[:3]
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    R = np.array([[cp * cy, cp * sy, -sp],
                  [sp * sr * cy - cr * sy, sr * sp * sy + cr * cy, cp * sr],
                  [cr * sp * cy + sr * sy, cr * sp * sy - sr * cy, cp * cr]])
    T = np.eye(4)
    T[:3, :3] = R.T
    T[:3, 3] = state[3:6]
    return T


class StereoVisualOdometry:
    """me::StereoVisualOdometry on the device.  One instance per camera rig."""

    def __init__(self, param: Parameters | None = None, ctx: Context | None = None, max_outer: int = 10000):
        self.m_param = param or Parameters()
        self.ctx = ctx or default_context()
        self.max_outer = max_outer
        self.m_state = np.zeros(6)
        self.m_inliers_idx = np.zeros(0, np.int32)
        self.m_pts3D = np.zeros((0, 4))

    def srand(self, seed: int):
        """srand(seed) for the RANSAC sampling stream of this context."""
        self.ctx.check(self.ctx.lib.me_vo_srand(self.ctx.h, seed), "me_vo_srand")

    def process(self, matches, init=None) -> bool:
        m = matches_array(matches)
        init = np.zeros(6) if init is None else np.asarray(init, np.float64).ravel()
        if init.shape != (6,):
            init = np.zeros(6)
        n = len(m)
        if n < 6:
            return False
        init = np.ascontiguousarray(init)
        motion = np.zeros(16)
        state = np.zeros(6)
        pts = np.zeros((n, 4))
        inl = np.zeros(n, np.int32)
        nin = ctypes.c_int(0)
        ok = ctypes.c_int(0)
        P = ctypes.POINTER
        cp = self.m_param.to_c()
        c = self.ctx
        c.check(c.lib.me_vo_process(c.h, vptr(m), n, init.ctypes.data_as(P(ctypes.c_double)), ctypes.byref(cp),
                                    self.max_outer, motion.ctypes.data_as(P(ctypes.c_double)),
                                    state.ctypes.data_as(P(ctypes.c_double)), pts.ctypes.data_as(P(ctypes.c_double)),
                                    inl.ctypes.data_as(P(ctypes.c_int)), ctypes.byref(nin), ctypes.byref(ok)),
                "me_vo_process")
        self.m_state = state
        self.m_pts3D = pts
        self.m_inliers_idx = inl[:nin.value].copy()
        return bool(ok.value)

    def getMotion(self) -> np.ndarray:
        return euler_motion(self.m_state)

    def getState(self) -> np.ndarray:
        return self.m_state.copy()

    def getPts3D(self) -> np.ndarray:
        return self.m_pts3D

    def getInliers_idx(self) -> list:
        return self.m_inliers_idx.tolist()

    def getParams(self) -> Parameters:
        return self.m_param
