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


# ------------------------------------------------------------------ monocular VO (§8f-4)
@dataclass
class MonoParameters:
    """MonoVisualOdometry::parameters with the VisualOdometry::parameters base
    (MonoVisualOdometry.h:21-28, VisualOdometry.h:19-33); the fields the mono
    path reads, same defaults."""
    prob: float = 0.99
    fu: float = 1.0
    fv: float = 1.0
    cu: float = 0.0
    cv: float = 0.0
    ransac: bool = True
    inlier_threshold: float = 2.0

    def to_c(self):
        from ._lib import MonoParamsC

        return MonoParamsC(self.fu, self.fv, self.cu, self.cv, self.prob, self.inlier_threshold, int(bool(self.ransac)))


class MonoVisualOdometry:
    """Mirror of me::MonoVisualOdometry (include/MotionEstimation/vo/
    MonoVisualOdometry.h:18-57, src/vo/MonoVisualOdometry.cpp:7-73).
    process() hands the matches to me_mono_vo_process: the five-point solve of
    every RANSAC sample on its own GPU lane, the Sampson scores of every
    model by a wave, the best model's recoverPose (decomposition, DLT
    triangulation and cheirality of every match under the four poses) on the
    device.  OpenCV's findEssentialMat / recoverPose are restated (parity
    unpinned); the RANSAC samples follow OpenCV's cv::RNG((uint64)-1)."""

    def __init__(self, param: MonoParameters | None = None, ctx: Context | None = None):
        self.param = param or MonoParameters()
        self.ctx = ctx or default_context()
        self._Rt = np.eye(4)
        self._E = np.eye(4)  # (the reference's ctor sets m_E = eye(4, 4))
        self._inliers: list = []
        self._outliers: list = []

    def process(self, matches) -> bool:
        """matches: (n, 4) {f1.x, f1.y, f2.x, f2.y} or a pair (f1 (n, 2), f2 (n, 2))."""
        if isinstance(matches, tuple):
            f1 = np.ascontiguousarray(matches[0], np.float32).reshape(-1, 2)
            f2 = np.ascontiguousarray(matches[1], np.float32).reshape(-1, 2)
        else:
            m = np.asarray(matches, np.float32).reshape(-1, 4)
            f1, f2 = np.ascontiguousarray(m[:, :2]), np.ascontiguousarray(m[:, 2:])
        n = len(f1)
        p = self.param.to_c()
        Rt, E = np.zeros(16), np.zeros(9)
        inl = np.zeros(max(n, 1), np.int32)
        ni, ok = ctypes.c_int(0), ctypes.c_int(0)
        c = self.ctx
        c.check(c.lib.me_mono_vo_process(c.h, f1.ctypes.data, f2.ctypes.data, n, ctypes.byref(p),
                                         Rt.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                         E.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), inl.ctypes.data,
                                         ctypes.byref(ni), ctypes.byref(ok)), "me_mono_vo_process")
        self._Rt = Rt.reshape(4, 4)
        # MonoVisualOdometry.cpp:9-52: fewer than 8 matches leaves m_E and the inlier / outlier lists
        # as they were; an empty E is assigned (an empty matrix) and the lists kept; otherwise all
        # three are replaced
        if n < 8:
            return bool(ok.value)
        if not np.any(E):
            self._E = np.zeros((0, 0))
            return bool(ok.value)
        self._E = E.reshape(3, 3)
        self._inliers = [int(i) for i in inl[:ni.value]]
        s = set(self._inliers)
        self._outliers = [i for i in range(n) if i not in s]
        return bool(ok.value)

    def getMotion(self) -> np.ndarray:
        return self._Rt.copy()

    def getEssentialMat(self) -> np.ndarray:
        return self._E.copy()

    def getInliersIdx(self) -> list:
        return list(self._inliers)

    def getOutliersIdx(self) -> list:
        return list(self._outliers)
