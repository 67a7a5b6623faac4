"""Track and pose containers mirroring include/MotionEstimation/core/feature_types.h.

* ``WBA_Point`` (feature_types.h:121-197): a feature track with its frame
  indices, 2x2 covariances and homogeneous 3-D point.  IDs come from one
  static counter PER FEATURE TYPE (mono ``Point2f`` vs stereo pair,
  :196-197), incremented only by the value constructor; copies keep the ID;
  assignment swaps features/indices/cov/pt/ID but not count/camID (:176-184).
  These IDs are the "track IDs" of the north star's bit-exact parity: the
  device kernels decide WHICH tracks survive (KLT status, NMS maxima order),
  this bookkeeping numbers them exactly as the reference does.
* ``CamPose`` (:201-243), ``StereoMatch`` / ``StereoOdoMatches`` (:90-115).
* ``nonMaxSupScanline3x3`` (:270, src/core/feature_types.cpp:253-351) runs on
  the GPU (nms.hip).
"""
from __future__ import annotations

import copy as _copy
from dataclasses import dataclass, field

import numpy as np

from ._lib import ME_HOST, Context, default_context, vptr
from .rotation_utils import Quat

_latest_id = {"mono": 0, "stereo": 0}


def _kind(feat) -> str:
    return "stereo" if isinstance(feat, tuple) and len(feat) == 2 and hasattr(feat[0], "__len__") else "mono"


class WBA_Point:
    """Windowed-BA track.  feat: (x, y) for mono, ((xl, yl), (xr, yr)) for stereo."""

    __slots__ = ("features", "indices", "cov", "pt", "count", "ID", "camID", "kind")

    def __init__(self, match, frame_nb: int, camIDber: int = 0, cov=None, pt=None):
        self.kind = _kind(match)
        self.features = [match]
        self.indices = [int(frame_nb)]
        self.cov = [np.zeros((2, 2)) if cov is None else np.asarray(cov, np.float64)]
        self.pt = np.array([0.0, 0.0, 0.0, 1.0]) if pt is None else np.asarray(pt, np.float64).copy()
        self.count = 1
        self.ID = _latest_id[self.kind]
        _latest_id[self.kind] += 1
        self.camID = camIDber

    @staticmethod
    def reset_ids(kind: str | None = None):
        """Test helper: the reference counter is process-global (static int)."""
        for k in ([kind] if kind else list(_latest_id)):
            _latest_id[k] = 0

    @staticmethod
    def latest_id(kind: str = "stereo") -> int:
        return _latest_id[kind]

    def copy(self) -> "WBA_Point":  # WBA_Point(const WBA_Point&): keeps ID, count, camID
        c = object.__new__(WBA_Point)
        c.kind = self.kind
        c.features = list(self.features)
        c.indices = list(self.indices)
        c.cov = [x.copy() for x in self.cov]
        c.pt = self.pt.copy()
        c.count = self.count
        c.ID = self.ID
        c.camID = self.camID
        return c

    def assign(self, other: "WBA_Point") -> "WBA_Point":
        """operator= (copy-and-swap): takes features/indices/cov/pt/ID, keeps count and camID."""
        tmp = other.copy()
        self.features, self.indices, self.cov, self.pt, self.ID = tmp.features, tmp.indices, tmp.cov, tmp.pt, tmp.ID
        return self

    def addMatch(self, match, frame_nb: int, cov=None):
        self.features.append(match)
        self.indices.append(int(frame_nb))
        self.cov.append(np.zeros((2, 2)) if cov is None else np.asarray(cov, np.float64))
        self.count += 1
        assert len(self.indices) == self.getLastFrameIdx() - self.getFirstFrameIdx() + 1, \
            "addMatch: frames must be contiguous (feature_types.h:140)"

    def pop(self):
        self.features.pop(0)
        self.indices.pop(0)
        self.cov.pop(0)

    def removeLastFeat(self):
        self.features.pop()
        self.indices.pop()
        self.cov.pop()

    def isValid(self) -> bool:
        return len(self.features) > 0

    def isTriangulated(self) -> bool:
        p = self.pt
        return not (p[0] == 0 and p[1] == 0 and p[2] == 0 and p[3] == 1)

    def findFeat(self, idx: int):
        for k, i in enumerate(self.indices):
            if i == idx:
                return True, self.features[k]
        return False, None

    def getLastFeat(self):
        return self.features[-1] if self.features else None

    def getFirstFeat(self):
        return self.features[0] if self.features else None

    def getFeat(self, idx: int):
        return self.features[idx]

    def getCov(self, idx: int):
        return self.cov[idx]

    def getLastFrameIdx(self) -> int:
        return self.indices[-1] if self.indices else 0xFFFFFFFF  # (unsigned)-1 on an empty track

    def getFirstFrameIdx(self) -> int:
        return self.indices[0] if self.indices else 0xFFFFFFFF

    def getFrameIdx(self, idx: int) -> int:
        return self.indices[idx]

    def getNbFeatures(self) -> int:
        return len(self.features)

    def getCount(self) -> int:
        return self.count

    def getID(self) -> int:
        return self.ID

    def getCameraID(self) -> int:
        return self.camID

    def get3DLocation(self) -> np.ndarray:
        return self.pt.copy()

    def set3DLocation(self, pt):
        self.pt = np.asarray(pt, np.float64).copy()

    def setCameraNum(self, i: int):
        self.camID = i

    def __repr__(self):
        return (f"Point {self.ID}: {self.getNbFeatures()} feats (from {self.getFirstFrameIdx()} to "
                f"{self.getLastFrameIdx()})")


@dataclass
class CamPose:
    """CamPose<Quat<double>, double> (feature_types.h:201-243); orientation maps world->camera."""
    ID: int = 0
    orientation: Quat = field(default_factory=Quat)
    position: np.ndarray = field(default_factory=lambda: np.zeros(3))
    Cov: np.ndarray = field(default_factory=lambda: np.zeros((6, 6)))

    def TrMat(self) -> np.ndarray:
        T = np.eye(4)
        T[:3, :3] = self.orientation.getR3()
        T[:3, 3] = self.position
        return T

    def __mul__(self, pose: "CamPose") -> "CamPose":
        """CamPose::operator* (feature_types.h:223-228): R1 R2 | R1 t2 + t1, keeps this ID and Cov."""
        return CamPose(self.ID, self.orientation * pose.orientation,
                       self.orientation * np.asarray(pose.position) + np.asarray(self.position),
                       np.array(self.Cov, np.float64, copy=True))


# ------------------------------------------------ pose-covariance propagation
# src/core/feature_types.cpp:171-251.  The reference writes a CV_32F identity
# into a CV_64F Jacobian with Mat::copyTo, which reallocates the ROI header
# instead of writing J: those blocks stay zero (reproduced):
# J[0:3, 6:9] in poseMultiplicationWithCovarianceReverse, J[3:6, 3:6] in
# invertPoseWithCovariance.
def poseMultiplicationWithCovariance(p1: CamPose, p2: CamPose, ID: int) -> CamPose:
    """P3 = P1 * P2 with Cov3 = J diag(Cov1, Cov2) J^T (feature_types.cpp:171-194)."""
    assert p1.Cov.size and p2.Cov.size, "Poses cannot be mulitplied (empty Cov matrix)"
    p3 = p1 * p2
    aug = np.zeros((12, 12))
    aug[:6, :6], aug[6:, 6:] = p1.Cov, p2.Cov
    q1, q2, q3 = p1.orientation, p2.orientation, p3.orientation
    J = np.zeros((6, 12))
    J[:3, :3] = np.eye(3)
    J[:3, 3:6] = q1.getH_qvec(p2.position)
    J[:3, 6:9] = q1.getR3()
    J[3:, 3:6] = q3.getH() @ q2.getQr() @ q1.getG()
    J[3:, 9:12] = q3.getH() @ q1.getQl() @ q2.getG()
    p3.ID = ID
    p3.Cov = J @ aug @ J.T
    return p3


def poseMultiplicationWithCovarianceReverse(p1: CamPose, p2: CamPose, ID: int) -> CamPose:
    """P3 = P2 * P1 with propagated covariance (feature_types.cpp:196-219)."""
    assert p1.Cov.size and p2.Cov.size, "Poses cannot be multiplied (empty Cov matrix)"
    p3 = p2 * p1
    aug = np.zeros((12, 12))
    aug[:6, :6], aug[6:, 6:] = p1.Cov, p2.Cov
    q1, q2, q3 = p1.orientation, p2.orientation, p3.orientation
    J = np.zeros((6, 12))
    J[:3, :3] = q2.getR3()
    # J[:3, 6:9] stays 0: the reference's CV_32F identity never reaches J
    J[:3, 9:12] = q2.getH_qvec(p1.position)
    J[3:, 3:6] = q3.getH() @ q2.getQl() @ q1.getG()
    J[3:, 9:12] = q3.getH() @ q1.getQr() @ q2.getG()
    p3.ID = ID
    p3.Cov = J @ aug @ J.T
    return p3


def invertPoseWithCovariance(p: CamPose) -> None:
    """In place: P <- P^-1 with Cov <- J Cov J^T (feature_types.cpp:221-236)."""
    assert p.Cov.size, "Pose cannot be inverted (empty Cov matrix)"
    qc = p.orientation.conj()
    J = np.zeros((6, 6))
    J[:3, :3] = -qc.getR3()
    J[:3, 3:6] = qc.getH_qvec(p.position)
    # J[3:6, 3:6] stays 0 (the reference's -eye(CV_32F) never reaches J)
    p.position = -(qc * np.asarray(p.position))
    p.orientation = qc
    p.Cov = J @ p.Cov @ J.T


def ScalePoseWithCovariance(p: CamPose, scale) -> None:
    """In place: t <- s t, Cov <- J diag(Cov, var_s) J^T (feature_types.cpp:238-251); scale = (s, var_s)."""
    assert p.Cov.size, "Pose cannot be scaled (empty Cov matrix)"
    aug = np.zeros((7, 7))
    aug[:6, :6] = p.Cov
    aug[6, 6] = scale[1]
    J = np.zeros((6, 7))
    J[:3, :3] = np.eye(3) * scale[0]
    J[3:, 3:6] = np.eye(3)
    J[:3, 6] = p.position
    p.Cov = J @ aug @ J.T
    p.position = np.asarray(p.position, np.float64) * scale[0]


@dataclass
class StereoMatch:
    f1: tuple
    f2: tuple
    m_score: float = -1.0


@dataclass
class StereoOdoMatches(StereoMatch):
    f3: tuple = (0.0, 0.0)
    f4: tuple = (0.0, 0.0)


def nonMaxSupScanline3x3(response, ctx: Context | None = None):
    """me::nonMaxSupScanline3x3: returns (maxima (n,2) [(row+0.5+dr, col+0.5+dc)], 8U mask)."""
    ctx = ctx or default_context()
    r = np.ascontiguousarray(response, np.float64)
    if r.ndim != 2:
        raise ValueError("response must be a 2-D CV_64F map")
    h, w = r.shape
    mask = np.zeros((h, w), np.uint8)
    cap = max(1, (h * w) // 2 + 1)
    mx = np.zeros(2 * cap)
    n = np.zeros(1, np.int32)
    import ctypes
    ctx.check(ctx.lib.me_nms_scanline3x3(ctx.h, ME_HOST, vptr(r), w, h, vptr(mask), vptr(mx), cap,
                                         n.ctypes.data_as(ctypes.POINTER(ctypes.c_int))), "me_nms_scanline3x3")
    k = int(n[0])
    return mx[:2 * min(k, cap)].reshape(-1, 2), mask
