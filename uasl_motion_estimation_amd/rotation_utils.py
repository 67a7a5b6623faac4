"""Host-side rotation helpers mirroring include/MotionEstimation/core/rotation_utils.h.

Only what the hot-path adapters need: Quat (normalised on construction,
rotation_utils.h:130, .cpp:217-226), getR3 (:232-237), exp_map_Quat /
log_map_Quat (:190-204, theta floor 1e-10, acos(w) with no sign fix) and the
StopCondition enum (:20).  PI is the reference's 3.14156592 (:15).
"""
from __future__ import annotations

import math
from enum import IntEnum

import numpy as np

PI = 3.14156592  # rotation_utils.h:15 (sic)


class StopCondition(IntEnum):
    NO_STOP = 0
    SMALL_GRADIENT = 1
    SMALL_INCREMENT = 2
    MAX_ITERATIONS = 3
    SMALL_DECREASE_FUNCTION = 4
    SMALL_REPROJ_ERROR = 5
    NO_CONVERGENCE = 6


def deg2Rad(deg: float) -> float:
    return deg * PI / 180


def rad2Deg(rad: float) -> float:
    return rad * 180 / PI


class Quat:
    __slots__ = ("w", "x", "y", "z")

    def __init__(self, w=1.0, x=0.0, y=0.0, z=0.0):
        self.w, self.x, self.y, self.z = float(w), float(x), float(y), float(z)
        self.normalize()

    def normalize(self):
        n = math.sqrt(self.w * self.w + self.x * self.x + self.y * self.y + self.z * self.z)
        if n != 0.0:
            self.w /= n
            self.x /= n
            self.y /= n
            self.z /= n

    def coeffs(self) -> np.ndarray:
        return np.array([self.w, self.x, self.y, self.z])

    def getR3(self) -> np.ndarray:
        w, x, y, z = self.w, self.x, self.y, self.z
        return np.array([[w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y)],
                         [2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x)],
                         [2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z]])

    def __repr__(self):
        return f"Quat({self.w}, {self.x}, {self.y}, {self.z})"

    # --- rotation_utils.h:148, 157-161, 240-268; rotation_utils.cpp:261-266, 306-308
    def conj(self) -> "Quat":
        return Quat(self.w, -self.x, -self.y, -self.z)

    def vec(self) -> np.ndarray:
        return np.array([self.x, self.y, self.z])

    def __mul__(self, q):
        """Quat * Quat (normalised result) or Quat * 3-vector (getR3() @ v)."""
        if isinstance(q, Quat):
            a = self
            return Quat(a.w * q.w - (a.x * q.x + a.y * q.y + a.z * q.z), a.w * q.x + a.x * q.w + a.y * q.z - a.z * q.y,
                        a.w * q.y - a.x * q.z + a.y * q.w + a.z * q.x, a.w * q.z + a.x * q.y - a.y * q.x + a.z * q.w)
        return self.getR3() @ np.asarray(q, np.float64)

    def getQl(self) -> np.ndarray:
        w, x, y, z = self.w, self.x, self.y, self.z
        return np.array([[w, -x, -y, -z], [x, w, -z, y], [y, z, w, -x], [z, -y, x, w]])

    def getQr(self) -> np.ndarray:
        w, x, y, z = self.w, self.x, self.y, self.z
        return np.array([[w, -x, -y, -z], [x, w, z, -y], [y, -z, w, x], [z, y, -x, w]])

    def getH(self) -> np.ndarray:
        """d(rotation vector) / d(quaternion), 3x4."""
        w = self.w
        c = 1.0 / (1 - w * w + 1e-20)
        d = math.acos(w) / math.sqrt(1 - w * w + 1e-20)
        k = 2 * c * (d * w - 1)
        return np.array([[k * self.x, 2 * d, 0, 0], [k * self.y, 0, 2 * d, 0], [k * self.z, 0, 0, 2 * d]])

    def getG(self) -> np.ndarray:
        """d(quaternion) / d(rotation vector), 4x3, at log(q)."""
        return Gq_v(log_map_Quat(self))

    def getH_qvec(self, x) -> np.ndarray:
        """d(q x) / d(rotation vector), 3x3."""
        x = np.asarray(x, np.float64)
        q = self.vec()
        D = np.zeros((3, 4))
        D[:, 0] = 2 * self.w * x + 2 * skew(q) @ x
        D[:, 1:] = 2 * (float(q @ x) * np.eye(3) + np.outer(q, x) - np.outer(x, q) - self.w * skew(x))
        return D @ self.getG()


def skew(v) -> np.ndarray:
    """rotation_utils.h:30."""
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]], np.float64)


def Gq_v(v) -> np.ndarray:
    """d(exp quaternion) / d(rotation vector), 4x3 (rotation_utils.cpp:357-368)."""
    v = np.asarray(v, np.float64)
    snorm = float(v @ v)
    norm = math.sqrt(snorm) + 1e-20
    a = math.cos(0.5 * norm) * norm - 2 * math.sin(0.5 * norm)
    sn = snorm * math.sin(0.5 * norm)
    M = np.vstack([-v * sn, 2 * sn * np.eye(3) + np.outer(v, v) * a])
    return 1 / (2 * norm ** 3) * M


def exp_map_Quat(vec) -> Quat:
    v = [float(a) for a in vec]
    norm = math.sqrt(v[0] ** 2 + v[1] ** 2 + v[2] ** 2)
    theta = 1e-10 if norm < 1e-10 else norm
    s = math.sin(theta / 2)
    q = Quat(math.cos(theta / 2), v[0] / theta * s, v[1] / theta * s, v[2] / theta * s)
    q.normalize()
    return q


def log_map_Quat(q: Quat) -> np.ndarray:
    norm = math.sqrt(q.x ** 2 + q.y ** 2 + q.z ** 2)
    theta = 1e-10 if norm < 1e-10 else norm
    a = float(np.arccos(q.w)) * 2.0  # no clamp: NaN for |w| > 1 like std::acos
    return a * (np.array([q.x, q.y, q.z]) / theta)
