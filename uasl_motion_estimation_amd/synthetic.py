"""Deterministic synthetic stereo streams (SURVEY §8d generator).

The reference ships no data and no tests, so every input of the parity tests
and of bench.py is generated here from a seed (seed = 20261015 + config):

* intrinsics fx = fy = 0.9 W, cx = W/2, cy = H/2, K0 = K1, baseline b = 0.5 m
  (the reference's default for a zero baseline, BundleAdjuster.h:389-390);
* camera path: forward 0.5 m / keyframe, yaw 0.3 deg / keyframe; poses are
  world->camera (p_cam = R X + t), the convention of both StereoReprojectionError
  (BundleAdjuster.h:153-160) and ScaleState (optimisation.cpp:175-178);
* landmarks Z ~ U[5, 50] m, track lengths U[2, W], sigma = 0.5 px noise
  (feat_var = 0.25 = TrackingInfo::feat_cov, file_IO.h:73), fixedFrames = 2;
* images: 8-bit 4-octave value-noise texture on piecewise fronto-parallel
  planes; the right image goes through a NON-monotone tone map, the
  multi-spectral case mutual information is meant for.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np

CONFIGS = {
    1: dict(width=640, height=480, n_feats=200, window=5),
    2: dict(width=640, height=480, n_feats=500, window=10),
    3: dict(width=1280, height=720, n_feats=2000, window=20),
    4: dict(width=3840, height=2160, n_feats=8000, window=30),
    5: dict(width=1280, height=720, n_feats=2000, window=50),
}
SEED0 = 20261015
BASELINE = 0.5


def intrinsics(width: int, height: int) -> np.ndarray:
    f = 0.9 * width
    return np.array([[f, 0.0, width / 2.0], [0.0, f, height / 2.0], [0.0, 0.0, 1.0]])


# ------------------------------------------------------------------ rotations
def rot_y(a: float) -> np.ndarray:
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])


def aa_to_R(aa: np.ndarray) -> np.ndarray:
    th = float(np.linalg.norm(aa))
    if th < 1e-12:
        return np.eye(3)
    w = aa / th
    Wx = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    return np.eye(3) + math.sin(th) * Wx + (1 - math.cos(th)) * Wx @ Wx


def R_to_aa(R: np.ndarray) -> np.ndarray:
    c = max(-1.0, min(1.0, (np.trace(R) - 1) / 2))
    th = math.acos(c)
    if th < 1e-12:
        return np.zeros(3)
    v = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    return v * th / (2 * math.sin(th))


def R_to_aa_robust(R: np.ndarray) -> np.ndarray:
    """Angle-axis of R through its quaternion (Shepperd): well defined up to
    and at a half turn, where R_to_aa's trace formula loses the axis."""
    m = np.asarray(R, np.float64)
    tr = np.trace(m)
    if tr > max(m[0, 0], m[1, 1], m[2, 2]):
        w = 0.5 * math.sqrt(1.0 + tr)
        v = np.array([m[2, 1] - m[1, 2], m[0, 2] - m[2, 0], m[1, 0] - m[0, 1]]) / (4.0 * w)
    else:
        i = int(np.argmax([m[0, 0], m[1, 1], m[2, 2]]))
        j, k = (i + 1) % 3, (i + 2) % 3
        r = math.sqrt(max(0.0, 1.0 + m[i, i] - m[j, j] - m[k, k]))
        v = np.zeros(3)
        v[i] = 0.5 * r
        v[j] = (m[j, i] + m[i, j]) / (2.0 * r)
        v[k] = (m[k, i] + m[i, k]) / (2.0 * r)
        w = (m[k, j] - m[j, k]) / (2.0 * r)
    if w < 0:
        w, v = -w, -v
    s = float(np.linalg.norm(v))
    if s < 1e-15:
        return np.zeros(3)
    return v / s * (2.0 * math.atan2(s, w))


def R_to_quat(R: np.ndarray) -> np.ndarray:
    """(w, x, y, z) with w >= 0, matching Quat::getR3 (rotation_utils.h:232-237)."""
    aa = R_to_aa(R)
    th = float(np.linalg.norm(aa))
    if th < 1e-12:
        return np.array([1.0, 0.0, 0.0, 0.0])
    ax = aa / th
    return np.concatenate([[math.cos(th / 2)], ax * math.sin(th / 2)])


def trajectory(window: int, first_id: int = 0):
    """World->camera poses (R, t) of `window` keyframes."""
    poses = []
    for i in range(window):
        k = first_id + i
        Rw = rot_y(math.radians(0.3 * k))  # camera->world rotation
        C = np.array([0.0, 0.0, 0.5 * k])
        R = Rw.T
        t = -R @ C
        poses.append((R, t))
    return poses


def project(K, b, R, t, X):
    p = R @ X + t
    xl = K[0, 0] * p[0] / p[2] + K[0, 2]
    y = K[1, 1] * p[1] / p[2] + K[1, 2]
    xr = K[0, 0] * (p[0] - b) / p[2] + K[0, 2]
    return np.array([xl, y, xr, y]), p


# ------------------------------------------------------------------ BA window
@dataclass
class BAProblem:
    cams: np.ndarray          # (W, 6) {t, angle-axis}
    pts: np.ndarray           # (N, 3)
    obs: np.ndarray           # (O, 4)
    cam_idx: np.ndarray       # (O,) int32
    pt_idx: np.ndarray        # (O,) int32
    K0: np.ndarray
    K1: np.ndarray
    baseline: float
    feat_var: float
    fixed_frames: int
    cams_true: np.ndarray = field(default=None)
    pts_true: np.ndarray = field(default=None)
    obs_dim: int = 4                      # 2: BundleAdjuster<2> (obs (O, 2) + cam_id)
    cam_id: np.ndarray = field(default=None)

    def copy(self):
        return BAProblem(self.cams.copy(), self.pts.copy(), self.obs, self.cam_idx, self.pt_idx, self.K0, self.K1,
                         self.baseline, self.feat_var, self.fixed_frames, self.cams_true, self.pts_true,
                         self.obs_dim, self.cam_id)


def ba_problem(seed: int, n_pts: int, window: int, width: int, height: int, noise: float = 0.5,
               fixed: int = 2, alive_frac: float = 0.7, outlier_frac: float = 0.02) -> BAProblem:
    rng = np.random.default_rng(seed)
    K = intrinsics(width, height)
    b = BASELINE
    poses = trajectory(window)
    margin = 12.0
    pts_true, obs, cidx, pidx = [], [], [], []
    j = 0
    tries = 0
    while j < n_pts and tries < 50 * n_pts:
        tries += 1
        L = int(rng.integers(2, window + 1))
        if rng.random() < alive_frac:
            end = window - 1
        else:
            end = int(rng.integers(L - 1, window))
        start = end - L + 1
        u = rng.uniform(margin, width - margin)
        v = rng.uniform(margin, height - margin)
        Z = rng.uniform(5.0, 50.0)
        R, t = poses[start]
        pc = np.array([(u - K[0, 2]) * Z / K[0, 0], (v - K[1, 2]) * Z / K[1, 1], Z])
        X = R.T @ (pc - t)
        ok = True
        rows = []
        for f in range(start, end + 1):
            m, p = project(K, b, poses[f][0], poses[f][1], X)
            if p[2] < 1.0 or not (margin <= m[0] < width - margin and margin <= m[1] < height - margin
                                  and margin <= m[2] < width - margin):
                ok = False
                break
            rows.append((f, m))
        if not ok:
            continue
        for f, m in rows:
            mm = m + rng.normal(0.0, noise, 4)
            mm[3] = mm[1] + rng.normal(0.0, noise)  # y of the right image observed independently
            if rng.random() < outlier_frac:
                mm[:2] += rng.normal(0.0, 8.0, 2)
            obs.append(mm)
            cidx.append(f)
            pidx.append(j)
        pts_true.append(X)
        j += 1
    pts_true = np.array(pts_true)
    cams_true = np.zeros((window, 6))
    for i, (R, t) in enumerate(poses):
        cams_true[i, :3] = t
        cams_true[i, 3:] = R_to_aa(R)
    # initial estimate: perturbed poses (2 cm, 0.2 deg) except the fixed ones,
    # points triangulated from the noisy first stereo observation
    cams = cams_true.copy()
    for i in range(fixed, window):
        cams[i, :3] += rng.normal(0.0, 0.02, 3)
        cams[i, 3:] += np.radians(rng.normal(0.0, 0.2, 3))
    obs = np.array(obs)
    cidx = np.array(cidx, dtype=np.int32)
    pidx = np.array(pidx, dtype=np.int32)
    pts = np.zeros_like(pts_true)
    first = np.full(len(pts_true), -1)
    for o in range(len(obs)):
        if first[pidx[o]] < 0:
            first[pidx[o]] = o
    for jj in range(len(pts_true)):
        o = first[jj]
        xl, yl, xr, _ = obs[o]
        d = max(xl - xr, 0.5)
        Z = K[0, 0] * b / d
        pc = np.array([(xl - K[0, 2]) * Z / K[0, 0], (yl - K[1, 2]) * Z / K[1, 1], Z])
        R = aa_to_R(cams[cidx[o], 3:])
        pts[jj] = R.T @ (pc - cams[cidx[o], :3])
    # keep the start feasible for the Ceres-style bounds (BundleAdjuster.h:455-460)
    Zmax = K[0, 0] * b / 0.1
    pts[:, 2] = np.clip(pts[:, 2], K[0, 0] * b / (2 * K[0, 2]) + 1e-3, Zmax - 1e-3)
    return BAProblem(cams, pts, obs, cidx, pidx, K.copy(), K.copy(), b, noise ** 2, fixed, cams_true, pts_true)


def ba_problem_mono(seed: int, n_pts: int, window: int, width: int, height: int, noise: float = 0.5,
                    fixed: int = 2, min_len: int = 3, right_frac: float = 0.3) -> BAProblem:
    """BundleAdjuster<2> window: the stereo window's tracks, each kept in ONE
    image (WBA_Point::camID 0 = left, 1 = right, BundleAdjuster.h:395-398) as
    Observation<2> {x, y}; tracks shorter than ``min_len`` frames dropped."""
    bp = ba_problem(seed, n_pts, window, width, height, noise=noise, fixed=fixed)
    rng = np.random.default_rng(seed + 7)
    cnt = np.bincount(bp.pt_idx, minlength=len(bp.pts))
    keep_pt = cnt >= min_len
    new_id = np.cumsum(keep_pt) - 1
    side = (rng.random(len(bp.pts)) < right_frac).astype(np.int32)  # per track
    sel = keep_pt[bp.pt_idx]
    o4 = bp.obs[sel]
    pid = bp.pt_idx[sel]
    cid = side[pid]
    obs = np.where(cid[:, None] == 0, o4[:, 0:2], o4[:, 2:4])
    return BAProblem(bp.cams, bp.pts[keep_pt].copy(), np.ascontiguousarray(obs), bp.cam_idx[sel].copy(),
                     new_id[pid].astype(np.int32), bp.K0, bp.K1, bp.baseline, bp.feat_var, fixed, bp.cams_true,
                     bp.pts_true[keep_pt], 2, np.ascontiguousarray(cid, np.int32))


# ------------------------------------------------------------------ images
def _value_noise(X, Y, rng_seed: int, octaves: int = 4, base: float = 0.35):
    out = np.zeros_like(X)
    amp, tot = 1.0, 0.0
    for o in range(octaves):
        cell = base / (2 ** o)
        gx, gy = X / cell, Y / cell
        ix, iy = np.floor(gx).astype(np.int64), np.floor(gy).astype(np.int64)
        fx, fy = gx - ix, gy - iy
        sx, sy = fx * fx * (3 - 2 * fx), fy * fy * (3 - 2 * fy)

        def h(a, c):
            v = (a * 73856093) ^ (c * 19349663) ^ (rng_seed * 83492791 + o * 2654435761)
            v = (v ^ (v >> 13)) * 1274126177
            v = v ^ (v >> 16)
            return (v & 0xFFFF).astype(np.float64) / 65535.0

        v00, v10, v01, v11 = h(ix, iy), h(ix + 1, iy), h(ix, iy + 1), h(ix + 1, iy + 1)
        val = (v00 * (1 - sx) + v10 * sx) * (1 - sy) + (v01 * (1 - sx) + v11 * sx) * sy
        out += amp * val
        tot += amp
        amp *= 0.55
    return out / tot


@dataclass
class Scene:
    planes: list           # (x0, x1, Z) world strips
    seed: int


def make_scene(seed: int) -> Scene:
    rng = np.random.default_rng(seed)
    edges = np.sort(rng.uniform(-40, 40, 9))
    planes = [(-1e9, edges[0], float(rng.uniform(8, 40)))]
    for a, c in zip(edges[:-1], edges[1:]):
        planes.append((float(a), float(c), float(rng.uniform(6, 45))))
    planes.append((float(edges[-1]), 1e9, float(rng.uniform(8, 40))))
    planes.append((-1e9, 1e9, 60.0))  # background: rays passing between strips
    return Scene(planes, seed)


def tone_map():
    v = np.arange(256, dtype=np.float64)
    lut = 127.5 + 120.0 * np.sin(2 * np.pi * v / 255.0 * 1.3 + 0.7)  # non-monotone
    return np.clip(np.rint(lut), 0, 255).astype(np.uint8)


def render(scene: Scene, K, R, t, width, height, shift=0.0):
    """8-bit image of the scene seen by camera (R, t) shifted by `shift` along its x axis."""
    u, v = np.meshgrid(np.arange(width, dtype=np.float64), np.arange(height, dtype=np.float64))
    d = np.stack([(u - K[0, 2]) / K[0, 0], (v - K[1, 2]) / K[1, 1], np.ones_like(u)], -1)
    Rw = R.T
    C = -Rw @ t + Rw @ np.array([shift, 0.0, 0.0])
    dw = d @ Rw.T
    # nearest plane per pixel first (the first plane reaching the minimum
    # depth, as a sequential s < best scan), then the texture once per pixel
    # at that plane's hit point: the same values as texturing every plane
    best = np.full(u.shape, np.inf)
    which = np.full(u.shape, -1, np.int32)
    for k, (x0, x1, Z) in enumerate(scene.planes):
        s = (Z - C[2]) / dw[..., 2]
        X = C[0] + s * dw[..., 0]
        hit = (s > 0) & (X >= x0) & (X < x1) & (s < best)
        best = np.where(hit, s, best)
        which = np.where(hit, k, which)
    tex = np.zeros(u.shape)
    for k, (x0, x1, Z) in enumerate(scene.planes):
        m = which == k
        if not m.any():
            continue
        dwm = dw[m]
        s = (Z - C[2]) / dwm[:, 2]
        X = C[0] + s * dwm[:, 0]
        Y = C[1] + s * dwm[:, 1]
        tex[m] = _value_noise(X, Y, scene.seed)
    img = np.clip(np.rint(tex * 255.0), 0, 255).astype(np.uint8)
    return img


def depth_at(scene: Scene, K, R, t, u, v):
    """Depth along the optical axis and world point for pixels (u, v)."""
    d = np.stack([(u - K[0, 2]) / K[0, 0], (v - K[1, 2]) / K[1, 1], np.ones_like(u)], -1)
    Rw = R.T
    C = -Rw @ t
    dw = d @ Rw.T
    best = np.full(u.shape, np.inf)
    for (x0, x1, Z) in scene.planes:
        s = (Z - C[2]) / dw[..., 2]
        X = C[0] + s * dw[..., 0]
        hit = (s > 0) & (X >= x0) & (X < x1) & (s < best)
        best = np.where(hit, s, best)
    Xw = C[None, :] + best[:, None] * dw
    return best, Xw


# ------------------------------------------------------------------ long sequences
# The strip scene above is a short-window fixture: the straight forward path
# flies through its planes within ~40 keyframes.  Long sequences (the
# config-5 10k-frame stream) use a heading-consistent arc -- 0.5 m chord and
# 0.3 deg yaw (to the right) per keyframe, a circle of radius
# 0.5 / (2 sin 0.15 deg) = 95.5 m (1200 keyframes per lap) -- inside a ring
# corridor that follows it: floor, ceiling and two cylindrical walls 6 m to
# either side, value-noise textured, so every keyframe sees the same kind of
# structure at 5-35 m.
#
# World frame: z up, the circle centred on the z axis, the camera plane at
# height ARC_H.  The reference's BA bounds the points in WORLD coordinates
# (Z in [fx b / (2 cx), fx b / 0.1], BundleAdjuster.h:442-460): with z the
# height, every point -- a far mismatch included, up to fx b / d_min = 288 m
# away, i.e. at most ~90 m above or below the camera -- stays feasible, and
# the world origin stays within ~130 m of every camera (the world->camera
# translation carries no large offset to cancel against).
YAW_STEP_DEG = 0.3
ARC_H = 100.0


def arc_radius(step: float = 0.5, yaw_deg: float = YAW_STEP_DEG) -> float:
    return step / (2.0 * math.sin(math.radians(yaw_deg) / 2.0))


def trajectory_arc(n: int, first_id: int = 0):
    """World->camera poses (R, t) on the arc: heading psi = 0.3 deg k, camera
    forward (cos psi, -sin psi, 0), down (0, 0, -1), right (-sin psi, -cos psi,
    0) -- towards the circle's centre -- and centre C = R0 (sin psi, cos psi, 0)
    + (0, 0, ARC_H)."""
    R0 = arc_radius()
    poses = []
    for i in range(n):
        psi = math.radians(YAW_STEP_DEG) * (first_id + i)
        c, s = math.cos(psi), math.sin(psi)
        Rw = np.array([[-s, 0.0, c], [-c, 0.0, -s], [0.0, -1.0, 0.0]])  # columns: right, down, forward
        C = np.array([R0 * s, R0 * c, ARC_H])
        R = Rw.T
        poses.append((R, -R @ C))
    return poses


@dataclass
class CorridorScene:
    seed: int
    radius: float                 # trajectory radius (corridor centre line), circle centred on the z axis
    half_width: float = 6.0       # walls at radius -+ half_width
    floor_z: float = ARC_H - 1.6
    ceil_z: float = ARC_H + 3.0


def render_corridor(scene: CorridorScene, K, R, t, width, height, shift=0.0):
    u, v = np.meshgrid(np.arange(width, dtype=np.float64), np.arange(height, dtype=np.float64))
    d = np.stack([(u - K[0, 2]) / K[0, 0], (v - K[1, 2]) / K[1, 1], np.ones_like(u)], -1)
    Rw = R.T
    C = -Rw @ t + Rw @ np.array([shift, 0.0, 0.0])
    dw = (d @ Rw.T).reshape(-1, 3)
    n = dw.shape[0]
    best = np.full(n, np.inf)
    surf = np.full(n, -1, np.int32)
    with np.errstate(divide="ignore", invalid="ignore"):
        for k, z in enumerate((scene.floor_z, scene.ceil_z)):
            s = (z - C[2]) / dw[:, 2]
            hit = (s > 0) & (s < best)
            best = np.where(hit, s, best)
            surf = np.where(hit, k, surf)
        a = dw[:, 0] ** 2 + dw[:, 1] ** 2
        bq = 2.0 * (C[0] * dw[:, 0] + C[1] * dw[:, 1])
        for k, r in ((2, scene.radius - scene.half_width), (3, scene.radius + scene.half_width)):
            c = C[0] * C[0] + C[1] * C[1] - r * r
            disc = bq * bq - 4.0 * a * c
            sq = np.sqrt(np.maximum(disc, 0.0))
            s1 = (-bq - sq) / (2.0 * a)
            s2 = (-bq + sq) / (2.0 * a)
            s = np.where(s1 > 0, s1, s2)
            hit = (disc >= 0) & (s > 0) & (s < best)
            best = np.where(hit, s, best)
            surf = np.where(hit, k, surf)
    tex = np.zeros(n)
    for k in range(4):
        m = surf == k
        if not m.any():
            continue
        P = C[None, :] + best[m, None] * dw[m]
        if k < 2:  # floor / ceiling: world (x, y)
            cu, cv = P[:, 0], P[:, 1]
        else:      # walls: arc length, height
            r = scene.radius + (-1 if k == 2 else 1) * scene.half_width
            cu, cv = r * np.arctan2(P[:, 1], P[:, 0]), P[:, 2]
        tex[m] = _value_noise(cu, cv, scene.seed * 4 + k)
    return np.clip(np.rint(tex.reshape(height, width) * 255.0), 0, 255).astype(np.uint8)


def _value_noise_torch(X, Y, rng_seed: int, octaves: int = 4, base: float = 0.35):
    """_value_noise on torch tensors (same integer hash, same interpolation)."""
    import torch

    out = torch.zeros_like(X)
    amp, tot = 1.0, 0.0
    for o in range(octaves):
        cell = base / (2 ** o)
        gx, gy = X / cell, Y / cell
        ix, iy = torch.floor(gx).to(torch.int64), torch.floor(gy).to(torch.int64)
        fx, fy = gx - ix.to(X.dtype), gy - iy.to(X.dtype)
        sx, sy = fx * fx * (3 - 2 * fx), fy * fy * (3 - 2 * fy)
        salt = (rng_seed * 83492791 + o * 2654435761) & 0xFFFFFFFFFFFFFFFF
        salt = salt - (1 << 64) if salt >= (1 << 63) else salt

        def h(a, c):
            v = (a * 73856093) ^ (c * 19349663) ^ salt
            v = (v ^ (v >> 13)) * 1274126177
            v = v ^ (v >> 16)
            return (v & 0xFFFF).to(X.dtype) / 65535.0

        v00, v10, v01, v11 = h(ix, iy), h(ix + 1, iy), h(ix, iy + 1), h(ix + 1, iy + 1)
        val = (v00 * (1 - sx) + v10 * sx) * (1 - sy) + (v01 * (1 - sx) + v11 * sx) * sy
        out += amp * val
        tot += amp
        amp *= 0.55
    return out / tot


def render_corridor_torch(scene: CorridorScene, K, R, t, width, height, shift=0.0, device="cuda"):
    """render_corridor on the GPU through torch (long synthetic sequences: a
    720p frame in milliseconds instead of ~0.6 s of numpy); returns a uint8
    (height, width) tensor on `device`."""
    import torch

    f64 = torch.float64
    v, u = torch.meshgrid(torch.arange(height, dtype=f64, device=device), torch.arange(width, dtype=f64, device=device),
                          indexing="ij")
    d = torch.stack([(u - K[0, 2]) / K[0, 0], (v - K[1, 2]) / K[1, 1], torch.ones_like(u)], -1).reshape(-1, 3)
    Rw = R.T
    C = -Rw @ t + Rw @ np.array([shift, 0.0, 0.0])
    dw = d @ torch.as_tensor(Rw.T.copy(), device=device)
    n = dw.shape[0]
    best = torch.full((n,), float("inf"), dtype=f64, device=device)
    surf = torch.full((n,), -1, dtype=torch.int32, device=device)
    for k, z in enumerate((scene.floor_z, scene.ceil_z)):
        s = (z - C[2]) / dw[:, 2]
        hit = (s > 0) & (s < best)
        best = torch.where(hit, s, best)
        surf = torch.where(hit, torch.full_like(surf, k), surf)
    a = dw[:, 0] ** 2 + dw[:, 1] ** 2
    bq = 2.0 * (C[0] * dw[:, 0] + C[1] * dw[:, 1])
    for k, r in ((2, scene.radius - scene.half_width), (3, scene.radius + scene.half_width)):
        c = C[0] * C[0] + C[1] * C[1] - r * r
        disc = bq * bq - 4.0 * a * c
        sq = torch.sqrt(torch.clamp(disc, min=0.0))
        s1 = (-bq - sq) / (2.0 * a)
        s2 = (-bq + sq) / (2.0 * a)
        s = torch.where(s1 > 0, s1, s2)
        hit = (disc >= 0) & (s > 0) & (s < best)
        best = torch.where(hit, s, best)
        surf = torch.where(hit, torch.full_like(surf, k), surf)
    tex = torch.zeros(n, dtype=f64, device=device)
    Cw = torch.as_tensor(C, device=device)
    for k in range(4):
        m = surf == k
        P = Cw[None, :] + best[m, None] * dw[m]
        if k < 2:
            cu, cv = P[:, 0], P[:, 1]
        else:
            r = scene.radius + (-1 if k == 2 else 1) * scene.half_width
            cu, cv = r * torch.atan2(P[:, 1], P[:, 0]), P[:, 2]
        tex[m] = _value_noise_torch(cu, cv, scene.seed * 4 + k)
    return torch.clamp(torch.round(tex.reshape(height, width) * 255.0), 0, 255).to(torch.uint8)


def corridor_frames_torch(seed: int, width: int, height: int, first_id: int, n: int, device="cuda"):
    """Stereo keyframes first_id .. first_id + n - 1 of the corridor sequence
    rendered on the GPU: [(left, right) uint8 device tensors, R, t]."""
    import torch

    scene = CorridorScene(seed, arc_radius())
    K = intrinsics(width, height)
    lut = torch.as_tensor(tone_map(), device=device)
    out = []
    for (R, t) in trajectory_arc(n, first_id):
        L = render_corridor_torch(scene, K, R, t, width, height, 0.0, device)
        Rr = lut[render_corridor_torch(scene, K, R, t, width, height, BASELINE, device).long()]
        out.append((L, Rr, R, t))
    return K, out


@dataclass
class StereoFrame:
    left: np.ndarray
    right: np.ndarray
    R: np.ndarray
    t: np.ndarray


def stereo_stream(seed: int, width: int, height: int, n_frames: int, first_id: int = 0, render_div: int = 1,
                  scene_kind: str = "strips"):
    """Stereo keyframes of the synthetic trajectory.  render_div > 1 renders
    each image at 1/render_div resolution and replicates pixels (4K test
    inputs in seconds instead of minutes; the geometry -- intrinsics, poses,
    depth_at -- stays at full resolution).  scene_kind "corridor": the arc
    trajectory in the ring corridor (long sequences, see trajectory_arc)."""
    corridor = scene_kind == "corridor"
    scene = CorridorScene(seed, arc_radius()) if corridor else make_scene(seed)
    K = intrinsics(width, height)
    lut = tone_map()
    frames = []
    d = max(1, int(render_div))
    w_r, h_r = -(-width // d), -(-height // d)
    K_r = intrinsics(w_r, h_r)

    rf = render_corridor if corridor else render

    def rend(R, t, shift=0.0):
        if d == 1:
            return rf(scene, K, R, t, width, height, shift=shift)
        img = rf(scene, K_r, R, t, w_r, h_r, shift=shift)
        return np.ascontiguousarray(np.kron(img, np.ones((d, d), np.uint8))[:height, :width])

    poses = list(trajectory_arc(n_frames, first_id) if corridor else trajectory(n_frames, first_id))
    jobs = [(R, t, sh) for (R, t) in poses for sh in (0.0, BASELINE)]
    # images are independent: rendered by a thread pool (numpy releases the GIL in the array work)
    workers = min(len(jobs), 16, os.cpu_count() or 1)
    if workers > 1:
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(workers) as ex:
            imgs = list(ex.map(lambda j: rend(*j), jobs))
    else:
        imgs = [rend(*j) for j in jobs]
    for k, (R, t) in enumerate(poses):
        frames.append(StereoFrame(imgs[2 * k], lut[imgs[2 * k + 1]], R, t))
    return scene, K, frames


def grid_features(rng, n, width, height, margin):
    """Jittered grid of n feature positions at least `margin` px from the border."""
    aspect = width / height
    ny = max(1, int(round(math.sqrt(n / aspect))))
    nx = max(1, int(math.ceil(n / ny)))
    xs = np.linspace(margin, width - margin - 1, nx)
    ys = np.linspace(margin, height - margin - 1, ny)
    gx, gy = np.meshgrid(xs, ys)
    pts = np.stack([gx.ravel(), gy.ravel()], -1)[:n]
    jit = rng.uniform(-0.45, 0.45, pts.shape) * np.array([xs[1] - xs[0] if nx > 1 else 0,
                                                           ys[1] - ys[0] if ny > 1 else 0])
    pts = np.clip(pts + jit, margin, np.array([width - margin - 1, height - margin - 1]))
    return pts


@dataclass
class ScaleProblem:
    """Flattened ScaleState (optimisation.h:76-98) of the last keyframe."""
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
    mask: np.ndarray | None = None


def scale_problem(seed: int, width: int, height: int, n_feats: int, window: int = 5, w: int = 5,
                  scale0: float = 1.02, frames=None, scene=None, right_frac: float = 0.25,
                  untriangulated_frac: float = 0.03, stale_frac: float = 0.05) -> ScaleProblem:
    """Tracks seen in the last keyframe of a window, 3-D points from the scene."""
    rng = np.random.default_rng(seed + 7)
    if frames is None:
        scene, K, frames = stereo_stream(seed, width, height, 2)
    K = intrinsics(width, height)
    fr = frames[-1]
    R, t = fr.R, fr.t
    pts = grid_features(rng, n_feats, width, height, 4 * w + 4)
    depth, Xw = depth_at(scene, K, R, t, pts[:, 0], pts[:, 1])
    Xh = np.concatenate([Xw, np.ones((len(Xw), 1))], 1)
    n_right = int(round(right_frac * n_feats))
    n_left = n_feats - n_right
    XL = Xh[:n_left].copy()
    XR = Xh[n_left:].copy()
    # right-detected tracks store the point shifted by the baseline in the
    # camera frame (optimisation.cpp:202-207 undoes exactly that)
    XR[:, :3] = XR[:, :3] - (R.T @ np.array([BASELINE, 0.0, 0.0]))[None, :]
    tri_l = (rng.random(n_left) >= untriangulated_frac).astype(np.uint8)
    tri_r = (rng.random(n_right) >= untriangulated_frac).astype(np.uint8)
    XL[tri_l == 0] = np.array([0, 0, 0, 1.0])
    XR[tri_r == 0] = np.array([0, 0, 0, 1.0])
    lframe = window - 1
    last_l = np.where(rng.random(n_left) < stale_frac, lframe - 1, lframe).astype(np.uint32)
    last_r = np.where(rng.random(n_right) < stale_frac, lframe - 1, lframe).astype(np.uint32)
    q = R_to_quat(R)
    return ScaleProblem(np.ascontiguousarray(XL), np.ascontiguousarray(XR), tri_l, tri_r, last_l, last_r, lframe,
                        K.copy(), K.copy(), q, t.copy(), q.copy(), t.copy(), scale0, BASELINE, w,
                        np.ascontiguousarray(fr.left), np.ascontiguousarray(fr.right))


def random_patches(seed: int, width: int, height: int, n: int, pw: int, ph: int):
    """Random images + corner lists for batched MI tests/benchmarks."""
    rng = np.random.default_rng(seed)
    scene, K, frames = stereo_stream(seed, width, height, 1)
    L, Rimg = frames[0].left, frames[0].right
    xyL = np.stack([rng.integers(0, width - pw + 1, n), rng.integers(0, height - ph + 1, n)], -1).astype(np.int32)
    d = rng.integers(-3, 40, n)
    xyR = np.stack([np.clip(xyL[:, 0] - d, 0, width - pw), np.clip(xyL[:, 1] + rng.integers(-1, 2, n), 0,
                                                                     height - ph)], -1).astype(np.int32)
    return L, Rimg, np.ascontiguousarray(xyL), np.ascontiguousarray(xyR)


def vo_matches(seed: int, n: int, width: int = 1280, height: int = 720, noise: float = 0.0,
               state=(0.004, -0.006, 0.003, 0.05, -0.02, 0.5), n_outliers: int = 0):
    """Quad matches (n, 8) float32 {f1, f2, f3, f4} of a stereo rig moving by
    `state` (Euler angles, translation) in the StereoVisualOdometry convention
    (project3D :22-32, reproject :116-141: X_cur = R4(state)^T X_prev + t).
    Returns (matches, params dict for vo.Parameters).  `noise` px of Gaussian
    noise on f3/f4; the first `n_outliers` rows get f3/f4 shifted 20-60 px."""
    rng = np.random.default_rng(seed)
    K = intrinsics(width, height)
    f, cu, cv = K[0, 0], K[0, 2], K[1, 2]
    b = BASELINE
    r, p, y = state[:3]
    cr, sr, cp, sp, cy, sy = (math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y))
    R = np.array([[cp * cy, cp * sy, -sp],
                  [sp * sr * cy - cr * sy, sr * sp * sy + cr * cy, cp * sr],
                  [cr * sp * cy + sr * sy, cr * sp * sy - sr * cy, cp * cr]])
    out = np.zeros((n, 8), np.float32)
    k = 0
    while k < n:
        u = rng.uniform(20, width - 20)
        v = rng.uniform(20, height - 20)
        Z = rng.uniform(5.0, 40.0)
        d = f * b / Z
        # f1/f2 as float32 first: project3D works on the float features
        f1 = np.float32([u, v])
        f2 = np.float32([u - d, v])
        dd = float(f1[0] - cu) - float(f2[0] - cu)
        if dd <= 0:
            continue
        Xp = np.array([(float(f1[0]) - cu) * b / dd, (float(f1[1]) - cv) * b / dd, f * b / dd])
        Xc = R.T @ Xp + np.asarray(state[3:6])
        if Xc[2] < 1.0:
            continue
        u3, v3 = f * Xc[0] / Xc[2] + cu, f * Xc[1] / Xc[2] + cv
        u4 = (f * Xc[0] - b * f) / Xc[2] + cu
        if not (0 <= u3 < width and 0 <= v3 < height and 0 <= u4 < width):
            continue
        f3 = np.array([u3, v3]) + (rng.normal(0, noise, 2) if noise else 0)
        f4 = np.array([u4, v3]) + (rng.normal(0, noise, 2) if noise else 0)
        if k < n_outliers:
            sh = rng.uniform(20, 60, 2) * rng.choice([-1, 1], 2)
            f3 = f3 + sh
            f4 = f4 + sh
        out[k] = (f1[0], f1[1], f2[0], f2[1], f3[0], f3[1], f4[0], f4[1])
        k += 1
    params = dict(baseline=b, fu1=f, fv1=f, fu2=f, fv2=f, cu1=cu, cu2=cu, cv1=cv, cv2=cv)
    return out, params


def mono_matches(seed: int, n: int, width: int = 1280, height: int = 720, noise: float = 0.3,
                 aa=(0.01, -0.02, 0.005), t=(0.3, -0.05, 1.0), n_outliers: int = 0, n_invalid: int = 0):
    """Two-view matches (f1 in view 1, f2 in view 2; the MonoVisualOdometry
    input, MonoVisualOdometry.cpp:7-17) of points 4-40 m in front of a
    camera that moves by X2 = R(aa) X1 + t (t normalised to 1 m: the mono scale
    is unobservable).  `noise` px Gaussian on both views; the first
    `n_outliers` matches get f2 shifted 15-60 px; the last `n_invalid` get
    f1.x = -1 (dropped by the reference's f1.x > 0 test).  Returns
    (f1 (n, 2) float32, f2 (n, 2) float32, params dict, R, t unit)."""
    rng = np.random.default_rng(seed)
    K = intrinsics(width, height)
    f, cu, cv = K[0, 0], K[0, 2], K[1, 2]
    R = aa_to_R(np.asarray(aa, np.float64))
    tv = np.asarray(t, np.float64)
    tv = tv / np.linalg.norm(tv)
    f1 = np.zeros((n, 2), np.float32)
    f2 = np.zeros((n, 2), np.float32)
    k = 0
    while k < n:
        u, v, Z = rng.uniform(10, width - 10), rng.uniform(10, height - 10), rng.uniform(4.0, 40.0)
        X1 = np.array([(u - cu) * Z / f, (v - cv) * Z / f, Z])
        X2 = R @ X1 + tv
        if X2[2] < 1.0:
            continue
        u2, v2 = f * X2[0] / X2[2] + cu, f * X2[1] / X2[2] + cv
        if not (0 <= u2 < width and 0 <= v2 < height):
            continue
        a = np.array([u, v]) + (rng.normal(0, noise, 2) if noise else 0)
        b = np.array([u2, v2]) + (rng.normal(0, noise, 2) if noise else 0)
        if k < n_outliers:
            b = b + rng.uniform(15, 60, 2) * rng.choice([-1, 1], 2)
        f1[k], f2[k] = a, b
        k += 1
    if n_invalid:
        f1[n - n_invalid:, 0] = -1.0
    return f1, f2, dict(fu=f, fv=f, cu=cu, cv=cv), R, tv
