"""Windowed stereo VO front-to-back on one stereo stream (the config-5 shape).

The reference is a library: its application (the loop that feeds
`Optimiser<ScaleState,...>` and `BundleAdjuster<4>` from tracked features)
lives outside it.  This module is that loop, written against the reference's
own data model so the hot-path calls see what the reference's callers would
pass them:

per keyframe t (every frame is a keyframe)
  1. KLT: the active tracks' last left features, L(t-1) -> L(t) (klt.hip);
     a track whose status is 0 or whose new position leaves the feature
     margin stops being tracked (it keeps its features in the window);
  2. MI stereo matching (build-defined, like KLT): every tracked or new
     feature is matched along the rectified epipolar line of R(t) by the
     batched mutual-information score (me_mi_scores, 11 x 11 patches, one
     candidate per integer disparity), best candidate + parabola sub-pixel
     refinement; a feature whose best disparity is at the range's edge is
     dropped;
  3. WBA_Point bookkeeping (include/MotionEstimation/core/feature_types.h:
     121-197): tracked features `addMatch((l, r), t)`; empty grid cells get
     new tracks (value constructor: ID = latestID++) triangulated from their
     stereo match at the predicted pose of t; `pop()` drops features that fell
     out of the window (tracks with none left are deleted);
  4. pose prediction for t: constant velocity on {t, angle-axis};
  5. scale LM: Optimiser<ScaleState, vector<pair<Mat,Mat>>>::optimise
     (optimisation.cpp:29-147) over the tracks seen in t, window poses,
     images of t (the frame's scale estimate is recorded);
  6. BundleAdjuster<4> over the last W keyframes (BundleAdjuster.h:208-229,
     :354-376 initialiseObservations with first_frame = the window's first
     keyframe ID, fixedFrames = 2, fixed LM iterations), poses and points
     written back.

Every decision above is a pure function of the images and of the hot-path
results, so a backend (GPU: libme_hip.so; tests: the oracle) that reproduces
the hot path reproduces the track IDs, feature positions and poses.  Host
bookkeeping is vectorised numpy over a structure-of-arrays track table; the
WBA_Point semantics are cross-checked in tests/test_pipeline.py by replaying
the event log through feature_types.WBA_Point.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from . import synthetic as S

PATCH = 11          # MI patch (11 x 11, window_size 5)
W_SCALE = 5         # ScaleState::window_size
MARGIN = 4 * W_SCALE + 4  # feature margin: every scale-LM ROI (incl. the +1 px NEQ patch) stays inside


# ------------------------------------------------------------------ rotations (host, FP64)
def aa_to_R(aa):
    return S.aa_to_R(np.asarray(aa, np.float64))


def R_to_quat(R):
    return S.R_to_quat(R)


@dataclass
class PipelineConfig:
    width: int
    height: int
    n_feats: int
    window: int
    ba_iters: int = 10
    scale_iters: int = 10
    fixed_frames: int = 2
    d_min: int = 2
    d_max: int = 128
    baseline: float = S.BASELINE
    feat_var: float = 0.25

    @staticmethod
    def from_config(c: int, **kw) -> "PipelineConfig":
        cfg = S.CONFIGS[c]
        return PipelineConfig(cfg["width"], cfg["height"], cfg["n_feats"], cfg["window"], **kw)


@dataclass
class FrameResult:
    t: int
    n_tracked: int
    n_new: int
    n_active: int
    n_window_pts: int
    n_window_obs: int
    scale: float
    scale_stop: int
    scale_iters: int
    ba_iters: int
    ba_cost: float
    pose: np.ndarray = field(repr=False)


class Backend:
    """The hot-path calls of the loop.  Images are handles returned by
    frame_images(); corner / point arrays are host numpy."""

    def frame_images(self, t: int, left: np.ndarray, right: np.ndarray):
        raise NotImplementedError

    def klt(self, prev, cur, pts: np.ndarray):
        """(n, 2) float32 -> (n, 2) float32, (n,) uint8 status."""
        raise NotImplementedError

    def mi_scores(self, imgs, xyL: np.ndarray, xyR: np.ndarray) -> np.ndarray:
        """MI of 11 x 11 pairs (left patch in L, right patch in R), float32."""
        raise NotImplementedError

    def scale_optimise(self, sp, params) -> dict:
        raise NotImplementedError

    def ba_solve(self, bp, iters: int):
        """(cams, pts, summary dict) after `iters` fixed LM iterations."""
        raise NotImplementedError


class GPUBackend(Backend):
    """libme_hip.so through the C ABI; images resident in HBM (one upload per frame)."""

    def __init__(self, ctx=None):
        from ._lib import default_context

        self.ctx = ctx or default_context()
        self._imgs = {}

    def frame_images(self, t, left, right):
        if t in self._imgs:
            return self._imgs[t]
        L = np.ascontiguousarray(left, np.uint8)
        R = np.ascontiguousarray(right, np.uint8)
        dL, dR = self.ctx.malloc(L.nbytes), self.ctx.malloc(R.nbytes)
        self.ctx.h2d(dL, L)
        self.ctx.h2d(dR, R)
        h = (dL, dR, L.shape, L, R)
        self._imgs[t] = h
        return h

    def release(self, t):
        h = self._imgs.pop(t, None)
        if h is not None:
            self.ctx.free(h[0])
            self.ctx.free(h[1])

    def close(self):
        for t in list(self._imgs):
            self.release(t)

    def klt(self, prev, cur, pts):
        import ctypes

        from ._lib import ME_DEVICE
        from .klt import klt_params

        n = len(pts)
        out = np.zeros((n, 2), np.float32)
        st = np.zeros(n, np.uint8)
        if n == 0:
            return out, st
        H, W = prev[2]
        c = self.ctx
        pts = np.ascontiguousarray(pts, np.float32)
        d_in, d_out, d_st = c.malloc(8 * n), c.malloc(8 * n), c.malloc(max(n, 16))
        try:
            c.h2d(d_in, pts)
            kp = klt_params()
            c.check(c.lib.me_klt_track(c.h, ME_DEVICE, ctypes.c_void_p(prev[0]), ctypes.c_void_p(cur[0]), W, H, W,
                                       ctypes.c_void_p(d_in), ctypes.c_void_p(d_out), ctypes.c_void_p(d_st), n,
                                       ctypes.byref(kp)), "me_klt_track")
            c.d2h(out, d_out)
            c.d2h(st, d_st)
        finally:
            for p in (d_in, d_out, d_st):
                c.free(p)
        return out, st

    def mi_scores(self, imgs, xyL, xyR):
        from .mutual_information import mi_scores_device

        n = len(xyL)
        out = np.zeros(n, np.float32)
        if n == 0:
            return out
        H, W = imgs[2]
        c = self.ctx
        xyL = np.ascontiguousarray(xyL, np.int32)
        xyR = np.ascontiguousarray(xyR, np.int32)
        dl, dr, do = c.malloc(xyL.nbytes), c.malloc(xyR.nbytes), c.malloc(4 * n)
        try:
            c.h2d(dl, xyL)
            c.h2d(dr, xyR)
            mi_scores_device(c, imgs[0], W, imgs[1], W, W, H, dl, dr, n, (PATCH, PATCH), do)
            c.d2h(out, do)
        finally:
            for p in (dl, dr, do):
                c.free(p)
        return out

    def scale_optimise(self, sp, params):
        from ._lib import ME_DEVICE
        from .optimisation import scale_optimise

        imgs = sp.imgs_handle
        return scale_optimise(sp, params, ctx=self.ctx, img_mem=ME_DEVICE, dev_imgs=(imgs[0], imgs[1]))

    def ba_solve(self, bp, iters):
        from .optimisation import SolverOptions, ba_solve

        return ba_solve(bp, SolverOptions.fixed_iterations(iters), ctx=self.ctx)


def _cell_jitter(t: int, cells: np.ndarray) -> np.ndarray:
    """Deterministic jitter in [-0.3, 0.3) per (frame, cell), two components."""
    h = (cells.astype(np.uint64) * np.uint64(2654435761) + np.uint64(t) * np.uint64(40503)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(2246822519)) & np.uint64(0xFFFFFFFF)
    a = (h & np.uint64(0xFFFF)).astype(np.float64) / 65536.0
    b = ((h >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.float64) / 65536.0
    return np.stack([a, b], -1) * 0.6 - 0.3


class WindowedStereoVO:
    """The loop of the module docstring.  `events` logs the WBA_Point calls
    (("new", id, t, (l, r)), ("add", id, t, (l, r)), ("pop", id), ("del", id))
    when log_events is set."""

    def __init__(self, cfg: PipelineConfig, backend: Backend, K=None, first_pose=None, velocity=None,
                 log_events: bool = False):
        self.cfg = cfg
        self.be = backend
        self.K = np.asarray(S.intrinsics(cfg.width, cfg.height) if K is None else K, np.float64)
        self.f, self.cx, self.cy = self.K[0, 0], self.K[0, 2], self.K[1, 2]
        # grid of feature cells over the margin-free interior
        aw, ah = cfg.width - 2 * MARGIN, cfg.height - 2 * MARGIN
        self.nx = max(1, int(round(math.sqrt(cfg.n_feats * aw / ah))))
        self.ny = max(1, int(math.ceil(cfg.n_feats / self.nx)))
        self.cw, self.ch = aw / self.nx, ah / self.ny
        # track table (structure of arrays, index = creation order = ID order)
        self.ids = np.zeros(0, np.int64)
        self.X = np.zeros((0, 3))
        self.active = np.zeros(0, bool)
        self.first = np.zeros(0, np.int64)   # first frame still held (after pops)
        self.last = np.zeros(0, np.int64)    # last frame observed
        self.latest_id = 0                   # WBA_Point<pair<Point2f,Point2f>>::latestID
        self.obs = {}                        # t -> (track indices int64, (n, 4) float32 {xl, yl, xr, yr})
        self.poses = {}                      # t -> {t, angle-axis} world -> camera
        self.first_pose = np.zeros(6) if first_pose is None else np.asarray(first_pose, np.float64)
        self.velocity = velocity             # prior {t, aa} step for the second frame
        self.prev_imgs = None
        self.prev_t = None
        self.log_events = log_events
        self.events = []
        self.results = []

    # ---------------------------------------------------------------- matching
    def stereo_match(self, imgs, uv: np.ndarray, d_pred=None, ratio: float = 1.2, half: int = 6):
        """MI disparity search for features uv (n, 2) float32 -> (xr float32, ok).

        Tracked features (d_pred given) search +-half px around the disparity
        their 3-D point predicts at the predicted pose; new features search
        [d_min, d_max] and must pass a uniqueness test (best MI >= ratio x
        the best outside +-2 px of it).  Best integer candidate, parabola
        sub-pixel refinement; the best must be an interior maximum."""
        cfg = self.cfg
        n = len(uv)
        if n == 0:
            return np.zeros(0, np.float32), np.zeros(0, bool)
        x0 = np.floor(uv[:, 0].astype(np.float64) - W_SCALE).astype(np.int64)  # Rect(x - w, ..) truncation
        y0 = np.floor(uv[:, 1].astype(np.float64) - W_SCALE).astype(np.int64)
        if d_pred is None:
            lo = np.full(n, cfg.d_min, np.int64)
            nd = cfg.d_max - cfg.d_min + 1
        else:
            dp = np.where(np.isfinite(d_pred), d_pred, -1e9)
            lo = np.clip(np.rint(dp).astype(np.int64) - half, cfg.d_min, cfg.d_max)
            nd = 2 * half + 1
        d = lo[:, None] + np.arange(nd, dtype=np.int64)[None, :]
        xr = x0[:, None] - d
        valid = (xr >= 0) & (d <= cfg.d_max)
        if d_pred is not None:
            valid &= np.isfinite(d_pred)[:, None] & (d_pred > 0)[:, None]
        xr_c = np.where(valid, xr, 0)
        xyL = np.stack([np.repeat(x0, nd), np.repeat(y0, nd)], -1)
        xyR = np.stack([xr_c.ravel(), np.repeat(y0, nd)], -1)
        sc = self.be.mi_scores(imgs, xyL, xyR).reshape(n, nd).astype(np.float64)
        sc = np.where(valid, sc, -np.inf)
        with np.errstate(invalid="ignore", divide="ignore"):  # -inf candidates (outside the image)
            return self._pick(uv, d, sc, nd, d_pred, ratio)

    def _pick(self, uv, d, sc, nd, d_pred, ratio):
        n = len(uv)
        rows = np.arange(n)
        k = np.argmax(sc, axis=1)
        best = sc[rows, k]
        ok = (k > 0) & (k < nd - 1) & np.isfinite(best)
        kk = np.clip(k, 1, nd - 2)
        s_m, s_0, s_p = sc[rows, kk - 1], sc[rows, kk], sc[rows, kk + 1]
        den = s_m - 2 * s_0 + s_p
        ok &= np.isfinite(s_m) & np.isfinite(s_p) & (den < 0)
        if d_pred is None:  # uniqueness against the best candidate outside +-2 px
            m = sc.copy()
            for j in range(-2, 3):
                m[rows, np.clip(k + j, 0, nd - 1)] = -np.inf
            second = m.max(axis=1)
            ok &= best >= ratio * second
        den_s = np.where(ok, den, -1.0)
        delta = np.where(ok, 0.5 * (s_m - s_p) / den_s, 0.0)
        disp = d[rows, kk].astype(np.float64) + delta
        xr_f = (uv[:, 0].astype(np.float64) - disp).astype(np.float32)
        ok &= xr_f >= MARGIN
        return xr_f, ok

    def _predicted_disparity(self, idx, pose):
        R = aa_to_R(pose[3:])
        Z = self.X[idx] @ R[2] + pose[2]
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.where(Z > 0, self.f * self.cfg.baseline / Z, np.nan)

    # ---------------------------------------------------------------- helpers
    def _in_margin(self, uv):
        cfg = self.cfg
        return ((uv[:, 0] >= MARGIN) & (uv[:, 0] < cfg.width - MARGIN) & (uv[:, 1] >= MARGIN)
                & (uv[:, 1] < cfg.height - MARGIN))

    def _predict_pose(self, t):
        if t == 0:
            return self.first_pose.copy()
        p1 = self.poses[t - 1]
        if t == 1 or (t - 2) not in self.poses:
            v = np.zeros(6) if self.velocity is None else np.asarray(self.velocity, np.float64)
        else:
            v = p1 - self.poses[t - 2]
        return p1 + v

    def _triangulate(self, uv, xr, pose):
        disp = uv[:, 0].astype(np.float64) - xr.astype(np.float64)
        Z = self.f * self.cfg.baseline / disp
        pc = np.stack([(uv[:, 0].astype(np.float64) - self.cx) * Z / self.f,
                       (uv[:, 1].astype(np.float64) - self.cy) * Z / self.f, Z], -1)
        R = aa_to_R(pose[3:])
        return (pc - pose[:3][None, :]) @ R  # R^T (pc - t), row form

    def _add_tracks(self, t, uv, xr, pose):
        n = len(uv)
        ids = np.arange(self.latest_id, self.latest_id + n, dtype=np.int64)
        self.latest_id += n
        self.ids = np.concatenate([self.ids, ids])
        self.X = np.concatenate([self.X, self._triangulate(uv, xr, pose)])
        self.active = np.concatenate([self.active, np.ones(n, bool)])
        self.first = np.concatenate([self.first, np.full(n, t, np.int64)])
        self.last = np.concatenate([self.last, np.full(n, t, np.int64)])
        return np.arange(len(self.ids) - n, len(self.ids), dtype=np.int64)

    # ---------------------------------------------------------------- one keyframe
    def process(self, t: int, left: np.ndarray, right: np.ndarray) -> FrameResult:
        cfg = self.cfg
        imgs = self.be.frame_images(t, left, right)
        pose = self._predict_pose(t)
        self.poses[t] = pose
        trk_idx = np.zeros(0, np.int64)
        trk_uv = np.zeros((0, 2), np.float32)
        # 1. KLT of the active tracks
        if self.prev_imgs is not None and self.active.any():
            act = np.flatnonzero(self.active)
            pi, puv = self.obs[self.prev_t]
            pos = np.searchsorted(pi, act)
            prev_uv = np.ascontiguousarray(puv[pos, :2])
            uv, st = self.be.klt(self.prev_imgs, imgs, prev_uv)
            keep = (st == 1) & self._in_margin(uv)
            self.active[act[~keep]] = False
            trk_idx, trk_uv = act[keep], uv[keep]
        # 2. stereo matching of the tracked features (around their predicted disparity)
        xr, ok = self.stereo_match(imgs, trk_uv, self._predicted_disparity(trk_idx, pose))
        self.active[trk_idx[~ok]] = False
        trk_idx, trk_uv, xr = trk_idx[ok], trk_uv[ok], xr[ok]
        n_tracked = len(trk_idx)
        # 3a. new tracks in empty cells
        occ = np.zeros(self.nx * self.ny, bool)
        if n_tracked:
            cx = np.clip(((trk_uv[:, 0] - MARGIN) / self.cw).astype(np.int64), 0, self.nx - 1)
            cy = np.clip(((trk_uv[:, 1] - MARGIN) / self.ch).astype(np.int64), 0, self.ny - 1)
            occ[cy * self.nx + cx] = True
        empty = np.flatnonzero(~occ)[: max(0, cfg.n_feats - n_tracked)]
        cyx = np.stack([empty % self.nx, empty // self.nx], -1).astype(np.float64)
        nuv = (MARGIN + (cyx + 0.5 + _cell_jitter(t, empty)) * np.array([self.cw, self.ch])).astype(np.float32)
        nxr, nok = self.stereo_match(imgs, nuv)
        nuv, nxr = nuv[nok], nxr[nok]
        new_idx = self._add_tracks(t, nuv, nxr, pose)
        # 3b. this frame's features (tracked first, then new; sorted by track = ID order)
        idx = np.concatenate([trk_idx, new_idx])
        feats = np.concatenate([np.concatenate([trk_uv, xr[:, None], trk_uv[:, 1:2]], 1),
                                np.concatenate([nuv, nxr[:, None], nuv[:, 1:2]], 1)]).astype(np.float32)
        o = np.argsort(idx, kind="stable")
        idx, feats = idx[o], feats[o]
        self.obs[t] = (idx, feats)
        self.last[idx] = t
        if self.log_events:
            is_new = np.zeros(len(self.ids), bool)
            is_new[new_idx] = True
            for i, fe in zip(idx, feats):
                self.events.append(("new" if is_new[i] else "add", int(self.ids[i]), t, tuple(float(v) for v in fe)))
        # 5. scale LM over the tracks seen in t
        sc = self._scale(t, imgs, idx)
        # 6. windowed BA
        nwp, nwo, bs = self._ba(t)
        # 3c. pop the features that leave the window with the next keyframe
        self._pop(t + 1 - cfg.window)
        self.prev_imgs, self.prev_t = imgs, t
        r = FrameResult(t, n_tracked, len(new_idx), int(self.active.sum()), nwp, nwo, sc["scale"], int(sc["stop"]),
                        int(sc["iterations"]), int(bs["iterations"]), float(bs["final_cost"]), self.poses[t].copy())
        self.results.append(r)
        return r

    def _scale(self, t, imgs, idx):
        from .optimisation import OptimisationParams

        pose = self.poses[t]
        R = aa_to_R(pose[3:])
        q = R_to_quat(R)
        Xh = np.concatenate([self.X[idx], np.ones((len(idx), 1))], 1)
        n = len(idx)
        sp = S.ScaleProblem(np.ascontiguousarray(Xh), np.zeros((0, 4)), np.ones(n, np.uint8), np.zeros(0, np.uint8),
                            np.full(n, t, np.uint32), np.zeros(0, np.uint32), t, self.K.copy(), self.K.copy(), q,
                            pose[:3].copy(), q.copy(), pose[:3].copy(), 1.0, self.cfg.baseline, W_SCALE, imgs[3],
                            imgs[4])
        sp.imgs_handle = imgs
        return self.be.scale_optimise(sp, OptimisationParams.fixed_iterations(self.cfg.scale_iters))

    def _ba(self, t):
        cfg = self.cfg
        f0 = max(0, t - cfg.window + 1)
        frames = [f for f in range(f0, t + 1) if f in self.obs]
        if t - f0 + 1 <= cfg.fixed_frames:
            return 0, 0, {"iterations": 0, "final_cost": float("nan")}
        ti = np.concatenate([self.obs[f][0] for f in frames])
        fe = np.concatenate([self.obs[f][1] for f in frames])
        fr = np.concatenate([np.full(len(self.obs[f][0]), f, np.int64) for f in frames])
        # initialiseObservations order (BundleAdjuster.h:354-376): points in track order, features in frame order
        o = np.lexsort((fr, ti))
        ti, fe, fr = ti[o], fe[o], fr[o]
        upts, pt_idx = np.unique(ti, return_inverse=True)
        cams = np.stack([self.poses[f] for f in range(f0, t + 1)])
        bp = S.BAProblem(cams, self.X[upts].copy(), fe.astype(np.float64), (fr - f0).astype(np.int32),
                         pt_idx.astype(np.int32), self.K.copy(), self.K.copy(), cfg.baseline, cfg.feat_var,
                         cfg.fixed_frames)
        c, p, s = self.be.ba_solve(bp, cfg.ba_iters)
        if s.get("status", 2) == 2:
            for k, f in enumerate(range(f0, t + 1)):
                self.poses[f] = np.asarray(c[k], np.float64).copy()
            self.X[upts] = p
        return len(upts), len(ti), s

    def _pop(self, new_first):
        """WBA_Point::pop() of every feature older than `new_first`; empty tracks deleted."""
        for f in [f for f in self.obs if f < new_first]:
            idx, _ = self.obs.pop(f)
            if self.log_events:
                for i in idx:
                    self.events.append(("pop", int(self.ids[i])))
            self.first[idx] = f + 1
        dead = (self.last < new_first)
        if dead.any():
            if self.log_events:
                for i in np.flatnonzero(dead):
                    self.events.append(("del", int(self.ids[i])))
            keep = ~dead
            remap = np.cumsum(keep) - 1
            self.ids, self.X, self.active = self.ids[keep], self.X[keep], self.active[keep]
            self.first, self.last = self.first[keep], self.last[keep]
            self.obs = {f: (remap[i], fe) for f, (i, fe) in self.obs.items()}


def synthetic_sequence(c: int, n_frames: int, seed: int | None = None, render_div: int = 1):
    """Stereo keyframes of config c's synthetic trajectory (0.5 m forward and
    0.3 deg yaw per keyframe), the true first pose and the per-frame motion
    prior used for the second keyframe."""
    cfg = S.CONFIGS[c]
    seed = S.SEED0 + c if seed is None else seed
    scene, K, frames = S.stereo_stream(seed, cfg["width"], cfg["height"], n_frames, render_div=render_div)
    poses = []
    for fr in frames:
        poses.append(np.concatenate([fr.t, S.R_to_aa(fr.R)]))
    return frames, K, poses[0], poses[1] - poses[0], poses
