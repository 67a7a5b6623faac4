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
import os
from dataclasses import dataclass, field

import numpy as np

from . import synthetic as S

ROCTX = os.environ.get("ME_ROCTX", "0") == "1"  # roctx ranges around the loop's stages (rocprofv3 --marker-trace)

PATCH = 11          # MI patch (11 x 11, window_size 5)
W_SCALE = 5         # ScaleState::window_size
MARGIN = 4 * W_SCALE + 4  # feature margin: every scale-LM ROI (incl. the +1 px NEQ patch) stays inside


# ------------------------------------------------------------------ rotations (host, FP64)
def aa_to_R(aa):
    return S.aa_to_R(np.asarray(aa, np.float64))


def R_to_quat(R):
    return S.R_to_quat(R)


# (-1)^k / (2k+1)! and (-1)^k / (2k+2)!: the same literals as vo_chain_kernel (csrc/ba.hip)
_ROT_A = (1.0, -0.16666666666666666, 0.008333333333333333, -0.0001984126984126984, 2.7557319223985893e-06,
          -2.505210838544172e-08, 1.6059043836821613e-10, -7.647163731819816e-13, 2.8114572543455206e-15,
          -8.22063524662433e-18, 1.9572941063391263e-20, -3.868170170630684e-23, 6.446950284384474e-26,
          -9.183689863795546e-29, 1.1309962886447716e-31, -1.216125041553518e-34, 1.151633562077195e-37,
          -9.67759295863189e-41, 7.265460179153071e-44, -4.902469756513544e-47, 2.9893108271424046e-50,
          -1.6552108677421951e-53, 8.359650847182804e-57, -3.866628513960594e-60)
_ROT_B = (0.5, -0.041666666666666664, 0.001388888888888889, -2.48015873015873e-05, 2.755731922398589e-07,
          -2.08767569878681e-09, 1.1470745597729725e-11, -4.779477332387385e-14, 1.5619206968586225e-16,
          -4.110317623312165e-19, 8.896791392450574e-22, -1.6117375710961184e-24, 2.4795962632247976e-27,
          -3.279889237069838e-30, 3.7699876288159054e-33, -3.8003907548547434e-36, 3.387157535521162e-39,
          -2.6882202662866363e-42, 1.911963205040282e-45, -1.2256174391283858e-48, 7.117406731291439e-52,
          -3.7618428812322616e-55, 1.817315401561479e-58, -8.055476070751236e-62)


def rot_series(aa):
    """Angle-axis -> rotation, R = I + A [a]x + B [a]x^2 with A = sin(th) / th
    and B = (1 - cos th) / th^2 as Taylor series in th^2 (24 terms, Horner):
    only +, -, * in a fixed order, so the device (me_vo_ba_chain) forms the
    same bits.  The loop's pose(t) re-prediction uses it (step 7)."""
    a0, a1, a2 = float(aa[0]), float(aa[1]), float(aa[2])
    t2 = (a0 * a0 + a1 * a1) + a2 * a2
    A, B = _ROT_A[23], _ROT_B[23]
    for k in range(22, -1, -1):
        A = A * t2 + _ROT_A[k]
        B = B * t2 + _ROT_B[k]
    av = (a0, a1, a2)
    K = ((0.0, -a2, a1), (a2, 0.0, -a0), (-a1, a0, 0.0))
    R = np.empty((3, 3))
    for i in range(3):
        for j in range(3):
            k2 = av[i] * av[j] - (t2 if i == j else 0.0)
            R[i, j] = ((1.0 if i == j else 0.0) + A * K[i][j]) + B * k2
    return R


def move_landmarks(X, R, pose, pose2, R2):
    """Landmarks triangulated at `pose` (rotation R) moved to `pose2`
    (rotation R2), camera-frame coordinates kept: x_c = R X + t, then
    R2^T (x_c - t2) -- elementwise, in the order vo_chain_kernel uses."""
    d = [(((X[:, 0] * R[k, 0] + X[:, 1] * R[k, 1]) + X[:, 2] * R[k, 2]) + pose[k]) - pose2[k] for k in range(3)]
    return np.stack([(d[0] * R2[0, k] + d[1] * R2[1, k]) + d[2] * R2[2, k] for k in range(3)], 1)


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


def match_host(be, imgs, uv, lo, nd, dvalid, unique: bool, d_max: int, ratio: float = 1.2):
    """MI disparity search, the numpy restatement (the oracle backend's
    matcher; the GPU backend runs the same on the device,
    me_mi_epipolar_match): feature k searches d = lo_k .. lo_k + nd - 1;
    returns (xr float32, ok).  Best integer candidate, parabola sub-pixel
    refinement, the best must be an interior maximum; with `unique` it must
    also be >= ratio x the best outside +-2 px of it."""
    n = len(uv)
    if n == 0:
        return np.zeros(0, np.float32), np.zeros(0, bool)
    x0 = np.floor(uv[:, 0].astype(np.float64) - W_SCALE).astype(np.int64)  # Rect(x - w, ..) truncation
    y0 = np.floor(uv[:, 1].astype(np.float64) - W_SCALE).astype(np.int64)
    d = lo[:, None] + np.arange(nd, dtype=np.int64)[None, :]
    xr = x0[:, None] - d
    P = 2 * W_SCALE + 1  # both patches inside the image (the right one: xr >= 0)
    H, W = imgs[2][:2]
    inside = (x0 >= 0) & (y0 >= 0) & (x0 + P <= W) & (y0 + P <= H)
    valid = (xr >= 0) & (d <= d_max) & inside[:, None]
    if dvalid is not None:
        valid &= dvalid[:, None]
    xr_c = np.where(valid, xr, 0)
    x0c, y0c = np.where(inside, x0, 0), np.where(inside, y0, 0)  # (scored -inf below: any in-image corner)
    xyL = np.stack([np.repeat(x0c, nd), np.repeat(y0c, nd)], -1)
    xyR = np.stack([xr_c.ravel(), np.repeat(y0c, nd)], -1)
    sc = be.mi_scores(imgs, xyL, xyR).reshape(n, nd).astype(np.float64)
    sc = np.where(valid, sc, -np.inf)
    with np.errstate(invalid="ignore", divide="ignore"):  # -inf candidates (outside the image)
        return _pick(uv, d, sc, nd, unique, ratio)


def _pick(uv, d, sc, nd, unique, ratio):
    n = len(uv)
    rows = np.arange(n)
    k = np.argmax(sc, axis=1)
    best = sc[rows, k]
    ok = (k > 0) & (k < nd - 1) & np.isfinite(best)
    kk = np.clip(k, 1, nd - 2)
    s_m, s_0, s_p = sc[rows, kk - 1], sc[rows, kk], sc[rows, kk + 1]
    den = s_m - 2 * s_0 + s_p
    ok &= np.isfinite(s_m) & np.isfinite(s_p) & (den < 0)
    if unique:  # uniqueness against the best candidate outside +-2 px
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


def new_cells(t: int, uv_good: np.ndarray, grid) -> np.ndarray:
    """New features of keyframe t: the good tracked features (uv_good) occupy
    their grid cell (trunc((u - MARGIN) / cw), trunc((v - MARGIN) / ch)),
    clamped, in FP64; the first max(0, n_feats - #good) empty cells in
    ascending order get a feature at MARGIN + (cell + 0.5 + jitter) * (cw, ch),
    rounded to float32 (me_vo_new_cells computes the same on the device)."""
    nx, ny, cw, ch, n_feats = grid
    occ = np.zeros(nx * ny, bool)
    if len(uv_good):
        cx = np.clip(((uv_good[:, 0].astype(np.float64) - MARGIN) / cw).astype(np.int64), 0, nx - 1)
        cy = np.clip(((uv_good[:, 1].astype(np.float64) - MARGIN) / ch).astype(np.int64), 0, ny - 1)
        occ[cy * nx + cx] = True
    empty = np.flatnonzero(~occ)[: max(0, n_feats - len(uv_good))]
    cyx = np.stack([empty % nx, empty // nx], -1).astype(np.float64)
    return (MARGIN + (cyx + 0.5 + _cell_jitter(t, empty)) * np.array([cw, ch])).astype(np.float32)


def camera_centre(pose) -> np.ndarray:
    """World position of a {t, angle-axis} world->camera pose: -R^T t (drift
    is measured on centres: the world->camera translation also carries the
    rotation error times the distance from the world origin)."""
    pose = np.asarray(pose, np.float64)
    return -aa_to_R(pose[3:]).T @ pose[:3]


def in_margin(uv, width, height):
    return ((uv[:, 0] >= MARGIN) & (uv[:, 0] < width - MARGIN) & (uv[:, 1] >= MARGIN)
            & (uv[:, 1] < height - MARGIN))


class Backend:
    """The hot-path calls of the loop.  Images are handles returned by
    frame_images(); corner / point arrays are host numpy.  The staged calls
    (klt_submit / klt_match, ba_submit / ba_result, scale_submit /
    scale_result) default to the plain ones run synchronously; the GPU
    backend queues them (front end and BA on separate streams)."""

    d_max = 128

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

    # ---- staged forms
    def klt_submit(self, prev, cur, pts):
        return (prev, cur, np.ascontiguousarray(pts, np.float32))

    def klt_match(self, h, imgs, lo, nd, dvalid):
        """KLT of the submitted points, then the MI search (lo, nd, dvalid per
        point) of those that pass the KLT gate: (uv, status, xr, ok)."""
        prev, cur, pts = h
        uv, st = self.klt(prev, cur, pts)
        H, W = imgs[2]
        keep = (st == 1) & in_margin(uv, W, H)
        xr = np.zeros(len(uv), np.float32)
        ok = np.zeros(len(uv), bool)
        xk, okk = match_host(self, imgs, uv[keep], lo[keep], nd, dvalid[keep], False, self.d_max)
        xr[keep], ok[keep] = xk, okk
        return uv, st, xr, ok

    def match(self, imgs, uv, lo, nd, unique):
        return match_host(self, imgs, uv, lo, nd, None, unique, self.d_max)

    def klt_match_new(self, h, imgs, lo, nd, dvalid, t, grid, d_min, nd_new):
        """klt_match, then the new features of the cells the good tracked
        features leave empty (new_cells) matched with the uniqueness test:
        (uv, status, xr, ok, new_uv, new_xr, new_ok)."""
        uv, st, xr, ok = self.klt_match(h, imgs, lo, nd, dvalid)
        H, W = imgs[2]
        good = (st == 1) & in_margin(uv, W, H) & ok
        nuv = new_cells(t, uv[good], grid)
        nxr, nok = self.match(imgs, nuv, np.full(len(nuv), d_min, np.int64), nd_new, True)
        return uv, st, xr, ok, nuv, nxr, nok

    def scale_submit(self, sp, params):
        self._scale_res = self.scale_optimise(sp, params)

    def scale_result(self) -> dict:
        r, self._scale_res = self._scale_res, None
        return r

    def ba_submit(self, bp, iters: int):
        self._ba_res = self.ba_solve(bp, iters)

    def ba_result(self):
        r, self._ba_res = self._ba_res, None
        return r

    # ---- device-resident BA window (GPU): observations appended per keyframe
    device_window = False

    def window_add(self, t, ids, feats):
        pass

    def window_pop(self, t):
        pass


class GPUBackend(Backend):
    """libme_hip.so through the C ABI; images resident in HBM (one upload per
    frame).  Two contexts of the device: `ctx` runs the BA, `tctx` the front
    end (KLT, the epipolar MI matcher, the scale LM), so the scale LM of frame
    t and the KLT of frame t + 1 run beside the BA of frame t.  Device buffers
    and page-locked staging are persistent (grow-only); per stage one H2D and
    one D2H."""

    def __init__(self, ctx=None, tctx=None, overlap: bool = True, front_cus: int = 4, match_on_ba: bool = False):
        from ._lib import Context, default_context

        self.ctx = ctx or default_context()
        self._own_t = tctx is None and overlap
        self.tctx = tctx or (Context(self.ctx.device) if overlap else self.ctx)
        # the two contexts run side by side on disjoint CU sets (front_cus of
        # every 16 CUs to the front end, whole XCDs: _lib.cu_split): the
        # persistent scale-LM kernel needs its workgroups co-resident, which
        # the BA's kernels on shared CUs would not leave room for
        self._masked = False
        front_cus = int(os.environ.get("ME_VO_FRONT_CUS", front_cus))  # A/B timing
        if self.tctx is not self.ctx and 0 < front_cus < 16:
            import torch

            from ._lib import cu_split
            ncu = torch.cuda.get_device_properties(self.ctx.device).multi_processor_count
            front, back = cu_split(ncu, front_cus)
            self.tctx.set_cu_mask(front)
            self.ctx.set_cu_mask(back)
            self._masked = True
        # the matchers run on the front end beside the BA of the previous
        # keyframe (the loop applies that BA only after the matching)
        self.mctx = self.ctx if match_on_ba else self.tctx
        self._scale_pool = None  # worker thread of the asynchronous scale LM
        self._ba_pool = self._ba_fut = None  # worker thread queueing the BA launches
        # one context for both sides (overlap=False or tctx=ctx): a context takes
        # one call at a time (me_hip.h), so neither the scale LM nor the BA
        # queueing runs on a worker thread -- both run inline, in loop order
        self.shared_ctx = self.tctx is self.ctx
        self.async_enqueue = os.environ.get("ME_VO_ASYNC_ENQUEUE", "1") == "1" and not self.shared_ctx
        self._imgs = {}
        # device-resident BA window: obs (4 doubles) | frame | track ID per
        # observation, frame by frame; [_wstart, _wend) live in store _wcur
        self._wcap = 0
        self._wstore = [None, None]
        self._wcaps = [0, 0]
        self._wcur = 0
        self._wend = 0
        self._wfrm = {}  # frame -> (offset, count)
        self._dev = {}   # name -> [ptr, bytes] on the device
        self._pin = {}   # name -> [ptr, bytes] page-locked host
        self._hview = {}  # page-locked ptr -> uint8 view of the whole buffer
        self._baq = []  # queued BA solves, oldest first (at most two: window t chained behind t - 1)
        self._bw_k = 0  # staging / device buffer set of the next window solve
        # window t's BA start formed on the device behind window t - 1's solve (me_vo_ba_chain)
        self.chain_window = os.environ.get("ME_VO_CHAIN", "1") == "1"
        self.tlog = None  # diagnostics: (event, frame, perf_counter) of BA enqueues / completions
        self._scale_res = None

    def reserve(self, cfg):
        """Size the BA side for the configuration's fullest window up front:
        the window stores, both solve buffer sets and the BA scratch (a buffer
        that grows mid-run waits for both contexts).  Bounds: every keyframe of
        the window contributes at most n_feats observations (tracked + new),
        and a landmark has at least one."""
        n_obs = cfg.window * cfg.n_feats + cfg.n_feats
        n_pts = n_obs
        nc = cfg.window
        cap = 2 * n_obs
        if self._wend == 0 and self._wcap < cap:
            for k in (0, 1):
                if self._wstore[k] is not None:
                    self.ctx.free(self._wstore[k])
                self._wstore[k] = self.ctx.malloc(40 * cap)
                self._wcaps[k] = cap
            self._wcap = cap
        nb = 48 * nc + 24 * n_pts + 4 * n_pts + 4 * nc
        for k in (0, 1):
            self._hbuf(f"bw{k}", nb)
            self._dbuf(f"bw{k}", nb)
            self._dbuf(f"bw_idx{k}", 8 * n_obs)
        for k in (0, 1):
            self._hbuf(f"w_add{k}", 40 * cfg.n_feats)
        self.ctx.check(self.ctx.lib.me_ba_reserve(self.ctx.h, nc, n_pts, n_obs, 4, cfg.fixed_frames), "me_ba_reserve")

    # ---- persistent buffers
    def _dbuf(self, name, nbytes):
        b = self._dev.get(name)
        if b is None or b[1] < nbytes:
            if b is not None:
                self.tctx.synchronize()
                self.ctx.synchronize()
                self.tctx.free(b[0])
            nb = max(4096, int(nbytes * 1.5))
            self._dev[name] = b = [self.tctx.malloc(nb), nb]
        return b[0]

    def _hbuf(self, name, nbytes):
        b = self._pin.get(name)
        if b is None or b[1] < nbytes:
            if b is not None:  # (both contexts copy from / to staging buffers, as _dbuf)
                self.tctx.synchronize()
                self.ctx.synchronize()
                self._hview.pop(b[0], None)
                self.tctx.host_free(b[0])
            nb = max(4096, int(nbytes * 1.5))
            self._pin[name] = b = [self.tctx.host_alloc(nb), nb]
            self._hview[b[0]] = self._map(b[0], nb)  # one numpy view of the whole buffer
        return b[0]

    @staticmethod
    def _map(ptr, nbytes):
        import ctypes

        return np.frombuffer((ctypes.c_char * nbytes).from_address(ptr), np.uint8, nbytes)

    def _view(self, ptr, dtype, count, offset=0):
        """count items of dtype at byte offset of the page-locked buffer ptr (a
        slice of the buffer's cached view: no ctypes type built per call)."""
        nbytes = np.dtype(dtype).itemsize * count
        if count == 0:
            return np.zeros(0, dtype)
        base = self._hview.get(ptr)
        if base is None:
            return self._map(ptr + offset, nbytes).view(dtype)
        return base[offset:offset + nbytes].view(dtype)

    def frame_images(self, t, left, right):
        if t in self._imgs:
            return self._imgs[t]
        L = np.ascontiguousarray(left, np.uint8)
        R = np.ascontiguousarray(right, np.uint8)
        # (on the front-end context: the BA context may be in use by the enqueue worker)
        dL, dR = self.tctx.malloc(L.nbytes), self.tctx.malloc(R.nbytes)
        self.tctx.h2d(dL, L)
        self.tctx.h2d(dR, R)
        h = (dL, dR, L.shape, L, R)
        self._imgs[t] = h
        return h

    def frame_images_device(self, t, left, right):
        """Images already resident on the device (e.g. rendered there): `left`
        / `right` expose data_ptr() and shape (torch uint8 tensors, kept
        referenced until release(t))."""
        if t in self._imgs:
            return self._imgs[t]
        shape = tuple(left.shape)
        ph = np.lib.stride_tricks.as_strided(np.zeros(1, np.uint8), shape=shape, strides=(0, 0))  # shape only
        h = (int(left.data_ptr()), int(right.data_ptr()), shape, ph, ph, (left, right))
        self._imgs[t] = h
        return h

    def release(self, t):
        h = self._imgs.pop(t, None)
        if h is not None and len(h) == 5:  # (device-resident inputs of frame_images_device are the caller's)
            self.tctx.free(h[0])
            self.tctx.free(h[1])

    def close(self):
        if self._scale_res is not None:
            self.scale_result()
        if self._scale_pool is not None:
            self._scale_pool.shutdown()
            self._scale_pool = None
        self._join_enqueue()
        while self._baq:
            self.ba_result()
        if self._ba_pool is not None:
            self._ba_pool.shutdown()
            self._ba_pool = None
        for st in self._wstore:
            if st is not None:
                self.ctx.free(st)
        self._wstore = [None, None]
        self._wcaps = [0, 0]
        for t in list(self._imgs):
            self.release(t)
        self.tctx.synchronize()
        for p, _ in self._dev.values():
            self.tctx.free(p)
        self._hview = {}
        for p, _ in self._pin.values():
            self.tctx.host_free(p)
        self._dev, self._pin = {}, {}
        if self._masked:
            self.ctx.set_cu_mask(None)
            self.tctx.set_cu_mask(None)
            self._masked = False
        if self._own_t:
            self.tctx.close()
            self._own_t = False

    # ---- plain calls (tests, tools)
    def klt(self, prev, cur, pts):
        h = self.klt_submit(prev, cur, pts)
        n = len(pts)
        if n == 0:
            return np.zeros((0, 2), np.float32), np.zeros(0, np.uint8)
        c = self.tctx
        hp = self._hbuf("out", 14 * n)
        dres = self._dbuf("res", 14 * n)
        c.copy_async(hp, dres, 13 * n)
        c.synchronize()
        return self._view(hp, np.float32, 2 * n).reshape(n, 2).copy(), self._view(hp, np.uint8, n, 12 * n).copy()

    def mi_scores(self, imgs, xyL, xyR):
        from .mutual_information import mi_scores_device

        n = len(xyL)
        if n == 0:
            return np.zeros(0, np.float32)
        H, W = imgs[2]
        c = self.tctx
        hp = self._hbuf("mi_in", 16 * n)
        self._view(hp, np.int32, 2 * n)[:] = np.asarray(xyL, np.int32).ravel()
        self._view(hp, np.int32, 2 * n, 8 * n)[:] = np.asarray(xyR, np.int32).ravel()
        d = self._dbuf("mi", 20 * n)
        c.copy_async(d, hp, 16 * n)
        mi_scores_device(c, imgs[0], W, imgs[1], W, W, H, d, d + 8 * n, n, (PATCH, PATCH), d + 16 * n)
        ho = self._hbuf("mi_out", 4 * n)
        c.copy_async(ho, d + 16 * n, 4 * n)
        c.synchronize()
        return self._view(ho, np.float32, n).copy()

    def scale_optimise(self, sp, params):
        from ._lib import ME_DEVICE
        from .optimisation import scale_optimise

        imgs = sp.imgs_handle
        return scale_optimise(sp, params, ctx=self.tctx, img_mem=ME_DEVICE, dev_imgs=(imgs[0], imgs[1]))

    def ba_solve(self, bp, iters):
        assert not self._baq, "ba_solve with window solves queued"
        self.ba_submit(bp, iters)
        return self.ba_result()

    # ---- staged calls
    # device result block of a KLT + match: uv (8n) | xr (4n) | status (n) | ok (n)
    def klt_submit(self, prev, cur, pts):
        import ctypes

        from ._lib import ME_DEVICE
        from .klt import klt_params

        n = len(pts)
        if n == 0:
            return (0, prev, cur)
        H, W = prev[2]
        c = self.tctx
        hp = self._hbuf("klt_in", 8 * n)
        self._view(hp, np.float32, 2 * n)[:] = np.asarray(pts, np.float32).ravel()
        d_in = self._dbuf("klt_in", 8 * n)
        dres = self._dbuf("res", 14 * n)
        c.copy_async(d_in, hp, 8 * n)
        kp = klt_params()
        c.check(c.lib.me_klt_track(c.h, ME_DEVICE, ctypes.c_void_p(prev[0]), ctypes.c_void_p(cur[0]), W, H, W,
                                   ctypes.c_void_p(d_in), ctypes.c_void_p(dres), ctypes.c_void_p(dres + 12 * n), n,
                                   ctypes.byref(kp)), "me_klt_track")
        return (n, prev, cur)

    def _epipolar(self, imgs, d_uv, d_lo, d_valid, d_status, n, nd, unique, d_xr, d_ok):
        import ctypes

        H, W = imgs[2]
        c = self.mctx
        V = ctypes.c_void_p
        c.check(c.lib.me_mi_epipolar_match(c.h, V(imgs[0]), V(imgs[1]), W, H, W, V(d_uv), V(d_lo),
                                           V(d_valid) if d_valid else None, V(d_status) if d_status else None, n, nd,
                                           PATCH, self.d_max, 1 if unique else 0, 1.2, float(MARGIN), V(d_xr),
                                           V(d_ok)), "me_mi_epipolar_match")

    def klt_match(self, h, imgs, lo, nd, dvalid):
        n = h[0]
        if n == 0:
            z = np.zeros(0, np.float32)
            return np.zeros((0, 2), np.float32), np.zeros(0, np.uint8), z, np.zeros(0, bool)
        c = self.mctx
        if c is not self.tctx:
            self.tctx.synchronize()  # the KLT results
        hp = self._hbuf("lo", 5 * n)
        self._view(hp, np.int32, n)[:] = lo
        self._view(hp, np.uint8, n, 4 * n)[:] = dvalid
        dl = self._dbuf("lo", 5 * n)
        c.copy_async(dl, hp, 5 * n)
        dres = self._dbuf("res", 14 * n)
        self._epipolar(imgs, dres, dl, dl + 4 * n, dres + 12 * n, n, nd, False, dres + 8 * n, dres + 13 * n)
        ho = self._hbuf("out", 14 * n)
        c.copy_async(ho, dres, 14 * n)
        c.synchronize()
        uv = self._view(ho, np.float32, 2 * n).reshape(n, 2).copy()
        xr = self._view(ho, np.float32, n, 8 * n).copy()
        st = self._view(ho, np.uint8, n, 12 * n).copy()
        ok = self._view(ho, np.uint8, n, 13 * n).astype(bool)
        return uv, st, xr, ok

    def klt_match_new(self, h, imgs, lo, nd, dvalid, t, grid, d_min, nd_new):
        """One submission and one round trip: the tracked features' matcher,
        me_vo_new_cells (the cells they leave empty) and the new features'
        matcher (me_mi_epipolar_match_count over the device count)."""
        import ctypes

        n = h[0]
        if n == 0:
            return Backend.klt_match_new(self, h, imgs, lo, nd, dvalid, t, grid, d_min, nd_new)
        c = self.mctx
        if c is not self.tctx:
            self.tctx.synchronize()  # the KLT results
        nx, ny, cw, ch, nf = grid
        H, W = imgs[2]
        V = ctypes.c_void_p
        hp = self._hbuf("lo", 5 * n)
        self._view(hp, np.int32, n)[:] = lo
        self._view(hp, np.uint8, n, 4 * n)[:] = dvalid
        dl = self._dbuf("lo", 5 * n)
        c.copy_async(dl, hp, 5 * n)
        dres = self._dbuf("res", 14 * n)
        self._epipolar(imgs, dres, dl, dl + 4 * n, dres + 12 * n, n, nd, False, dres + 8 * n, dres + 13 * n)
        # new-feature block: count (16 B) | uv (8 nf) | xr (4 nf) | lo (4 nf) | ok (nf)
        m = max(nf, 1)
        dn = self._dbuf("new", 16 + 17 * m)
        c.check(c.lib.me_vo_new_cells(c.h, V(dres), V(dres + 12 * n), V(dres + 13 * n), n, W, H, float(MARGIN), nx,
                                      ny, float(cw), float(ch), nf, t, d_min, V(dn + 16), V(dn + 16 + 12 * m), V(dn)),
                "me_vo_new_cells")
        c.check(c.lib.me_mi_epipolar_match_count(c.h, V(imgs[0]), V(imgs[1]), W, H, W, V(dn + 16), V(dn + 16 + 12 * m),
                                                 V(dn), m, nd_new, PATCH, self.d_max, 1, 1.2, float(MARGIN),
                                                 V(dn + 16 + 8 * m), V(dn + 16 + 16 * m)),
                "me_mi_epipolar_match_count")
        o = 16 * ((14 * n + 15) // 16)
        ho = self._hbuf("out", o + 16 + 17 * m)
        c.copy_async(ho, dres, 14 * n)
        c.copy_async(ho + o, dn, 16 + 17 * m)
        c.synchronize()
        uv = self._view(ho, np.float32, 2 * n).reshape(n, 2).copy()
        xr = self._view(ho, np.float32, n, 8 * n).copy()
        st = self._view(ho, np.uint8, n, 12 * n).copy()
        ok = self._view(ho, np.uint8, n, 13 * n).astype(bool)
        k = int(self._view(ho, np.int32, 1, o)[0])
        nuv = self._view(ho, np.float32, 2 * k, o + 16).reshape(k, 2).copy()
        nxr = self._view(ho, np.float32, k, o + 16 + 8 * m).copy()
        nok = self._view(ho, np.uint8, k, o + 16 + 16 * m).astype(bool)
        return uv, st, xr, ok, nuv, nxr, nok

    def match(self, imgs, uv, lo, nd, unique):
        n = len(uv)
        if n == 0:
            return np.zeros(0, np.float32), np.zeros(0, bool)
        c = self.mctx
        hp = self._hbuf("m_in", 12 * n)
        self._view(hp, np.float32, 2 * n)[:] = np.asarray(uv, np.float32).ravel()
        self._view(hp, np.int32, n, 8 * n)[:] = lo
        d = self._dbuf("m", 17 * n)
        c.copy_async(d, hp, 12 * n)
        self._epipolar(imgs, d, d + 8 * n, 0, 0, n, nd, unique, d + 12 * n, d + 16 * n)
        ho = self._hbuf("m_out", 5 * n)
        c.copy_async(ho, d + 12 * n, 5 * n)
        c.synchronize()
        return self._view(ho, np.float32, n).copy(), self._view(ho, np.uint8, n, 4 * n).astype(bool)

    def scale_submit(self, sp, params):
        """The scale LM on the front-end context, run by a worker thread: the
        arguments are built here, the worker only makes the C calls (which
        release the GIL), and the loop yields once so the worker starts before
        the loop's next Python stretch; the loop books the keyframe and queues
        the next BA meanwhile; scale_result joins it."""
        import time

        from ._lib import ME_DEVICE
        from .optimisation import ScaleCall

        imgs = sp.imgs_handle
        call = ScaleCall(sp, params, ctx=self.tctx, img_mem=ME_DEVICE, dev_imgs=(imgs[0], imgs[1]))
        if self.shared_ctx:  # (no second caller on the context: run it now, in loop order)
            from concurrent.futures import Future

            self._join_enqueue()
            fut = Future()
            fut.set_result(call.run())
            self._scale_res = (fut, call)
            return
        if self._scale_pool is None:
            from concurrent.futures import ThreadPoolExecutor

            self._scale_pool = ThreadPoolExecutor(max_workers=1)
        self._scale_res = (self._scale_pool.submit(call.run), call)
        time.sleep(0)  # (a GIL hand-over: the worker enters the C call now, not at the loop's next blocking call)

    def scale_result(self) -> dict:
        r, self._scale_res = self._scale_res, None
        if r is None:
            return None
        fut, call = r
        fut.result()
        return call.result()

    # ---- device-resident BA window
    device_window = True

    def _wview(self, k):
        """(obs, frame, id) device pointers of store k (capacity _wcap)."""
        base = self._wstore[k]
        return base, base + 32 * self._wcap, base + 36 * self._wcap

    def window_add(self, t, ids, feats):
        """Append keyframe t's observations (one H2D); the live window is
        compacted into the other store when the tail is full (stream-ordered
        copies; a BA in flight reads the current store, which the compaction
        only reads, and the other store's last solve has completed).  The
        staging alternates by keyframe parity: the copy from the other set,
        two keyframes back, ran before that keyframe's BA, which the loop has
        waited for."""
        self._join_enqueue()  # (stream order: the previous window's solve is queued before these copies)
        n = len(ids)
        live0 = min((o for o, _ in self._wfrm.values()), default=self._wend)
        live = self._wend - live0
        c = self.ctx
        if self._wend + n > self._wcap:
            cap = max(1 << 16, 2 * (live + n), self._wcap)
            k = 1 - self._wcur
            if self._wcaps[k] < cap:  # (the other store is reused when it is large enough: a free waits for the device)
                if self._wstore[k] is not None:
                    c.free(self._wstore[k])
                self._wstore[k] = c.malloc(40 * cap)
                self._wcaps[k] = cap
            cap = self._wcaps[k]
            old = self._wcap
            if live:
                ob, fb, ib = self._wstore[self._wcur], self._wstore[self._wcur] + 32 * old, \
                    self._wstore[self._wcur] + 36 * old
                self._wcap = cap
                no, nf, ni = self._wview(k)
                c.d2d(no, ob + 32 * live0, 32 * live)
                c.d2d(nf, fb + 4 * live0, 4 * live)
                c.d2d(ni, ib + 4 * live0, 4 * live)
            self._wcap = cap
            self._wcur = k
            self._wfrm = {f: (o - live0, m) for f, (o, m) in self._wfrm.items()}
            self._wend = live
        if n:
            hp = self._hbuf(f"w_add{t & 1}", 40 * n)
            self._view(hp, np.float64, 4 * n)[:] = np.asarray(feats, np.float64).ravel()
            self._view(hp, np.int32, n, 32 * n)[:] = t
            self._view(hp, np.int32, n, 36 * n)[:] = ids
            o, f, i = self._wview(self._wcur)
            e = self._wend
            c.copy_async(o + 32 * e, hp, 32 * n)
            c.copy_async(f + 4 * e, hp + 32 * n, 4 * n)
            c.copy_async(i + 4 * e, hp + 36 * n, 4 * n)
        self._wfrm[t] = (self._wend, n)
        self._wend += n

    def window_pop(self, t):
        self._wfrm.pop(t, None)

    def ba_submit_window(self, t, f0, win_ids, X, cams, iters, chain=None):
        """Queue the BA of the device-resident window [f0, t]: the window's
        track IDs, points and cameras go up (one H2D), the observation indices
        are built on the device (me_ba_window_indices), the solve runs on the
        device-resident problem (me_ba_solve_async, ME_DEVICE).  `chain`
        (WindowedStereoVO._chain_args): the cameras and points sent are the
        loop's state before the previous window's result, which
        me_vo_ba_chain applies on the device behind that window's solve, so
        this solve is queued before the previous one completes.  Two buffer
        sets alternate (the previous window's stays in use until its wait)."""
        import ctypes
        import time

        from ._lib import ME_DEVICE, BAProblemC, VOWindowC
        from .optimisation import SolverOptions

        self._join_enqueue()  # (the previous window's queueing: this one may chain from it)
        off0 = self._wfrm[f0][0]
        n_obs = self._wend - off0
        npts, nc = len(win_ids), len(cams)
        c = self.ctx
        k = self._bw_k
        self._bw_k ^= 1
        # cams | pts (solved in place) | win_ids | chain: cam_src -- one page-locked block, one H2D
        o_ids = 48 * nc + 24 * npts
        o_cs = o_ids + 4 * npts
        nb = o_cs + 4 * nc
        hp = self._hbuf(f"bw{k}", nb)
        self._view(hp, np.float64, 6 * nc)[:] = np.asarray(cams, np.float64).ravel()
        self._view(hp, np.float64, 3 * npts, 48 * nc)[:] = np.asarray(X, np.float64).ravel()
        self._view(hp, np.int32, npts, o_ids)[:] = win_ids
        d = self._dbuf(f"bw{k}", nb)
        di = self._dbuf(f"bw_idx{k}", 8 * max(n_obs, 1))
        w = VOWindowC()
        w.stage, w.dev, w.stage_bytes = hp, d, nb if chain is not None else o_cs
        if chain is not None:
            assert chain["nc"] == nc and self._baq and self._baq[-1][0] == "dev"
            self._view(hp, np.int32, nc, o_cs)[:] = chain["cam_src"]
            prev = self._baq[-1][6]  # (device IDs, count) of the window solved before this one
            w.chain = 1
            w.cam_src, w.prev_ids, w.n_prev, w.new_from = d + o_cs, prev[0], prev[1], chain["new_from"]
            a = w.args
            a.pose[:] = [float(x) for x in chain["pose"]]
            a.R[:] = [float(x) for x in np.asarray(chain["R"], np.float64).ravel()]
            a.vel[:] = [float(x) for x in chain["vel"]]
            a.k1, a.k0, a.mode = chain["k1"], chain["k0"], chain["mode"]
        o, f, i = self._wview(self._wcur)
        w.win_ids, w.frame, w.ids, w.first_frame = d + o_ids, f + 4 * off0, i + 4 * off0, f0
        p = BAProblemC()
        p.n_cams, p.n_pts, p.n_obs = nc, npts, n_obs
        p.cams = ctypes.cast(d, ctypes.POINTER(ctypes.c_double))
        p.pts = ctypes.cast(d + 48 * nc, ctypes.POINTER(ctypes.c_double))
        p.obs = ctypes.cast(o + 32 * off0, ctypes.POINTER(ctypes.c_double))
        p.cam_idx = ctypes.cast(di, ctypes.POINTER(ctypes.c_int32))
        p.pt_idx = ctypes.cast(di + 4 * n_obs, ctypes.POINTER(ctypes.c_int32))
        K = np.asarray(self._K, np.float64).ravel()
        p.K0[:] = [float(x) for x in K]
        p.K1[:] = [float(x) for x in K]
        p.baseline, p.feat_var, p.fixed_frames = self._calib
        p.mem, p.obs_dim = ME_DEVICE, 4
        opt = SolverOptions.fixed_iterations(iters).to_c()

        def enqueue():  # H2D, the chained start, the window's indices, the solve: one C call (no GIL)
            if self.tlog is not None:
                self.tlog.append(("enq0", t, time.perf_counter()))
            c.check(c.lib.me_vo_window_submit(c.h, ctypes.byref(w), ctypes.byref(p), ctypes.byref(opt)),
                    "me_vo_window_submit")
            if self.tlog is not None:
                self.tlog.append(("enq", t, time.perf_counter()))

        # Queued by a worker thread (the C call releases the GIL): the loop
        # goes on -- it waits for the previous window (me_ba_wait_out may run
        # beside the queueing: the library's solve queue is locked), applies
        # it and starts the next keyframe.  Stream work of this ctx from the
        # loop thread (window_add) joins the worker first.
        fut = None
        if self.async_enqueue:
            if self._ba_pool is None:
                from concurrent.futures import ThreadPoolExecutor

                self._ba_pool = ThreadPoolExecutor(max_workers=1)
            fut = self._ba_fut = self._ba_pool.submit(enqueue)
        else:
            enqueue()
        self._baq.append(("dev", p, opt, w, nc, npts, (d + o_ids, npts), fut))
        return n_obs

    def _join_enqueue(self):
        if self._ba_fut is not None:  # (and its errors)
            fut, self._ba_fut = self._ba_fut, None
            fut.result()

    def ba_submit(self, bp, iters):
        """Queue the window's solve on the BA context (me_ba_solve_async: the
        host arrays are staged into page-locked memory at once)."""
        from ._lib import BAOptionsC  # noqa: F401
        from .optimisation import SolverOptions, ba_struct

        keep = []
        p, cams, pts = ba_struct(bp, keep)
        o = SolverOptions.fixed_iterations(iters).to_c()
        c = self.ctx
        import ctypes
        self._join_enqueue()
        c.check(c.lib.me_ba_solve_async(c.h, ctypes.byref(p), ctypes.byref(o)), "me_ba_solve_async")
        self._baq.append(("host", p, o, cams, pts, keep))

    def ba_result(self):
        """The oldest queued solve: (cams, pts, summary).  A device-resident
        window's result comes from the staging its solve read back into
        (me_ba_wait_out): no wait on a solve queued behind it."""
        import ctypes

        from ._lib import BASummaryC
        from .optimisation import _summary

        rec = self._baq.pop(0)
        s = BASummaryC()
        c = self.ctx
        if rec[0] == "dev":
            _, p, o, w, nc, npts, _, fut = rec
            if fut is not None:  # this window's own queueing (a newer one's may run on beside the wait)
                fut.result()
                if fut is self._ba_fut:
                    self._ba_fut = None
            cams = np.empty((nc, 6), np.float64)
            pts = np.empty((npts, 3), np.float64)
            c.check(c.lib.me_ba_wait_out(c.h, ctypes.byref(s), cams.ctypes.data_as(ctypes.c_void_p),
                                         pts.ctypes.data_as(ctypes.c_void_p)), "me_ba_wait_out")
            if self.tlog is not None:
                import time

                self.tlog.append(("done", None, time.perf_counter()))
            return cams, pts, _summary(s)
        c.check(c.lib.me_ba_wait(c.h, ctypes.byref(s)), "me_ba_wait")
        _, p, o, cams, pts, keep = rec
        return cams, pts, _summary(s)


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
    when log_events is set.

    The loop is lagged by definition (process): BA(t - 1) enters the state
    after keyframe t is matched and booked, so on the GPU the BA of t - 1 runs
    while the host tracks, matches and books t, and the BA context idles only
    while BA(t - 1) is applied and BA(t) queued.  Every backend takes the same
    decisions; `overlap` only tells the GPU backend to run the front end on its
    own context (overlap=False: one context and one stream; the scale LM and
    the BA queueing then run inline on the loop thread, in loop order).  Call
    finish() after the last keyframe."""

    def __init__(self, cfg: PipelineConfig, backend: Backend, K=None, first_pose=None, velocity=None,
                 log_events: bool = False, overlap: bool = False):
        self.cfg = cfg
        self.be = backend
        self.be.d_max = cfg.d_max
        if hasattr(backend, "reserve"):
            backend.reserve(cfg)
        self.K = np.asarray(S.intrinsics(cfg.width, cfg.height) if K is None else K, np.float64)
        self.f, self.cx, self.cy = self.K[0, 0], self.K[0, 2], self.K[1, 2]
        # grid of feature cells over the margin-free interior
        aw, ah = cfg.width - 2 * MARGIN, cfg.height - 2 * MARGIN
        self.nx = max(1, int(round(math.sqrt(cfg.n_feats * aw / ah))))
        self.ny = max(1, int(math.ceil(cfg.n_feats / self.nx)))
        self.cw, self.ch = aw / self.nx, ah / self.ny
        # track table (structure of arrays, index = creation order = ID order):
        # ids, X, active, first (first frame still held, after pops), last
        # (last frame observed) are views of the first n rows of capacity
        # buffers, two sets: appends write the tail in place, a pop compacts
        # into the other set (one copy per keyframe instead of two)
        self._tab = [None, None]
        self._tcur, self._tn = 0, 0
        self._gen, self._remap = 0, None  # compactions so far, and the last one's index map
        self._tab_alloc(0, 4096)
        self._tab_view()
        self.latest_id = 0                   # WBA_Point<pair<Point2f,Point2f>>::latestID
        self.obs = {}                        # t -> (track IDs int64, ascending; (n, 4) float32 {xl, yl, xr, yr})
        self.poses = {}                      # t -> {t, angle-axis} world -> camera
        self.first_pose = np.zeros(6) if first_pose is None else np.asarray(first_pose, np.float64)
        self.velocity = velocity             # prior {t, aa} step for the second frame
        self.prev_imgs = None
        self.prev_t = None
        self.log_events = log_events
        self.overlap = overlap
        self._ev = []                        # compact event records, expanded by .events
        self.results = []
        self._pending = None                 # frame whose BA (and, once _complete runs, scale LM) are queued
        self._scale_args = None
        self.stage_s = {"host": 0.0, "wait": 0.0}  # host bookkeeping vs time blocked in the backend
        self.wait_by_stage = {}  # backend call -> seconds blocked in it

    @property
    def events(self):
        out = []
        for rec in self._ev:
            if rec[0] == "frame":
                _, ids, t, feats, is_new = rec
                out.extend(("new" if nw else "add", int(i), t, tuple(float(v) for v in fe))
                           for i, fe, nw in zip(ids, feats, is_new))
            else:
                out.extend((rec[0], int(i)) for i in rec[1])
        return out

    # ---------------------------------------------------------------- matching
    def search_window(self, d_pred=None, half: int = 6):
        """Disparity candidates per feature: tracked features (d_pred given)
        search +-half px around the disparity their 3-D point predicts at the
        predicted pose; new features search [d_min, d_max] (uniqueness test).
        Returns (lo, nd, dvalid)."""
        cfg = self.cfg
        if d_pred is None:
            return None, cfg.d_max - cfg.d_min + 1, None
        dp = np.where(np.isfinite(d_pred), d_pred, -1e9)
        lo = np.clip(np.rint(dp).astype(np.int64) - half, cfg.d_min, cfg.d_max)
        with np.errstate(invalid="ignore"):
            dvalid = np.isfinite(d_pred) & (d_pred > 0)
        return lo, 2 * half + 1, dvalid

    def stereo_match(self, imgs, uv: np.ndarray, d_pred=None, ratio: float = 1.2, half: int = 6):
        """MI disparity search for features uv (n, 2) float32 -> (xr float32, ok)."""
        n = len(uv)
        lo, nd, dvalid = self.search_window(d_pred, half)
        if lo is None:
            lo = np.full(n, self.cfg.d_min, np.int64)
        return match_host(self.be, imgs, uv, lo, nd, dvalid, d_pred is None, self.cfg.d_max, ratio)

    def _predicted_disparity(self, idx, pose):
        R = aa_to_R(pose[3:])
        Z = self.X[idx] @ R[2] + pose[2]
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.where(Z > 0, self.f * self.cfg.baseline / Z, np.nan)

    # ---------------------------------------------------------------- helpers
    def _in_margin(self, uv):
        return in_margin(uv, self.cfg.width, self.cfg.height)

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

    _TAB = (("ids", np.int64, ()), ("X", np.float64, (3,)), ("active", bool, ()), ("first", np.int64, ()),
            ("last", np.int64, ()))

    def _tab_alloc(self, k, cap):
        self._tab[k] = {nm: np.zeros((cap,) + sh, dt) for nm, dt, sh in self._TAB}

    def _tab_view(self):
        b, n = self._tab[self._tcur], self._tn
        self.ids, self.X, self.active = b["ids"][:n], b["X"][:n], b["active"][:n]
        self.first, self.last = b["first"][:n], b["last"][:n]

    def _add_tracks(self, t, uv, xr, pose):
        n = len(uv)
        n0 = self._tn
        b = self._tab[self._tcur]
        if n0 + n > len(b["ids"]):  # grow: the live rows into a larger set
            cap = 2 * (n0 + n)
            self._tab_alloc(self._tcur, cap)
            for nm, _, _ in self._TAB:
                self._tab[self._tcur][nm][:n0] = b[nm][:n0]
            b = self._tab[self._tcur]
        b["ids"][n0:n0 + n] = np.arange(self.latest_id, self.latest_id + n, dtype=np.int64)
        self.latest_id += n
        b["X"][n0:n0 + n] = self._triangulate(uv, xr, pose)
        b["active"][n0:n0 + n] = True
        b["first"][n0:n0 + n] = t
        b["last"][n0:n0 + n] = t
        self._tn = n0 + n
        self._tab_view()
        return np.arange(n0, n0 + n, dtype=np.int64)

    def _wait(self, fn, *a):
        import time

        from ._lib import roctx_range
        t0 = time.perf_counter()
        name = getattr(fn, "__name__", "stage")
        with roctx_range(name, ROCTX):
            r = fn(*a)
        dt = time.perf_counter() - t0
        self.stage_s["wait"] += dt
        self.wait_by_stage[name] = self.wait_by_stage.get(name, 0.0) + dt
        return r

    # ---------------------------------------------------------------- one keyframe
    def process(self, t: int, left: np.ndarray, right: np.ndarray):
        """Keyframe t.  The loop definition (both backends, overlap or not):
        the BA of keyframe t - 1 enters the state (poses, landmarks) only after
        keyframe t is matched and booked -- keyframe t's prediction, matching
        and new tracks use the state after BA(t - 2) -- so BA(t - 1) runs on
        the device while the host tracks, matches and books keyframe t, and
        BA(t) is queued as soon as BA(t - 1) is applied:
          1. KLT of the active tracks (L(t-1) -> L(t)) queued;
          2. pops of keyframe t-1's completion (features leaving the window);
          3. pose(t) predicted (constant velocity, lagged state);
          4. KLT gate + MI matching of the tracked features, new features of
             the cells they leave empty (one round trip);
          5. WBA_Point bookkeeping of t (addMatch, new tracks triangulated at
             the predicted pose);
          6. scale LM of keyframe t-1 (front end, beside BA(t-1));
          7. BA(t-1) applied, keyframe t-1's FrameResult; pose(t) predicted
             again from the refined poses and t's new landmarks moved with
             it (camera-frame coordinates kept);
          8. keyframe t's observations appended, BA(t) queued."""
        import time
        t_in = time.perf_counter()
        w0 = self.stage_s["wait"]
        cfg = self.cfg
        imgs = self.be.frame_images(t, left, right)
        # 1. KLT of the active tracks, queued first (it needs only frame t-1's features)
        kh = None
        if self.prev_imgs is not None and self.active.any():
            act = np.flatnonzero(self.active)
            pid, puv = self.obs[self.prev_t]
            aid = self.ids[act]
            # (the active tracks are exactly the features of keyframe t-1, in ID order, as a rule)
            pos = np.arange(len(pid)) if len(aid) == len(pid) and np.array_equal(aid, pid) else np.searchsorted(pid, aid)
            kh = self.be.klt_submit(self.prev_imgs, imgs, np.ascontiguousarray(puv[pos, :2]))
        # 2. pops of frame t-1's completion (active tracks keep their order)
        if self._pending is not None:
            self._pop(self._pending[0] + 1 - cfg.window)
        # 3. prediction from the lagged state
        pose = self._predict_pose(t)
        self.poses[t] = pose
        trk_idx = np.zeros(0, np.int64)
        trk_uv = np.zeros((0, 2), np.float32)
        xr = np.zeros(0, np.float32)
        grid = (self.nx, self.ny, self.cw, self.ch, cfg.n_feats)
        _, nd_new, _ = self.search_window()
        if kh is not None:
            # 4. KLT gate + stereo matching of the tracked features (around their predicted disparity),
            # then the new features of the cells they leave empty -- one backend round trip
            act = np.flatnonzero(self.active)
            lo, nd, dvalid = self.search_window(self._predicted_disparity(act, pose))
            uv, st, xr_all, ok, nuv, nxr, nok = self._wait(self.be.klt_match_new, kh, imgs, lo, nd, dvalid, t, grid,
                                                           cfg.d_min, nd_new)
            good = (st == 1) & self._in_margin(uv) & ok
            self.active[act[~good]] = False
            trk_idx, trk_uv, xr = act[good], uv[good], xr_all[good]
        else:
            nuv = new_cells(t, trk_uv, grid)
            nxr, nok = self._wait(self.be.match, imgs, nuv, np.full(len(nuv), cfg.d_min, np.int64), nd_new, True)
        # 6. frame t-1's scale LM queued now (front end, beside BA(t-1); its inputs are the lagged state,
        # untouched by this frame's bookkeeping): the GPU backend runs it on a worker thread
        if self._scale_args is not None:
            self._scale_submit(*self._scale_args)
            self._scale_args = None
        n_tracked = len(trk_idx)
        nuv, nxr = nuv[nok], nxr[nok]
        # 5. bookkeeping: new tracks, this frame's features (tracked first, then new; sorted by track = ID order)
        new_idx = self._add_tracks(t, nuv, nxr, pose)
        idx = np.concatenate([trk_idx, new_idx])
        feats = np.concatenate([np.concatenate([trk_uv, xr[:, None], trk_uv[:, 1:2]], 1),
                                np.concatenate([nuv, nxr[:, None], nuv[:, 1:2]], 1)]).astype(np.float32)
        o = np.argsort(idx, kind="stable")
        idx, feats = idx[o], feats[o]
        fid = self.ids[idx]
        self.obs[t] = (fid, feats)
        self.last[idx] = t
        if self.log_events:
            is_new = np.zeros(len(self.ids), bool)
            is_new[new_idx] = True
            self._ev.append(("frame", self.ids[idx].copy(), t, feats.copy(), is_new[idx]))
        new_ids = self.ids[new_idx]
        R_pose = aa_to_R(pose[3:])
        # 8 (chained). A backend that can form BA(t)'s start on the device from BA(t-1)'s result queues
        # BA(t) now, behind BA(t-1): the same values as step 7 forms on the host below
        chain = self._chain_args(t, pose, R_pose, new_ids)
        if chain is not None:
            self.be.window_add(t, fid.astype(np.int32), feats)
            ba = self._ba_submit(t, chain)
        # 7. frame t-1's BA applied
        done = self._complete_ba()
        # pose(t) again from the refined poses; the new landmarks of t keep their camera-frame coordinates
        pose2 = self._predict_pose(t)
        if not np.array_equal(pose2, pose) and len(new_ids):
            j = np.searchsorted(self.ids, new_ids)
            self.X[j] = move_landmarks(self.X[j], R_pose, pose, pose2, rot_series(pose2[3:]))
        self.poses[t] = pose2
        # 8. the window's observations, BA(t) queued; the scale LM over the tracks seen in t is queued by
        # the next keyframe (beside this BA; the scale only enters the frame's result)
        if chain is None:
            self.be.window_add(t, fid.astype(np.int32), feats)
            ba = self._ba_submit(t)
        self._scale_args = (t, imgs, fid.copy())
        self._pending = (t, n_tracked, len(new_idx), int(self.active.sum()), ba)
        self.prev_imgs, self.prev_t = imgs, t
        # 9. frame t-1's FrameResult (its scale LM result), while BA(t) runs
        self._complete_result(done)
        self.stage_s["host"] += (time.perf_counter() - t_in) - (self.stage_s["wait"] - w0)

    def finish(self):
        """Complete the last queued keyframe (its pops, scale LM, BA)."""
        import time
        t_in = time.perf_counter()
        w0 = self.stage_s["wait"]
        if self._pending is not None:
            self._pop(self._pending[0] + 1 - self.cfg.window)
        if self._scale_args is not None:
            self._scale_submit(*self._scale_args)
            self._scale_args = None
        self._complete_result(self._complete_ba())
        self.stage_s["host"] += (time.perf_counter() - t_in) - (self.stage_s["wait"] - w0)

    def _complete_ba(self):
        """Frame t-1 (the pending one): its BA result applied (its pops ran
        before the next keyframe's matching, its scale LM is queued)."""
        if self._pending is None:
            return None
        t, n_tracked, n_new, n_active, ba = self._pending
        self._pending = None
        nwp, nwo, bs = self._ba_finish(ba)
        return (t, n_tracked, n_new, n_active, nwp, nwo, bs)

    def _complete_result(self, done):
        """Frame t-1's FrameResult: its scale LM result and its BA summary."""
        if done is None:
            return
        t, n_tracked, n_new, n_active, nwp, nwo, bs = done
        sc = self._wait(self.be.scale_result)
        self.results.append(FrameResult(t, n_tracked, n_new, n_active, nwp, nwo, sc["scale"], int(sc["stop"]),
                                        int(sc["iterations"]), int(bs["iterations"]), float(bs["final_cost"]),
                                        self.poses[t].copy()))

    def _scale_submit(self, t, imgs, tids):
        from .optimisation import OptimisationParams

        idx = np.searchsorted(self.ids, tids)  # (tracks seen in t are alive: their last frame is t)
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
        self._wait(self.be.scale_submit, sp, OptimisationParams.fixed_iterations(self.cfg.scale_iters))

    def _chain_args(self, t, pose, R_pose, new_ids):
        """Step 7's inputs for a backend that chains BA(t) behind BA(t-1) on
        the device (None: step 7 on the host, then BA(t) queued): per window
        camera / landmark its source in BA(t-1)'s result (-1 none, -2 new in
        t), the pose(t) prediction form, the first prediction and its rotation."""
        if not getattr(self.be, "chain_window", False) or self._pending is None or self._pending[4] is None:
            return None
        cfg = self.cfg
        f0 = max(0, t - cfg.window + 1)
        if t - f0 + 1 <= cfg.fixed_frames:
            return None
        pt, pf0, pwids = self._pending[4][:3]
        nc = t - f0 + 1
        k1 = t - 1 - f0
        if t == 1 or (t - 2) not in self.poses:
            mode, k0 = 0, -1
            vel = np.zeros(6) if self.velocity is None else np.asarray(self.velocity, np.float64)
        elif t - 2 >= f0:
            mode, k0, vel = 1, t - 2 - f0, np.zeros(6)
        else:
            return None
        if k1 < 0 or pt != t - 1:
            return None
        cam_src = np.array([f - pf0 if pf0 <= f <= pt else -1 for f in range(f0, t)] + [-1], np.int32)
        # the landmarks' sources are found on the device by track ID (window t-1's IDs are ascending; the
        # tracks new in t hold the largest IDs)
        new_from = int(new_ids[0]) if len(new_ids) else 2 ** 31 - 1
        return dict(cam_src=cam_src, new_from=new_from, pose=np.asarray(pose, np.float64), R=R_pose, vel=vel,
                    k1=k1, k0=k0, mode=mode, nc=nc)

    def _ba_submit(self, t, chain=None):
        """The window's BA problem in initialiseObservations order
        (BundleAdjuster.h:354-376: points in track order, each track's
        features in frame order), built in O(observations): the window's
        points are the tracks seen in [f0, t] (last >= f0), their features
        are contiguous in frames (addMatch, feature_types.h:140), so track
        j's features land at offset_j + (f - max(first_j, f0))."""
        cfg = self.cfg
        f0 = max(0, t - cfg.window + 1)
        if t - f0 + 1 <= cfg.fixed_frames:
            return None
        win = self.last >= f0
        upts = np.flatnonzero(win)
        if self.be.device_window:  # observations already on the device, frame by frame
            cams = np.stack([self.poses[f] for f in range(f0, t + 1)])
            assert self.latest_id < 2 ** 31
            self.be._K, self.be._calib = self.K, (cfg.baseline, cfg.feat_var, cfg.fixed_frames)
            n_obs = self._wait(self.be.ba_submit_window, t, f0, self.ids[upts].astype(np.int32), self.X[upts], cams,
                               cfg.ba_iters, chain)
            return (t, f0, self.ids[upts].copy(), n_obs, upts, self._gen)
        bp = self.ba_problem(t, f0, upts)
        self._wait(self.be.ba_submit, bp, cfg.ba_iters)
        return (t, f0, self.ids[upts].copy(), len(bp.obs), upts, self._gen)

    def ba_problem(self, t, f0, upts):
        """The window [f0, t]'s BA problem on the host (host-path backends;
        diagnostics)."""
        cfg = self.cfg
        local = np.cumsum(self.last >= f0) - 1      # table index -> window point index
        first = np.maximum(self.first[upts], f0)
        cnt = self.last[upts] - first + 1
        off = np.zeros(len(cnt) + 1, np.int64)
        np.cumsum(cnt, out=off[1:])
        n_obs = int(off[-1])
        fe = np.empty((n_obs, 4), np.float64)
        cam = np.empty(n_obs, np.int32)
        pti = np.empty(n_obs, np.int32)
        seen = 0
        for f in range(f0, t + 1):
            if f not in self.obs:
                continue
            fid, feats = self.obs[f]
            j = local[np.searchsorted(self.ids, fid)]
            q = off[j] + (f - first[j])
            fe[q] = feats
            cam[q] = f - f0
            pti[q] = j
            seen += len(fid)
        assert seen == n_obs, "window tracks must have contiguous features in the window"
        cams = np.stack([self.poses[f] for f in range(f0, t + 1)])
        return S.BAProblem(cams, self.X[upts], fe, cam, pti, self.K.copy(), self.K.copy(), cfg.baseline, cfg.feat_var,
                           cfg.fixed_frames)

    def _ba_finish(self, ba):
        if ba is None:
            return 0, 0, {"iterations": 0, "final_cost": float("nan")}
        t, f0, wids, nobs, upts, gen = ba
        c, p, s = self._wait(self.be.ba_result)
        # the window's tracks now (a pop may have compacted the table since the submit -- its index map;
        # a track popped out of the table, seen only in the window's first keyframe, needs no landmark)
        if gen == self._gen:
            j, live = upts, np.ones(len(upts), bool)
        elif gen + 1 == self._gen:
            j = self._remap[upts]
            live = j >= 0
            j = np.maximum(j, 0)
        else:  # (not reached by the loop: one pop at most between a window's submit and its result)
            j = np.minimum(np.searchsorted(self.ids, wids), max(len(self.ids) - 1, 0))
            live = (self.ids[j] == wids) if len(self.ids) else np.zeros(len(wids), bool)
        if s.get("status", 2) != 2 and os.environ.get("ME_VO_DUMP_FAILED"):  # diagnostics: the failed window
            upts = j[live]
            bp = self.ba_problem(t, f0, upts)
            np.savez(os.environ["ME_VO_DUMP_FAILED"], cams=bp.cams, pts=bp.pts, obs=bp.obs, cam_idx=bp.cam_idx,
                     pt_idx=bp.pt_idx, K=bp.K0, t=t, f0=f0, ids=self.ids[upts], first=self.first[upts],
                     last=self.last[upts], status=s.get("status"), termination=s.get("termination"))
            os.environ.pop("ME_VO_DUMP_FAILED")
        if s.get("status", 2) == 2:
            c = np.asarray(c, np.float64)  # (a fresh array per result: its rows are kept as the poses)
            for k, f in enumerate(range(f0, t + 1)):
                self.poses[f] = c[k]
            self.X[j[live]] = np.asarray(p)[live]
        return len(wids), nobs, s

    def _pop(self, new_first):
        """WBA_Point::pop() of every feature older than `new_first`; empty tracks deleted."""
        for f in [f for f in self.obs if f < new_first]:
            fid, _ = self.obs.pop(f)
            self.be.window_pop(f)
            if self.log_events:
                self._ev.append(("pop", fid.copy()))
            # (the tracks seen in f are those whose first held frame is f: frames pop oldest first and
            # a track's features are contiguous -- WBA_Point::pop of each of them)
            self.first[self.first == f] = f + 1
        dead = (self.last < new_first)
        if dead.any():
            if self.log_events:
                self._ev.append(("del", self.ids[np.flatnonzero(dead)].copy()))
            keep = ~dead  # (the observation store holds IDs: nothing to re-index)
            n2 = int(keep.sum())
            k = 1 - self._tcur
            cap = len(self._tab[self._tcur]["ids"])
            if self._tab[k] is None or len(self._tab[k]["ids"]) < cap:
                self._tab_alloc(k, cap)
            src, dst = self._tab[self._tcur], self._tab[k]
            for nm, _, _ in self._TAB:
                np.compress(keep, src[nm][:self._tn], axis=0, out=dst[nm][:n2])
            remap = np.cumsum(keep) - 1  # old table index -> new (-1: deleted)
            remap[dead] = -1
            self._remap, self._gen = remap, self._gen + 1
            self._tcur, self._tn = k, n2
            self._tab_view()


def synthetic_sequence(c: int, n_frames: int, seed: int | None = None, render_div: int = 1, first_id: int = 0):
    """Stereo keyframes of config c's synthetic sequence (0.5 m forward along
    the heading and 0.3 deg yaw per keyframe: the arc through the ring
    corridor, synthetic.trajectory_arc, any length), the true first pose and
    the per-frame motion prior used for the second keyframe.  first_id starts
    the sequence at keyframe first_id of the arc (chunked long runs)."""
    cfg = S.CONFIGS[c]
    seed = S.SEED0 + c if seed is None else seed
    scene, K, frames = S.stereo_stream(seed, cfg["width"], cfg["height"], n_frames, first_id=first_id,
                                       render_div=render_div, scene_kind="corridor")
    poses = []
    for fr in frames:
        poses.append(np.concatenate([fr.t, S.R_to_aa_robust(fr.R)]))
    return frames, K, poses[0], poses[1] - poses[0], poses


class NativeStereoVO:
    """The windowed stereo VO loop of WindowedStereoVO with the GPU backend,
    every step in native code behind the C ABI (me_vo_loop_*, csrc/vo_loop.hip):
    the Python layer only hands images in and reads results out.  Same
    decisions, events, results and poses as WindowedStereoVO(GPUBackend)
    (tests/test_pipeline.py, test_native_loop_*).  Two contexts of the device as GPUBackend sets
    them up: `ctx` runs the window solves, `tctx` (front_cus of every 16 CUs,
    whole XCDs) the KLT, the matchers and the scale LM; overlap=False runs
    everything on `ctx` (no worker threads).  Images: numpy (copied in) or
    device tensors exposing data_ptr() (kept referenced for two keyframes)."""

    def __init__(self, cfg: PipelineConfig, ctx=None, K=None, first_pose=None, velocity=None, log_events=False,
                 overlap: bool = True, front_cus: int = 4, tctx=None, async_enqueue: bool = True):
        import ctypes

        from ._lib import Context, VOLoopConfigC, cu_split, default_context

        self.cfg = cfg
        self.ctx = ctx or default_context()
        self._own_t = tctx is None and overlap
        self.tctx = tctx or (Context(self.ctx.device) if overlap else self.ctx)
        self._masked = False
        front_cus = int(os.environ.get("ME_VO_FRONT_CUS", front_cus))
        if self.tctx is not self.ctx and 0 < front_cus < 16:
            import torch

            ncu = torch.cuda.get_device_properties(self.ctx.device).multi_processor_count
            front, back = cu_split(ncu, front_cus)
            self.tctx.set_cu_mask(front)
            self.ctx.set_cu_mask(back)
            self._masked = True
        self.lib = self.ctx.lib
        self.K = np.asarray(S.intrinsics(cfg.width, cfg.height) if K is None else K, np.float64)
        c = VOLoopConfigC()
        self.lib.me_vo_loop_default_config(ctypes.byref(c))
        c.width, c.height, c.n_feats, c.window = cfg.width, cfg.height, cfg.n_feats, cfg.window
        c.ba_iters, c.scale_iters, c.fixed_frames, c.d_min, c.d_max = (cfg.ba_iters, cfg.scale_iters,
                                                                      cfg.fixed_frames, cfg.d_min, cfg.d_max)
        c.baseline, c.feat_var = float(cfg.baseline), float(cfg.feat_var)
        c.K[:] = [float(x) for x in self.K.ravel()]
        c.first_pose[:] = [float(x) for x in (np.zeros(6) if first_pose is None else np.asarray(first_pose))]
        c.has_velocity = int(velocity is not None)
        if velocity is not None:
            c.velocity[:] = [float(x) for x in np.asarray(velocity)]
        c.log_events = int(log_events)
        c.async_enqueue = int(async_enqueue)
        h = ctypes.c_void_p()
        self.ctx.check(self.lib.me_vo_loop_create(self.ctx.h, self.tctx.h, ctypes.byref(c), ctypes.byref(h)),
                       "me_vo_loop_create")
        self.h = h
        self.log_events = log_events
        self._keep = {}  # device images of the last two keyframes (the loop reads them until process(t + 1))

    def _check(self, rc, what):
        if rc != 0:
            from ._lib import MEError

            msg = self.lib.me_vo_loop_last_error(self.h)
            raise MEError(rc, f"{what}: {msg.decode() if msg else ''}")

    def _order_after_torch(self, device):
        """The loop reads device images on its own streams: order those after
        the torch stream that produced them, without a host wait.  A
        CU-masked ctx stream is a blocking stream and already orders after
        work on the legacy null stream; recording an event on the null
        stream would also wait for every blocking stream's work -- the BA in
        flight -- and serialise the pipeline, so from the null stream only
        non-blocking loop streams get an event wait."""
        import ctypes

        import torch

        cur = torch.cuda.current_stream(device)
        waiters = []
        for c in {self.ctx, self.tctx}:
            sp = c.stream_ptr()
            if cur.cuda_stream == 0:
                fl = ctypes.c_uint()
                c.check(c.lib.me_stream_flags(c.h, ctypes.byref(fl)), "me_stream_flags")
                if fl.value == 0:  # blocking: ordered after the null stream already
                    continue
            if sp != cur.cuda_stream:
                waiters.append(sp)
        if waiters:
            ev = torch.cuda.Event()
            ev.record(cur)
            for sp in waiters:
                torch.cuda.ExternalStream(sp, device=device).wait_event(ev)

    def process(self, t: int, left, right):
        import ctypes

        from ._lib import ME_DEVICE, ME_HOST

        shape = (self.cfg.height, self.cfg.width)
        if hasattr(left, "data_ptr"):
            import torch

            for name, im in (("left", left), ("right", right)):
                if not (isinstance(im, torch.Tensor) and im.dtype == torch.uint8 and tuple(im.shape) == shape
                        and im.is_contiguous() and im.is_cuda and im.device.index == self.ctx.device):
                    raise ValueError(f"NativeStereoVO.process: {name} must be a contiguous uint8 tensor of shape "
                                     f"{shape} on cuda:{self.ctx.device}, got "
                                     f"{getattr(im, 'dtype', None)} {tuple(getattr(im, 'shape', ()))} "
                                     f"on {getattr(im, 'device', None)}")
            self._order_after_torch(left.device)
            self._keep[t] = (left, right)
            self._keep.pop(t - 2, None)
            rc = self.lib.me_vo_loop_process(self.h, t, ctypes.c_void_p(left.data_ptr()),
                                             ctypes.c_void_p(right.data_ptr()), ME_DEVICE)
        else:
            L, R = np.asarray(left), np.asarray(right)
            for name, im in (("left", L), ("right", R)):
                if im.dtype != np.uint8 or im.shape != shape:
                    raise ValueError(f"NativeStereoVO.process: {name} must be a uint8 array of shape {shape}, "
                                     f"got {im.dtype} {im.shape}")
            L, R = np.ascontiguousarray(L), np.ascontiguousarray(R)
            rc = self.lib.me_vo_loop_process(self.h, t, L.ctypes.data, R.ctypes.data, ME_HOST)
        self._check(rc, "me_vo_loop_process")

    def finish(self):
        self._check(self.lib.me_vo_loop_finish(self.h), "me_vo_loop_finish")

    def close(self):
        if getattr(self, "h", None):
            self.lib.me_vo_loop_destroy(self.h)
            self.h = None
        self._keep = {}
        if self._masked:
            self.ctx.set_cu_mask(None)
            self.tctx.set_cu_mask(None)
            self._masked = False
        if self._own_t:
            self.tctx.close()
            self._own_t = False

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- results (the attributes WindowedStereoVO exposes)
    @property
    def results(self):
        import ctypes

        from ._lib import VOFrameResultC

        n = ctypes.c_int()
        self._check(self.lib.me_vo_loop_results(self.h, None, 0, ctypes.byref(n)), "results")
        arr = (VOFrameResultC * max(n.value, 1))()
        self._check(self.lib.me_vo_loop_results(self.h, arr, n.value, ctypes.byref(n)), "results")
        return [FrameResult(r.t, r.n_tracked, r.n_new, r.n_active, r.n_window_pts, r.n_window_obs, r.scale,
                            r.scale_stop, r.scale_iters, r.ba_iters, r.ba_cost, np.array(r.pose[:], np.float64))
                for r in arr[:n.value]]

    def event_records(self) -> np.ndarray:
        """The WBA_Point event log as a numpy record array (kind 0 new, 1 add, 2 pop, 3 del)."""
        import ctypes

        from ._lib import VO_EVENT_DTYPE

        n = ctypes.c_long()
        self._check(self.lib.me_vo_loop_events(self.h, None, 0, ctypes.byref(n)), "events")
        a = np.zeros(n.value, VO_EVENT_DTYPE)
        if n.value:
            self._check(self.lib.me_vo_loop_events(self.h, a.ctypes.data, n.value, ctypes.byref(n)), "events")
        return a

    @property
    def events(self):
        """WindowedStereoVO.events: ("new"|"add", id, t, (xl, yl, xr, yr)), ("pop", id), ("del", id)."""
        out = []
        kinds = ("new", "add", "pop", "del")
        for e in self.event_records():
            k = int(e["kind"])
            if k < 2:
                out.append((kinds[k], int(e["id"]), int(e["t"]), tuple(float(v) for v in e["feat"])))
            else:
                out.append((kinds[k], int(e["id"])))
        return out

    def _tracks(self):
        import ctypes

        n = ctypes.c_int()
        self._check(self.lib.me_vo_loop_tracks(self.h, None, None, None, None, None, 0, ctypes.byref(n)), "tracks")
        m = n.value
        ids, X = np.zeros(m, np.int64), np.zeros((m, 3))
        act, first, last = np.zeros(m, np.uint8), np.zeros(m, np.int64), np.zeros(m, np.int64)
        self._check(self.lib.me_vo_loop_tracks(self.h, ids.ctypes.data, X.ctypes.data, act.ctypes.data,
                                               first.ctypes.data, last.ctypes.data, m, ctypes.byref(n)), "tracks")
        return ids, X, act.astype(bool), first, last

    @property
    def ids(self):
        return self._tracks()[0]

    @property
    def X(self):
        return self._tracks()[1]

    @property
    def active(self):
        return self._tracks()[2]

    @property
    def poses(self) -> dict:
        import ctypes

        n = ctypes.c_int()
        self._check(self.lib.me_vo_loop_poses(self.h, None, None, 0, ctypes.byref(n)), "poses")
        ts, ps = np.zeros(n.value, np.int32), np.zeros((n.value, 6))
        self._check(self.lib.me_vo_loop_poses(self.h, ts.ctypes.data, ps.ctypes.data, n.value, ctypes.byref(n)),
                    "poses")
        return {int(t): ps[i] for i, t in enumerate(ts)}

    @property
    def obs(self) -> dict:
        """Keyframe -> (track IDs, (n, 4) float32 features) of the observations still held."""
        import ctypes

        n = ctypes.c_int()
        self._check(self.lib.me_vo_loop_frames(self.h, None, 0, ctypes.byref(n)), "frames")
        ts = np.zeros(n.value, np.int32)
        self._check(self.lib.me_vo_loop_frames(self.h, ts.ctypes.data, n.value, ctypes.byref(n)), "frames")
        out = {}
        for t in ts:
            m = ctypes.c_int()
            self._check(self.lib.me_vo_loop_frame_obs(self.h, int(t), None, None, 0, ctypes.byref(m)), "obs")
            ids, fe = np.zeros(m.value, np.int64), np.zeros((m.value, 4), np.float32)
            self._check(self.lib.me_vo_loop_frame_obs(self.h, int(t), ids.ctypes.data, fe.ctypes.data, m.value,
                                                      ctypes.byref(m)), "obs")
            out[int(t)] = (ids, fe)
        return out

    def _stats(self):
        import ctypes

        s = (ctypes.c_double * 9)()
        self._check(self.lib.me_vo_loop_stats(self.h, s, 9), "stats")
        return list(s)

    @property
    def latest_id(self) -> int:
        return int(self._stats()[2])

    @property
    def stage_s(self) -> dict:
        s = self._stats()
        return {"host": s[0], "wait": s[1]}

    @property
    def wait_by_stage(self) -> dict:
        s = self._stats()
        names = ("klt_match_new", "match", "scale_submit", "ba_submit_window", "ba_result", "scale_result")
        return {nm: v for nm, v in zip(names, s[3:])}
