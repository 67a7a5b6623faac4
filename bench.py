#!/usr/bin/env python3
"""Headline benchmark: frames/s + BA iter/s, 2000 feats x 20-keyframe window (BASELINE.json, config 3).

One step = one stereo frame of the hot path on one batch of synthetic input,
inputs resident in HBM when the timed region starts:
  1. KLT: 2000 features tracked from the previous to the current left image
     (3 pyramid levels, 21x21 window)            -> klt.hip
  2. MI stereo-scale optimisation of the current keyframe (2000 tracks,
     11x11 MI patches, reference OptimisationParams defaults) -> scale.hip / mi
  3. windowed stereo BA: 2000 landmarks x 20 keyframes, 10 LM iterations
     (fixed work, tolerances off)   -> ba.hip (FP64 MFMA Schur)

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process
per GPU, each rank processes its own independent stereo stream (weak scaling,
no collective on the data path; config-3 windows are below the landmark count
at which the RCCL-sharded BA pays).  The barrier and the MAX over
ranks of the timed region stay; value = frames of all ranks / that time.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--frames", type=int, default=4, help="distinct synthetic frames cycled per rank")
    ap.add_argument("--ba-iters", type=int, default=10)
    ap.add_argument("--scale-iters", type=int, default=10,
                    help="MAX_NB_ITER of the frame's scale LM; tolerances off (SURVEY 8d frame definition)")
    ap.add_argument("--cpu-runs", type=int, default=5, help="runs of the 1-thread CPU-baseline sample (median)")
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="processes of the all-cores CPU figure (0: the host cores this process may use, <= 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lib", default=None, help="development A/B only: load this libme_hip.so build")
    ap.add_argument("--vo-matches", type=int, default=2000,
                    help="matches of the StereoVisualOdometry::process line (SURVEY 8f rank 1; 0: off)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run each frame's KLT, scale LM and BA back to back on one stream (no KLT/back-end overlap)")
    ap.add_argument("--overlap", choices=("frontend", "klt"), default="frontend",
                    help="two-stream pipeline: the front end (KLT + scale LM) of frame t+1 beside frame t's BA "
                         "(frontend), or only KLT of frame t+1 beside the scale LM + BA of frame t (klt)")
    ap.add_argument("--front-cus", type=int, default=8,
                    help="frontend overlap: the tracker context's stream runs on CUs i with i %% 16 < F and the "
                         "back-end stream on the others (me_set_cu_mask; whole XCDs per side, _lib.cu_split); 0: shared CUs")
    ap.add_argument("--streams", default="2,4",
                    help="extra measurement: S independent replica streams per GPU (one context, HIP stream and "
                         "host thread each, every stream's frames sequential), for each S of this comma list, "
                         "reported as multi_stream; the headline value stays one pipelined stream per GPU "
                         "(config 5's 8-GPU throughput story is replicas: this is its one-GPU part); '1': off")
    ap.add_argument("--sharded-ba", type=int, default=1,
                    help="config-4 landmark-sharded BA line (SURVEY 8e): over RCCL across the ranks when --gpus > 1, "
                         "two contexts on one GPU (host exchange, the crossover point) at N = 1; 0: off")
    ap.add_argument("--sharded-reps", type=int, default=3)
    ap.add_argument("--vo-loop", choices=("native", "python"), default="native",
                    help="the VO loop lines' host loop: native (me_vo_loop_*, C++) or the Python WindowedStereoVO")
    ap.add_argument("--comm", choices=("nccl", "gloo"), default="nccl",
                    help="torch.distributed backend for N > 1 (gloo: the sharded BA exchanges host-staged through "
                         "me_comm_create_callback -- rehearses the N-rank branch without RCCL)")
    ap.add_argument("--rank-device", choices=("local", "zero"), default="local",
                    help="GPU per rank: LOCAL_RANK (default) or device 0 for every rank (tests: N ranks on one GPU, "
                         "--comm gloo only)")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the RCCL process group even at one rank (exercises the RCCL exchange path)")
    ap.add_argument("--pipeline-frames", type=int, default=40,
                    help="keyframes of the end-to-end windowed VO line at the headline config (KLT -> epipolar MI "
                         "matching -> WBA_Point tracks -> scale LM -> sliding-window BA, pipelined); 0: off")
    ap.add_argument("--pipeline-c5-frames", type=int, default=64,
                    help="keyframes of the same loop at config 5 (W = 50: the window fills and slides); 0: off")
    ap.add_argument("--mi-pairs", type=int, default=1 << 20, help="pairs of the batched MI-kernel roofline line (0: off)")
    ap.add_argument("--timing", choices=("dominant", "all", "none"), default="dominant",
                    help="HIP-event timing inside the timed region: only the dominant kernel family (default; "
                         "the Schur family's sampled launches carry the events themselves, hipExtLaunchKernelGGL: "
                         "the kernel's own begin/end timestamps; other families record two events around the "
                         "launch), every family, or none")
    ap.add_argument("--timing-every", type=int, default=8,
                    help="time every k-th launch of the timed family inside the timed region (HIP events; "
                         "config 3: ~40 of the 330 Schur launches, the frame rate ~1.3 %% below --timing none)")
    ap.add_argument("--profile-steps", type=int, default=3,
                    help="untimed steps with every family timed, to pick the dominant family")
    return ap.parse_args()


class FrameData:
    pass


SCALE_ITERS = 10  # the frame's scale-LM MAX_NB_ITER (set from --scale-iters)


def scale_counters(ctx, stats):
    """Per-solve LM counters (me_scale_last_counters) into the frame statistics."""
    v = [ctypes.c_long() for _ in range(4)]
    ctx.check(ctx.lib.me_scale_last_counters(ctx.h, *[ctypes.byref(x) for x in v]), "me_scale_last_counters")
    stats["scale_res_evals"] += v[0].value
    stats["scale_rejections"] += v[2].value
    stats["scale_executed"] += v[3].value


def new_stats():
    return dict(frames=0, ba_iters=0, scale_iters=0, scale_res_evals=0, scale_rejections=0, scale_executed=0)


def make_frames(cfg: dict, seed: int, n_frames: int):
    from uasl_motion_estimation_amd import synthetic as S

    W, H, N, win = cfg["width"], cfg["height"], cfg["n_feats"], cfg["window"]
    scene, K, stream = S.stereo_stream(seed, W, H, n_frames + 1)
    frames = []
    rng = np.random.default_rng(seed)
    for f in range(n_frames):
        fd = FrameData()
        fd.prev = stream[f].left
        fd.cur = stream[f + 1]
        fd.klt_pts = S.grid_features(rng, N, W, H, 12).astype(np.float32)
        fd.scale = S.scale_problem(seed + f, W, H, N, window=win, w=5, frames=stream[: f + 2], scene=scene)
        fd.ba = S.ba_problem(seed * 7 + f, N, win, W, H)
        frames.append(fd)
    return frames


def upload_images(ctx, frames):
    """Device copies of every image, KLT point list and BA window (inputs
    resident in HBM before timing)."""
    from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, DeviceScaleTracks

    keep = []
    for fd in frames:
        for name, img in (("d_prev", fd.prev), ("d_curL", fd.cur.left), ("d_curR", fd.cur.right)):
            img = np.ascontiguousarray(img)
            p = ctypes.c_void_p()
            ctx.check(ctx.lib.me_malloc(ctx.h, ctypes.byref(p), img.nbytes))
            ctx.check(ctx.lib.me_memcpy_h2d(ctx.h, p, img.ctypes.data, img.nbytes))
            setattr(fd, name, p.value)
            keep.append(p.value)
        n = len(fd.klt_pts)
        for name, nbytes in (("d_pts_in", 8 * n), ("d_pts_out", 8 * n), ("d_status", n)):
            p = ctypes.c_void_p()
            ctx.check(ctx.lib.me_malloc(ctx.h, ctypes.byref(p), max(nbytes, 16)))
            setattr(fd, name, p.value)
        ctx.check(ctx.lib.me_memcpy_h2d(ctx.h, ctypes.c_void_p(fd.d_pts_in), fd.klt_pts.ctypes.data, 8 * n))
        fd.dba = DeviceBAProblem(fd.ba, ctx)  # BA window resident in HBM
        fd.dscale = DeviceScaleTracks(fd.scale, ctx)  # scale-state tracks resident in HBM
    return keep


class _Calls:
    """The C-ABI argument blocks of one frame, built once (as a C++ caller
    would keep them): per frame only the scalars that change are reset."""

    def __init__(self, ctx, fd, kp, ba_opts):
        from uasl_motion_estimation_amd._lib import ME_DEVICE, BASummaryC
        from uasl_motion_estimation_amd.optimisation import OptimisationParams, scale_struct

        H, W = fd.prev.shape
        n = len(fd.klt_pts)
        self.klt = (ctx.h, ME_DEVICE, ctypes.c_void_p(fd.d_prev), ctypes.c_void_p(fd.d_curL), W, H, W,
                    ctypes.c_void_p(fd.d_pts_in), ctypes.c_void_p(fd.d_pts_out), ctypes.c_void_p(fd.d_status), n,
                    ctypes.byref(kp))
        self.keep = []
        self.sc = scale_struct(fd.scale, self.keep, ME_DEVICE, (fd.d_curL, fd.d_curR), fd.dscale.d)
        self.scale0 = self.sc.scale
        self.sp = OptimisationParams.fixed_iterations(SCALE_ITERS).to_c()
        self.stop, self.it, self.nmi = ctypes.c_int(), ctypes.c_int(), ctypes.c_long()
        self.scale = (ctx.h, ctypes.byref(self.sc), ctypes.byref(self.sp), 0, ctypes.byref(self.stop),
                      ctypes.byref(self.it), None, 0, ctypes.byref(self.nmi))
        self.bp = fd.dba.struct()
        self.bo = ba_opts.to_c()
        self.bs = BASummaryC()
        self.ba = (ctx.h, ctypes.byref(self.bp), ctypes.byref(self.bo), ctypes.byref(self.bs))


def _calls(ctx, fd, kp, ba_opts):
    """The frame's argument blocks for this context (built once per context)."""
    m = fd.__dict__.setdefault("_calls", {})
    c = m.get(id(ctx))
    if c is None:
        c = m[id(ctx)] = _Calls(ctx, fd, kp, ba_opts)
    return c


def gpu_step(ctx, fd, kp, ba_opts, stats):
    """One frame, sequential on the ctx stream: KLT, scale LM, BA."""
    c = _calls(ctx, fd, kp, ba_opts)
    ctx.check(ctx.lib.me_klt_track(*c.klt), "klt")
    back_end(ctx, fd, kp, ba_opts, stats)


def back_end(ctx, fd, kp, ba_opts, stats):
    """Scale LM + BA of one frame on the ctx stream (blocking, as the reference's optimise())."""
    c = _calls(ctx, fd, kp, ba_opts)
    lib = ctx.lib
    c.sc.scale = c.scale0  # every replay of the frame starts from the same scale
    ctx.check(lib.me_scale_optimise(*c.scale), "me_scale_optimise")
    stats["scale_iters"] += c.it.value
    scale_counters(ctx, stats)
    fd.dba.reset()  # same starting point every time the frame is replayed (device copy)
    ctx.check(lib.me_ba_solve(*c.ba), "me_ba_solve")
    stats["ba_iters"] += c.bs.iterations
    stats["frames"] += 1


class _Hip:
    """HIP events through the runtime (plumbing for the two-stream frame pipeline)."""

    def __init__(self):
        self.rt = ctypes.CDLL("libamdhip64.so")
        self.rt.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        self.rt.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self.rt.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        self.rt.hipEventDestroy.argtypes = [ctypes.c_void_p]

    def event(self):
        e = ctypes.c_void_p()
        assert self.rt.hipEventCreateWithFlags(ctypes.byref(e), 2) == 0  # hipEventDisableTiming
        return e

    def record(self, e, stream):
        assert self.rt.hipEventRecord(e, stream) == 0

    def wait(self, stream, e):
        assert self.rt.hipStreamWaitEvent(stream, e, 0) == 0


class FramePipeline:
    """Two-stream frame pipeline on one GPU.

    overlap="frontend" (default): the front end of frame t+1 (KLT, then the
    MI scale LM, both on the tracker context's HIP stream) runs while the back
    end of frame t (the windowed BA, queued whole with me_ba_solve_async on
    the back-end context's stream) runs beside it -- the usual VO split of a
    tracking front end and a BA back end (the BA of keyframe t refines the
    window; frame t+1's motion estimate starts from frame t's front-end pose).
    Frame t's BA waits (stream-side) on an event recorded after frame t's
    scale LM, so every dependency the back end has on its front end is kept;
    per frame the work is exactly the sequential gpu_step's (one KLT, one
    scale LM, one BA).

    overlap="klt": only KLT of frame t+1 runs on the tracker stream; the scale
    LM stays on the back-end stream between the BAs (round-1 pipeline)."""

    def __init__(self, ctx, tctx, hip, overlap="frontend"):
        self.ctx, self.tctx, self.hip, self.overlap = ctx, tctx, hip, overlap
        self.ev = [hip.event(), hip.event()]
        self.s_main = ctypes.c_void_p(ctx.lib.me_get_stream(ctx.h))
        self.s_trk = ctypes.c_void_p(tctx.lib.me_get_stream(tctx.h))

    @property
    def scale_ctx(self):
        """The context whose argument blocks hold the frames' scale-LM results."""
        return self.tctx if self.overlap == "frontend" else self.ctx

    def _klt(self, fd, kp, ba_opts, k):
        c = _calls(self.tctx, fd, kp, ba_opts)
        self.tctx.check(self.tctx.lib.me_klt_track(*c.klt), "klt")
        self.hip.record(self.ev[k & 1], self.s_trk)

    def _scale(self, cx, fd, kp, ba_opts, stats):
        c = _calls(cx, fd, kp, ba_opts)
        c.sc.scale = c.scale0  # every replay of the frame starts from the same scale
        cx.check(cx.lib.me_scale_optimise(*c.scale), "me_scale_optimise")
        stats["scale_iters"] += c.it.value
        scale_counters(cx, stats)

    def run(self, frames, n, kp, ba_opts, stats, first=0):
        if n <= 0:
            return
        # the contexts' streams may have been re-created (me_set_cu_mask) since the last run
        self.s_main = ctypes.c_void_p(self.ctx.lib.me_get_stream(self.ctx.h))
        self.s_trk = ctypes.c_void_p(self.tctx.lib.me_get_stream(self.tctx.h))
        if self.overlap == "frontend":
            return self._run_frontend(frames, n, kp, ba_opts, stats, first)
        ctx, lib = self.ctx, self.ctx.lib
        self._klt(frames[first % len(frames)], kp, ba_opts, 0)
        pend = None
        for t in range(n):
            fd = frames[(first + t) % len(frames)]
            c = _calls(ctx, fd, kp, ba_opts)
            self.hip.wait(self.s_main, self.ev[t & 1])  # frame t's back end after its tracks
            self._scale(ctx, fd, kp, ba_opts, stats)
            if t + 1 < n:  # issued once the scale LM is done: it overlaps the BA's latency-bound kernels
                self._klt(frames[(first + t + 1) % len(frames)], kp, ba_opts, t + 1)
            if pend is not None:  # frame t-1's BA finished before this scale LM ran (same stream)
                self._ba_wait(pend, stats)
            fd.dba.reset()
            ctx.check(lib.me_ba_solve_async(ctx.h, ctypes.byref(c.bp), ctypes.byref(c.bo)), "me_ba_solve_async")
            pend = c
        self._ba_wait(pend, stats)

    def _run_frontend(self, frames, n, kp, ba_opts, stats, first):
        ctx, lib = self.ctx, self.ctx.lib
        pend = None
        for t in range(n):
            fd = frames[(first + t) % len(frames)]
            # front end of frame t on the tracker stream: KLT, scale LM (blocking
            # host call), while frame t-1's BA runs on the back-end stream
            self._klt(fd, kp, ba_opts, t)
            self._scale(self.tctx, fd, kp, ba_opts, stats)
            self.hip.record(self.ev[t & 1], self.s_trk)
            c = _calls(ctx, fd, kp, ba_opts)
            self.hip.wait(self.s_main, self.ev[t & 1])  # frame t's back end after its front end
            fd.dba.reset()
            # queued behind frame t-1's BA (two solves may be queued per context): the
            # back-end stream never waits for the host to build this plan
            ctx.check(lib.me_ba_solve_async(ctx.h, ctypes.byref(c.bp), ctypes.byref(c.bo)), "me_ba_solve_async")
            if pend is not None:
                self._ba_wait(pend, stats)
            pend = c
        self._ba_wait(pend, stats)

    def _ba_wait(self, c, stats):
        self.ctx.check(self.ctx.lib.me_ba_wait(self.ctx.h, ctypes.byref(c.bs)), "me_ba_wait")
        stats["ba_iters"] += c.bs.iterations
        stats["frames"] += 1


def cpu_payload(fd):
    """The host inputs of one frame (what the oracle leg needs; picklable)."""
    return (fd.prev, fd.cur.left, fd.klt_pts, fd.scale, fd.ba)


def cpu_frame(payload, ba_iters, scale_iters):
    """One frame on the CPU restatement (oracle/, 1 thread): KLT, scale LM, BA.
    Returns its outputs (the parity leg compares them with the GPU's)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O  # CPU baseline leg only
    from uasl_motion_estimation_amd.optimisation import OptimisationParams

    prev, cur, pts, sp, bp = payload
    kp, kst = O.klt(prev, cur, pts)
    sc = O.scale_optimise(sp, **OptimisationParams.fixed_iterations(scale_iters).oracle_kw())
    cams, pps, s = O.ba_solve(bp, max_num_iterations=ba_iters, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    return dict(klt=kp, klt_status=kst, scale=sc, cams=cams, pts=pps, ba=s)


def _pin_init(cores):
    """Pool initializer: pin this worker process to one core of the shared
    queue (the `taskset -c` of BASELINE.md / SURVEY §8d, done in-process)."""
    try:
        core = cores.get(timeout=5)
        os.sched_setaffinity(0, {core})
    except Exception:  # pragma: no cover  (affinity not permitted: unpinned, reported as such)
        pass


def _cpu_worker(args):
    """All-cores leg: one process runs its frames back to back (spawned before
    this bench touched the GPU, pinned to its own core)."""
    payloads, ba_iters, scale_iters = args
    t0 = time.perf_counter()
    for pl in payloads:
        cpu_frame(pl, ba_iters, scale_iters)
    return len(payloads), time.perf_counter() - t0


def _cpu_single(args):
    """1-thread leg in a process pinned to one core: one warm-up frame, then
    `runs` passes over the distinct frames; per-pass frames/s."""
    pls, ba_iters, scale_iters, runs = args
    cpu_frame(pls[0], ba_iters, scale_iters)
    rates, tot_t, ba_it = [], 0.0, 0
    for _ in range(max(1, runs)):
        t1 = time.perf_counter()
        for pl in pls:
            ba_it += cpu_frame(pl, ba_iters, scale_iters)["ba"]["iterations"]
        dt = time.perf_counter() - t1
        rates.append(len(pls) / dt)
        tot_t += dt
    return rates, tot_t, ba_it, sorted(os.sched_getaffinity(0))


def host_cpu():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    return model, os.cpu_count() or 1, avail


def gpu_outputs(ctx, fd, sctx=None):
    """Outputs of the last timed replay of a frame, read back after the timed
    region: KLT points/status (device buffers), the scale LM result (the
    frame's argument block) and the BA window (device-resident problem)."""
    n = len(fd.klt_pts)
    kp = np.zeros((n, 2), np.float32)
    kst = np.zeros(n, np.uint8)
    ctx.check(ctx.lib.me_memcpy_d2h(ctx.h, kp.ctypes.data, ctypes.c_void_p(fd.d_pts_out), kp.nbytes))
    ctx.check(ctx.lib.me_memcpy_d2h(ctx.h, kst.ctypes.data, ctypes.c_void_p(fd.d_status), kst.nbytes))
    c = fd._calls[id(ctx)]
    cs = fd._calls[id(sctx or ctx)]  # the context that ran the frame's scale LM
    cams, pts = fd.dba.download()
    return dict(klt=kp, klt_status=kst, scale=dict(stop=cs.stop.value, iterations=cs.it.value, scale=cs.sc.scale),
                cams=cams, pts=pts, ba=dict(iterations=c.bs.iterations, successful_steps=c.bs.successful_steps))


def compare(g, o):
    """Parity bars of the tests (tests/test_gpu_configs.py) on one frame."""
    klt = bool(np.array_equal(g["klt_status"], o["klt_status"])
               and np.array_equal(g["klt"].view(np.uint32), np.asarray(o["klt"], np.float32).view(np.uint32)))
    gs, os_ = g["scale"], o["scale"]
    scale = (gs["stop"] == os_["stop"] and gs["iterations"] == os_["iterations"]
             and abs(gs["scale"] - os_["scale"]) <= 1e-9 * abs(os_["scale"]))

    def rel(a, b):
        return float(np.max(np.abs(a - b) / (np.abs(b) + 1e-3)))  # 1e-6 rel with a 1e-9 floor ~ this at |b| >= 1e-3

    ba_ok = (g["ba"]["iterations"] == o["ba"]["iterations"]
             and g["ba"]["successful_steps"] == o["ba"]["successful_steps"]
             and np.allclose(g["cams"], o["cams"], rtol=1e-6, atol=1e-9)
             and np.allclose(g["pts"], o["pts"], rtol=1e-6, atol=1e-9))
    return dict(klt_bit_exact=klt, scale_match=bool(scale), ba_match=bool(ba_ok),
                ba_max_rel=max(rel(g["cams"], o["cams"]), rel(g["pts"], o["pts"])))


# Algorithmic work per launch of each kernel family: (bound,
# amount, unit, peak).  Bytes are the algorithmic HBM bytes of one launch;
# flops are the useful FP64 MFMA flops (no padding).  cam_solve (BA_SOLVE)
# is a single-workgroup dependency chain with no HBM/MFMA roofline.
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
MI_COUNTERS = "r06_mi_reg"  # SQ counters of the current batch MI kernel (tools/gpu.sh sq)
PEAK_F64_MFMA_TFS = 78.6   # MI355X FP64 matrix spec


def alg_work(family: str, cfg: dict, frames):
    N = cfg["n_feats"]
    hbm = lambda b: ("hbm", float(b), "GB/s", PEAK_HBM_GBS)  # noqa: E731
    if family == "SCALE_RES":
        return hbm(262.0 * N)                  # 2x121 px + 2 corners + out per track
    if family == "SCALE_NEQ":
        return hbm(234.0 * N)                  # x0 100 B + x1 u x2 110 B + corners + out
    if family == "KLT":
        return hbm((2 * 22 * 22 + 2 * 2 * 22 * 22 + 16) * 4.0 * N)  # I, dIx, dIy windows (+1 border) x 3 levels
    fd = frames[0].ba
    no, npt = len(fd.obs), len(fd.pts)
    n6 = 6 * (len(fd.cams) - fd.fixed_frames)
    if family == "BA_LINEARIZE":
        return hbm(no * (32 + 8 + 24 + 48 + 320.0 + 72 + 144 + 216))  # in: obs, idx, point, camera; out: r+J, V_o/g_o, W_o, camera pieces
    if family == "BA_POINTS":
        return hbm(no * 72.0 + npt * (72 + 72 + 72 + 24))             # V_o/g_o in; V, g, L_p, z out
    if family == "BA_SCHUR":
        # useful Schur-fill flops: per landmark with k observations by variable
        # cameras 108 k + 216 k (k + 1) / 2 + 60 -- not the padded dense GEMM the kernel runs
        k = np.bincount(fd.pt_idx[fd.cam_idx >= fd.fixed_frames], minlength=npt).astype(np.float64)
        return ("mfma", float(np.sum(108.0 * k + 108.0 * k * (k + 1) + 60.0)), "TFLOP/s", PEAK_F64_MFMA_TFS)
    if family == "BA_STEP":
        return hbm(no * (144 + 320 + 32 + 8 + 8 + 48.0) + npt * (24 + 72 + 72 + 48))  # W_o, r+J, obs, idx, cams | point
    return None


# kernels of each timed family (the PMC traffic of a family launch is their sum)
FAMILY_KERNELS = {
    "SCALE_RES": ["scale_res_ctrl_kernel"], "SCALE_NEQ": ["scale_neq_ctrl_kernel"], "KLT": ["klt_kernel"],
    "BA_LINEARIZE": ["linearize_kernel"],
    "BA_SCHUR": ["pt_schur_kernel"], "BA_SOLVE": ["cam_solve_kernel"],
    "BA_STEP": ["pt_step_kernel"], "MI": ["mi_quad_kernel"],
}


# PMC traffic = 2 x FETCH_SIZE + WRITE_SIZE (tools/summarise.py pmc).  The MI355X
# guide calibrates the x2 on FETCH_SIZE only for 16-byte-per-lane streaming
# reads (and WRITE_SIZE for 16-byte streaming stores); none of these kernels
# is such a stream (pt_schur_kernel: 8-byte double gathers of W / obs rows and
# written-through partial tiles; mi_quad_kernel: byte patch rows; KLT:
# unaligned dwords), so their absolute traffic is uncalibrated -- ratios
# between variants of one kernel stand.
TRAFFIC_CALIBRATION = ("uncalibrated: 2 x FETCH_SIZE + WRITE_SIZE, the guide's correction for 16-B/lane streaming "
                       "reads applied to a kernel that is not one; ratios between variants hold")


def pmc_traffic(family: str):
    """HBM bytes per family launch from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, written by tools/summarise.py pmc from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this same bench); None if absent."""
    import glob
    import re

    # newest = highest round / version numbers (natural order: v10 after v9)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")),
                   key=lambda f: ([int(x) for x in re.findall(r"\d+", os.path.basename(f))], os.path.basename(f)))
    ks = FAMILY_KERNELS.get(family, [])
    for f in reversed(files):  # the newest summary that profiled this family's kernels
        d = json.load(open(f))
        if ks and all(k in d for k in ks):
            return float(sum(d[k]["traffic_bytes"] for k in ks))
    return None


def rocprof_avg_ms(family: str):
    """Average duration (ms) of the family's kernel in the newest committed
    headline-frame rocprofv3 summary (profiles/*_kernel_stats.txt written by
    tools/gpu.sh prof: the bench's config-3 frame without event timing), and
    that file's name; (None, None) if absent.  The live HIP-event average
    brackets each sampled launch with two event packets on the BA stream, so
    it also carries the dependent-launch gap and the events' own cost."""
    import glob
    import re

    ks = FAMILY_KERNELS.get(family, [])
    files = [f for f in glob.glob(os.path.join(ROOT, "profiles", "*_kernel_stats.txt")) if "_bench_" not in f]
    files.sort(key=lambda f: ([int(x) for x in re.findall(r"\d+", os.path.basename(f))], os.path.basename(f)))
    for f in reversed(files):
        best = None
        for line in open(f):
            m = re.match(r"\s*(?:void )?(\S+?)(?:<[^>]*>)?\s+(\d+)\s+([\d.]+) us\s+([\d.]+) us/call", line)
            if m and ks and m.group(1) in ks and (best is None or int(m.group(2)) > best[0]):
                best = (int(m.group(2)), float(m.group(4)))
        if best:
            return best[1] * 1e-3, os.path.basename(f)
    return None, None


def mi_batch_roofline(ctx, frames, n_pairs: int, reps: int = 10):
    """Batched MI patch scores (A1, 11x11) on n_pairs pairs of the resident
    frame images: the north-star MI kernel measured on its own (HIP events
    on the ctx stream), algorithmic bytes 262 B per pair."""
    from uasl_motion_estimation_amd.mutual_information import mi_scores_device

    fd = frames[0]
    H, W = fd.cur.left.shape
    rng = np.random.default_rng(7)
    xyL = np.stack([rng.integers(0, W - 11, n_pairs), rng.integers(0, H - 11, n_pairs)], -1).astype(np.int32)
    xyR = xyL.copy()
    xyR[:, 0] = np.clip(xyL[:, 0] - rng.integers(0, 40, n_pairs), 0, W - 11)
    dL, dR, dout = ctx.malloc(xyL.nbytes), ctx.malloc(xyR.nbytes), ctx.malloc(4 * n_pairs)
    ctx.h2d(dL, xyL)
    ctx.h2d(dR, xyR)
    run = lambda: mi_scores_device(ctx, fd.d_curL, W, fd.d_curR, W, W, H, dL, dR, n_pairs, (11, 11), dout)  # noqa: E731
    run()
    run()
    ctx.synchronize()
    ctx.timing_reset()
    ctx.timing(True)
    for _ in range(reps):
        run()
    ctx.synchronize()
    ctx.timing(False)
    n, ms = ctx.timing_read("MI")
    for p in (dL, dR, dout):
        ctx.free(p)
    avg = ms / max(n, 1)
    achieved = 262.0 * n_pairs / (avg * 1e-3) / 1e9
    kernel = "mi_lane_kernel" if os.environ.get("ME_MI_KERNEL") == "lane" else "mi_quad_kernel"
    out = {"bound": "hbm", "achieved": round(achieved, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
           "frac": round(achieved / PEAK_HBM_GBS, 5), "traffic": pmc_traffic("MI"),
           "traffic_calibration": TRAFFIC_CALIBRATION, "kernel": kernel,
           "pairs": n_pairs, "avg_launch_ms": round(avg, 5), "pairs_per_s": round(n_pairs / (avg * 1e-3), 1)}
    # VALU-issue roofline: the kernel's wave instructions per pair (SQ_INSTS_VALU of the committed
    # tools/gpu.sh sq pass) against one wave64 VALU instruction per SIMD per 2 cycles (1024 SIMDs,
    # 2.4 GHz: MI355X_MICROARCH.md "Wave scheduling" / v_fma_f32 row -- 32 lanes per cycle; one wave
    # alone issues every 4, but the kernel keeps ~8 waves per CU resident)
    cpath = os.path.join(ROOT, "profiles", MI_COUNTERS + ".json")
    if os.path.exists(cpath):
        cnt = json.load(open(cpath))
        vpp = cnt.get("valu_insts_per_pair", cnt.get("insts_valu_per_pair"))  # (round-5 / tools/summarise.py keys)
        if kernel in cnt.get("kernel", "") and vpp:
            peak = 1024 * 2.4e9 / 2 / 1e9
            ach = vpp * n_pairs / (avg * 1e-3) / 1e9
            out["valu_issue"] = {"bound": "valu-issue", "achieved": round(ach, 1), "peak": round(peak, 1),
                                 "unit": "G wave-instr/s", "frac": round(ach / peak, 4),
                                 "valu_insts_per_pair": round(vpp, 2),
                                 "resident_waves_per_cu": round(cnt["resident_waves_per_cu"], 2),
                                 "counters": "profiles/" + MI_COUNTERS + ".txt"}
    return out


def stereo_vo_line(ctx, n: int, reps: int = 5, cpu: bool = True):
    """StereoVisualOdometry::process (src/vo/StereoVisualOdometry.cpp:34-114):
    200 RANSAC hypotheses + GN refinement on n synthetic quad matches
    (noise 0.005 px, the parity-test setup), device vs the oracle (1 thread)."""
    from uasl_motion_estimation_amd import synthetic as S
    from uasl_motion_estimation_amd.vo import Parameters, StereoVisualOdometry

    m, p = S.vo_matches(12, n, noise=0.005)
    vo = StereoVisualOdometry(Parameters(**{k: v for k, v in p.items() if k in Parameters.__dataclass_fields__}),
                              ctx=ctx)
    vo.srand(1)
    vo.process(m)
    t0 = time.perf_counter()
    for _ in range(reps):
        vo.srand(1)
        ok = vo.process(m)
    gpu_ms = (time.perf_counter() - t0) * 1e3 / reps
    out = {"matches": n, "ms_per_process": round(gpu_ms, 3), "ok": bool(ok), "inliers": len(vo.getInliers_idx())}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle as O  # CPU baseline leg only

        seq = O.libc_rand_seq(1, 16 * 200 + 64)
        t0 = time.perf_counter()
        O.vo_process(m, p, rand_seq=seq)
        out["cpu_ms_per_process"] = round((time.perf_counter() - t0) * 1e3, 3)
        out["cpu_cores"] = 1
    return out


def _shard_parity(cams, pts, lo, hi, s_sh, ref_cams, ref_pts, s_ref):
    """Sharded vs single-device solve of the same window: max relative
    difference of cameras and of this rank's landmarks, equal iteration and
    successful-step counts (tolerance 1e-6, the north-star pose bar)."""
    def rel(a, b):
        a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
        return float(np.max(np.abs(a - b) / (np.abs(b) + 1e-9))) if a.size else 0.0

    return {"cams_max_rel": rel(cams, ref_cams), "pts_max_rel": rel(pts, ref_pts[lo:hi]),
            "same_iterations": s_sh["iterations"] == s_ref["iterations"]
            and s_sh["successful_steps"] == s_ref["successful_steps"]}


def _parity_ok(p):
    return bool(p["same_iterations"] and p["cams_max_rel"] <= 1e-6 and p["pts_max_rel"] <= 1e-6)


def crossover_model(ctx, opts, reps, xch_lb_us=None):
    """Where landmark sharding pays, from one GPU: the device time of the
    largest rank's shard (1/G of the landmarks, all cameras, the same fixed
    LM iterations) plus two all-reduces per iteration, priced two ways:
    (a) at the MEASURED per-exchange cost of the 1-rank RCCL communicator on
    this GPU (xch_lb_us, from rccl_1rank: a lower bound -- a real ring over
    xGMI adds hops), and (b) at the library gate's per-exchange estimate
    (me_ba_shard_exchange_us); `gate` is me_ba_shard_worthwhile's decision
    for the window at G ranks.  A prediction for the driver's 8-GPU run, not
    a measurement."""
    from uasl_motion_estimation_amd import synthetic as S
    from uasl_motion_estimation_amd._lib import load_library
    from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, shard_landmarks, shard_worthwhile

    lib = load_library()
    est = {G: lib.me_ba_shard_exchange_us(G) for G in (2, 4, 8)}
    rows = []
    for name, (npts, win, w, h, seed) in {"config 3 (2000 x 20)": (2000, 20, 1280, 720, 3),
                                          "config 4 (8000 x 30)": (8000, 30, 3840, 2160, 4),
                                          "VO window at W = 50 (8000 x 50)": (8000, 50, 1280, 720, 5)}.items():
        bp = S.ba_problem(S.SEED0 + seed, npts, win, w, h)
        row = {"window": name, "observations": len(bp.obs)}
        t1 = None
        for G in (1, 2, 4, 8):
            local = bp if G == 1 else shard_landmarks(bp, 0, G)[0]
            d = DeviceBAProblem(local, ctx)
            d.solve(opts)
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                d.reset()
                s1 = d.solve(opts)
            el = (time.perf_counter() - t0) / reps
            d.close()
            if G == 1:
                t1 = el
                row["ms_1gpu"] = round(1e3 * el, 3)
                continue
            row[f"ms_shard_{G}"] = round(1e3 * el, 3)
            if xch_lb_us is not None:
                pred = el + 2 * s1["iterations"] * xch_lb_us * 1e-6
                row[f"predicted_speedup_{G}gpu_measured_1rank_xch"] = round(t1 / pred, 2)
            pred = el + 2 * s1["iterations"] * est[G] * 1e-6
            row[f"predicted_ms_{G}gpu"] = round(1e3 * pred, 3)
            row[f"predicted_speedup_{G}gpu"] = round(t1 / pred, 2)
            row[f"gate_{G}gpu"] = shard_worthwhile(len(bp.obs), G)
        rows.append(row)
    return {"xch_us_measured_1rank_lower_bound": None if xch_lb_us is None else round(xch_lb_us, 2),
            "xch_us_gate_estimate": {str(G): v for G, v in est.items()}, "rows": rows}


def hbm_copy_gbs(ctx, nbytes: int = 1 << 30, reps: int = 20):
    """Measured HBM bandwidth of this GPU (read + write bytes / time): the
    library's 16-byte-per-lane nontemporal streaming copy of a 1 GiB buffer
    (me_hbm_copy_gbs, the best of tools/ubench/copy.hip's sweep, ~6.0 TB/s;
    the MI355X guide quotes 6.29 TB/s for a float4 copy) -- the measured
    denominator beside the 8 TB/s datasheet peak
    (SURVEY §8d).  (Round 5 used a torch uint8 copy_, 4.8-4.9 TB/s, which
    inflated every frac_vs_measured_copy by ~1.3x)"""
    g = ctypes.c_double()
    ctx.check(ctx.lib.me_hbm_copy_gbs(ctx.h, nbytes, reps, ctypes.byref(g)), "me_hbm_copy_gbs")
    return round(g.value, 1)


def exchange_us(ctx, comm, barrier, sizes, reps=50):
    """Measured cost (us) of one in-place sum all-reduce of n doubles through
    the library's communicator on the ctx stream, per size: the packed
    camera-system exchange (~17k doubles at W = 30) and the step scalars (5)."""
    out = {}
    for n in sizes:
        d = ctx.malloc(8 * n)
        ctx.h2d(d, np.zeros(n))
        for _ in range(5):
            comm.allreduce(d, n)
        ctx.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            comm.allreduce(d, n)
        ctx.synchronize()
        out[str(n)] = round((time.perf_counter() - t0) / reps * 1e6, 2)
        ctx.free(d)
    return out


def sharded_ba_line(args, ctx, dist, world, rank, local_rank, barrier):
    """Config-4 window (8000 landmarks x 30 keyframes, args.ba_iters LM
    iterations) solved (a) unsharded on this GPU and (b) landmark-sharded with
    the library's communicator (me_ba_solve_comm: one packed all-reduce after
    the Schur pass and one of the step scalars per LM iteration): native RCCL
    across the world's ranks (one GPU each), or, at N = 1, RCCL at one rank
    (the exchange's own overhead) and two contexts of this GPU with a
    host-staged thread exchange.  Every mode is checked against the
    single-device solve of the same window (parity).  Shards are resident in
    HBM (reset by a device copy); timing: barrier + MAX over ranks."""
    import threading

    import torch

    from uasl_motion_estimation_amd import synthetic as S
    from uasl_motion_estimation_amd._lib import Context, load_library
    from uasl_motion_estimation_amd.optimisation import (Comm, DeviceBAProblem, SolverOptions, ThreadAllReduce,
                                                         rccl_comm, shard_landmarks, shard_worthwhile)

    c = S.CONFIGS[4]
    bp = S.ba_problem(S.SEED0 + 4, c["n_feats"], c["window"], c["width"], c["height"])
    opts = SolverOptions.fixed_iterations(args.ba_iters)
    reps = max(1, args.sharded_reps)
    full = DeviceBAProblem(bp, ctx)
    full.solve(opts)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        full.reset()
        s1 = full.solve(opts)
    t_single = (time.perf_counter() - t0) / reps
    ref_cams, ref_pts = full.download()
    full.close()
    out = {"workload": f"config 4 BA: {len(bp.pts)} landmarks x {len(bp.cams)} keyframes, {len(bp.obs)} observations, "
                       f"{args.ba_iters} LM iterations", "single_gpu_ms": round(1e3 * t_single, 3),
           "single_gpu_ba_iter_per_s": round(s1["iterations"] / t_single, 1),
           "exchanges_per_lm_iteration": 2}

    def timed_comm(d, comm):
        d.reset()
        d.solve_comm(comm, opts)
        barrier()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            d.reset()
            ss = d.solve_comm(comm, opts)
        ctx.synchronize()
        return (time.perf_counter() - t0) / reps, ss

    if dist is not None:
        from uasl_motion_estimation_amd.optimisation import host_staged_allreduce

        gloo = args.comm == "gloo"
        local, (lo, hi) = shard_landmarks(bp, rank, world)
        d = DeviceBAProblem(local, ctx)
        if gloo:
            # host-staged exchange: the kernels and the callback's copies ordered on one torch stream
            stream = torch.cuda.Stream(device=ctx.device)
            torch.cuda.set_stream(stream)
            ctx.set_stream(stream.cuda_stream)
            comm = Comm.callback(ctx, world, rank, host_staged_allreduce())
        else:
            comm = rccl_comm(ctx)
        try:
            cal = comm.exchange_us()  # measured by the communicator at creation (max over the ranks)
            gate_cal = comm.shard_worthwhile(len(bp.obs))
            el, ss = timed_comm(d, comm)
            cams, pts = d.download()
            xus = exchange_us(ctx, comm, barrier, [17000, 5])
        finally:
            comm.close()
            if gloo:
                ctx.set_stream(None)
                torch.cuda.set_stream(torch.cuda.default_stream(ctx.device))
        d.close()
        par = _shard_parity(cams, pts, lo, hi, ss, ref_cams, ref_pts, s1)
        tt = torch.tensor([el, par["cams_max_rel"], par["pts_max_rel"], 0.0 if par["same_iterations"] else 1.0],
                          device="cpu" if gloo else f"cuda:{local_rank}", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt[0].item())
        par = {"cams_max_rel": float("%.3g" % tt[1].item()), "pts_max_rel": float("%.3g" % tt[2].item()),
               "same_iterations": tt[3].item() == 0.0}
        par["ok"] = _parity_ok(par)
        out.update({"mode": (f"landmark-sharded over a host-staged gloo exchange (me_comm_create_callback), {world} "
                             f"ranks" + (" on one GPU" if args.rank_device == "zero" else ", one GPU each")) if gloo
                    else f"landmark-sharded over native RCCL (me_comm), {world} ranks, one GPU each",
                    "ranks": world, "sharded_ms": round(1e3 * el, 3),
                    "gate_would_shard": gate_cal,
                    "gate_inputs": {"calibrated_exchange_us": {k: round(v, 2) for k, v in cal.items()},
                                    "per_exchange_us": round(0.5 * (cal["system"] + cal["scalars"]), 2),
                                    "built_in_estimate_us": round(load_library().me_ba_shard_exchange_us(world), 2),
                                    "gate_at_built_in_estimate": shard_worthwhile(len(bp.obs), world)},
                    "exchange_us": xus,
                    "sharded_ba_iter_per_s": round(ss["iterations"] / el, 1),
                    "speedup_vs_single_gpu": round(t_single / el, 3), "landmarks_rank0": hi - lo if rank == 0 else None,
                    "parity_vs_single_gpu": par})
        return out
    # N = 1 (a) native RCCL at one rank: the exchange's overhead on the same window
    try:
        comm = Comm.rccl(ctx, 1, 0, Comm.unique_id())
        d = DeviceBAProblem(bp, ctx)
        el1, ss1 = timed_comm(d, comm)
        cams, pts = d.download()
        d.close()
        xus1 = exchange_us(ctx, comm, barrier, [17000, 5])
        comm.close()
        par = _shard_parity(cams, pts, 0, len(bp.pts), ss1, ref_cams, ref_pts, s1)
        par = {k: (float("%.3g" % v) if isinstance(v, float) else v) for k, v in par.items()}
        par["ok"] = _parity_ok(par)
        xch_lb = max(0.0, (el1 - t_single) / max(1, 2 * ss1["iterations"])) * 1e6
        out["rccl_1rank"] = {"ms": round(1e3 * el1, 3), "overhead_vs_single_gpu": round(el1 / t_single - 1.0, 4),
                             "us_per_exchange_in_solve": round(xch_lb, 2), "exchange_us": xus1,
                             "parity_vs_single_gpu": par}
    except Exception as e:  # reported, never fatal
        xch_lb = None
        out["rccl_1rank"] = {"error": f"{type(e).__name__}: {e}"}
    # (b) two contexts on this GPU, threads + host exchange (the crossover point)
    ranks = 2
    ctxs = [Context(local_rank) for _ in range(ranks)]
    parts = [shard_landmarks(bp, r, ranks) for r in range(ranks)]
    shards = [DeviceBAProblem(parts[r][0], ctxs[r]) for r in range(ranks)]
    res, errs = [None] * ranks, []

    ar = ThreadAllReduce(ranks)
    comms = [None] * ranks

    def mk(r):  # (collective: the communicators calibrate their exchanges at creation, outside the timing)
        try:
            comms[r] = Comm.callback(ctxs[r], ranks, r, ar.callback(r, ctxs[r]))
        except Exception as e:  # pragma: no cover
            errs.append(e)

    def run(r):
        try:
            for _ in range(reps):
                shards[r].reset()
                res[r] = shards[r].solve_comm(comms[r], opts)
            ctxs[r].synchronize()
        except Exception as e:  # pragma: no cover
            errs.append(e)

    def in_threads(fn):
        th = [threading.Thread(target=fn, args=(r,)) for r in range(ranks)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        return time.perf_counter() - t0

    in_threads(mk)
    in_threads(run)
    el = in_threads(run) / reps
    cal2 = comms[0].exchange_us() if comms[0] is not None else None
    for cm in comms:
        if cm is not None:
            cm.close()
    pars = []
    for r in range(ranks):
        cams, pts = shards[r].download()
        lo, hi = parts[r][1]
        pars.append(_shard_parity(cams, pts, lo, hi, res[r], ref_cams, ref_pts, s1))
    for sh in shards:
        sh.close()
    for cc in ctxs:
        cc.close()
    if errs:
        raise errs[0]
    par = {"cams_max_rel": float("%.3g" % max(p["cams_max_rel"] for p in pars)),
           "pts_max_rel": float("%.3g" % max(p["pts_max_rel"] for p in pars)),
           "same_iterations": all(p["same_iterations"] for p in pars)}
    par["ok"] = _parity_ok(par)
    out["crossover_model"] = crossover_model(ctx, opts, reps, xch_lb)
    out.update({"mode": "landmark-sharded over 2 contexts of one GPU (threads, host-staged exchange through "
                        "me_comm_create_callback)", "ranks": ranks,
                "sharded_ms": round(1e3 * el, 3), "sharded_ba_iter_per_s": round(res[0]["iterations"] / el, 1),
                "speedup_vs_single_gpu": round(t_single / el, 3), "parity_vs_single_gpu": par,
                "calibrated_exchange_us": None if cal2 is None else {k: round(v, 2) for k, v in cal2.items()}})
    return out


def _frame_event_records(vo):
    """The keyframe (new / addMatch) events of a loop's WBA_Point log as me_vo_event records, in log order."""
    from uasl_motion_estimation_amd._lib import VO_EVENT_DTYPE

    if hasattr(vo, "event_records"):
        e = vo.event_records()
        return e[e["kind"] < 2]
    recs = [r for r in vo._ev if r[0] == "frame"]
    n = sum(len(r[1]) for r in recs)
    out = np.zeros(n, VO_EVENT_DTYPE)
    k = 0
    for _, ids, t, feats, is_new in recs:
        m = len(ids)
        out["kind"][k:k + m] = np.where(is_new, 0, 1)
        out["t"][k:k + m] = t
        out["id"][k:k + m] = ids
        out["feat"][k:k + m] = feats
        k += m
    return out


def pipeline_line(args, ctx, cpu: bool, c: int, n: int, warm: int = 6, parity_prefix: int = 0):
    """The windowed stereo VO loop itself (uasl_motion_estimation_amd/
    pipeline.py) on one synthetic stream of config c: per keyframe KLT, the
    epipolar MI matcher (tracked and new features), the WBA_Point
    bookkeeping, the scale LM and the sliding-window BA (10 LM iterations),
    every decision taken on the host from the hot path's results.  The loop
    runs pipelined (KLT and scale LM on a front-end context beside the BA,
    WindowedStereoVO(overlap=True)).  Images are uploaded before the timed
    loop; the host bookkeeping (numpy) is inside it.  Frames/s over the
    keyframes after `warm`; host time = bookkeeping outside the backend
    calls, wait = time blocked on device results; a second, event-timed pass
    gives the device time per kernel family.  With cpu=True the same loop runs
    sequentially on the oracle backend (1 thread) and its track IDs, feature
    positions and poses are compared with the GPU's.  parity_prefix = P > 0
    (cpu=False): the oracle runs the first P keyframes only and the GPU run's
    keyframe records (WBA_Point events, per-keyframe results and poses at
    completion) of those keyframes are compared with it -- keyframe k's
    decisions depend only on keyframes <= k + 1."""
    from uasl_motion_estimation_amd import pipeline as PL

    t0 = time.perf_counter()
    fr, K, p0, v, truth = PL.synthetic_sequence(c, n)
    gen = time.perf_counter() - t0
    cfg = PL.PipelineConfig.from_config(c)

    native = args.vo_loop == "native"

    def run(timed_families=False, log=False):
        from types import SimpleNamespace

        import torch

        if native:  # the loop in C++ (me_vo_loop_*); the images device-resident before timing
            dev = [(torch.from_numpy(fr[t].left).to(f"cuda:{ctx.device}"),
                    torch.from_numpy(fr[t].right).to(f"cuda:{ctx.device}")) for t in range(n)]
            torch.cuda.synchronize()
            vo = PL.NativeStereoVO(cfg, ctx, K, p0, v, log_events=log, overlap=True)
            tctx, be = vo.tctx, None

            def proc(t):
                vo.process(t, *dev[t])
        else:
            be = PL.GPUBackend(ctx)
            for t in range(n):
                be.frame_images(t, fr[t].left, fr[t].right)  # resident before timing
            ctx.synchronize()
            vo = PL.WindowedStereoVO(cfg, be, K, p0, v, log_events=log, overlap=True)
            tctx = be.tctx

            def proc(t):
                vo.process(t, fr[t].left, fr[t].right)
        for t in range(warm):
            proc(t)
        # (no finish() here: the loop applies BA(t-1) after keyframe t's matching, so the timed span
        # starts in steady state, with the last warm-up keyframe's BA in flight)
        for cc in (ctx, tctx):
            cc.timing_reset()
            cc.timing(timed_families)
        h0, w0 = vo.stage_s["host"], vo.stage_s["wait"]
        ws0 = dict(vo.wait_by_stage)
        t1 = time.perf_counter()
        for t in range(warm, n):
            proc(t)
        vo.finish()
        el = time.perf_counter() - t1
        fam = {}
        if timed_families:
            for name in ("MI", "SCALE_RES", "SCALE_NEQ", "BA_LINEARIZE", "BA_SCHUR", "BA_SOLVE", "BA_STEP", "KLT",
                         "PYR"):
                ms = sum(cc.timing_read(name)[1] for cc in (ctx, tctx))
                if ms > 0:
                    fam[name] = round(1e3 * ms / (n - warm), 1)
            for cc in (ctx, tctx):
                cc.timing(False)
        stage, wbs = vo.stage_s, vo.wait_by_stage
        ws = {k: round(1e3 * (v_ - ws0.get(k, 0.0)) / (n - warm), 3) for k, v_ in wbs.items()}
        # a snapshot of what the line reads (the native loop's state goes with close())
        snap = SimpleNamespace(results=vo.results, poses=vo.poses, ids=vo.ids, latest_id=vo.latest_id,
                               events=vo.events if log else None,
                               frame_events=_frame_event_records(vo) if log else None)
        if native:
            vo.close()
        else:
            be.close()
        return snap, el, (stage["host"] - h0), (stage["wait"] - w0), fam, ws

    # the timed run keeps no event log (a test artefact); the family-timed run logs the events
    # the parity leg compares (the same decisions: events are only recorded, never read back)
    vo, el, host_s, wait_s, _, ws = run(log=False)
    vo_ev, _, _, _, fam, _ = run(timed_families=True, log=cpu or parity_prefix > 0)
    m = n - warm
    last = vo.results[-1]
    out = {"workload": f"config {c}: {cfg.width}x{cfg.height} stereo, {cfg.n_feats} features, {cfg.window}-keyframe "
                       f"sliding window, {n} keyframes (KLT + epipolar MI matching + tracks + scale LM + "
                       f"{cfg.ba_iters}-iteration BA per keyframe), pipelined on two contexts",
           "host_loop": "native (me_vo_loop_*, C++)" if native else "python (WindowedStereoVO)",
           "frames_per_s": round(m / el, 2), "ms_per_frame": round(1e3 * el / m, 3), "frames_timed": m,
           "host_ms_per_frame": round(1e3 * host_s / m, 3), "wait_ms_per_frame": round(1e3 * wait_s / m, 3),
           "wait_ms_per_frame_by_call": ws,
           "device_us_per_frame": fam,
           "window_landmarks_last": last.n_window_pts, "window_observations_last": last.n_window_obs,
           "tracked_last": last.n_tracked, "tracks_created": int(vo.latest_id),
           "drift_m_last": round(float(np.abs(PL.camera_centre(vo.poses[n - 1]) -
                                              PL.camera_centre(truth[n - 1])).max()), 4),
           "render_s": round(gen, 1)}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from pipeline_oracle import OracleBackend  # CPU baseline / parity leg only

        ov = PL.WindowedStereoVO(cfg, OracleBackend(), K, p0, v, log_events=True)
        t1 = time.perf_counter()
        for t in range(n):
            ov.process(t, fr[t].left, fr[t].right)
        ov.finish()
        ct = time.perf_counter() - t1
        pose_rel = max(float(np.max(np.abs(vo_ev.poses[t] - ov.poses[t]) / (np.abs(ov.poses[t]) + 1e-3)))
                       for t in range(n))
        out["cpu_baseline"] = {"frames_per_s": round(n / ct, 3), "cores": 1, "kind": "port",
                               "sample": f"the same {n} keyframes on the oracle backend, sequential, 1 thread; "
                                         f"{ct:.1f} s"}
        out["parity"] = {"events_bit_exact": vo_ev.events == ov.events,
                         "track_ids_equal": bool(np.array_equal(vo_ev.ids, ov.ids)),
                         "timed_run_same_poses": all(np.array_equal(vo.poses[t], vo_ev.poses[t]) for t in range(n)),
                         "pose_max_rel_diff": float("%.3g" % pose_rel)}
    elif parity_prefix > 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from pipeline_oracle import OracleBackend  # parity leg only
        P = min(parity_prefix, n)
        ov = PL.WindowedStereoVO(cfg, OracleBackend(), K, p0, v, log_events=True)
        for t in range(P):
            ov.process(t, fr[t].left, fr[t].right)
        ov.finish()
        fg = vo_ev.frame_events
        fg = fg[fg["t"] < P]
        fo = _frame_event_records(ov)
        ev_ok = len(fg) == len(fo) and all(np.array_equal(fg[k], fo[k]) for k in ("kind", "t", "id")) and \
            np.array_equal(fg["feat"].view(np.uint32), fo["feat"].view(np.uint32))
        rg, ro = vo_ev.results[:P], ov.results[:P]
        same = all((a.n_tracked, a.n_new, a.n_window_pts, a.n_window_obs, a.ba_iters, a.scale_stop, a.scale_iters)
                   == (b.n_tracked, b.n_new, b.n_window_pts, b.n_window_obs, b.ba_iters, b.scale_stop, b.scale_iters)
                   for a, b in zip(rg, ro)) and len(rg) == len(ro) == P
        pose_rel = max(float(np.max(np.abs(a.pose - b.pose) / (np.abs(b.pose) + 1e-3))) for a, b in zip(rg, ro))
        out["parity"] = {"keyframes_checked": P, "events_bit_exact": bool(ev_ok), "results_equal": bool(same),
                         "pose_max_rel_diff": float("%.3g" % pose_rel),
                         "ok": bool(ev_ok and same and pose_rel <= 1e-6)}
    return out


def multi_stream(args, cfg, seed, local_rank, kp, ba_opts, barrier, S_):
    """S independent stereo streams on this GPU, each sequential (its own
    context = HIP stream + scratch, its own host thread; ctypes releases the
    GIL inside the library): whole-GPU throughput of small latency-bound
    frames.  Returns frames/s over all streams and the per-stream rate.
    Several persistent scale-LM grids and camera solves run at once here: the
    cross-workgroup launches rely on no co-residency (csrc/roster.hpp)."""
    import threading

    from uasl_motion_estimation_amd._lib import Context

    ctxs = [Context(local_rank) for _ in range(S_)]
    fr = []
    for k, c in enumerate(ctxs):
        f = make_frames(cfg, seed + 7919 * (k + 1), args.frames)
        upload_images(c, f)
        fr.append(f)
    stats = [new_stats() for _ in range(S_)]
    for k in range(S_):
        for i in range(args.warmup):
            gpu_step(ctxs[k], fr[k][i % len(fr[k])], kp, ba_opts, stats[k])
        ctxs[k].synchronize()
    stats = [new_stats() for _ in range(S_)]
    errs = []

    def run(k):
        try:
            for i in range(args.steps):
                gpu_step(ctxs[k], fr[k][i % len(fr[k])], kp, ba_opts, stats[k])
            ctxs[k].synchronize()
        except Exception as e:  # pragma: no cover
            errs.append(e)

    barrier()
    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(k,)) for k in range(S_)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    if errs:
        raise errs[0]
    nfr = sum(st["frames"] for st in stats)
    return {"streams": S_, "frames": nfr, "value": round(nfr / el, 2), "unit": "frames/s",
            "per_stream": round(nfr / el / S_, 2), "ba_iter_per_s": round(sum(st["ba_iters"] for st in stats) / el, 1),
            "frame": "sequential per stream (KLT, scale LM, BA on one context: no front-end / BA overlap)"}


def main():
    global SCALE_ITERS
    args = parse()
    SCALE_ITERS = args.scale_iters
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rank_device == "zero":  # (tests: every rank on GPU 0; RCCL cannot run two ranks on one GPU)
        assert args.comm == "gloo" or world == 1, "--rank-device zero needs --comm gloo"
        local_rank = 0
    pool = pool1 = None
    model, ncpu, avail = host_cpu()
    cpu_workers = args.cpu_workers or min(16, avail)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # CPU legs: worker processes started before anything touches the GPU,
        # each pinned to its own core (1-thread leg: the first allowed core;
        # all-cores leg: the next cpu_workers cores)
        import multiprocessing as mp

        mpc = mp.get_context("spawn")
        cores = sorted(os.sched_getaffinity(0))
        q1 = mpc.Queue()
        q1.put(cores[0])
        pool1 = mpc.Pool(1, initializer=_pin_init, initargs=(q1,))
        if cpu_workers > 1:
            qa = mpc.Queue()
            for k in range(cpu_workers):
                qa.put(cores[k % len(cores)])
            pool = mpc.Pool(cpu_workers, initializer=_pin_init, initargs=(qa,))
    import torch

    dist = None
    if world > 1 or args.dist:
        from datetime import timedelta

        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        if "MASTER_ADDR" not in os.environ:  # --dist at one rank without a launcher
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29511", RANK="0", WORLD_SIZE="1")
        dist.init_process_group(args.comm, timeout=timedelta(seconds=180))
    from uasl_motion_estimation_amd import synthetic as S
    from uasl_motion_estimation_amd._lib import Context, KT
    from uasl_motion_estimation_amd.klt import klt_params
    from uasl_motion_estimation_amd.optimisation import SolverOptions

    if args.lib:
        from uasl_motion_estimation_amd import _lib

        _lib.load_library(args.lib)
    cfg = S.CONFIGS[args.config]
    seed = S.SEED0 + args.config + 1000 * rank
    t0 = time.time()
    frames = make_frames(cfg, seed, args.frames)
    gen_s = time.time() - t0
    ctx = Context(local_rank)
    upload_images(ctx, frames)
    kp = klt_params()
    ba_opts = SolverOptions.fixed_iterations(args.ba_iters)

    def barrier():
        if dist is not None:
            dist.barrier()

    fam_names = ("MI", "SCALE_RES", "SCALE_NEQ", "BA_LINEARIZE", "BA_POINTS", "BA_SCHUR", "BA_SOLVE", "BA_STEP",
                 "KLT", "PYR")
    stats = new_stats()
    for i in range(args.warmup):
        gpu_step(ctx, frames[i % len(frames)], kp, ba_opts, stats)
    ctx.synchronize()
    pipe = tctx = None
    ncu = torch.cuda.get_device_properties(local_rank).multi_processor_count

    def cu_split(on):
        """Frontend overlap: disjoint CU sets for the two streams (only around the pipelined
        runs; the side measurements use the whole device).  The latency-bound BA kernels and
        the persistent scale LM otherwise share every CU's issue slots and slow each other."""
        if pipe is None or args.overlap != "frontend" or not 0 < args.front_cus < 16:
            return
        from uasl_motion_estimation_amd._lib import cu_split
        front, back = cu_split(ncu, args.front_cus)  # whole XCDs per side (ME_CU_SPLIT=interleaved: shared)
        tctx.set_cu_mask(front if on else None)
        ctx.set_cu_mask(back if on else None)
    if not args.no_pipeline:
        tctx = Context(local_rank)  # tracker context: its own HIP stream and scratch
        pipe = FramePipeline(ctx, tctx, _Hip(), args.overlap)
        cu_split(True)
        pipe.run(frames, max(args.warmup, 2), kp, ba_opts, new_stats())
        tctx.synchronize()
        ctx.synchronize()
        cu_split(False)
    # untimed profile steps with every family timed: per-family device time and
    # the dominant family (by device time) among those with a roofline
    ctx.timing_reset()
    ctx.timing(True)
    pstats = new_stats()
    for i in range(args.profile_steps):
        gpu_step(ctx, frames[i % len(frames)], kp, ba_opts, pstats)
    ctx.synchronize()
    ctx.timing(False)
    prof = {f: ctx.timing_read(f) for f in fam_names}
    rl = {f: alg_work(f, cfg, frames) for f in fam_names if prof[f][0] > 0}
    npf = max(1, pstats["frames"])
    # per-frame device-time budget of every family (the latency-bound ones included)
    budget = {f: {"launches_per_frame": round(prof[f][0] / npf, 2), "us_per_launch": round(1e3 * prof[f][1] / prof[f][0], 2),
                  "us_per_frame": round(1e3 * prof[f][1] / npf, 1)} for f in fam_names if prof[f][0] > 0}
    # the MI that runs in the frame (scale LM residual launches, speculative candidates included):
    # 262 algorithmic bytes per executed track evaluation
    mi_in_frame = None
    if prof["SCALE_RES"][0] > 0:
        b = 262.0 * cfg["n_feats"] * pstats["scale_executed"]
        a_gbs = b / (prof["SCALE_RES"][1] * 1e-3) / 1e9
        mi_in_frame = {"bound": "hbm", "achieved": round(a_gbs, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                       "frac": round(a_gbs / PEAK_HBM_GBS, 5), "kernel": "scale_res_ctrl_kernel",
                       "track_evaluations_per_frame": round(cfg["n_feats"] * pstats["scale_executed"] / npf, 1),
                       "us_per_frame": budget["SCALE_RES"]["us_per_frame"],
                       # the whole persistent LM launch (control phases and waits included) per track evaluation
                       "ns_per_track_evaluation": round(1e6 * prof["SCALE_RES"][1] /
                                                        (cfg["n_feats"] * pstats["scale_executed"]), 2)}
    # the persistent scale LM (one launch per frame) is the whole LM control loop with its
    # phase waits, not one kernel's pass over its data: reported as mi_in_frame, not as the roofline kernel
    persistent_scale = "SCALE_RES" in budget and budget["SCALE_RES"]["launches_per_frame"] <= 1.5
    dom = max((f for f in rl if rl[f] is not None and not (f == "SCALE_RES" and persistent_scale)),
              key=lambda f: prof[f][1])
    # timed region: HIP events on the ctx stream around the dominant family only
    ctx.timing_reset()
    if args.timing != "none":
        ctx.timing(True, None if args.timing == "all" else [dom])
        # every k-th launch of the family: a live average over the timed region whose event
        # records perturb the stream k times less (--timing-every 1: every launch)
        ctx.timing_sample(args.timing_every)
    stats = new_stats()
    cu_split(True)
    barrier()
    torch.cuda.synchronize()
    ctx.synchronize()
    t_start = time.perf_counter()
    if pipe is None:
        for i in range(args.steps):
            gpu_step(ctx, frames[i % len(frames)], kp, ba_opts, stats)
    else:
        pipe.run(frames, args.steps, kp, ba_opts, stats)
        tctx.synchronize()
    ctx.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    cu_split(False)
    barrier()
    ctx.timing(False)
    ctx.timing_sample(1)
    fams = {f: ctx.timing_read(f) for f in fam_names}
    t_max = elapsed
    frames_total = stats["frames"]
    ba_total = stats["ba_iters"]
    if dist is not None:
        tdev = "cpu" if args.comm == "gloo" else f"cuda:{local_rank}"
        tt = torch.tensor([elapsed], device=tdev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
        cnt = torch.tensor([stats["frames"], stats["ba_iters"]], device=tdev, dtype=torch.float64)
        dist.all_reduce(cnt)
        frames_total, ba_total = int(cnt[0].item()), int(cnt[1].item())
    value = frames_total / t_max
    bound, amount, unit, peak = rl[dom]
    n_l, ms_l = fams[dom] if fams[dom][0] > 0 else prof[dom]
    if dom == "SCALE_RES":  # executed evaluations per launch (speculative candidate batches)
        amount = 262.0 * cfg["n_feats"] * (stats if fams[dom][0] > 0 else pstats)["scale_executed"] / n_l
    avg_ms = ms_l / n_l
    scale_u = 1e9 if unit == "GB/s" else 1e12
    achieved = amount / (avg_ms * 1e-3) / scale_u
    roofline = {"bound": bound, "achieved": round(achieved, 3), "peak": peak, "unit": unit,
                "frac": round(achieved / peak, 5), "traffic": pmc_traffic(dom),
                "traffic_calibration": TRAFFIC_CALIBRATION, "kernel": dom,
                "kernels": FAMILY_KERNELS.get(dom), "avg_launch_ms": round(avg_ms, 5), "work_per_launch": amount,
                "timed_live": fams[dom][0] > 0, "timed_launches": n_l, "sampled_every": args.timing_every}
    rp_ms, rp_file = rocprof_avg_ms(dom)
    if rp_ms:  # the same kernel in the committed rocprofv3 summary of the headline frame
        a_rp = amount / (rp_ms * 1e-3) / scale_u
        roofline.update({"rocprof_avg_launch_ms": round(rp_ms, 5), "rocprof_summary": f"profiles/{rp_file}",
                         "achieved_rocprof": round(a_rp, 3), "frac_rocprof": round(a_rp / peak, 5)})
    if "BA_SOLVE" in budget:  # the frame's largest kernel has no HBM/MFMA roofline: a latency budget
        b = budget["BA_SOLVE"]
        roofline["solve"] = {"kernel": "cam_solve_kernel", "bound": "latency (dependent blocked-Cholesky chain)",
                             "us_per_lm_iteration": b["us_per_launch"], "launches_per_frame": b["launches_per_frame"],
                             "us_per_frame": b["us_per_frame"],
                             "share_of_step": round(b["us_per_frame"] * 1e-3 / (t_max * 1e3 / max(frames_total, 1)
                                                                                  * max(world, 1)), 4)}
    copy_gbs = hbm_copy_gbs(ctx)
    if unit == "GB/s":
        roofline["peak_measured_copy"] = copy_gbs
        roofline["frac_vs_measured_copy"] = round(achieved / copy_gbs, 5)
    mi_rl = mi_batch_roofline(ctx, frames, args.mi_pairs) if args.mi_pairs > 0 else None
    for r_ in (mi_rl, mi_in_frame):
        if r_ is not None:
            r_["peak_measured_copy"] = copy_gbs
            r_["frac_vs_measured_copy"] = round(r_["achieved"] / copy_gbs, 5)
    multi = [multi_stream(args, cfg, seed, local_rank, kp, ba_opts, barrier, S_)
             for S_ in sorted({int(x) for x in str(args.streams).split(",") if x.strip()}) if S_ > 1] or None
    pipe_line = pipe_c5 = None
    if args.pipeline_frames > 0 and rank == 0:
        cpu_leg = world == 1 and not args.no_cpu_baseline
        pipe_line = pipeline_line(args, ctx, cpu_leg, args.config, args.pipeline_frames)
        if args.pipeline_c5_frames > 0:
            pipe_c5 = pipeline_line(args, ctx, False, 5, args.pipeline_c5_frames, parity_prefix=16)
    sharded = None
    if args.sharded_ba:
        try:
            sharded = sharded_ba_line(args, ctx, dist, world, rank, local_rank, barrier)
        except Exception as e:  # reported, never fatal to the headline line
            sharded = {"error": f"{type(e).__name__}: {e}"}
    vo_line = stereo_vo_line(ctx, args.vo_matches, cpu=rank == 0 and world == 1 and not args.no_cpu_baseline) \
        if args.vo_matches > 0 else None
    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # parity of the timed frames: the last timed replay of each distinct
        # frame (read back after the timed region) against the oracle
        outs = [cpu_frame(cpu_payload(fd), args.ba_iters, args.scale_iters) for fd in frames]
        cmp = [compare(gpu_outputs(ctx, fd, pipe.scale_ctx if pipe else None), o) for fd, o in zip(frames, outs)]
        parity = {"frames_checked": len(cmp), "klt_bit_exact": all(c["klt_bit_exact"] for c in cmp),
                  "scale_match": all(c["scale_match"] for c in cmp), "ba_match": all(c["ba_match"] for c in cmp),
                  "ba_max_rel_diff": float("%.3g" % max(c["ba_max_rel"] for c in cmp))}
        parity["ok"] = parity["klt_bit_exact"] and parity["scale_match"] and parity["ba_match"]
        # 1 thread, pinned to one core: median of cpu_runs runs over the distinct frames (one warm-up frame first)
        pls = [cpu_payload(fd) for fd in frames]
        rates, tot_t, ba_it, pinned = pool1.apply(_cpu_single, ((pls, args.ba_iters, args.scale_iters,
                                                                args.cpu_runs),))
        cpu = {"value": round(float(np.median(rates)), 4), "unit": "frames/s", "cores": 1, "kind": "port",
               "sample": f"median of {len(rates)} runs x {len(pls)} config-{args.config} frames (KLT + MI scale LM "
                         f"(<= {args.scale_iters} it.) + {args.ba_iters}-iteration BA) on the oracle restatement, "
                         f"1 thread pinned to core {pinned if len(pinned) > 1 else pinned[0]}, after 1 warm-up "
                         f"frame; {tot_t:.1f} s",
               "pinned_cores": pinned,
               "runs_frames_per_s": [round(r, 4) for r in rates],
               "ba_iter_per_s": round(ba_it / tot_t, 3), "cpu_model": model, "nproc": ncpu,
               "cores_available": avail}
        if pool is not None:
            per = [(pls * 2, args.ba_iters, args.scale_iters)] * cpu_workers
            t1 = time.perf_counter()
            res = pool.map(_cpu_worker, per)
            wall = time.perf_counter() - t1
            nf_all = sum(r[0] for r in res)
            cpu["all_cores"] = {"value": round(nf_all / wall, 3), "unit": "frames/s", "cores": cpu_workers,
                                "sample": f"{cpu_workers} processes x {2 * len(pls)} frames (independent frames, "
                                          f"one process pinned per core: an upper bound for a multi-threaded "
                                          f"CPU path); "
                                          f"{wall:.1f} s"}
            if avail > cpu_workers:
                # the GPU box grants one GPU's job 16 cores; the frames are independent, so the
                # host's other cores would add linearly at best: a stated upper bound, not a run
                cpu["all_cores"]["linear_extrapolation_to_cores_available"] = {
                    "value": round(nf_all / wall * avail / cpu_workers, 3), "cores": avail}
    for pl_ in (pool, pool1):
        if pl_ is not None:
            pl_.close()
            pl_.join()
    if rank == 0:
        out = {
            "metric": "frames/sec + BA iter/sec, 2000 feats x 20-keyframe window, 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * t_max / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8+f32 (MI), f64 (BA)",
            "data": "synthetic",
            "config": {"workload": f"config {args.config}: {cfg['width']}x{cfg['height']} stereo, "
                                   f"{cfg['n_feats']} feats, {cfg['window']}-keyframe window, 11x11 MI patches",
                       "frame": f"KLT + MI scale LM (LM, MAX_NB_ITER {args.scale_iters}, tolerances off) + "
                                f"{args.ba_iters} BA LM iterations",
                       "frame_kind": "composite: the three stages on independent synthetic inputs of the config's "
                                     "shape (the connected VO loop is the `pipeline` line)",
                       "parallelism": f"{world} independent streams (one per GPU)",
                       "pipeline": None if pipe is None else (
                           ("front end (KLT + scale LM) of frame t+1 overlaps the BA of frame t" + (
                               f" on disjoint CUs ({args.front_cus} of every 16 for the front end)"
                               if 0 < args.front_cus < 16 else "")) if args.overlap == "frontend" else "KLT of frame t+1 overlaps the BA of frame t") +
                           " (two HIP streams, event dependency per frame)"},
            "ba_iter_per_s": round(ba_total / t_max, 2),
            "scale_lm_per_frame": {k: round(stats[k2] / max(1, stats["frames"]), 3) for k, k2 in
                                   (("iterations", "scale_iters"), ("residual_evaluations", "scale_res_evals"),
                                    ("rejections", "scale_rejections"), ("executed_evaluations", "scale_executed"))},
            "parity": parity,
            "roofline": roofline,
            "mi_roofline": mi_rl,
            "multi_stream": multi,
            "sharded_ba": sharded,
            "pipeline": pipe_line,
            "pipeline_config5": pipe_c5,
            "stereo_vo": vo_line,
            "cpu_baseline": cpu,
            "hbm_copy_GBs_measured": copy_gbs,
            "kernel_ms_profile": {f: [prof[f][0], round(prof[f][1], 3)] for f in prof},
            "kernel_budget_per_frame": budget,
            "mi_in_frame": mi_in_frame,
            "gen_s": round(gen_s, 1),
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
