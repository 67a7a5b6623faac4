"""End-to-end windowed stereo VO (uasl_motion_estimation_amd/pipeline.py).

CPU: the loop on the oracle backend, its WBA_Point bookkeeping replayed
through feature_types.WBA_Point (include/MotionEstimation/core/
feature_types.h:121-197: IDs from the value constructor, contiguous
addMatch, pop of the oldest feature).
GPU: the same loop on libme_hip.so (pipelined: KLT, the device epipolar
matcher and the scale LM on a front-end context beside the BA) vs the
oracle backend, sequential: track IDs and feature positions bit-exact,
poses 1e-6, over 56 keyframes of a sliding W = 50 window.
"""
import numpy as np
import pytest

from uasl_motion_estimation_amd import pipeline as PL
from uasl_motion_estimation_amd.feature_types import WBA_Point


def _run(cfg_id, n_frames, backend, window=None, ba_iters=5, log=True, frames=None, overlap=False):
    if frames is None:
        frames = PL.synthetic_sequence(cfg_id, n_frames)
    fr, K, p0, v, truth = frames
    kw = dict(ba_iters=ba_iters)
    cfg = PL.PipelineConfig.from_config(cfg_id, **kw)
    if window is not None:
        cfg.window = window
    vo = PL.WindowedStereoVO(cfg, backend, K, p0, v, log_events=log, overlap=overlap)
    for t in range(n_frames):
        vo.process(t, fr[t].left, fr[t].right)
    vo.finish()
    return vo


def test_pipelined_loop_equals_sequential_loop(oracle):
    """overlap=True (KLT of t queued before frame t-1 completes, BA and scale
    LM queued) takes exactly the decisions of the sequential loop."""
    from pipeline_oracle import OracleBackend

    frames = PL.synthetic_sequence(1, 10)
    a = _run(1, 10, OracleBackend(), window=4, ba_iters=2, frames=frames)
    b = _run(1, 10, OracleBackend(), window=4, ba_iters=2, frames=frames, overlap=True)
    assert a.events == b.events and np.array_equal(a.ids, b.ids) and np.array_equal(a.X, b.X)
    assert all(np.array_equal(a.poses[t], b.poses[t]) for t in a.poses)
    assert [r.n_window_obs for r in a.results] == [r.n_window_obs for r in b.results]


def _replay(vo):
    """WBA_Point calls of the event log; returns {id: WBA_Point} of the live tracks."""
    WBA_Point.reset_ids("stereo")
    live = {}
    for ev in vo.events:
        kind, tid = ev[0], ev[1]
        if kind == "new":
            _, _, t, f = ev
            p = WBA_Point(((f[0], f[1]), (f[2], f[3])), t)
            assert p.getID() == tid  # latestID++ in creation order
            live[tid] = p
        elif kind == "add":
            _, _, t, f = ev
            live[tid].addMatch(((f[0], f[1]), (f[2], f[3])), t)  # asserts contiguous frames (:140)
        elif kind == "pop":
            live[tid].pop()
        else:  # del: every feature popped
            assert not live[tid].isValid()
            del live[tid]
    return live


def test_pipeline_bookkeeping_matches_wba_point(oracle):
    from pipeline_oracle import OracleBackend

    vo = _run(1, 9, OracleBackend(), window=4, ba_iters=2)
    live = _replay(vo)
    # the pipeline's track table and observation store hold exactly the live WBA_Points
    assert sorted(live) == sorted(int(i) for i in vo.ids)
    per_track = {int(i): [] for i in vo.ids}
    for t in sorted(vo.obs):
        fid, fe = vo.obs[t]
        for i, f in zip(fid, fe):
            per_track[int(i)].append((t, tuple(float(x) for x in f)))
    for tid, p in live.items():
        got = per_track[tid]
        assert [g[0] for g in got] == p.indices
        assert [g[1] for g in got] == [(a[0], a[1], b[0], b[1]) for a, b in p.features]
    r = vo.results[-1]
    assert r.n_tracked > 0.5 * vo.cfg.n_feats and r.ba_iters == 2
    # the window slid: no feature older than window - 1 keyframes remains
    assert min(vo.obs) == 9 - 4


def test_pipeline_tracks_the_synthetic_trajectory(oracle):
    from pipeline_oracle import OracleBackend

    frames = PL.synthetic_sequence(1, 8)
    vo = _run(1, 8, OracleBackend(), window=5, ba_iters=5, log=False, frames=frames)
    truth = frames[4]
    err = max(np.abs(PL.camera_centre(vo.poses[t]) - PL.camera_centre(truth[t])).max() for t in range(8))
    assert err < 0.1  # metres over 8 keyframes of 0.5 m: VO drift, not a convention error


N_SLIDE = 56  # config 5: the W = 50 window fills at keyframe 49 and slides 6 times


@pytest.fixture(scope="module")
def seq5():
    return PL.synthetic_sequence(5, N_SLIDE)


_ORACLE_RUNS = {}


def _oracle_run(seq5, window, n):
    """The sequential oracle loop on config 5's keyframes (cached per module: the Python GPU loop and
    the native loop are both checked against it)."""
    from pipeline_oracle import OracleBackend

    key = (window, n)
    if key not in _ORACLE_RUNS:
        _ORACLE_RUNS[key] = _run(5, n, OracleBackend(), window=window, frames=seq5, ba_iters=10)
    return _ORACLE_RUNS[key]


def _check_against_oracle(g, o, window, n):
    if window == 50:  # the window slid: its oldest keyframe is n - 50, and pops happened
        assert min(g.obs) == n - window and any(ev[0] == "pop" for ev in g.events)
    assert g.events == o.events  # track IDs, frames and feature positions, bit for bit
    assert np.array_equal(g.ids, o.ids)
    gr, orr = g.results, o.results
    assert len(gr) == len(orr) == n
    for rg, ro in zip(gr, orr):
        assert (rg.n_tracked, rg.n_new, rg.n_window_pts, rg.n_window_obs, rg.ba_iters) == \
            (ro.n_tracked, ro.n_new, ro.n_window_pts, ro.n_window_obs, ro.ba_iters), (rg, ro)
        assert (rg.scale_stop, rg.scale_iters) == (ro.scale_stop, ro.scale_iters), (rg, ro)
        np.testing.assert_allclose(rg.scale, ro.scale, rtol=1e-6)
    gp, op = g.poses, o.poses
    for t in gp:
        np.testing.assert_allclose(gp[t], op[t], rtol=1e-6, atol=1e-9)
    # every landmark within 1e-6 (measured: 1.5e-10 at most; the round-4 bar let
    # 0.1 % of them exceed it), and every landmark reprojects into the last
    # keyframe (left and right image, each loop's own pose) within 1e-6 pixel
    # (measured: 6.7e-9)
    rel = np.abs(g.X - o.X) / (np.abs(o.X) + 1e-9)
    dpx = _reproj_diff(g, o, max(gp))
    print("landmarks: max rel %.3g; max reprojection difference %.3g px" % (rel.max(), dpx.max()))
    assert rel.max() < 1e-6, (rel.max(), int((rel > 1e-6).sum()))
    assert dpx.max() < 1e-6, (dpx.max(), int((dpx >= 1e-6).sum()))


def _reproj_diff(g, o, t):
    from uasl_motion_estimation_amd import synthetic as S

    K, b = np.asarray(o.K), float(o.cfg.baseline)
    out = []
    for vo in (g, o):
        pose = np.asarray(vo.poses[t], np.float64)
        P = np.asarray(vo.X, np.float64) @ S.aa_to_R(pose[3:]).T + pose[:3]
        out.append(P)
    front = (out[0][:, 2] > 1.0) & (out[1][:, 2] > 1.0)
    px = []
    for P in out:
        P = P[front]
        px.append(np.stack([K[0, 0] * P[:, 0] / P[:, 2] + K[0, 2], K[1, 1] * P[:, 1] / P[:, 2] + K[1, 2],
                            K[0, 0] * (P[:, 0] - b) / P[:, 2] + K[0, 2]], 1))
    return np.abs(px[0] - px[1]).max(1) if len(px[0]) else np.zeros(1)


@pytest.mark.gpu
@pytest.mark.parametrize("window,n", [(50, N_SLIDE), (8, 24)])
def test_pipeline_gpu_matches_oracle(ctx, oracle, seq5, window, n):
    """Config 5 (1280 x 720, 2000 features, W = 50 sliding window) over 56
    keyframes -- the window fills and slides (pops of the oldest keyframe,
    feature_types.h:142) -- and a W = 8 window over 24 keyframes (many pops
    and track deletions)."""
    be = PL.GPUBackend(ctx)  # front end on its own context, the loop pipelined
    try:
        g = _run(5, n, be, window=window, frames=seq5, overlap=True, ba_iters=10)
    finally:
        be.close()
    _check_against_oracle(g, _oracle_run(seq5, window, n), window, n)


def _native(ctx, n, window, frames, log=True, **kw):
    fr, K, p0, v, truth = frames
    cfg = PL.PipelineConfig.from_config(5, ba_iters=10)
    cfg.window = window
    vo = PL.NativeStereoVO(cfg, ctx, K, p0, v, log_events=log, **kw)
    for t in range(n):
        vo.process(t, fr[t].left, fr[t].right)
    vo.finish()
    return vo


@pytest.mark.gpu
@pytest.mark.parametrize("window,n", [(50, N_SLIDE), (8, 24)])
def test_native_loop_matches_oracle(ctx, oracle, seq5, window, n):
    """The loop in native code (me_vo_loop_*, csrc/vo_loop.hip) against the
    sequential oracle loop: WBA_Point events bit for bit, results, poses and
    landmarks to 1e-6 -- the same bar as the Python GPU loop."""
    g = _native(ctx, n, window, seq5)
    try:
        _check_against_oracle(g, _oracle_run(seq5, window, n), window, n)
    finally:
        g.close()


class _DevFrame:
    def __init__(self, left, right):
        self.left, self.right = left, right


@pytest.mark.gpu
def test_native_loop_shared_context_and_device_images(ctx, seq5):
    """overlap=False (one context: the scale LM and the window queueing inline)
    and device-resident images (ME_DEVICE) take the overlapped host-image run's
    decisions and values bit for bit."""
    import torch

    a = _native(ctx, 16, 8, seq5)
    b = _native(ctx, 16, 8, seq5, overlap=False)
    fr = seq5[0]
    # (no torch.cuda.synchronize(): process() orders the loop's streams after
    # the producing torch stream itself)
    dev = [_DevFrame(torch.from_numpy(fr[t].left).cuda(), torch.from_numpy(fr[t].right).cuda()) for t in range(16)]
    c = _native(ctx, 16, 8, (dev,) + tuple(seq5[1:]))
    try:
        ea = a.event_records()
        for o in (b, c):
            assert np.array_equal(ea, o.event_records())
            assert np.array_equal(a.ids, o.ids) and np.array_equal(a.X, o.X)
            pa, po = a.poses, o.poses
            assert all(np.array_equal(pa[t], po[t]) for t in pa)
            ra = np.array([(r.scale, r.ba_cost) for r in a.results])
            assert np.array_equal(ra, np.array([(r.scale, r.ba_cost) for r in o.results]), equal_nan=True)
    finally:
        for o in (a, b, c):
            o.close()


@pytest.mark.gpu
def test_native_loop_rejects_images_that_do_not_match_the_config(ctx, seq5):
    """the native loop copies width x height bytes from the
    caller's pointer, so NativeStereoVO.process checks dtype, shape,
    contiguity and device first and raises; the loop is untouched by a
    rejected call and the next correct keyframe goes through."""
    import torch

    fr, K, p0, v, truth = seq5
    cfg = PL.PipelineConfig.from_config(5, ba_iters=10)
    cfg.window = 8
    vo = PL.NativeStereoVO(cfg, ctx, K, p0, v)
    try:
        L, R = fr[0].left, fr[0].right
        bad = [(L[:-1], R), (L, R[:, :-1]), (L.astype(np.float32), R), (L, R.T)]
        for a, b in bad:
            with pytest.raises(ValueError):
                vo.process(0, a, b)
        dL, dR = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
        strided = torch.zeros((L.shape[0], 2 * L.shape[1]), dtype=torch.uint8, device=dL.device)[:, ::2]
        for a, b in [(dL[:-1], dR), (dL.float(), dR), (dL.t(), dR), (dL, dR.cpu()), (strided, dR)]:
            with pytest.raises(ValueError):
                vo.process(0, a, b)
        vo.process(0, L, R)
        vo.process(1, dL, dR)
    finally:
        vo.close()


def _write_cli_input(path, frames, n, window):
    fr, K, p0, v, truth = frames
    cfg = PL.PipelineConfig.from_config(5, ba_iters=10)
    iv = np.array([cfg.width, cfg.height, cfg.n_feats, window, cfg.ba_iters, cfg.scale_iters, cfg.fixed_frames,
                   cfg.d_min, cfg.d_max, n, 1], np.int32)
    dv = np.concatenate([[cfg.baseline, cfg.feat_var], np.asarray(K, np.float64).ravel(), p0, v]).astype(np.float64)
    with open(path, "wb") as fh:
        fh.write(iv.tobytes())
        fh.write(dv.tobytes())
        for t in range(n):
            fh.write(np.ascontiguousarray(fr[t].left, np.uint8).tobytes())
            fh.write(np.ascontiguousarray(fr[t].right, np.uint8).tobytes())


@pytest.mark.gpu
def test_cpp_host_drives_the_loop(ctx, seq5, tmp_path):
    """A compiled C++ caller (tests/cpp/vo_loop_cli.cpp over me::WindowedStereoVO
    in include/MotionEstimationAMD/motion_estimation_amd.hpp, no Python in the
    process) runs the loop: its results, WBA_Point events, poses and track
    table equal the Python-driven native loop's bit for bit."""
    import os
    import subprocess

    from uasl_motion_estimation_amd._lib import VO_EVENT_DTYPE

    n, window = 16, 8
    cli = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "vo_loop_cli")
    assert os.path.exists(cli), "tests/cpp/vo_loop_cli not built (__graft_entry__.build())"
    _write_cli_input(tmp_path / "in.bin", seq5, n, window)
    r = subprocess.run([cli, str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0, r.stderr
    buf = (tmp_path / "out.bin").read_bytes()
    pos = 0

    def take(dtype, count):
        nonlocal pos
        a = np.frombuffer(buf, dtype, count, pos)
        pos += a.nbytes
        return a

    nres = int(take(np.int64, 1)[0])
    rdt = np.dtype([("t", "i4"), ("n_tracked", "i4"), ("n_new", "i4"), ("n_active", "i4"), ("nwp", "i4"),
                    ("nwo", "i4"), ("scale", "f8"), ("stop", "i4"), ("sit", "i4"), ("bit", "i4"), ("cost", "f8"),
                    ("pose", "f8", 6)], align=True)
    res = take(rdt, nres)
    ev = take(VO_EVENT_DTYPE, int(take(np.int64, 1)[0]))
    pdt = np.dtype([("t", "i4"), ("pad", "i4"), ("pose", "f8", 6)])
    ps = take(pdt, int(take(np.int64, 1)[0]))
    nt = int(take(np.int64, 1)[0])
    ids = take(np.int64, nt)
    X = take(np.float64, 3 * nt).reshape(nt, 3)
    assert pos == len(buf)
    py = _native(ctx, n, window, seq5)
    try:
        assert np.array_equal(ev, py.event_records())
        assert np.array_equal(ids, py.ids) and np.array_equal(X, py.X)
        pp = py.poses
        assert [int(t) for t in ps["t"]] == sorted(pp) and all(np.array_equal(p["pose"], pp[int(p["t"])]) for p in ps)
        pr = py.results
        assert nres == n == len(pr)
        assert [(int(a["t"]), int(a["n_tracked"]), int(a["n_new"])) for a in res] == [(b.t, b.n_tracked, b.n_new)
                                                                                        for b in pr]
        assert np.array_equal(np.array([(a["scale"], a["cost"]) for a in res]),
                              np.array([(b.scale, b.ba_cost) for b in pr]), equal_nan=True)  # (no-BA keyframes: NaN cost)
    finally:
        py.close()


@pytest.mark.gpu
def test_pipeline_gpu_chained_equals_unchained(ctx, seq5):
    """BA(t) queued behind BA(t - 1), its start formed on the device from
    BA(t - 1)'s result (me_vo_ba_chain: refined poses and landmarks, pose(t)
    predicted again, t's new landmarks moved), is the state the host forms in
    step 7: events, poses and landmarks bit for bit against the loop that
    waits for BA(t - 1) before queueing BA(t)."""
    runs = []
    for chain in (True, False):
        be = PL.GPUBackend(ctx)
        be.chain_window = chain
        try:
            runs.append(_run(5, 24, be, window=8, frames=seq5, overlap=True, ba_iters=10))
        finally:
            be.close()
    a, b = runs
    assert a.events == b.events and np.array_equal(a.ids, b.ids)
    assert np.array_equal(a.X, b.X)
    assert all(np.array_equal(a.poses[t], b.poses[t]) for t in a.poses)
    assert [r.ba_iters for r in a.results] == [r.ba_iters for r in b.results]
    assert np.array_equal([r.ba_cost for r in a.results], [r.ba_cost for r in b.results], equal_nan=True)


@pytest.mark.gpu
def test_pipeline_gpu_chained_equals_unchained_after_failed_ba(ctx, seq5):
    """the chained start after a FAILED BA(t - 1) -- the device
    chain (vo_chain_kernel) keeps the host's poses and landmarks when the
    previous solve ended with termination 2, the host loop skips the write
    back for status 3.  Every second window solve fails (test hook
    me_debug_solve_flags(2048): each of its camera solves fails, every LM
    step is invalid, the solve ends after max_num_consecutive_invalid_steps
    with the parameters untouched); events, poses and landmarks bit for bit
    between the chained and the unchained loop, and the native loop takes
    the same decisions."""
    import ctypes

    hook = ctx.lib.me_debug_solve_flags
    hook.argtypes = [ctypes.c_void_p, ctypes.c_int]
    runs = []
    for chain in (True, False):
        be = PL.GPUBackend(ctx)
        be.chain_window = chain
        assert hook(ctx.h, 2048) == 0
        try:
            runs.append(_run(5, 16, be, window=8, frames=seq5, overlap=True, ba_iters=10))
        finally:
            hook(ctx.h, 0)
            be.close()
    a, b = runs
    assert a.events == b.events and np.array_equal(a.ids, b.ids)
    assert np.array_equal(a.X, b.X)
    assert all(np.array_equal(a.poses[t], b.poses[t]) for t in a.poses)
    assert [r.ba_iters for r in a.results] == [r.ba_iters for r in b.results]
    assert np.array_equal([r.ba_cost for r in a.results], [r.ba_cost for r in b.results], equal_nan=True)
    # the hook did fail windows: a failed solve leaves the predicted poses, so the
    # run leaves the unhooked run's poses
    be = PL.GPUBackend(ctx)
    try:
        ref = _run(5, 16, be, window=8, frames=seq5, overlap=True, ba_iters=10)
    finally:
        be.close()
    assert not all(np.array_equal(a.poses[t], ref.poses[t]) for t in a.poses)
    assert hook(ctx.h, 2048) == 0
    try:
        n = _native(ctx, 16, 8, seq5)
    finally:
        hook(ctx.h, 0)
    try:
        assert n.events == a.events and np.array_equal(n.ids, a.ids)
        assert [r.ba_iters for r in n.results] == [r.ba_iters for r in a.results]
        for t in a.poses:
            np.testing.assert_allclose(n.poses[t], a.poses[t], rtol=1e-9, atol=1e-12)
    finally:
        n.close()


def test_rot_series_equals_rodrigues():
    """The loop's pose(t) re-prediction rotation (pipeline.rot_series: a
    Taylor series in theta^2, the device chain's arithmetic) against the
    closed-form Rodrigues rotation, up to pi."""
    rng = np.random.default_rng(3)
    for _ in range(500):
        a = rng.normal(0, 1.0, 3)
        a *= min(1.0, np.pi / np.linalg.norm(a))
        np.testing.assert_allclose(PL.rot_series(a), PL.aa_to_R(a), rtol=0, atol=1e-14)
    assert np.array_equal(PL.rot_series(np.zeros(3)), np.eye(3))


@pytest.mark.gpu
@pytest.mark.parametrize("unique", [False, True])
def test_gpu_epipolar_matcher_equals_host_restatement(ctx, oracle, unique):
    """me_mi_epipolar_match (device MI scores + FP64 pick) = match_host (MI
    scores + the numpy pick) bit for bit, on features across a config-3
    stereo pair: per-feature windows (tracked form, with invalid features)
    and the full [d_min, d_max] range with the uniqueness test (new form)."""
    from pipeline_oracle import OracleBackend

    fr = PL.synthetic_sequence(3, 2)[0]
    be = PL.GPUBackend(ctx)
    try:
        imgs = be.frame_images(0, fr[0].left, fr[0].right)
        rng = np.random.default_rng(7)
        n = 600
        uv = np.stack([rng.uniform(PL.MARGIN, 1280 - PL.MARGIN, n), rng.uniform(PL.MARGIN, 720 - PL.MARGIN, n)],
                      -1).astype(np.float32)
        # features whose patch leaves the image: scored -inf on both sides, never read
        e = 48
        # (patch corner floor(u - 5): x0 < 0 for u < 5, x0 + 11 > 1280 for u >= 1275)
        uv[:e // 4, 0] = rng.uniform(0, 4.9, e // 4)
        uv[e // 4:e // 2, 0] = rng.uniform(1275, 1280, e // 4)
        uv[e // 2:3 * e // 4, 1] = rng.uniform(0, 4.9, e // 4)
        uv[3 * e // 4:e, 1] = rng.uniform(715, 720, e // 4)
        if unique:
            lo, nd, dvalid = np.full(n, 2, np.int64), 127, None
            got = be.match(imgs, uv, lo, nd, True)
        else:
            lo = rng.integers(2, 120, n).astype(np.int64)
            nd = 13
            dvalid = rng.random(n) > 0.1
            # tracked form with per-feature validity (device layout uv | lo | xr | valid | ok)
            c = be.mctx  # (the stream the backend's matcher runs on)
            d = be._dbuf("t_uv", 18 * n)
            hp = be._hbuf("t_uv", 18 * n)
            be._view(hp, np.float32, 2 * n)[:] = uv.ravel()
            be._view(hp, np.int32, n, 8 * n)[:] = lo
            be._view(hp, np.uint8, n, 16 * n)[:] = dvalid
            c.copy_async(d, hp, 18 * n)
            be._epipolar(imgs, d, d + 8 * n, d + 16 * n, 0, n, nd, False, d + 12 * n, d + 17 * n)
            c.copy_async(hp, d, 18 * n)
            c.synchronize()
            got = (be._view(hp, np.float32, n, 12 * n).copy(), be._view(hp, np.uint8, n, 17 * n).astype(bool))
        ob = OracleBackend()
        oimgs = ob.frame_images(0, fr[0].left, fr[0].right)
        ref = PL.match_host(ob, oimgs, uv, lo, nd, dvalid, unique, 128)
    finally:
        be.close()
    assert np.array_equal(got[1], ref[1])
    assert np.array_equal(got[0][ref[1]].view(np.uint32), ref[0][ref[1]].view(np.uint32))
    assert ref[1].sum() > n // 4  # the comparison covers many accepted matches
    assert not ref[1][:e].any()  # the border features match nothing


@pytest.mark.gpu
def test_pipeline_gpu_shared_context_equals_overlapped(ctx, seq5):
    """GPUBackend(overlap=False): one context for the front end and the BA (the
    scale LM and the BA queueing inline, no worker thread calling the same
    context) takes the overlapped loop's decisions bit for bit."""
    a_be = PL.GPUBackend(ctx, overlap=False)
    assert a_be.shared_ctx and not a_be.async_enqueue
    try:
        a = _run(5, 16, a_be, window=8, frames=seq5, ba_iters=10)
    finally:
        a_be.close()
    b_be = PL.GPUBackend(ctx)
    try:
        b = _run(5, 16, b_be, window=8, frames=seq5, overlap=True, ba_iters=10)
    finally:
        b_be.close()
    assert a.events == b.events and np.array_equal(a.ids, b.ids)
    for t in a.poses:
        assert np.array_equal(a.poses[t], b.poses[t]), t
    assert np.array_equal(a.X, b.X)
    assert [(r.scale, r.scale_iters, r.ba_iters) for r in a.results] == [(r.scale, r.scale_iters, r.ba_iters)
                                                                          for r in b.results]
