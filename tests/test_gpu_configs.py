"""GPU parity at the BASELINE configurations' full sizes (configs 2-5), and
the scale optimiser's LM rejection path.

Every case runs the product path (libme_hip.so through the C ABI) and the
CPU restatement (oracle/) on the same seeded synthetic input:
  * BA (BundleAdjuster<4>::optimise, BundleAdjuster.h:431-476): same
    iteration / successful-step counts, cameras and points within 1e-6
    relative (1e-9 absolute floor) at fixed iteration counts;
  * scale LM (Optimiser<ScaleState,...>::optimise, optimisation.cpp:29-147,
    run_LM_step :685-730): same stop condition, iterations, residual /
    normal-equation evaluation counts and LM rejections; trace and scale
    within 1e-9 relative;
  * KLT: positions and status bit-exact.
"""
import dataclasses

import numpy as np
import pytest

from uasl_motion_estimation_amd import synthetic as S
from uasl_motion_estimation_amd.optimisation import OptimisationParams

pytestmark = pytest.mark.gpu


def _ba_fixed(ctx, oracle, bp, iters):
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve

    cams, pts, s = ba_solve(bp.copy(), SolverOptions.fixed_iterations(iters), ctx=ctx)
    rc, rp, rs = oracle.ba_solve(bp, max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                                 parameter_tolerance=0.0)
    assert s["iterations"] == rs["iterations"] == iters, (s, rs)
    assert s["successful_steps"] == rs["successful_steps"], (s, rs)
    assert s["status"] == rs["status"] == 2
    np.testing.assert_allclose(cams, rc, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(pts, rp, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(s["final_cost"], rs["final_cost"], rtol=1e-9)


def _scale_check(ctx, oracle, sp, params: OptimisationParams, test=False):
    from uasl_motion_estimation_amd.optimisation import scale_optimise

    got = scale_optimise(sp, params, test=test, ctx=ctx)
    ref = oracle.scale_optimise(sp, test=int(test), **params.oracle_kw())
    assert int(got["stop"]) == ref["stop"], (got["stop"], ref)
    assert got["iterations"] == ref["iterations"]
    assert (got["res_evals"], got["neq_evals"], got["rejections"]) == \
        (ref["res_evals"], ref["neq_evals"], ref["rejections"]), (got, ref)
    n = len(sp.X_left) + len(sp.X_right)
    assert got["track_evals"] == n * (got["res_evals"] + (0 if test else 2 * got["neq_evals"]))
    np.testing.assert_allclose(got["scale"], ref["scale"], rtol=1e-9)
    np.testing.assert_allclose(got["trace"], ref["trace"], rtol=1e-9)
    return got, ref


# ------------------------------------------------------------------ LM rejection path
@pytest.fixture(scope="module")
def sp300():
    return S.scale_problem(3, 640, 480, 300)


@pytest.mark.parametrize("scale0,kw,stop", [
    (1.02, {}, 2),                                   # rejections, then SMALL_INCREMENT after an accepted step
    (0.9, dict(alpha=5.0, incr_tol=1e-6), 4),        # rejections, then SMALL_DECREASE_FUNCTION
    (0.9, dict(v=float("inf")), 6),                  # NO_CONVERGENCE (v2 <= v)
    (1.2, dict(minim=False), 2),                     # maximisation: rho sign flipped
    (1.02, dict(alpha=20.0), 2),
])
def test_scale_lm_rejections(ctx, oracle, sp300, scale0, kw, stop):
    sp = dataclasses.replace(sp300, scale=scale0)
    got, ref = _scale_check(ctx, oracle, sp, OptimisationParams(**kw))
    assert ref["rejections"] > 0 and ref["stop"] == stop


def test_scale_lm_fixed_iterations_long_streak(ctx, oracle, sp300):
    """Tolerances off: the final rejection streak runs until mu overflows and
    the step is exactly 0 (~33 rejections); most late candidates equal the
    current state bit for bit and are decided without an evaluation."""
    got, ref = _scale_check(ctx, oracle, sp300, OptimisationParams.fixed_iterations(10))
    assert ref["rejections"] >= 30


def test_scale_gn_fixed_iterations(ctx, oracle, sp300):
    """GN with tolerances off runs MAX_NB_ITER + 1 iterations and reports NO_STOP (SURVEY A-2)."""
    p = dataclasses.replace(OptimisationParams.fixed_iterations(10), type=0)
    got, ref = _scale_check(ctx, oracle, sp300, p)
    assert ref["iterations"] == 11 and ref["stop"] == 0


# ------------------------------------------------------------------ config-sized scale LM
def _cfg_scale_problem(c: int, frame: int, render_div: int = 1):
    """The bench's scale problem of config c, frame `frame` (bench.py make_frames)."""
    cfg = S.CONFIGS[c]
    seed = S.SEED0 + c
    scene, K, stream = S.stereo_stream(seed, cfg["width"], cfg["height"], frame + 2, render_div=render_div)
    return S.scale_problem(seed + frame, cfg["width"], cfg["height"], cfg["n_feats"], window=cfg["window"], w=5,
                           frames=stream[: frame + 2], scene=scene)


@pytest.fixture(scope="module")
def sp_cfg3():
    return [_cfg_scale_problem(3, f) for f in (0, 1)]


@pytest.mark.parametrize("frame", [0, 1])
@pytest.mark.parametrize("mode", ["default", "fixed10"])
def test_scale_config3_2000_tracks(ctx, oracle, sp_cfg3, frame, mode):
    sp = sp_cfg3[frame]
    assert len(sp.X_left) + len(sp.X_right) == 2000 and sp.imgL.shape == (720, 1280)
    p = OptimisationParams() if mode == "default" else OptimisationParams.fixed_iterations(10)
    _scale_check(ctx, oracle, sp, p)


def test_scale_config2_500_tracks(ctx, oracle):
    sp = _cfg_scale_problem(2, 0)
    assert len(sp.X_left) + len(sp.X_right) == 500
    _scale_check(ctx, oracle, sp, OptimisationParams())
    _scale_check(ctx, oracle, sp, OptimisationParams.fixed_iterations(10))


def test_scale_config4_8000_tracks_4k(ctx, oracle):
    sp = _cfg_scale_problem(4, 0, render_div=4)
    assert len(sp.X_left) + len(sp.X_right) == 8000 and sp.imgL.shape == (2160, 3840)
    _scale_check(ctx, oracle, sp, OptimisationParams.fixed_iterations(10))


@pytest.fixture(scope="module")
def stream_cfg4():
    """Config 4's first stereo pairs rendered natively at 3840x2160
    (render_div=1: every pixel rendered, no pixel replication)."""
    cfg = S.CONFIGS[4]
    scene, K, stream = S.stereo_stream(S.SEED0 + 4, cfg["width"], cfg["height"], 2, render_div=1)
    return scene, stream


def test_scale_config4_8000_tracks_native_4k(ctx, oracle, stream_cfg4):
    """Config 4's scale LM on natively rendered 4K images (VERDICT r3 item 1;
    the render_div=4 case above keeps ~3x3 distinct values per 11x11 patch)."""
    cfg = S.CONFIGS[4]
    scene, stream = stream_cfg4
    sp = S.scale_problem(S.SEED0 + 4, cfg["width"], cfg["height"], cfg["n_feats"], window=cfg["window"], w=5,
                         frames=stream[:2], scene=scene)
    assert len(sp.X_left) + len(sp.X_right) == 8000 and sp.imgL.shape == (2160, 3840)
    # the images really are native: neighbouring columns / rows differ (a 4x
    # replicated render has identical 4-pixel runs: fraction 0)
    assert np.mean(sp.imgL[:, 0::4] != sp.imgL[:, 1::4]) > 0.5 and np.mean(sp.imgL[0::4] != sp.imgL[1::4]) > 0.5
    _scale_check(ctx, oracle, sp, OptimisationParams.fixed_iterations(10))
    _scale_check(ctx, oracle, sp, OptimisationParams())


def test_klt_config4_8000_features_native_4k(ctx, oracle, stream_cfg4):
    """KLT of 8000 features on a native 3840x2160 pair, bit-exact against the
    oracle's restatement (positions and status)."""
    from uasl_motion_estimation_amd.klt import calcOpticalFlowPyrLK

    c = S.CONFIGS[4]
    _, stream = stream_cfg4
    rng = np.random.default_rng(S.SEED0 + 4)
    pts = S.grid_features(rng, c["n_feats"], c["width"], c["height"], 12).astype(np.float32)
    assert len(pts) == 8000
    got, gst = calcOpticalFlowPyrLK(stream[0].left, stream[1].left, pts, ctx=ctx)
    ref, rst = oracle.klt(stream[0].left, stream[1].left, pts)
    assert np.array_equal(gst, rst)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert gst.mean() > 0.8


# ------------------------------------------------------------------ config-sized BA windows
def test_ba_config3_2000x20_10_iterations(ctx, oracle):
    c = S.CONFIGS[3]
    bp = S.ba_problem(S.SEED0 + 3, c["n_feats"], c["window"], c["width"], c["height"])
    assert len(bp.pts) == 2000 and len(bp.cams) == 20
    _ba_fixed(ctx, oracle, bp, 10)


def test_ba_config3_bench_window(ctx, oracle):
    """The exact BA window bench.py times first (make_frames: seed * 7 + frame)."""
    c = S.CONFIGS[3]
    seed = S.SEED0 + 3
    _ba_fixed(ctx, oracle, S.ba_problem(seed * 7 + 0, c["n_feats"], c["window"], c["width"], c["height"]), 10)


@pytest.mark.parametrize("cfg,iters", [(3, 10), (4, 4)])
def test_ba_fused_assembly_identical(ctx, monkeypatch, cfg, iters):
    """S assembly inside the camera-solve launch (default; LDS form at config 3,
    global-memory form at config 4) vs its own s_assemble launch
    (ME_BA_NOFUSEASM=1): the same sums in the same order, so bit-identical
    cameras, points and summary."""
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve

    c = S.CONFIGS[cfg]
    bp = S.ba_problem(S.SEED0 + cfg, c["n_feats"], c["window"], c["width"], c["height"])
    out = {}
    for sep in ("0", "1"):
        monkeypatch.setenv("ME_BA_NOFUSEASM", sep)
        out[sep] = ba_solve(bp.copy(), SolverOptions.fixed_iterations(iters), ctx=ctx)
    (c0, p0, s0), (c1, p1, s1) = out["0"], out["1"]
    assert np.array_equal(c0, c1) and np.array_equal(p0, p1)
    assert (s0["iterations"], s0["successful_steps"], s0["final_cost"]) == \
        (s1["iterations"], s1["successful_steps"], s1["final_cost"])


def test_ba_config4_8000x30(ctx, oracle):
    c = S.CONFIGS[4]
    bp = S.ba_problem(S.SEED0 + 4, c["n_feats"], c["window"], c["width"], c["height"])
    assert len(bp.pts) == 8000 and len(bp.cams) == 30
    _ba_fixed(ctx, oracle, bp, 10)  # (the bench's 10 iterations, unsharded -- VERDICT r4)


def test_ba_config5_2000x50(ctx, oracle):
    c = S.CONFIGS[5]
    bp = S.ba_problem(S.SEED0 + 5, c["n_feats"], c["window"], c["width"], c["height"])
    assert len(bp.pts) == 2000 and len(bp.cams) == 50
    _ba_fixed(ctx, oracle, bp, 10)


# ------------------------------------------------------------------ config-sized KLT
def test_klt_config3_2000_features(ctx, oracle):
    from uasl_motion_estimation_amd.klt import calcOpticalFlowPyrLK

    c = S.CONFIGS[3]
    seed = S.SEED0 + 3
    scene, K, stream = S.stereo_stream(seed, c["width"], c["height"], 2)
    rng = np.random.default_rng(seed)
    pts = S.grid_features(rng, c["n_feats"], c["width"], c["height"], 12).astype(np.float32)
    got, gst = calcOpticalFlowPyrLK(stream[0].left, stream[1].left, pts, ctx=ctx)
    ref, rst = oracle.klt(stream[0].left, stream[1].left, pts)
    assert np.array_equal(gst, rst)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert gst.mean() > 0.8


# ------------------------------------------------------------------ A7: ScaleState::compute_residuals
@pytest.mark.parametrize("which", ["cfg1", "cfg3"])
def test_scale_state_mi_matches_oracle(ctx, oracle, which, sp300, sp_cfg3):
    """Evident intent of optimisation.cpp:230-278 (parity unpinned: the
    reference's stacking copies nothing): float MI of the stacked pairs, bit-exact."""
    from uasl_motion_estimation_amd.optimisation import scale_state_mi

    sp = sp300 if which == "cfg1" else sp_cfg3[1]
    mi, n = scale_state_mi(sp, ctx=ctx)
    rmi, rn = oracle.scale_state_mi(sp)
    assert n == rn > 0
    assert np.float32(mi).view(np.uint32) == np.float32(rmi).view(np.uint32)


def test_scale_state_mi_empty_is_an_error(ctx, sp300):
    from uasl_motion_estimation_amd import MEError
    from uasl_motion_estimation_amd.optimisation import scale_state_mi

    sp = dataclasses.replace(sp300, tri_left=np.zeros_like(sp300.tri_left))
    with pytest.raises(MEError):
        scale_state_mi(sp, ctx=ctx)


# ------------------------------------------------------------------ CU-partitioned concurrent front end / back end
def test_cu_masked_frontend_backend_overlap(oracle, sp_cfg3):
    """bench.py's frontend overlap: a tracker context whose stream is restricted
    to half the CUs (me_set_cu_mask) runs the config-3 scale LM while a
    back-end context on the other half runs the config-3 BA queued with
    me_ba_solve_async -- both concurrently on the device, both equal to the
    oracle; then the masks are lifted and the BA replays bit-identically."""
    import ctypes

    import torch

    from uasl_motion_estimation_amd._lib import BASummaryC, Context
    from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, SolverOptions

    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    front, back = Context(0), Context(0)
    try:
        front.set_cu_mask([i for i in range(ncu) if i % 16 < 8])
        back.set_cu_mask([i for i in range(ncu) if i % 16 >= 8])
        c = S.CONFIGS[3]
        bp = S.ba_problem(S.SEED0 + 3, c["n_feats"], c["window"], c["width"], c["height"])
        d = DeviceBAProblem(bp, back)
        st, opts = d.struct(), SolverOptions.fixed_iterations(10).to_c()
        back.check(back.lib.me_ba_solve_async(back.h, ctypes.byref(st), ctypes.byref(opts)), "me_ba_solve_async")
        _scale_check(front, oracle, sp_cfg3[0], OptimisationParams.fixed_iterations(10))  # while the BA runs
        s = BASummaryC()
        back.check(back.lib.me_ba_wait(back.h, ctypes.byref(s)), "me_ba_wait")
        cams, pts = d.download()
        rc, rp, rs = oracle.ba_solve(bp, max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                                     parameter_tolerance=0.0)
        assert s.iterations == rs["iterations"] == 10 and s.successful_steps == rs["successful_steps"]
        np.testing.assert_allclose(cams, rc, rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(pts, rp, rtol=1e-6, atol=1e-9)
        back.set_cu_mask(None)  # all CUs again: same device results
        d.reset()
        back.check(back.lib.me_ba_solve(back.h, ctypes.byref(st), ctypes.byref(opts), ctypes.byref(s)), "me_ba_solve")
        cams2, pts2 = d.download()
        assert np.array_equal(cams, cams2) and np.array_equal(pts, pts2)
        d.close()
    finally:
        front.close()
        back.close()


def test_klt_many_features_rare_weights(ctx, oracle):
    """40 000 features at random sub-pixel positions of a config-3 pair (about
    a million LK iterations): the bilinear weight jw11 = 16384 - the other three
    comes out -1 in about 1e-5 of them, where the packed-byte dot product of the
    staged footprint words cannot hold it (klt.hip takes the per-tap sum there).
    Bit-exact against the restatement."""
    from uasl_motion_estimation_amd.klt import calcOpticalFlowPyrLK

    c = S.CONFIGS[3]
    seed = S.SEED0 + 3
    scene, K, stream = S.stereo_stream(seed, c["width"], c["height"], 2)
    rng = np.random.default_rng(20261018)
    n = 40000
    pts = np.stack([rng.uniform(30, c["width"] - 30, n), rng.uniform(30, c["height"] - 30, n)], 1).astype(np.float32)
    got, gst = calcOpticalFlowPyrLK(stream[0].left, stream[1].left, pts, ctx=ctx)
    ref, rst = oracle.klt(stream[0].left, stream[1].left, pts)
    assert np.array_equal(gst, rst)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


# ------------------------------------------------------------------ co-residency roster (csrc/roster.hpp)
@pytest.fixture
def roster_now(ctx):
    """Test hook me_debug_solve_flags(8192): every roster on this ctx closes at
    once, so the persistent scale LM and the camera solve's workers run on
    whichever workgroups had joined by then (usually a few: the rest leave
    at once and their units are dealt over the joined ones; with none, block
    0 works alone), and the camera solve's block 0 claims every fused
    assembly unit not yet claimed without waiting (roster.hpp CLAIM)."""
    import ctypes

    hook = ctx.lib.me_debug_solve_flags
    hook.argtypes = [ctypes.c_void_p, ctypes.c_int]

    def set_(on):
        assert hook(ctx.h, 8192 if on else 0) == 0

    yield set_
    set_(False)


def test_roster_scale_lm_identical_at_any_participant_count(ctx, oracle, sp_cfg3, roster_now):
    """the persistent scale LM no longer assumes its grid
    co-resident.  With the roster closed at once the phases run on fewer
    workgroups: the same stop, counts, scale and trace bit for bit, and the
    oracle's."""
    from uasl_motion_estimation_amd.optimisation import scale_optimise

    sp = sp_cfg3[0]
    out = []
    for on in (False, True):
        roster_now(on)
        out.append(scale_optimise(sp, OptimisationParams(), ctx=ctx))
    a, b = out
    for k in ("stop", "iterations", "res_evals", "neq_evals", "rejections", "track_evals"):
        assert a[k] == b[k], k
    assert np.float64(a["scale"]).tobytes() == np.float64(b["scale"]).tobytes()
    assert np.array_equal(np.asarray(a["trace"]), np.asarray(b["trace"]))
    _scale_check(ctx, oracle, sp, OptimisationParams())  # (hook still on)


@pytest.mark.parametrize("cfg,iters", [(3, 10), (5, 4)])
def test_roster_camera_solve_identical_at_any_participant_count(ctx, roster_now, cfg, iters):
    """The camera solve's fused assembly units (config 3, LDS form: claimed
    by block 0 as well as by the assemblers) and trailing tiles (config 5,
    global-memory form with workers, dealt over whichever workers joined the
    roster): bit-identical cameras, points and summary."""
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve

    c = S.CONFIGS[cfg]
    bp = S.ba_problem(S.SEED0 + cfg, c["n_feats"], c["window"], c["width"], c["height"])
    out = []
    for on in (False, True):
        roster_now(on)
        out.append(ba_solve(bp.copy(), SolverOptions.fixed_iterations(iters), ctx=ctx))
    (c0, p0, s0), (c1, p1, s1) = out
    assert np.array_equal(c0, c1) and np.array_equal(p0, p1)
    assert (s0["iterations"], s0["successful_steps"], s0["final_cost"]) == \
        (s1["iterations"], s1["successful_steps"], s1["final_cost"])
