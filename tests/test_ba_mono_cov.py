"""BundleAdjuster<2> (mono / stereo-right windows) and pose covariance.

Reference: include/MotionEstimation/optimisation/BundleAdjuster.h
  * StandardReprojectionError :71-103 (camID 0), StereoRightError :106-139
    (camID != 0, p.x += cam[0] - baseline), chosen in BundleAdjuster<2>::optimise
    :395-398, K[0] only, a zero baseline replaced by 0.5 (:389-390);
  * extract_covariance :478-528 (ceres::Covariance over the camera blocks,
    constant cameras -> zero block).
CPU tests pin the oracle restatement (finite differences, a numpy inverse of
J^T J built independently); GPU tests compare libme_hip.so with the oracle.
Bars: residuals 1e-12 rel, Jacobians 1e-9 rel, poses/points 1e-6 rel at fixed
iterations (as the stereo BA), covariance 1e-6 rel.  Parity vs Ceres itself is
unpinned (no Ceres here)."""
import numpy as np
import pytest

from uasl_motion_estimation_amd import synthetic as S


@pytest.fixture(scope="module")
def mono():
    return S.ba_problem_mono(41, 120, 7, 640, 480)


def _res(oracle, bp, cams, pts, o):
    b = bp.copy()
    b.cams, b.pts = cams, pts
    return oracle.ba_evaluate(b)[0][o]


def test_oracle_mono_jacobian_matches_finite_differences(oracle, mono):
    r, Jc, Jp = oracle.ba_evaluate(mono)
    assert r.shape == (len(mono.obs), 2)
    for o in (int(np.argmax(mono.cam_id == 0)), int(np.argmax(mono.cam_id == 1))):
        ci, pi = mono.cam_idx[o], mono.pt_idx[o]
        h = 1e-6
        num_c = np.zeros((2, 6))
        for j in range(6):
            cp, cm = mono.cams.copy(), mono.cams.copy()
            cp[ci, j] += h
            cm[ci, j] -= h
            num_c[:, j] = (_res(oracle, mono, cp, mono.pts, o) - _res(oracle, mono, cm, mono.pts, o)) / (2 * h)
        num_p = np.zeros((2, 3))
        for j in range(3):
            pp, pm = mono.pts.copy(), mono.pts.copy()
            pp[pi, j] += h
            pm[pi, j] -= h
            num_p[:, j] = (_res(oracle, mono, mono.cams, pp, o) - _res(oracle, mono, mono.cams, pm, o)) / (2 * h)
        np.testing.assert_allclose(Jc[o], num_c, rtol=1e-5, atol=1e-5 * np.abs(num_c).max())
        np.testing.assert_allclose(Jp[o], num_p, rtol=1e-5, atol=1e-5 * np.abs(num_p).max())


def test_oracle_mono_residual_models(oracle, mono):
    """camID 0 projects with K[0] from the camera centre, camID 1 from the
    right camera (x shifted by the baseline), both with the left y."""
    from uasl_motion_estimation_amd.synthetic import aa_to_R

    r, _, _ = oracle.ba_evaluate(mono)
    K, b, sinv = mono.K0, mono.baseline, 1.0 / np.sqrt(mono.feat_var)
    for o in range(0, len(mono.obs), 17):
        cam = mono.cams[mono.cam_idx[o]]
        p = aa_to_R(cam[3:]) @ mono.pts[mono.pt_idx[o]] + cam[:3]
        if mono.cam_id[o]:
            p[0] -= b
        pred = np.array([K[0, 0] * p[0] / p[2] + K[0, 2], K[1, 1] * p[1] / p[2] + K[1, 2]])
        np.testing.assert_allclose(r[o], sinv * (pred - mono.obs[o]), rtol=1e-9, atol=1e-9)


def test_oracle_mono_zero_baseline_is_half_metre(oracle, mono):
    b0 = mono.copy()
    b0.baseline = 0.0
    b5 = mono.copy()
    b5.baseline = 0.5
    assert np.array_equal(oracle.ba_evaluate(b0)[0], oracle.ba_evaluate(b5)[0])


def _numpy_covariance(oracle, bp):
    """(J^T J)^-1 camera blocks from the oracle's residual Jacobians, Huber-corrected here."""
    r, Jc, Jp = oracle.ba_evaluate(bp)
    nf = min(max(bp.fixed_frames, 0), len(bp.cams))
    m, npt = len(bp.cams) - nf, len(bp.pts)
    n = 6 * m + 3 * npt
    J = np.zeros((r.size, n))
    D = r.shape[1]
    for o in range(len(r)):
        s = float(r[o] @ r[o])
        sc = np.sqrt(1.0 / np.sqrt(s)) if s > 1.0 else 1.0
        rows = slice(D * o, D * o + D)
        ci = bp.cam_idx[o] - nf
        if ci >= 0:
            J[rows, 6 * ci:6 * ci + 6] = sc * Jc[o]
        J[rows, 6 * m + 3 * bp.pt_idx[o]:6 * m + 3 * bp.pt_idx[o] + 3] = sc * Jp[o]
    C = np.linalg.inv(J.T @ J)
    out = np.zeros((len(bp.cams), 6, 6))
    for i in range(nf, len(bp.cams)):
        k = 6 * (i - nf)
        out[i] = C[k:k + 6, k:k + 6]
    return out


@pytest.mark.parametrize("kind", ["stereo", "mono"])
def test_oracle_covariance_matches_numpy_inverse(oracle, kind):
    bp = S.ba_problem(42, 60, 5, 640, 480) if kind == "stereo" else S.ba_problem_mono(43, 80, 6, 640, 480)
    cov = oracle.ba_covariance(bp)
    ref = _numpy_covariance(oracle, bp)
    assert cov is not None
    assert not cov[:bp.fixed_frames].any()
    np.testing.assert_allclose(cov, ref, rtol=1e-6, atol=1e-9 * np.abs(ref).max())


def test_oracle_covariance_unobserved_camera_fails(oracle):
    bp = S.ba_problem(44, 30, 4, 640, 480)
    keep = bp.cam_idx != 3  # the last (variable) camera loses all its observations
    bp.obs, bp.cam_idx, bp.pt_idx = bp.obs[keep], bp.cam_idx[keep], bp.pt_idx[keep]
    assert oracle.ba_covariance(bp) is None


# ---------------------------------------------------------------- GPU parity
@pytest.mark.gpu
def test_gpu_mono_residuals_and_jacobians(ctx, oracle, mono):
    from uasl_motion_estimation_amd.optimisation import ba_cost, ba_evaluate

    r, Jc, Jp = ba_evaluate(mono, ctx=ctx)
    rr, rJc, rJp = oracle.ba_evaluate(mono)
    assert r.shape == rr.shape == (len(mono.obs), 2)
    np.testing.assert_allclose(r, rr, rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(Jc, rJc, rtol=1e-9, atol=1e-12 * np.abs(rJc).max())
    np.testing.assert_allclose(Jp, rJp, rtol=1e-9, atol=1e-12 * np.abs(rJp).max())
    np.testing.assert_allclose(ba_cost(mono, ctx=ctx), oracle.ba_cost(mono), rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,w,fixed,iters", [(45, 120, 7, 2, 10), (46, 300, 10, 1, 8), (47, 60, 5, 2, 50)])
def test_gpu_mono_solve(ctx, oracle, seed, n, w, fixed, iters):
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve

    bp = S.ba_problem_mono(seed, n, w, 640, 480, fixed=fixed)
    if iters == 50:  # default options (Ceres tolerances)
        cams, pts, s = ba_solve(bp, ctx=ctx)
        rc, rp, rs = oracle.ba_solve(bp)
    else:
        cams, pts, s = ba_solve(bp, SolverOptions.fixed_iterations(iters), ctx=ctx)
        rc, rp, rs = oracle.ba_solve(bp, max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                                     parameter_tolerance=0.0)
    assert s["iterations"] == rs["iterations"] and s["successful_steps"] == rs["successful_steps"], (s, rs)
    assert s["status"] == rs["status"] == 2
    np.testing.assert_allclose(cams, rc, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(pts, rp, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["stereo", "mono"])
def test_gpu_covariance(ctx, oracle, kind):
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_covariance, ba_solve

    bp = S.ba_problem(48, 200, 8, 640, 480) if kind == "stereo" else S.ba_problem_mono(49, 200, 8, 640, 480)
    cams, pts, _ = ba_solve(bp, SolverOptions.fixed_iterations(5), ctx=ctx)
    bp.cams, bp.pts = cams, pts
    cov = ba_covariance(bp, ctx=ctx)
    ref = oracle.ba_covariance(bp)
    assert cov is not None and ref is not None
    assert not cov[:bp.fixed_frames].any()
    np.testing.assert_allclose(cov, ref, rtol=1e-6, atol=1e-9 * np.abs(ref).max())


@pytest.mark.gpu
def test_gpu_covariance_unobserved_block_fails(ctx, oracle):
    """A landmark without observations is not a Ceres parameter block, so
    extract_covariance's block count check fails (BundleAdjuster.h:490-495) and
    no covariance is produced; here its zero V block makes J^T J singular."""
    from uasl_motion_estimation_amd.optimisation import ba_covariance

    bp = S.ba_problem(50, 40, 4, 640, 480)
    bp.pts = np.vstack([bp.pts, [[0.5, 0.2, 10.0]]])
    assert ba_covariance(bp, ctx=ctx) is None
    assert oracle.ba_covariance(bp) is None


@pytest.mark.gpu
def test_gpu_bundle_adjuster_mono_api(ctx, oracle):
    """BundleAdjuster<2> through the reference-shaped API: WBA_Point mono tracks,
    camera IDs, compute_cov -> getPosesCovariance."""
    from uasl_motion_estimation_amd.feature_types import CamPose, WBA_Point
    from uasl_motion_estimation_amd.optimisation import BundleAdjuster, CalibrationParameters, SolverOptions
    from uasl_motion_estimation_amd.rotation_utils import exp_map_Quat

    bp = S.ba_problem_mono(51, 60, 5, 640, 480)
    first_id = 100
    cams = [CamPose(first_id + i, exp_map_Quat(c[3:]), np.array(c[:3])) for i, c in enumerate(bp.cams)]
    tracks = []
    for j in range(len(bp.pts)):
        sel = np.nonzero(bp.pt_idx == j)[0]
        t = WBA_Point((float(bp.obs[sel[0], 0]), float(bp.obs[sel[0], 1])), first_id + int(bp.cam_idx[sel[0]]),
                      int(bp.cam_id[sel[0]]))
        for o in sel[1:]:
            t.addMatch((float(bp.obs[o, 0]), float(bp.obs[o, 1])), first_id + int(bp.cam_idx[o]))
        t.set3DLocation(np.array([*bp.pts[j], 1.0]))
        tracks.append(t)
    calib = CalibrationParameters([bp.K0], bp.feat_var, bp.baseline, compute_cov=True)
    ba = BundleAdjuster(calib, cams, tracks, ctx=ctx, options=SolverOptions.fixed_iterations(6))
    assert ba.M == 2 and ba.getNbObservations() == len(bp.obs)
    assert ba.optimise(bp.fixed_frames).name == "SUCCESSFUL"
    covs = ba.getPosesCovariance()
    assert len(covs) == len(bp.cams) and not np.any(covs[0])
    assert all(np.all(np.linalg.eigvalsh(c) > 0) for c in covs[bp.fixed_frames:])
