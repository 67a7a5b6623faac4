"""Monocular VO: MonoVisualOdometry::process
(src/vo/MonoVisualOdometry.cpp:7-73) -- OpenCV findEssentialMat (five-point
+ RANSAC / LMedS) and recoverPose, restated (oracle/mono.cpp; parity
unpinned: OpenCV is absent, the reference ships no fixtures).

CPU: the oracle's five-point solver recovers the true essential matrix from
five exact correspondences; the whole process() recovers a synthetic
two-view motion, rejects the outliers and follows the reference's early
exits.  GPU: me_mono_vo_process equals the oracle -- the same inlier indices
bit for bit, motion and E within 1e-9 -- on RANSAC and LMedS runs with
outliers and invalid matches."""
import numpy as np
import pytest

from uasl_motion_estimation_amd import synthetic as S


def _true_E(R, t):
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    E = tx @ R
    return E / np.linalg.norm(E)


def test_oracle_five_point_exact(oracle):
    rng = np.random.default_rng(0)
    worst = 0.0
    for _ in range(200):
        R = S.aa_to_R(rng.normal(0, 0.1, 3))
        t = rng.normal(0, 1, 3)
        t /= np.linalg.norm(t)
        X = np.stack([rng.uniform(-5, 5, 5), rng.uniform(-3, 3, 5), rng.uniform(4, 40, 5)], 1)
        X2 = X @ R.T + t
        x1, x2 = X[:, :2] / X[:, 2:], X2[:, :2] / X2[:, 2:]
        Es = oracle.five_point(x1, x2)
        assert 1 <= len(Es) <= 10
        for E in Es:  # every solution satisfies the five epipolar constraints and det(E) = 0
            r = [abs(np.r_[x2[i], 1] @ E @ np.r_[x1[i], 1]) for i in range(5)]
            assert max(r) < 1e-9
        Et = _true_E(R, t)
        worst = max(worst, min(min(np.abs(E - Et).max(), np.abs(E + Et).max()) for E in Es))
    assert worst < 1e-6


def test_oracle_cv_rng_subsets(oracle):
    a = oracle.cv_rng_subsets(100, 50)
    b = oracle.cv_rng_subsets(100, 50)
    assert a.shape == (50, 5) and np.array_equal(a, b)  # cv::RNG((uint64)-1): deterministic
    assert all(len(set(r)) == 5 for r in a) and a.min() >= 0 and a.max() < 100
    assert len(oracle.cv_rng_subsets(4, 3)) == 0  # fewer than 5 points: no subset


@pytest.mark.parametrize("case", ["clean", "outliers", "lmeds"])
def test_oracle_mono_recovers_motion(oracle, case):
    no = 0 if case == "clean" else 150
    f1, f2, p, R, t = S.mono_matches(11, 800, noise=0.3, n_outliers=no, n_invalid=7)
    ok, Rt, E, inl, st = oracle.mono_vo_process(f1, f2, ransac=0 if case == "lmeds" else 1, **p)
    assert ok == 1
    assert np.abs(Rt[:3, :3] - R).max() < 5e-3 and np.abs(Rt[:3, 3] - t).max() < 3e-2
    assert abs(np.linalg.det(Rt[:3, :3]) - 1) < 1e-9 and abs(np.linalg.norm(Rt[:3, 3]) - 1) < 1e-9
    assert np.all(np.diff(inl) > 0) and not np.isin(np.arange(800 - 7, 800), inl).any()  # invalid matches skipped
    assert (inl < no).sum() <= 0.05 * max(no, 1)  # the outliers are rejected
    assert len(inl) > 0.8 * (800 - 7 - no)


def test_oracle_mono_early_exits(oracle):
    f1, f2, p, R, t = S.mono_matches(12, 7)
    ok, Rt, E, inl, st = oracle.mono_vo_process(f1, f2, **p)
    assert ok == 0 and np.array_equal(Rt, np.eye(4)) and len(inl) == 0  # < 8 matches (:67-71)
    f1, f2, p, R, t = S.mono_matches(12, 20, n_invalid=17)  # 3 valid: no essential matrix (:22-26)
    ok, Rt, E, inl, st = oracle.mono_vo_process(f1, f2, **p)
    assert ok == 0 and np.array_equal(Rt, np.eye(4)) and not E.any()
    f1, f2, p, R, t = S.mono_matches(12, 9, noise=0.2)  # 9 inliers at most: < 10 (:46-49)
    ok, Rt, E, inl, st = oracle.mono_vo_process(f1, f2, **p)
    assert ok == 0 and np.array_equal(Rt, np.eye(4)) and len(inl) <= 9


# ------------------------------------------------------------------ GPU
CASES = {
    "ransac_clean": dict(seed=21, n=600, noise=0.3, no=0, ni=0, ransac=1),
    "ransac_outliers": dict(seed=22, n=2000, noise=0.5, no=500, ni=13, ransac=1),
    "ransac_heavy": dict(seed=23, n=1000, noise=0.5, no=450, ni=0, ransac=1),
    "lmeds": dict(seed=24, n=800, noise=0.3, no=120, ni=5, ransac=0),
    "small": dict(seed=25, n=12, noise=0.2, no=0, ni=0, ransac=1),
    "threshold0": dict(seed=26, n=300, noise=0.3, no=30, ni=0, ransac=1, thr=0.0),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_gpu_mono_matches_oracle(ctx, oracle, name):
    from uasl_motion_estimation_amd.vo import MonoParameters, MonoVisualOdometry

    c = CASES[name]
    f1, f2, p, R, t = S.mono_matches(c["seed"], c["n"], noise=c["noise"], n_outliers=c["no"], n_invalid=c["ni"])
    thr = c.get("thr", 2.0)
    ok_o, Rt_o, E_o, inl_o, st = oracle.mono_vo_process(f1, f2, ransac=c["ransac"], inlier_threshold=thr, **p)
    vo = MonoVisualOdometry(MonoParameters(ransac=bool(c["ransac"]), inlier_threshold=thr, **p), ctx=ctx)
    ok = vo.process((f1, f2))
    assert ok == bool(ok_o)
    assert vo.getInliersIdx() == [int(i) for i in inl_o]  # indices bit for bit
    np.testing.assert_allclose(vo.getMotion(), Rt_o, rtol=0, atol=1e-9)
    if E_o.any():
        np.testing.assert_allclose(vo.getEssentialMat(), E_o, rtol=0, atol=1e-9)
    if ok:
        assert np.abs(vo.getMotion()[:3, :3] - R).max() < 1e-2
        assert set(vo.getOutliersIdx()) | set(vo.getInliersIdx()) == set(range(c["n"]))


@pytest.mark.gpu
def test_gpu_mono_too_few_matches(ctx):
    from uasl_motion_estimation_amd.vo import MonoVisualOdometry

    f1, f2, p, R, t = S.mono_matches(3, 7)
    vo = MonoVisualOdometry(ctx=ctx)
    assert not vo.process((f1, f2)) and np.array_equal(vo.getMotion(), np.eye(4))


@pytest.mark.gpu
def test_gpu_mono_early_exits_keep_state(ctx):
    """MonoVisualOdometry.cpp:9-52: < 8 matches returns before touching m_E and the
    inlier / outlier lists; an empty E is assigned (empty) and the lists are kept."""
    from uasl_motion_estimation_amd.vo import MonoParameters, MonoVisualOdometry

    f1, f2, p, R, t = S.mono_matches(21, 600, noise=0.3)
    vo = MonoVisualOdometry(MonoParameters(**p), ctx=ctx)
    assert vo.process((f1, f2))
    E0, inl0, out0 = vo.getEssentialMat(), vo.getInliersIdx(), vo.getOutliersIdx()
    a1, a2, *_ = S.mono_matches(3, 7)
    assert not vo.process((a1, a2)) and np.array_equal(vo.getMotion(), np.eye(4))
    assert np.array_equal(vo.getEssentialMat(), E0) and vo.getInliersIdx() == inl0 and vo.getOutliersIdx() == out0
    b1, b2, *_ = S.mono_matches(12, 20, n_invalid=17)  # 3 valid: no essential matrix
    assert not vo.process((b1, b2)) and np.array_equal(vo.getMotion(), np.eye(4))
    assert vo.getEssentialMat().size == 0 and vo.getInliersIdx() == inl0 and vo.getOutliersIdx() == out0
