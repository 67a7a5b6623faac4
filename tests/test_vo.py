"""Stereo VO: me_vo_process vs the oracle restatement of
StereoVisualOdometry::process (src/vo/StereoVisualOdometry.cpp:34-92).

Bars: process() result, inlier list (index order) and the RANSAC sampling are
exact; the motion matrix agrees to 1e-6 relative (FP64, the device sums
residuals / normal equations in a different order and solves by Cholesky-free
Householder QR like the oracle).  The reference only leaves its GN/LM loop
when a stop condition fires before k reaches the condition's enum value
(:277): noisy or outlier-contaminated data never
terminates there.  Those cases are checked as "both sides report the hang".
Parity unpinned: the reference ships no VO fixtures.
"""
import numpy as np
import pytest

from uasl_motion_estimation_amd import synthetic as S

TRUTH = np.array((0.004, -0.006, 0.003, 0.05, -0.02, 0.5))


def glibc_random_r(seed: int, count: int):
    """Pure-Python restatement of glibc random_r TYPE_3 (srandom_r + 310 discards)."""
    seed = seed or 1
    r = [0] * 34
    r[0] = seed
    for i in range(1, 31):
        hi, lo = divmod(r[i - 1], 127773) if r[i - 1] >= 0 else (-((-r[i - 1]) // 127773), -((-r[i - 1]) % 127773))
        w = 16807 * lo - 2836 * hi
        if w < 0:
            w += 2147483647
        r[i] = w
    st = [x & 0xFFFFFFFF for x in r[:31]]
    f, b = 3, 0
    out = []
    for k in range(310 + count):
        st[f] = (st[f] + st[b]) & 0xFFFFFFFF
        v = st[f] >> 1
        f = (f + 1) % 31
        b = (b + 1) % 31
        if k >= 310:
            out.append(v)
    return out


# ---------------------------------------------------------------- CPU: oracle
@pytest.mark.parametrize("seed", [1, 2, 42, 20261015])
def test_glibc_rand_restatement(oracle, seed):
    assert glibc_random_r(seed, 2000) == oracle.libc_rand_seq(seed, 2000).tolist()


def test_oracle_vo_recovers_motion(oracle):
    from uasl_motion_estimation_amd.vo import euler_motion

    m, p = S.vo_matches(3, 400)
    rc, M, inl = oracle.vo_process(m, p)
    assert rc == 1 and inl.tolist() == list(range(400))
    assert np.allclose(M, euler_motion(TRUTH), atol=1e-6)


def test_oracle_vo_lm_from_close_init(oracle):
    from uasl_motion_estimation_amd.vo import euler_motion

    m, p = S.vo_matches(4, 300, noise=0.005)
    p.update(method=1)
    rc, M, inl = oracle.vo_process(m, p, init=TRUTH + 1e-3)
    assert rc == 1 and len(inl) == 300
    assert np.allclose(M, euler_motion(TRUTH), atol=1e-4)


@pytest.mark.parametrize("kw", [dict(noise=0.5), dict(n_outliers=20)])
def test_oracle_vo_reference_loop_never_exits(oracle, kw):
    m, p = S.vo_matches(5, 300, **kw)
    rc, _, _ = oracle.vo_process(m, p, max_outer=500)
    assert rc == -2


def test_oracle_vo_too_few_matches(oracle):
    m, p = S.vo_matches(6, 5)
    rc, M, inl = oracle.vo_process(m, p)
    assert rc == 0 and len(inl) == 0 and np.allclose(M, np.eye(4))


def test_vo_parameters_defaults():
    """StereoVisualOdometry::parameters() / VisualOdometry::parameters() defaults."""
    from uasl_motion_estimation_amd.vo import Method, Parameters

    p = Parameters()
    assert (p.method, p.step_size, p.eps, p.e1, p.e2, p.e3, p.e4) == (Method.GN, 1.0, 1e-9, 1e-3, 1e-12, 1e-12, 1e-15)
    assert (p.max_iter, p.nb_fixed_frames, p.ransac, p.n_ransac, p.inlier_threshold) == (100, 2, True, 200, 2.0)
    assert (p.baseline, p.weighting, p.fu1, p.fv1, p.fu2, p.fv2) == (1.0, False, 1.0, 1.0, 1.0, 1.0)
    assert (p.cu1, p.cu2, p.cv1, p.cv2) == (0.0, 0.0, 0.0, 0.0)


# ---------------------------------------------------------------- GPU parity
def _run(ctx, oracle, m, p, seed, init=None, max_outer=10000):
    from uasl_motion_estimation_amd.vo import Parameters, StereoVisualOdometry

    vo = StereoVisualOdometry(Parameters(**p), ctx=ctx, max_outer=max_outer)
    vo.srand(seed)
    ok = vo.process(m, init)
    rc, M, inl = oracle.vo_process(m, p, rand_seq=oracle.libc_rand_seq(seed, 16 * vo.m_param.n_ransac + 64),
                                   init=init, max_outer=max_outer)
    return vo, ok, rc, M, inl


@pytest.mark.gpu
def test_gpu_rand_stream_is_glibc(ctx, oracle):
    import ctypes

    got = []
    ctx.check(ctx.lib.me_vo_srand(ctx.h, 77))
    v = ctypes.c_int()
    for _ in range(500):
        ctx.check(ctx.lib.me_vo_rand(ctx.h, ctypes.byref(v)))
        got.append(v.value)
    assert got == oracle.libc_rand_seq(77, 500).tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("case", [
    dict(n=400, seed=11),
    dict(n=2000, seed=12, noise=0.005),
    dict(n=7, seed=13),
    dict(n=6, seed=14),
    dict(n=300, seed=15, noise=0.01, n_ransac=50, inlier_threshold=0.02),
    dict(n=1000, seed=16, noise=0.005, ransac=False),
    dict(n=600, seed=17, noise=0.005, method=1, init=True),
    dict(n=20000, seed=18, noise=0.002),
])
def test_gpu_vo_parity(ctx, oracle, case):
    from uasl_motion_estimation_amd.vo import euler_motion

    case = dict(case)
    n, seed = case.pop("n"), case.pop("seed")
    noise = case.pop("noise", 0.0)
    init = TRUTH + 1e-3 if case.pop("init", False) else None
    m, p = S.vo_matches(seed, n, noise=noise)
    p.update(case)
    vo, ok, rc, M, inl = _run(ctx, oracle, m, p, seed, init=init)
    assert rc in (0, 1)
    assert ok == bool(rc)
    assert vo.getInliers_idx() == inl.tolist()
    got = vo.getMotion()
    assert np.allclose(got, M, rtol=1e-6, atol=1e-9), np.abs(got - M).max()
    if rc:
        assert np.allclose(got, euler_motion(TRUTH), atol=1e-3)
    X = vo.getPts3D()
    assert X.shape == (n, 4) and np.allclose(X[:, 3], 1.0)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(noise=0.5), dict(n_outliers=20), dict(method=1)])
def test_gpu_vo_reports_reference_hang(ctx, oracle, kw):
    from uasl_motion_estimation_amd._lib import MEError

    kw = dict(kw)
    method = kw.pop("method", 0)
    m, p = S.vo_matches(21, 300, **kw)
    p.update(method=method)
    rc, _, _ = oracle.vo_process(m, p, rand_seq=oracle.libc_rand_seq(5, 4000), max_outer=300)
    assert rc == -2
    from uasl_motion_estimation_amd.vo import Parameters, StereoVisualOdometry

    vo = StereoVisualOdometry(Parameters(**p), ctx=ctx, max_outer=300)
    vo.srand(5)
    with pytest.raises(MEError) as e:
        vo.process(m)
    assert e.value.code == -5


@pytest.mark.gpu
def test_gpu_vo_keeps_state_below_six_matches(ctx, oracle):
    from uasl_motion_estimation_amd.vo import Parameters, StereoVisualOdometry

    m, p = S.vo_matches(31, 200)
    vo = StereoVisualOdometry(Parameters(**p), ctx=ctx)
    vo.srand(1)
    assert vo.process(m)
    M0, in0 = vo.getMotion(), vo.getInliers_idx()
    assert not vo.process(m[:5])  # :41-42 returns before touching the state
    assert np.array_equal(vo.getMotion(), M0) and vo.getInliers_idx() == in0
