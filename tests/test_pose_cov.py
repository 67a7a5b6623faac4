"""Pose-covariance propagation (src/core/feature_types.cpp:171-251).

The product (uasl_motion_estimation_amd.feature_types, host FP64 like the
reference) is compared with the oracle's loop restatement (oracle/pose.cpp);
the oracle is pinned by finite differences of the pose product for every
Jacobian block the reference actually writes, and by the two blocks the
reference's CV_32F copyTo never writes (zero, reproduced).  Tolerance 1e-12
relative (different evaluation order of the same FP64 products)."""
import numpy as np
import pytest

from uasl_motion_estimation_amd.feature_types import (CamPose, ScalePoseWithCovariance, invertPoseWithCovariance,
                                                      poseMultiplicationWithCovariance,
                                                      poseMultiplicationWithCovarianceReverse)
from uasl_motion_estimation_amd.rotation_utils import Quat, exp_map_Quat, log_map_Quat


def _pose(rng, ID=0):
    rv = rng.normal(0, 0.4, 3)
    q = exp_map_Quat(rv)
    t = rng.normal(0, 2.0, 3)
    A = rng.normal(0, 0.1, (6, 6))
    return CamPose(ID, q, t, A @ A.T + 1e-3 * np.eye(6))


@pytest.mark.parametrize("seed", range(5))
def test_multiplication_matches_oracle(oracle, seed):
    rng = np.random.default_rng(seed)
    p1, p2 = _pose(rng, 3), _pose(rng, 4)
    for rev, fn in ((False, poseMultiplicationWithCovariance), (True, poseMultiplicationWithCovarianceReverse)):
        p3 = fn(p1, p2, 9)
        q3, t3, c3 = oracle.pose_mul_cov(p1.orientation.coeffs(), p1.position, p1.Cov, p2.orientation.coeffs(),
                                         p2.position, p2.Cov, rev)
        assert p3.ID == 9
        np.testing.assert_allclose(p3.orientation.coeffs(), q3, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(p3.position, t3, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(p3.Cov, c3, rtol=1e-10, atol=1e-13 * np.abs(c3).max())


@pytest.mark.parametrize("seed", range(5))
def test_inverse_and_scale_match_oracle(oracle, seed):
    rng = np.random.default_rng(100 + seed)
    p = _pose(rng)
    q, t, c = oracle.pose_invert_cov(p.orientation.coeffs(), p.position, p.Cov)
    invertPoseWithCovariance(p)
    np.testing.assert_allclose(p.orientation.coeffs(), q, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(p.position, t, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(p.Cov, c, rtol=1e-10, atol=1e-13 * np.abs(c).max())
    p = _pose(rng)
    t, c = oracle.pose_scale_cov(p.position, p.Cov, 1.7, 0.04)
    ScalePoseWithCovariance(p, (1.7, 0.04))
    np.testing.assert_allclose(p.position, t, rtol=1e-14)
    np.testing.assert_allclose(p.Cov, c, rtol=1e-12, atol=1e-15)


def _rv(q):
    return np.asarray(log_map_Quat(q))


def _numeric_jacobian(p1, p2, reverse, h=1e-6):
    """d(t3, rotvec3) / d(t1, rotvec1, t2, rotvec2) of the pose product by central differences."""
    def prod(x):
        a = CamPose(0, exp_map_Quat(x[3:6]), x[0:3], np.zeros((6, 6)))
        b = CamPose(0, exp_map_Quat(x[9:12]), x[6:9], np.zeros((6, 6)))
        c = b * a if reverse else a * b
        return np.concatenate([c.position, _rv(c.orientation)])
    x0 = np.concatenate([p1.position, _rv(p1.orientation), p2.position, _rv(p2.orientation)])
    J = np.zeros((6, 12))
    for k in range(12):
        d = np.zeros(12)
        d[k] = h
        J[:, k] = (prod(x0 + d) - prod(x0 - d)) / (2 * h)
    return J


@pytest.mark.parametrize("reverse", [False, True])
def test_oracle_jacobian_blocks_are_the_pose_product_derivatives(oracle, reverse):
    """Each block of J written by the reference equals the finite-difference
    derivative; the block behind the CV_32F copyTo is zero instead."""
    rng = np.random.default_rng(7)
    p1, p2 = _pose(rng), _pose(rng)
    Jn = _numeric_jacobian(p1, p2, reverse)
    # recover J column blocks from the oracle: Cov3 = J E_k J^T with unit covariance on one block
    for blk in range(4):
        c1, c2 = np.zeros((6, 6)), np.zeros((6, 6))
        (c1 if blk < 2 else c2)[3 * (blk % 2):3 * (blk % 2) + 3, 3 * (blk % 2):3 * (blk % 2) + 3] = np.eye(3)
        _, _, c3 = oracle.pose_mul_cov(p1.orientation.coeffs(), p1.position, c1, p2.orientation.coeffs(),
                                       p2.position, c2, reverse)
        Jb = Jn[:, 3 * blk:3 * blk + 3]
        quirk = reverse and blk == 2  # J(0:3, 6:9) never written
        if quirk:
            assert np.abs(c3).max() < 1e-300 or np.allclose(c3[:3, :3], 0.0)
            continue
        np.testing.assert_allclose(c3, Jb @ Jb.T, rtol=1e-5, atol=1e-6 * max(1.0, np.abs(c3).max()))


def test_inverse_rotation_block_is_zero_as_in_the_reference(oracle):
    rng = np.random.default_rng(11)
    p = _pose(rng)
    c = np.zeros((6, 6))
    c[3:, 3:] = np.eye(3)  # only rotation uncertainty
    p.Cov = c
    invertPoseWithCovariance(p)
    assert np.allclose(p.Cov[3:, 3:], 0.0)  # J(3:6, 3:6) = -eye(CV_32F) never reaches J
    assert np.abs(p.Cov[:3, :3]).max() > 0    # translation picks up the rotation uncertainty
