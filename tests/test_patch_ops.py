"""A3: comparePC, applyCCOEFFNormed, quantise (src/core/mutual_information.cpp:14-25,
136-140, 48-53).  CPU tests pin the oracle with known answers and an
independent numpy restatement; GPU tests compare libme_hip.so with the oracle:
comparePC and quantise bit-exact, applyCCOEFFNormed bit-exact against the
restatement (its OpenCV MatExpr rounding is itself unpinned: no OpenCV here)."""
import numpy as np
import pytest


def _patches(seed, n, r, c, scale=1.0):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((n, r, c)) * scale).astype(np.float32), \
        (rng.standard_normal((n, r, c)) * scale).astype(np.float32)


def _numpy_compare_pc(a, b):
    s = np.float32(0)
    s1 = np.float32(0)
    s2 = np.float32(0)
    for x, y in zip(a.ravel(), b.ravel()):
        s = np.float32(s + np.float32(x * y))
        s1 = np.float32(np.float64(s1) + np.float64(x) * np.float64(x))
        s2 = np.float32(np.float64(s2) + np.float64(y) * np.float64(y))
    return np.float32(s / np.sqrt(np.float32(s1 * s2)))


def test_oracle_compare_pc_matches_numpy_restatement(oracle):
    A, B = _patches(1, 20, 7, 9)
    got = oracle.compare_pc(A, B)
    ref = np.array([_numpy_compare_pc(a, b) for a, b in zip(A, B)], np.float32)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_oracle_known_answers(oracle):
    A, _ = _patches(2, 5, 11, 11)
    np.testing.assert_allclose(oracle.compare_pc(A, A), 1.0, rtol=1e-6)
    np.testing.assert_allclose(oracle.compare_pc(A, -A), -1.0, rtol=1e-6)
    np.testing.assert_allclose(oracle.ccoeff_normed(A + 3.0, A + 3.0), 1.0, rtol=1e-6)
    img = np.arange(256, dtype=np.uint8).reshape(16, 16)
    q = oracle.quantise(img, 0, 8)  # 256 / 8 = 32 levels of width 8... here: v / 32 + 0
    assert np.array_equal(q, (np.arange(256) // 32).astype(np.uint8).reshape(16, 16))
    q = oracle.quantise(img, 10, 74)  # d = 64 -> v / 4 + 10
    assert np.array_equal(q, ((np.arange(256) // 4) + 10).astype(np.uint8).reshape(16, 16))
    q = oracle.quantise(img, 200, 100)  # negative width: C division (256 / -100 = -2) and uchar wrap-around
    d = int(256 / -100)
    exp = np.array([(int(v / d) & 0xFF) + 200 for v in range(256)]) & 0xFF
    assert np.array_equal(q.ravel(), exp.astype(np.uint8))


# ---------------------------------------------------------------- GPU parity

@pytest.mark.gpu
@pytest.mark.parametrize("shape,n", [((11, 11), 1), ((11, 11), 5000), ((10, 10), 777), ((3, 17), 64), ((1, 1), 3)])
def test_gpu_compare_pc_bit_exact(ctx, oracle, shape, n):
    from uasl_motion_estimation_amd.mutual_information import comparePC

    A, B = _patches(3 + n, n, *shape, scale=40.0)
    got = np.atleast_1d(np.asarray(comparePC(A if n > 1 else A[0], B if n > 1 else B[0], ctx=ctx), np.float32))
    ref = oracle.compare_pc(A, B)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("shape,n", [((11, 11), 4096), ((10, 10), 33), ((5, 3), 1)])
def test_gpu_ccoeff_normed(ctx, oracle, shape, n):
    from uasl_motion_estimation_amd.mutual_information import applyCCOEFFNormed

    A, B = _patches(9 + n, n, *shape, scale=30.0)
    A += 128.0
    B += 128.0
    got = np.atleast_1d(np.asarray(applyCCOEFFNormed(A if n > 1 else A[0], B if n > 1 else B[0], ctx=ctx),
                                   np.float32))
    ref = oracle.ccoeff_normed(A, B)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("lo,hi", [(0, 8), (10, 74), (0, 255), (200, 100), (5, 6)])
def test_gpu_quantise_bit_exact(ctx, oracle, lo, hi):
    from uasl_motion_estimation_amd.mutual_information import quantise

    rng = np.random.default_rng(lo * 7 + hi)
    img = rng.integers(0, 256, (37, 53), dtype=np.uint8)
    ref = oracle.quantise(img, lo, hi)
    got = quantise(img.copy(), (lo, hi), ctx=ctx)
    assert np.array_equal(got, ref)


@pytest.mark.gpu
def test_gpu_quantise_rejects_empty_range(ctx):
    from uasl_motion_estimation_amd._lib import MEError
    from uasl_motion_estimation_amd.mutual_information import quantise

    with pytest.raises(MEError):
        quantise(np.zeros((4, 4), np.uint8), (7, 7), ctx=ctx)
