"""The C++ mirror of the reference API (include/MotionEstimationAMD) driven by a
compiled C++ caller (tests/cpp/adapter_cli) — the binding a maintainer adds
under the reference's src/ (INTEGRATION.md)."""
import os
import struct
import subprocess

import numpy as np
import pytest

from uasl_motion_estimation_amd import synthetic as S

CLI = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "adapter_cli")


def _run(mode, payload, tmp_path, check=True):
    i, o = tmp_path / f"{mode}.in", tmp_path / f"{mode}.out"
    i.write_bytes(payload)
    p = subprocess.run([CLI, mode, str(i), str(o)], capture_output=True, text=True, timeout=300)
    if check:
        assert p.returncode == 0, p.stderr
    return p, (o.read_bytes() if o.exists() else b"")


def _mi_payload(L, R):
    return struct.pack("<ii", *L.shape) + L.tobytes() + R.tobytes()


def test_cli_is_built_and_fails_loudly_without_a_device(tmp_path):
    assert os.path.exists(CLI), "build() compiles tests/cpp/adapter_cli"
    try:
        import torch

        if torch.cuda.is_available():
            pytest.skip("device present")
    except ImportError:
        pass
    L = np.zeros((11, 11), np.uint8)
    p, _ = _run("mi", _mi_payload(L, L), tmp_path, check=False)
    assert p.returncode == 1 and "me_create" in p.stderr  # no silent CPU fallback


@pytest.mark.gpu
def test_cpp_mi_and_entropy_bit_exact(tmp_path, oracle):
    rng = np.random.default_rng(7)
    L = rng.integers(0, 256, (11, 11), dtype=np.uint8)
    R = np.clip(L.astype(int) + rng.integers(-30, 30, L.shape), 0, 255).astype(np.uint8)
    _, out = _run("mi", _mi_payload(L, R), tmp_path)
    mi, h, threw = struct.unpack("<ffi", out)
    assert np.float32(mi) == np.float32(oracle.mutual_information(L, R))
    assert np.float32(h) == np.float32(oracle.entropy(L))
    assert threw == 1


@pytest.mark.gpu
def test_cpp_nms_bit_exact(tmp_path, oracle):
    rng = np.random.default_rng(8)
    r = np.round(rng.random((40, 50)) * 6) / 6
    _, out = _run("nms", struct.pack("<ii", *r.shape) + r.tobytes(), tmp_path)
    n = struct.unpack_from("<i", out)[0]
    mx = np.frombuffer(out, np.float64, 2 * n, 4).reshape(n, 2)
    mask = np.frombuffer(out, np.uint8, r.size, 4 + 16 * n).reshape(r.shape)
    rmx, rmask = oracle.nms(r)
    assert np.array_equal(mx, rmx) and np.array_equal(mask, rmask)


def _ba_payload(bp, compute_cov=0):
    od = getattr(bp, "obs_dim", 4)
    payload = struct.pack("<iiiiii", len(bp.cams), len(bp.pts), len(bp.obs), bp.fixed_frames, od, compute_cov)
    payload += np.asarray(bp.K0, np.float64).tobytes() + np.asarray(bp.K1, np.float64).tobytes()
    payload += struct.pack("<dd", bp.baseline, bp.feat_var)
    payload += np.ascontiguousarray(bp.cams, np.float64).tobytes() + np.ascontiguousarray(bp.pts).tobytes()
    payload += np.ascontiguousarray(bp.obs, np.float64).tobytes()
    payload += np.ascontiguousarray(bp.cam_idx, np.int32).tobytes() + np.ascontiguousarray(bp.pt_idx).tobytes()
    if od == 2:
        payload += np.ascontiguousarray(bp.cam_id, np.int32).tobytes()
    return payload


def _ba_result(out, bp):
    status, iters, cost = struct.unpack_from("<iid", out)
    off = 16
    cams = np.frombuffer(out, np.float64, 6 * len(bp.cams), off).reshape(-1, 6)
    off += 48 * len(bp.cams)
    pts = np.frombuffer(out, np.float64, 3 * len(bp.pts), off).reshape(-1, 3)
    off += 24 * len(bp.pts)
    (ncov,) = struct.unpack_from("<i", out, off)
    cov = np.frombuffer(out, np.float64, 36 * ncov, off + 4).reshape(-1, 6, 6)
    return status, iters, cost, cams, pts, cov


@pytest.mark.gpu
def test_cpp_bundle_adjuster_matches_oracle(tmp_path, oracle):
    bp = S.ba_problem(20261020, 150, 6, 640, 480)
    _, out = _run("ba", _ba_payload(bp), tmp_path)
    status, iters, cost, cams, pts, cov = _ba_result(out, bp)
    rc, rp, rs = oracle.ba_solve(bp)
    assert status == 2 and iters == rs["iterations"]  # Status::SUCCESSFUL
    assert len(cov) == 0
    np.testing.assert_allclose(cams, rc, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(pts, rp, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(cost, rs["final_cost"], rtol=1e-8)


@pytest.mark.gpu
def test_cpp_bundle_adjuster_over_rccl_comm_bit_identical(tmp_path):
    """BundleAdjuster<4>::optimise(fixed, &comm) with a one-rank RCCL
    amd::Comm (me_ba_solve_comm, the packed exchange) = the plain solve."""
    bp = S.ba_problem(20261020, 150, 6, 640, 480)
    _, a = _run("ba", _ba_payload(bp), tmp_path)
    _, b = _run("ba_rccl", _ba_payload(bp), tmp_path)
    assert a == b


@pytest.mark.gpu
def test_cpp_mono_bundle_adjuster_with_covariance(tmp_path, oracle):
    bp = S.ba_problem_mono(20261021, 150, 6, 640, 480)
    _, out = _run("ba", _ba_payload(bp, compute_cov=1), tmp_path)
    status, iters, cost, cams, pts, cov = _ba_result(out, bp)
    rc, rp, rs = oracle.ba_solve(bp)
    assert status == 2 and iters == rs["iterations"]
    np.testing.assert_allclose(cams, rc, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(pts, rp, rtol=1e-6, atol=1e-9)
    after = bp.copy()
    after.cams, after.pts = rc, rp
    rcov = oracle.ba_covariance(after)
    np.testing.assert_allclose(cov, rcov, rtol=1e-5, atol=1e-8 * np.abs(rcov).max())


def _scale_payload(sp, fixed10, thr, mask=None):
    nL, nR = len(sp.X_left), len(sp.X_right)
    rows, cols = sp.imgL.shape
    b = struct.pack("<8i", nL, nR, sp.window_size, int(sp.lframe), int(fixed10), int(mask is not None), rows, cols)
    b += np.asarray(sp.K1, np.float64).tobytes() + np.asarray(sp.K2, np.float64).tobytes()
    b += np.asarray(sp.q1, np.float64).tobytes() + np.asarray(sp.t1, np.float64).tobytes()
    b += np.asarray(sp.q2, np.float64).tobytes() + np.asarray(sp.t2, np.float64).tobytes()
    b += struct.pack("<ddd", sp.scale, sp.baseline, thr)
    b += np.ascontiguousarray(sp.X_left, np.float64).tobytes() + np.ascontiguousarray(sp.X_right, np.float64).tobytes()
    b += np.asarray(sp.tri_left, np.uint8).tobytes() + np.asarray(sp.tri_right, np.uint8).tobytes()
    b += np.asarray(sp.last_left, np.uint32).tobytes() + np.asarray(sp.last_right, np.uint32).tobytes()
    if mask is not None:
        b += np.asarray(mask, np.uint8).tobytes()
    return b + np.ascontiguousarray(sp.imgL).tobytes() + np.ascontiguousarray(sp.imgR).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("fixed10,masked", [(0, False), (1, False), (0, True)])
def test_cpp_scale_optimiser_matches_oracle(tmp_path, oracle, fixed10, masked):
    """Optimiser<ScaleState, vector<pair<Mat,Mat>>> through the C++ mirror:
    the ScaleState is flattened by me::amd::flatten_scale_state, the template
    the reference-side binding instantiates on its own ScaleState."""
    import dataclasses

    from uasl_motion_estimation_amd.optimisation import OptimisationParams

    sp = S.scale_problem(20261022, 640, 480, 400)
    mask = None
    if masked:  # keep every row the reference can index (A-6): mask out a few tracks on both sides
        mask = np.ones(len(sp.X_left) + len(sp.X_right), np.uint8)
        mask[::17] = 0
        mask[len(sp.X_left):] = 1
    thr = 1.2
    _, out = _run("scale", _scale_payload(sp, fixed10, thr, mask), tmp_path)
    stop, iters, scale = struct.unpack_from("<iid", out)
    off = 16
    (nres,) = struct.unpack_from("<i", out, off)
    res0 = np.frombuffer(out, np.float64, nres, off + 4)
    off += 4 + 8 * nres
    (ninl,) = struct.unpack_from("<i", out, off)
    inl = np.frombuffer(out, np.int32, ninl, off + 4)
    off += 4 + 4 * ninl
    jac, smi = struct.unpack_from("<dd", out, off)

    params = OptimisationParams.fixed_iterations(10) if fixed10 else OptimisationParams()
    spm = dataclasses.replace(sp, mask=mask)
    assert np.array_equal(res0, oracle.scale_residuals(sp))
    ref = oracle.scale_optimise(spm, **params.oracle_kw())
    assert stop == ref["stop"] and iters == ref["iterations"]
    np.testing.assert_allclose(scale, ref["scale"], rtol=1e-9)
    after = dataclasses.replace(sp, scale=scale)
    assert np.array_equal(inl, oracle.scale_inliers(after, thr))
    np.testing.assert_allclose(jac, oracle.scale_jacobian(dataclasses.replace(after, mask=mask)), rtol=1e-12)
    rmi, _ = oracle.scale_state_mi(sp)
    assert np.float32(smi) == np.float32(rmi)


@pytest.mark.gpu
def test_cpp_stereo_vo_matches_oracle(tmp_path, oracle):
    m, p = S.vo_matches(12, 300, noise=0.005)
    b = struct.pack("<ii", len(m), 1)
    b += struct.pack("<9d", p["baseline"], p["fu1"], p["fv1"], p["fu2"], p["fv2"], p["cu1"], p["cu2"], p["cv1"],
                     p["cv2"])
    b += np.ascontiguousarray(m, np.float32).tobytes()
    _, out = _run("vo", b, tmp_path)
    (ok,) = struct.unpack_from("<i", out)
    motion = np.frombuffer(out, np.float64, 16, 4).reshape(4, 4)
    (ninl,) = struct.unpack_from("<i", out, 4 + 128)
    inl = np.frombuffer(out, np.int32, ninl, 8 + 128)
    rc, rM, rinl = oracle.vo_process(m, p)
    assert rc in (0, 1) and bool(ok) == bool(rc)
    assert np.array_equal(inl, rinl)
    np.testing.assert_allclose(motion, rM, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
def test_cpp_mono_vo_matches_oracle(tmp_path, oracle):
    """me::MonoVisualOdometry (the C++ mirror of MonoVisualOdometry.h) over the
    C ABI = the oracle's restated findEssentialMat + recoverPose."""
    f1, f2, p, R, t = S.mono_matches(31, 500, noise=0.4, n_outliers=80, n_invalid=4)
    b = struct.pack("<ii", len(f1), 1) + struct.pack("<4d", p["fu"], p["fv"], p["cu"], p["cv"])
    b += np.ascontiguousarray(np.concatenate([f1, f2], 1), np.float32).tobytes()
    _, out = _run("mono", b, tmp_path)
    (ok,) = struct.unpack_from("<i", out)
    motion = np.frombuffer(out, np.float64, 16, 4).reshape(4, 4)
    (ninl,) = struct.unpack_from("<i", out, 4 + 128)
    inl = np.frombuffer(out, np.int32, ninl, 8 + 128)
    rok, rRt, rE, rinl, _ = oracle.mono_vo_process(f1, f2, **p)
    assert ok == rok == 1
    assert np.array_equal(inl, rinl)
    np.testing.assert_allclose(motion, rRt, rtol=0, atol=1e-9)
