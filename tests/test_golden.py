"""Golden fixtures (tests/golden/*.npz, written by tests/golden/make_golden.py).

CPU: the oracle reproduces its committed outputs (guards the restatement
against silent drift).  GPU: the product path, called through the C ABI,
reproduces them — bit-exact for MI / NMS / KLT / scale-state rows, 1e-6
relative for BA parameters (FP64 reductions in a different order).
"""
import numpy as np
import pytest

import golden_io as G


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


# ------------------------------------------------------------------ CPU (oracle)
@pytest.mark.parametrize("side", [10, 11])
def test_oracle_reproduces_mi_golden(oracle, side):
    d = G.load(f"mi_p{side}")
    out = oracle.mi_scores(d["imgL"], d["imgR"], d["xyL"], d["xyR"], side, side)
    assert np.array_equal(bits(out), bits(d["mi"]))
    x, y = d["xyL"][0]
    xr, yr = d["xyR"][0]
    hl, hr, hj = oracle.histograms(d["imgL"][y:y + side, x:x + side], d["imgR"][yr:yr + side, xr:xr + side])
    assert np.array_equal(hl, d["hist_l0"]) and np.array_equal(hr, d["hist_r0"]) and np.array_equal(hj, d["hist_j0"])


def test_oracle_reproduces_nms_golden(oracle):
    d = G.load("nms")
    mx, mask = oracle.nms(d["response"])
    assert np.array_equal(mx, d["maxima"]) and np.array_equal(mask, d["mask"])


def test_oracle_reproduces_klt_golden(oracle):
    d = G.load("klt")
    out, st = oracle.klt(d["prev"], d["next"], d["pts"])
    assert np.array_equal(out, d["out"]) and np.array_equal(st, d["status"])


def test_oracle_reproduces_scale_golden(oracle):
    d = G.load("scale")
    sp = G.scale_problem(d)
    res = oracle.scale_residuals(sp)
    assert np.array_equal(res, d["residuals"])
    JJ, e = oracle.scale_normal_equations(sp, res)
    assert (JJ, e) == (d["JJ"], d["e"])
    assert oracle.scale_jacobian(sp) == d["jacobian"]
    r = oracle.scale_optimise(G.scale_problem(d))
    assert r["scale"] == d["opt_scale"] and r["iterations"] == d["opt_iterations"] and r["stop"] == d["opt_stop"]


def test_oracle_reproduces_ba_golden(oracle):
    d = G.load("ba_cfg1")
    bp = G.ba_problem(d)
    r, Jc, Jp = oracle.ba_evaluate(bp)
    np.testing.assert_allclose(r, d["residuals"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(Jc, d["Jc"], rtol=1e-12, atol=1e-12)
    cams, pts, s = oracle.ba_solve(bp, max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                                   parameter_tolerance=0.0)
    np.testing.assert_allclose(cams, d["cams_fixed10"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(pts, d["pts_fixed10"], rtol=1e-10, atol=1e-12)
    assert s["iterations"] == d["iters_fixed10"]


# ------------------------------------------------------------------ GPU (product)
@pytest.mark.gpu
@pytest.mark.parametrize("side", [10, 11])
def test_gpu_mi_matches_golden(ctx, side):
    from uasl_motion_estimation_amd.mutual_information import mi_scores

    d = G.load(f"mi_p{side}")
    out = mi_scores(d["imgL"], d["imgR"], d["xyL"], d["xyR"], (side, side), ctx=ctx)
    assert np.array_equal(bits(out), bits(d["mi"]))


@pytest.mark.gpu
def test_gpu_nms_matches_golden(ctx):
    from uasl_motion_estimation_amd.feature_types import nonMaxSupScanline3x3

    d = G.load("nms")
    mx, mask = nonMaxSupScanline3x3(d["response"], ctx=ctx)
    assert np.array_equal(mx, d["maxima"]) and np.array_equal(mask, d["mask"])


@pytest.mark.gpu
def test_gpu_klt_matches_golden(ctx):
    from uasl_motion_estimation_amd.klt import calcOpticalFlowPyrLK

    d = G.load("klt")
    out, st = calcOpticalFlowPyrLK(d["prev"], d["next"], d["pts"], ctx=ctx)
    assert np.array_equal(out, d["out"]) and np.array_equal(st, d["status"])


@pytest.mark.gpu
def test_gpu_scale_matches_golden(ctx):
    from uasl_motion_estimation_amd.optimisation import (scale_jacobian, scale_normal_equations, scale_optimise,
                                                         scale_residuals)

    d = G.load("scale")
    sp = G.scale_problem(d)
    res = scale_residuals(sp, ctx=ctx)
    assert np.array_equal(res, d["residuals"])
    JJ, e = scale_normal_equations(sp, res, ctx=ctx)
    np.testing.assert_allclose([JJ, e], [d["JJ"], d["e"]], rtol=1e-12)
    np.testing.assert_allclose(scale_jacobian(sp, ctx=ctx), d["jacobian"], rtol=1e-12)
    r = scale_optimise(G.scale_problem(d), ctx=ctx)
    assert int(r["stop"]) == int(d["opt_stop"]) and r["iterations"] == d["opt_iterations"]
    np.testing.assert_allclose(r["scale"], d["opt_scale"], rtol=1e-9)


@pytest.mark.gpu
def test_gpu_ba_matches_golden(ctx):
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_evaluate, ba_reduced_system, ba_solve

    d = G.load("ba_cfg1")
    bp = G.ba_problem(d)
    r, Jc, Jp = ba_evaluate(bp, ctx=ctx)
    np.testing.assert_allclose(r, d["residuals"], rtol=1e-12, atol=1e-9)
    Sm, b = ba_reduced_system(bp, ctx=ctx)
    np.testing.assert_allclose(Sm, d["S"], rtol=1e-9, atol=1e-9 * np.abs(d["S"]).max())
    np.testing.assert_allclose(b, d["b"], rtol=1e-9, atol=1e-9 * np.abs(d["b"]).max())
    cams, pts, s = ba_solve(G.ba_problem(d), SolverOptions.fixed_iterations(10), ctx=ctx)
    np.testing.assert_allclose(cams, d["cams_fixed10"], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(pts, d["pts_fixed10"], rtol=1e-6, atol=1e-9)
    cams, pts, s = ba_solve(G.ba_problem(d), ctx=ctx)
    assert s["iterations"] == d["iters_default"] and s["status"] == d["status_default"]
    np.testing.assert_allclose(cams, d["cams_default"], rtol=1e-6, atol=1e-9)
