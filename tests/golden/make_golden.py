#!/usr/bin/env python3
"""Writes the golden fixtures of tests/golden/ from the oracle restatement.

The reference ships no golden vectors for this path and cannot be built here
(SURVEY §8c), so these fixtures are regression anchors produced by the
CPU restatement (oracle/, test infrastructure) on seeded synthetic inputs;
its correctness is pinned separately by tests/test_oracle.py.  Run from the
repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import golden_io as G  # noqa: E402
import oracle as O  # noqa: E402
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402


def mi(side, seed):
    L, R, xyL, xyR = S.random_patches(seed, 96, 64, 256, side, side)
    out = O.mi_scores(L, R, xyL, xyR, side, side)
    hl, hr, hj = O.histograms(L[xyL[0, 1]:xyL[0, 1] + side, xyL[0, 0]:xyL[0, 0] + side],
                              R[xyR[0, 1]:xyR[0, 1] + side, xyR[0, 0]:xyR[0, 0] + side])
    G.save(f"mi_p{side}", imgL=L, imgR=R, xyL=xyL, xyR=xyR, mi=out, hist_l0=hl, hist_r0=hr, hist_j0=hj)


def nms():
    rng = np.random.default_rng(20261015)
    r = np.round(rng.random((48, 64)) * 8) / 8.0 + 0.125  # quantised: plateaus and ties
    r[10:14, 20:30] = 2.0                                # a flat block
    mx, mask = O.nms(r)
    G.save("nms", response=r, maxima=mx, mask=mask)


def klt():
    sc, K, fr = S.stereo_stream(20261016, 160, 120, 2)
    rng = np.random.default_rng(3)
    pts = S.grid_features(rng, 48, 160, 120, 12).astype(np.float32)
    out, st = O.klt(fr[0].left, fr[1].left, pts)
    G.save("klt", prev=fr[0].left, next=fr[1].left, pts=pts, out=out, status=st)


def scale():
    sp = S.scale_problem(20261017, 160, 120, 60, window=5, w=5)
    res = O.scale_residuals(sp)
    JJ, e = O.scale_normal_equations(sp, res)
    jac = O.scale_jacobian(sp)
    r = O.scale_optimise(sp)
    G.save("scale", residuals=res, JJ=JJ, e=e, jacobian=jac, opt_scale=r["scale"], opt_stop=r["stop"],
           opt_iterations=r["iterations"], **G.dataclass_arrays("sp_", sp))


def ba():
    bp = S.ba_problem(20261018, 200, 5, 640, 480)
    cams, pts, s = O.ba_solve(bp, max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    r, Jc, Jp = O.ba_evaluate(bp)
    Sm, b, _ = O.ba_reduced_system(bp)
    cams_d, pts_d, s_d = O.ba_solve(bp)  # reference options (function_tolerance 1e-3)
    G.save("ba_cfg1", cams_fixed10=cams, pts_fixed10=pts, cost_fixed10=s["final_cost"],
           iters_fixed10=s["iterations"], residuals=r, Jc=Jc, Jp=Jp, S=Sm, b=b, cams_default=cams_d,
           pts_default=pts_d, iters_default=s_d["iterations"], status_default=s_d["status"],
           **G.dataclass_arrays("bp_", bp))


if __name__ == "__main__":
    os.makedirs(G.GOLDEN, exist_ok=True)
    mi(11, 20261011)
    mi(10, 20261012)
    nms()
    klt()
    scale()
    ba()
    for f in sorted(os.listdir(G.GOLDEN)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(G.GOLDEN, f)))
