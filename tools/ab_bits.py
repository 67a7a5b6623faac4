"""Bit-level A/B of two libme_hip.so builds on the BA windows of configs 3-5
(10 fixed LM iterations): each build runs in its own process (the library is
loaded once per process) and writes cams / pts; the parent compares them.
Usage: ab_bits.py LIB_A LIB_B"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [(3, 0), (3, 1), (4, 0), (5, 0), (2, 0)]


def run(lib, out):
    sys.path.insert(0, ROOT)
    import torch  # noqa: F401

    from uasl_motion_estimation_amd import _lib
    if lib != "default":
        _lib.load_library(lib)
    from uasl_motion_estimation_amd import synthetic as S
    from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve
    res = {}
    for c, k in CASES:
        cfg = S.CONFIGS[c]
        bp = S.ba_problem(S.SEED0 * 7 + c + 100 * k, cfg["n_feats"], cfg["window"], cfg["width"], cfg["height"])
        cams, pts, s = ba_solve(bp.copy(), SolverOptions.fixed_iterations(10))
        res[f"c{c}_{k}_cams"], res[f"c{c}_{k}_pts"] = cams, pts
        res[f"c{c}_{k}_it"] = np.array([s["iterations"], s["successful_steps"]])
    np.savez(out, **res)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        run(sys.argv[2], sys.argv[3])
        sys.exit(0)
    d = tempfile.mkdtemp()
    outs = []
    for i, lib in enumerate(sys.argv[1:3]):
        o = os.path.join(d, f"{i}.npz")
        subprocess.run([sys.executable, __file__, "--child", lib, o], check=True)
        outs.append(np.load(o))
    a, b = outs
    for key in a.files:
        same = np.array_equal(a[key].view(np.uint64) if a[key].dtype == np.float64 else a[key],
                              b[key].view(np.uint64) if b[key].dtype == np.float64 else b[key])
        rel = float(np.max(np.abs(a[key] - b[key]) / (np.abs(b[key]) + 1e-9))) if a[key].size else 0.0
        print(f"{key}: {'identical' if same else 'DIFFER'} max rel {rel:.3g}", flush=True)
