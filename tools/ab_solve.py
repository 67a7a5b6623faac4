"""A/B of libme_hip.so builds on the BA camera solve (BA_SOLVE family time per
launch) and the whole config-3 BA (10 LM iterations), plus result agreement.
Usage: ab_solve.py LIB [LIB...]  (each run in its own process by the caller)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch  # noqa: F401
from uasl_motion_estimation_amd import _lib
lib = sys.argv[1]
if lib != "default":
    _lib.load_library(lib)
from uasl_motion_estimation_amd import synthetic as S
from uasl_motion_estimation_amd._lib import Context
from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, SolverOptions
ctx = Context(0)
out = {}
for c in (3, 4, 5):
    cfg = S.CONFIGS[c]
    bp = S.ba_problem(S.SEED0 * 7 + c, cfg["n_feats"], cfg["window"], cfg["width"], cfg["height"])
    d = DeviceBAProblem(bp, ctx)
    opts = SolverOptions.fixed_iterations(10)
    d.solve(opts)
    ctx.synchronize()
    ctx.timing_reset(); ctx.timing(True, ["BA_SOLVE"])
    for _ in range(5):
        d.reset(); d.solve(opts)
    ctx.synchronize(); ctx.timing(False)
    n, ms = ctx.timing_read("BA_SOLVE")
    t0 = time.perf_counter()
    for _ in range(10):
        d.reset(); s = d.solve(opts)
    ctx.synchronize()
    el = (time.perf_counter() - t0) / 10
    cams, pts = d.download()
    np.save(f"/tmp/ab_{os.path.basename(os.path.dirname(lib)) or 'default'}_{c}.npy", cams)
    print(lib, "config", c, "solve us/launch", round(1e3 * ms / max(n, 1), 2), "BA ms", round(1e3 * el, 3),
          "iters", s["iterations"], "cost", s["final_cost"], flush=True)
