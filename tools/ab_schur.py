"""A/B of the Schur pass variants (ME_SCHUR_SORT, ME_SCHUR_PTS, ...) on the
bench's BA windows: per-family BA kernel time (HIP events) and the wall time
of the whole 10-iteration solve (plan included), configs 3 / 4 and the
8000 x 50 window of the config-5 VO loop's size.  One process per variant
(the caller sets the env); TAG labels the line."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402

if os.environ.get("LIB"):
    from uasl_motion_estimation_amd import _lib as _l

    _l.load_library(os.environ["LIB"])

from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import Context  # noqa: E402
from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, SolverOptions  # noqa: E402

ctx = Context(0)
fams = ("BA_LINEARIZE", "BA_SCHUR", "BA_SOLVE", "BA_STEP")
cases = {"c3": (2000, 20, 1280, 720), "c4": (8000, 30, 3840, 2160), "w50": (8000, 50, 1280, 720)}
for name, (n, w, W, H) in cases.items():
    bp = S.ba_problem(S.SEED0 * 7 + w, n, w, W, H)
    d = DeviceBAProblem(bp, ctx)
    o = SolverOptions.fixed_iterations(10)
    d.solve(o)
    ctx.synchronize()
    walls = []
    for _ in range(5):
        d.reset()
        ctx.synchronize()
        t0 = time.perf_counter()
        s = d.solve(o)
        ctx.synchronize()
        walls.append(time.perf_counter() - t0)
    ctx.timing_reset()
    ctx.timing(True)
    for _ in range(3):
        d.reset()
        s = d.solve(o)
    ctx.synchronize()
    ctx.timing(False)
    r = {}
    for f in fams:
        k, ms = ctx.timing_read(f)
        r[f] = round(1e3 * ms / max(k, 1), 2)
    print(os.environ.get("TAG", ""), name, "wall_ms %.3f" % (1e3 * min(walls)), "us/launch", r,
          "iters", s["iterations"], "final %.12e" % s["final_cost"], flush=True)
    d.close()
