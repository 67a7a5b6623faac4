"""Per-family BA kernel times (HIP events, all families) on the bench's config-3/4/5 windows, 10 LM iterations.
Env knobs (ME_SCHUR_PTS, ME_SOLVE_SKIP, ...) select A/B variants."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401
if os.environ.get("LIB"):
    from uasl_motion_estimation_amd import _lib as _l
    _l.load_library(os.environ["LIB"])
from uasl_motion_estimation_amd import synthetic as S
from uasl_motion_estimation_amd._lib import Context
from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, SolverOptions
ctx = Context(0)
fams = ("BA_LINEARIZE", "BA_SCHUR", "BA_SOLVE", "BA_STEP")
for c in [int(x) for x in os.environ.get("CONFIGS", "3,4,5").split(",")]:
    cfg = S.CONFIGS[c]
    bp = S.ba_problem(S.SEED0 * 7 + c, cfg["n_feats"], cfg["window"], cfg["width"], cfg["height"])
    d = DeviceBAProblem(bp, ctx)
    o = SolverOptions.fixed_iterations(10)
    d.solve(o); ctx.synchronize()
    ctx.timing_reset(); ctx.timing(True)
    for _ in range(5):
        d.reset(); s = d.solve(o)
    ctx.synchronize(); ctx.timing(False)
    r = {}
    for f in fams:
        n, ms = ctx.timing_read(f)
        r[f] = round(1e3 * ms / max(n, 1), 2)
    print(os.environ.get("TAG", ""), "config", c, "us/launch", r, "final", s["final_cost"], flush=True)
    d.close()
