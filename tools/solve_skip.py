"""cam_solve time with phases removed (ME_SOLVE_SKIP bits: 1 diag math, 2 panel, 4 trailing, 8 backward; results invalid)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401
from uasl_motion_estimation_amd import _lib
if len(sys.argv) > 1 and sys.argv[1] != "default":
    _lib.load_library(sys.argv[1])
from uasl_motion_estimation_amd import synthetic as S
from uasl_motion_estimation_amd._lib import Context
from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve
ctx = Context(0)
for c in (3,):
    cfg = S.CONFIGS[c]
    bp = S.ba_problem(S.SEED0 * 7 + c, cfg["n_feats"], cfg["window"], cfg["width"], cfg["height"])
    row = {}
    for sk in (0, 1, 2, 4, 8, 15, 256):
        os.environ["ME_SOLVE_SKIP"] = str(sk)
        ba_solve(bp.copy(), SolverOptions.fixed_iterations(10), ctx=ctx)
        ctx.timing_reset(); ctx.timing(True, ["BA_SOLVE"])
        for _ in range(3):
            ba_solve(bp.copy(), SolverOptions.fixed_iterations(10), ctx=ctx)
        ctx.synchronize(); ctx.timing(False)
        n, ms = ctx.timing_read("BA_SOLVE")
        row[sk] = round(1e3 * ms / max(n, 1), 1)
    print("config", c, "us/solve by skip mask", row, flush=True)
