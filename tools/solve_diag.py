"""Timing diagnostics of the BA camera solve phases (ME_SOLVE_SKIP masks).
Results of skipped runs are invalid; only the BA_SOLVE kernel time matters."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np
from uasl_motion_estimation_amd import synthetic as S
from uasl_motion_estimation_amd._lib import Context
from uasl_motion_estimation_amd.optimisation import SolverOptions, ba_solve

ctx = Context(0)
c = S.CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 3]
bp = S.ba_problem(7, c["n_feats"], c["window"], c["width"], c["height"])
opts = SolverOptions.fixed_iterations(10)
for mask in [0, 1, 2, 4, 8, 16, 32, 64, 127]:
    os.environ["ME_SOLVE_SKIP"] = str(mask)
    ba_solve(bp, opts, ctx=ctx)
    ctx.timing_reset()
    ctx.timing(True)
    for _ in range(3):
        ba_solve(bp, opts, ctx=ctx)
    ctx.timing(False)
    res = {f: ctx.timing_read(f) for f in ("BA_SOLVE", "BA_SCHUR", "BA_POINTS", "BA_STEP", "BA_LINEARIZE")}
    print(mask, {k: round(v[1] / max(v[0], 1) * 1e3, 1) for k, v in res.items()}, flush=True)
