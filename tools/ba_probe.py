#!/usr/bin/env python3
"""Development probe: per-family HIP-event times of one config-3 BA solve (10 LM iterations)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import Context  # noqa: E402
from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, SolverOptions  # noqa: E402

cfg = S.CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 3]
ctx = Context(0)
bp = S.ba_problem(S.SEED0 * 7, cfg["n_feats"], cfg["window"], cfg["width"], cfg["height"])
d = DeviceBAProblem(bp, ctx)
opts = SolverOptions.fixed_iterations(10)
for _ in range(2):
    d.reset()
    d.solve(opts)
ctx.synchronize()
ctx.timing_reset()
ctx.timing(True)
for _ in range(5):
    d.reset()
    d.solve(opts)
ctx.synchronize()
ctx.timing(False)
out = []
for f in ("BA_LINEARIZE", "BA_SCHUR", "BA_SOLVE", "BA_STEP"):
    n, ms = ctx.timing_read(f)
    out.append("%s %.2f us" % (f, 1e3 * ms / max(n, 1)))
print("probe=%s  " % os.environ.get("ME_SCHUR_PROBE", "0") + "  ".join(out))
