"""Wall time of one BA solve (10 LM iterations, HIP events around 20 queued solves, per-kernel
timing off) on the bench's config-3/4/5 windows.  Env knobs (ME_SCHUR_*, ME_LIB) select A/B
variants.  Usage: ba_wall.py [CONFIGS]  (e.g. 3,4,8000x50)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import Context  # noqa: E402
from uasl_motion_estimation_amd.optimisation import DeviceBAProblem, SolverOptions  # noqa: E402

ctx = Context(0)
out = {}
for c in (sys.argv[1] if len(sys.argv) > 1 else "3,4,5").split(","):
    if "x" in c:  # NFEATSxWINDOW at 1280x720
        nf, w = (int(v) for v in c.split("x"))
        bp = S.ba_problem(S.SEED0 * 7 + w, nf, w, 1280, 720)
    else:
        cfg = S.CONFIGS[int(c)]
        bp = S.ba_problem(S.SEED0 * 7 + int(c), cfg["n_feats"], cfg["window"], cfg["width"], cfg["height"])
    d = DeviceBAProblem(bp, ctx)
    o = SolverOptions.fixed_iterations(10)
    for _ in range(3):
        d.reset()
        s = d.solve(o)
    ctx.synchronize()
    best = []
    for rep in range(3):
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        ctx.synchronize()
        import time
        w0 = time.perf_counter()
        for _ in range(20):
            d.reset()
            s = d.solve(o)
        ctx.synchronize()
        best.append((time.perf_counter() - w0) / 20 * 1e3)
    out[c] = (round(min(best), 4), s["iterations"], s["final_cost"])
    d.close()
print(os.environ.get("TAG", ""), "ms per solve (best of 3 x 20):", out, flush=True)
