"""A/B of the spin-synchronised launches: the persistent
scale LM (config 3, 2 000 tracks, default LM) and the camera solve with
trailing workers (config 5 window, 2 000 x 50, 10 LM iterations), timed with
wall clocks around back-to-back solves.  Run once per library build
(ME_LIB=tools/abl/coop/libme_hip.so selects the cooperative-launch build) and
under `rocprofv3 --kernel-trace --stats` for the per-kernel averages
(tools/coop_ab.sh).  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import Context  # noqa: E402
from uasl_motion_estimation_amd.optimisation import (DeviceBAProblem, OptimisationParams,  # noqa: E402
                                                     SolverOptions, scale_optimise)

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = Context(0)
cfg = S.CONFIGS[3]
seed = S.SEED0 + 3
scene, K, stream = S.stereo_stream(seed, cfg["width"], cfg["height"], 2)
sp = S.scale_problem(seed, cfg["width"], cfg["height"], cfg["n_feats"], window=cfg["window"], w=5,
                     frames=stream[:2], scene=scene)
out = {"lib": os.environ.get("ME_LIB", "tree")}
for _ in range(3):
    r = scale_optimise(sp, OptimisationParams(), ctx=ctx)
t0 = time.perf_counter()
for _ in range(reps):
    r = scale_optimise(sp, OptimisationParams(), ctx=ctx)
out["scale_lm_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 4)
out["scale_lm"] = {k: r[k] for k in ("iterations", "res_evals", "rejections")}
c5 = S.CONFIGS[5]
bp = S.ba_problem(S.SEED0 + 5, c5["n_feats"], c5["window"], c5["width"], c5["height"])
d = DeviceBAProblem(bp, ctx)
o = SolverOptions.fixed_iterations(10)
for _ in range(3):
    d.reset()
    s = d.solve(o)
ctx.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    d.reset()
    s = d.solve(o)
ctx.synchronize()
out["ba_config5_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 4)
out["ba_config5_iterations"] = s["iterations"]
print(json.dumps(out))
