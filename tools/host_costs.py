"""Host-side cost of queuing one frame's work (wall time of each C-ABI call on the host):
me_klt_track, me_scale_optimise (blocking), me_ba_solve_async (queue only), me_ba_wait."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import bench  # noqa: E402
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import Context  # noqa: E402
from uasl_motion_estimation_amd.klt import klt_params  # noqa: E402
from uasl_motion_estimation_amd.optimisation import SolverOptions  # noqa: E402

cfg = S.CONFIGS[3]
frames = bench.make_frames(cfg, S.SEED0 + 3, 4)
ctx = Context(0)
bench.upload_images(ctx, frames)
kp = klt_params()
bo = SolverOptions.fixed_iterations(10)
st = bench.new_stats()
for fd in frames:
    bench.gpu_step(ctx, fd, kp, bo, st)
ctx.synchronize()
T = {k: [] for k in ("klt", "scale", "ba_async", "ba_wait", "reset")}
for r in range(5):
    for fd in frames:
        c = bench._calls(ctx, fd, kp, bo)
        t = time.perf_counter(); ctx.check(ctx.lib.me_klt_track(*c.klt)); T["klt"].append(time.perf_counter() - t)
        ctx.synchronize()
        c.sc.scale = c.scale0
        t = time.perf_counter(); ctx.check(ctx.lib.me_scale_optimise(*c.scale)); T["scale"].append(time.perf_counter() - t)
        t = time.perf_counter(); fd.dba.reset(); T["reset"].append(time.perf_counter() - t)
        t = time.perf_counter()
        ctx.check(ctx.lib.me_ba_solve_async(ctx.h, ctypes.byref(c.bp), ctypes.byref(c.bo)))
        T["ba_async"].append(time.perf_counter() - t)
        t = time.perf_counter(); ctx.check(ctx.lib.me_ba_wait(ctx.h, ctypes.byref(c.bs))); T["ba_wait"].append(time.perf_counter() - t)
for k, v in T.items():
    v = sorted(v)
    print("%-9s median %8.1f us  min %8.1f  max %8.1f" % (k, 1e6 * v[len(v) // 2], 1e6 * v[0], 1e6 * v[-1]))
