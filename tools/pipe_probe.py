"""Host timeline of the front-end/back-end frame pipeline (bench.FramePipeline,
overlap=frontend): wall time spent in each call per frame, no profiler."""
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
tctx = Context(0)
split = int(os.environ.get("CUSPLIT", "0"))  # front-end CUs out of every 16
if split:
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    tctx.set_cu_mask([i for i in range(ncu) if i % 16 < split])
    ctx.set_cu_mask([i for i in range(ncu) if i % 16 >= split])
pipe = bench.FramePipeline(ctx, tctx, bench._Hip(), os.environ.get("OVERLAP", "frontend"))
pipe.run(frames, 4, kp, bo, bench.new_stats())
ctx.synchronize(); tctx.synchronize()
T = {}


def tm(name, f, *a):
    t = time.perf_counter()
    r = f(*a)
    T.setdefault(name, []).append(time.perf_counter() - t)
    return r


n = 40
pend = None
t0 = time.perf_counter()
for t in range(n):
    fd = frames[t % 4]
    tm("klt", pipe._klt, fd, kp, bo, t)
    tm("scale", pipe._scale, tctx, fd, kp, bo, bench.new_stats())
    pipe.hip.record(pipe.ev[t & 1], pipe.s_trk)
    if pend is not None:
        tm("ba_wait", pipe._ba_wait, pend, bench.new_stats())
    c = bench._calls(ctx, fd, kp, bo)
    pipe.hip.wait(pipe.s_main, pipe.ev[t & 1])
    tm("reset", fd.dba.reset)
    tm("ba_async", ctx.lib.me_ba_solve_async, ctx.h, ctypes.byref(c.bp), ctypes.byref(c.bo))
    pend = c
pipe._ba_wait(pend, bench.new_stats())
el = time.perf_counter() - t0
print("CUSPLIT", split, "frames/s %.1f  ms/frame %.3f" % (n / el, 1e3 * el / n))
for k, v in T.items():
    v = sorted(v)
    print("%-9s median %8.1f us  min %8.1f  max %8.1f  mean %8.1f" % (k, 1e6 * v[len(v) // 2], 1e6 * v[0], 1e6 * v[-1],
                                                                   1e6 * sum(v) / len(v)))
