"""BA time per config-3 frame window on the back-end stream: whole GPU, half the CUs (the
pipeline's mask), and half the CUs while the front end (KLT + scale LM) runs on the other half."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import Context  # noqa: E402
from uasl_motion_estimation_amd.klt import klt_params  # noqa: E402
from uasl_motion_estimation_amd.optimisation import SolverOptions  # noqa: E402

cfg = S.CONFIGS[3]
frames = bench.make_frames(cfg, S.SEED0 + 3, 4)
ctx, tctx = Context(0), Context(0)
bench.upload_images(ctx, frames)
kp = klt_params()
bo = SolverOptions.fixed_iterations(10)
ncu = torch.cuda.get_device_properties(0).multi_processor_count
F = int(os.environ.get("FRONT", "8"))


def ba_run(n, front=False):
    st = bench.new_stats()
    t0 = time.perf_counter()
    pend = None
    for t in range(n):
        fd = frames[t % 4]
        c = bench._calls(ctx, fd, kp, bo)
        fd.dba.reset()
        ctx.check(ctx.lib.me_ba_solve_async(ctx.h, ctypes.byref(c.bp), ctypes.byref(c.bo)))
        if front:
            ct = bench._calls(tctx, fd, kp, bo)
            tctx.check(tctx.lib.me_klt_track(*ct.klt))
            ct.sc.scale = ct.scale0
            tctx.check(tctx.lib.me_scale_optimise(*ct.scale))
        if pend is not None:
            ctx.check(ctx.lib.me_ba_wait(ctx.h, ctypes.byref(pend.bs)))
        pend = c
    ctx.check(ctx.lib.me_ba_wait(ctx.h, ctypes.byref(pend.bs)))
    ctx.synchronize(); tctx.synchronize()
    return 1e3 * (time.perf_counter() - t0) / n


for mode in ("full", "half", "half+front", "full+front"):
    if mode.startswith("half"):
        tctx.set_cu_mask([i for i in range(ncu) if i % 16 < F])
        ctx.set_cu_mask([i for i in range(ncu) if i % 16 >= F])
    else:
        tctx.set_cu_mask(None)
        ctx.set_cu_mask(None)
    ba_run(8, "front" in mode)
    print("%-11s ms per BA window: %.3f" % (mode, ba_run(60, "front" in mode)), flush=True)
