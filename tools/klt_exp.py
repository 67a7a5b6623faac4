"""KLT timing experiment (development only): klt_kernel time vs max_iters /
levels on the config-3 frame, HIP-event timed through the library's
family timer."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import ME_DEVICE, Context  # noqa: E402
from uasl_motion_estimation_amd.klt import klt_params  # noqa: E402

W, H, N = 1280, 720, 2000
scene, K, stream = S.stereo_stream(20261018, W, H, 2)
rng = np.random.default_rng(0)
pts = S.grid_features(rng, N, W, H, 12).astype(np.float32)
ctx = Context()
dp = ctx.malloc(W * H); dn = ctx.malloc(W * H); din = ctx.malloc(8 * N); dout = ctx.malloc(8 * N); dst = ctx.malloc(N)
ctx.h2d(dp, np.ascontiguousarray(stream[0].left)); ctx.h2d(dn, np.ascontiguousarray(stream[1].left))
ctx.h2d(din, pts)
lib = ctx.lib
for levels, iters in [(3, 30), (3, 10), (3, 3), (3, 1), (0, 30), (0, 1), (1, 30), (3, 0)]:
    kp = klt_params(max_level=levels, max_iters=iters)
    lib.me_timing_enable(ctx.h, 1 << 8)
    lib.me_timing_reset(ctx.h)
    for _ in range(20):
        ctx.check(lib.me_klt_track(ctx.h, ME_DEVICE, ctypes.c_void_p(dp), ctypes.c_void_p(dn), W, H, W,
                                   ctypes.c_void_p(din), ctypes.c_void_p(dout), ctypes.c_void_p(dst), N,
                                   ctypes.byref(kp)), "klt")
    ctx.synchronize()
    cnt, ms = ctypes.c_long(), ctypes.c_double()
    lib.me_timing_read(ctx.h, 8, ctypes.byref(cnt), ctypes.byref(ms))
    print(f"levels {levels + 1} iters {iters:2d}: {1000 * ms.value / max(cnt.value, 1):8.1f} us/launch", flush=True)
