"""Timing of the VO loop's epipolar MI matcher (me_mi_epipolar_match) at the
config-3 loop's two shapes: ~1 860 tracked features x 13 candidates and ~260
new features x 127 candidates (HIP events, MI family).  LIB=... loads a
variant build."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: F401,E402

if os.environ.get("LIB"):
    from uasl_motion_estimation_amd import _lib as _l

    _l.load_library(os.environ["LIB"])
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import Context  # noqa: E402

ctx = Context(0)
cfg = S.CONFIGS[3]
scene, K, fr = S.stereo_stream(S.SEED0 + 3, cfg["width"], cfg["height"], 1)
L, R = np.ascontiguousarray(fr[0].left), np.ascontiguousarray(fr[0].right)
H, W = L.shape
dL, dR = ctx.malloc(L.nbytes), ctx.malloc(R.nbytes)
ctx.h2d(dL, L)
ctx.h2d(dR, R)
rng = np.random.default_rng(1)
V = ctypes.c_void_p
for n, nd, lo0, uniq in ((1864, 13, None, 0), (264, 127, 2, 1)):
    uv = np.stack([rng.uniform(160, W - 30, n), rng.uniform(30, H - 30, n)], -1).astype(np.float32)
    lo = (np.full(n, lo0) if lo0 is not None else rng.integers(2, 100, n)).astype(np.int32)
    du, dl, dx, do = ctx.malloc(uv.nbytes), ctx.malloc(lo.nbytes), ctx.malloc(4 * n), ctx.malloc(n)
    ctx.h2d(du, uv)
    ctx.h2d(dl, lo)
    run = lambda: ctx.check(ctx.lib.me_mi_epipolar_match(ctx.h, V(dL), V(dR), W, H, W, V(du), V(dl), None, None, n, nd,  # noqa: E731
                                                         11, 128, uniq, 1.2, 24.0, V(dx), V(do)), "epi")
    run()
    ctx.synchronize()
    ctx.timing_reset()
    ctx.timing(True)
    for _ in range(20):
        run()
    ctx.synchronize()
    ctx.timing(False)
    k, ms = ctx.timing_read("MI")
    xr = np.zeros(n, np.float32)
    ctx.d2h(xr, dx)
    print(os.environ.get("TAG", ""), f"n {n} nd {nd}: {1e3 * ms / max(k, 1):.1f} us/launch  checksum {float(np.nansum(xr)):.6f}",
          flush=True)
