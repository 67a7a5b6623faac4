"""KLT kernel timing on the config-3 frame (2000 features, 1280 x 720, the
bench's parameters), HIP-event timed through the library's family timer;
with --check the results are compared with the oracle restatement (bit-exact).
Usage: klt_bench.py [--reps R] [--check 0|1] [--lib LIB]"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--check", type=int, default=1)
ap.add_argument("--lib", default=None)
args = ap.parse_args()
from uasl_motion_estimation_amd import _lib  # noqa: E402

if args.lib:
    _lib.load_library(args.lib)
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import ME_DEVICE, Context  # noqa: E402
from uasl_motion_estimation_amd.klt import klt_params  # noqa: E402

W, H, N = 1280, 720, 2000
scene, K, stream = S.stereo_stream(20261018, W, H, 2)
rng = np.random.default_rng(0)
pts = S.grid_features(rng, N, W, H, 12).astype(np.float32)
ctx = Context()
dp, dn, din, dout, dst = ctx.malloc(W * H), ctx.malloc(W * H), ctx.malloc(8 * N), ctx.malloc(8 * N), ctx.malloc(N)
L0, L1 = np.ascontiguousarray(stream[0].left), np.ascontiguousarray(stream[1].left)
ctx.h2d(dp, L0)
ctx.h2d(dn, L1)
ctx.h2d(din, pts)
lib = ctx.lib
kp = klt_params()


def run():
    ctx.check(lib.me_klt_track(ctx.h, ME_DEVICE, ctypes.c_void_p(dp), ctypes.c_void_p(dn), W, H, W,
                               ctypes.c_void_p(din), ctypes.c_void_p(dout), ctypes.c_void_p(dst), N, ctypes.byref(kp)),
              "klt")


for _ in range(3):
    run()
ctx.synchronize()
lib.me_timing_enable(ctx.h, 1 << 8)
lib.me_timing_reset(ctx.h)
for _ in range(args.reps):
    run()
ctx.synchronize()
cnt, ms = ctypes.c_long(), ctypes.c_double()
lib.me_timing_read(ctx.h, 8, ctypes.byref(cnt), ctypes.byref(ms))
lib.me_timing_enable(ctx.h, 0)
print(f"klt_kernel: {1000 * ms.value / max(cnt.value, 1):.2f} us/launch ({N} features, {W}x{H})", flush=True)
if args.check:
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O  # checker only

    got = np.zeros(2 * N, np.float32)
    gst = np.zeros(N, np.uint8)
    ctx.d2h(got, dout)
    ctx.d2h(gst, dst)
    ref_pts, ref_st = O.klt(L0, L1, pts)
    same = np.array_equal(got.view(np.uint32), np.ascontiguousarray(ref_pts, np.float32).ravel().view(np.uint32)) \
        and np.array_equal(gst, ref_st)
    print(f"klt parity vs oracle: {'bit-exact' if same else 'MISMATCH'}", flush=True)
    if not same:
        sys.exit(1)
