#!/usr/bin/env python3
"""Development microbenchmark of the batched MI kernel (mi.hip, >= 32768 pairs):
1M 11x11 pairs at random corners of a config-3 synthetic stereo frame, HIP-event
timing on the ctx stream, and a self-check of the batch kernel against the
small-batch group kernel (parity-tested separately) on the same pairs."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from uasl_motion_estimation_amd import synthetic as S  # noqa: E402
from uasl_motion_estimation_amd._lib import Context  # noqa: E402
from uasl_motion_estimation_amd.mutual_information import mi_scores_device  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pairs", type=int, default=1 << 20)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--check", type=int, default=1)
ap.add_argument("--lib", default=None, help="load this libme_hip.so build (timing experiments)")
a = ap.parse_args()
if a.lib:
    from uasl_motion_estimation_amd import _lib

    _lib.load_library(a.lib)
cfg = S.CONFIGS[3]
scene, K, stream = S.stereo_stream(S.SEED0 + 3, cfg["width"], cfg["height"], 2)
L, R = np.ascontiguousarray(stream[1].left), np.ascontiguousarray(stream[1].right)
H, W = L.shape
ctx = Context(0)
n = a.pairs
rng = np.random.default_rng(7)
xyL = np.stack([rng.integers(0, W - 11, n), rng.integers(0, H - 11, n)], -1).astype(np.int32)
xyR = xyL.copy()
xyR[:, 0] = np.clip(xyL[:, 0] - rng.integers(0, 40, n), 0, W - 11)
dLi, dRi = ctx.malloc(L.nbytes), ctx.malloc(R.nbytes)
ctx.h2d(dLi, L)
ctx.h2d(dRi, R)
dL, dR, dout = ctx.malloc(xyL.nbytes), ctx.malloc(xyR.nbytes), ctx.malloc(4 * n)
ctx.h2d(dL, xyL)
ctx.h2d(dR, xyR)
run = lambda: mi_scores_device(ctx, dLi, W, dRi, W, W, H, dL, dR, n, (11, 11), dout)  # noqa: E731
run()
ctx.synchronize()
ctx.timing_reset()
ctx.timing(True)
for _ in range(a.reps):
    run()
ctx.synchronize()
ctx.timing(False)
cnt, ms = ctx.timing_read("MI")
avg = ms / cnt
print("pairs %d  avg %.4f ms  %.3f Gpairs/s  %.1f GB/s (262 B/pair)  frac %.4f" %
      (n, avg, n / avg / 1e6, 262 * n / avg / 1e6, 262 * n / avg / 1e6 / 8000))
if a.check:
    got = np.zeros(n, np.float32)
    ctx.d2h(got, dout)
    m = min(n, 200000)
    ref = np.zeros(m, np.float32)
    chunk = 30000
    for s in range(0, m, chunk):
        e = min(m, s + chunk)
        mi_scores_device(ctx, dLi, W, dRi, W, W, H, dL + 8 * s, dR + 8 * s, e - s, (11, 11), dout + 4 * s)
    ctx.synchronize()
    ctx.d2h(ref, dout)
    bad = np.flatnonzero(got[:m].view(np.uint32) != ref.view(np.uint32))
    print("self-check vs group kernel on %d pairs: %d mismatches" % (m, len(bad)))
    if len(bad):
        sys.exit(1)
