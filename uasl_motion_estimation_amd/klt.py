"""Pyramidal Lucas-Kanade tracking on MI355X (klt.hip).

Build-defined (the reference has no tracker): OpenCV-style
calcOpticalFlowPyrLK defaults (21x21 window, 3 pyramid levels, 30 iterations,
eps 0.01, min-eigenvalue 1e-4) with an integer/fixed-point formulation that
makes the device result bit-identical to its CPU restatement (oracle/klt.cpp).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import ME_HOST, Context, KLTParamsC, default_context, vptr


def klt_params(win=21, max_level=3, max_iters=30, eps=0.01, min_eig=1e-4) -> KLTParamsC:
    k = KLTParamsC()
    k.win, k.max_level, k.max_iters, k.eps, k.min_eig = win, max_level, max_iters, eps, min_eig
    return k


def calcOpticalFlowPyrLK(prev, nxt, pts, ctx: Context | None = None, **kw):
    """Track pts (n, 2) float32 from prev to nxt.  Returns (pts_out (n,2), status (n,) uint8)."""
    ctx = ctx or default_context()
    prev = np.ascontiguousarray(prev, np.uint8)
    nxt = np.ascontiguousarray(nxt, np.uint8)
    if prev.shape != nxt.shape or prev.ndim != 2:
        raise ValueError("prev/next must be equal-size grayscale images")
    pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 2)
    h, w = prev.shape
    out = np.zeros_like(pts)
    st = np.zeros(len(pts), np.uint8)
    kp = klt_params(**kw)
    ctx.check(ctx.lib.me_klt_track(ctx.h, ME_HOST, vptr(prev), vptr(nxt), w, h, w, vptr(pts), vptr(out), vptr(st),
                                   len(pts), ctypes.byref(kp)), "me_klt_track")
    return out, st
