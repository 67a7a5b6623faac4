"""Mutual-information patch scores on MI355X.

Mirrors include/MotionEstimation/core/mutual_information.h:
``computeMutualInformation(L, R)`` (src/core/mutual_information.cpp:55-86),
``computeEntropy(img)`` (:28-45), ``comparePC`` (:14-25),
``applyCCOEFFNormed`` (:136-140) and ``quantise`` (:48-53), plus the batched
forms the optimisers use.
All compute runs in libme_hip.so (mi.hip); results are bit-identical to the
reference's float values.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import ME_DEVICE, ME_HOST, Context, default_context, vptr


def _as_u8(img) -> np.ndarray:
    """cv::Mat::convertTo(CV_8U): saturate_cast<uchar> = round-half-even + clamp."""
    a = np.asarray(img)
    if a.dtype != np.uint8:
        a = np.clip(np.rint(a.astype(np.float64)), 0, 255).astype(np.uint8)
    if a.ndim != 2:
        raise ValueError("computeMutualInformation expects single-channel 2-D images")
    return np.ascontiguousarray(a)


def computeMutualInformation(imgL, imgR, ctx: Context | None = None) -> float:
    """me::computeMutualInformation(const cv::Mat&, const cv::Mat&) -> float (bits)."""
    ctx = ctx or default_context()
    L, R = _as_u8(imgL), _as_u8(imgR)
    if L.size == 0 or R.size == 0:
        raise ValueError("empty image (assert at mutual_information.cpp:57)")
    if L.shape != R.shape:
        raise ValueError("calcHist needs images of the same size")
    h, w = L.shape
    out = np.zeros(1, np.float32)
    ctx.check(ctx.lib.me_mutual_information(ctx.h, ME_HOST, vptr(L), w, vptr(R), w, w, h, vptr(out)),
              "me_mutual_information")
    return float(out[0])


def computeEntropy(img, ctx: Context | None = None) -> float:
    """me::computeEntropy(const cv::Mat&) -> float (bits)."""
    ctx = ctx or default_context()
    a = _as_u8(img)
    h, w = a.shape
    out = np.zeros(1, np.float32)
    ctx.check(ctx.lib.me_entropy(ctx.h, ME_HOST, vptr(a), w, w, h, vptr(out)), "me_entropy")
    return float(out[0])


def mi_scores(imgL, imgR, xyL, xyR, patch=(11, 11), ctx: Context | None = None) -> np.ndarray:
    """Batched MI of n patch pairs with integer top-left corners xyL/xyR (n, 2)."""
    ctx = ctx or default_context()
    L, R = _as_u8(imgL), _as_u8(imgR)
    xyL = np.ascontiguousarray(xyL, np.int32)
    xyR = np.ascontiguousarray(xyR, np.int32)
    n = len(xyL)
    pw, ph = patch
    out = np.zeros(n, np.float32)
    if n == 0:
        return out
    ctx.check(ctx.lib.me_mi_scores(ctx.h, ME_HOST, vptr(L), L.shape[1], vptr(R), R.shape[1], L.shape[1], L.shape[0],
                                   vptr(xyL), vptr(xyR), n, pw, ph, vptr(out)), "me_mi_scores")
    return out


def mi_scores_device(ctx: Context, dL: int, strideL: int, dR: int, strideR: int, width: int, height: int,
                     dxyL: int, dxyR: int, n: int, patch, dout: int):
    """Asynchronous form on device pointers (e.g. torch tensors' data_ptr())."""
    pw, ph = patch
    ctx.check(ctx.lib.me_mi_scores(ctx.h, ME_DEVICE, ctypes.c_void_p(dL), strideL, ctypes.c_void_p(dR), strideR,
                                   width, height, ctypes.c_void_p(dxyL), ctypes.c_void_p(dxyR), n, pw, ph,
                                   ctypes.c_void_p(dout)), "me_mi_scores(device)")


def _float_pairs(A, B):
    A = np.ascontiguousarray(A, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    single = A.ndim == 2
    if single:
        A, B = A[None], B[None]
    if A.shape != B.shape or A.ndim != 3 or A.shape[1] == 0 or A.shape[2] == 0:
        raise ValueError("patch pairs must be equal-size, non-empty float patches")
    return A, B, single


def _pair_op(fn, name, A, B, ctx):
    ctx = ctx or default_context()
    A, B, single = _float_pairs(A, B)
    out = np.zeros(len(A), np.float32)
    ctx.check(getattr(ctx.lib, fn)(ctx.h, ME_HOST, vptr(A), vptr(B), len(A), A.shape[1], A.shape[2], vptr(out)), fn)
    return float(out[0]) if single else out


def comparePC(PC1, PC2, ctx: Context | None = None):
    """me::comparePC(const Mat&, const Mat&) -> float; (n, r, c) stacks give n scores."""
    return _pair_op("me_compare_pc", "comparePC", PC1, PC2, ctx)


def applyCCOEFFNormed(r1, r2, ctx: Context | None = None):
    """me::applyCCOEFFNormed(const Mat&, const Mat&) -> float; (n, r, c) stacks give n scores."""
    return _pair_op("me_ccoeff_normed", "applyCCOEFFNormed", r1, r2, ctx)


def quantise(img, rng, ctx: Context | None = None) -> np.ndarray:
    """me::quantise(cv::Mat& img, pair<uchar,uchar> range): returns the quantised copy
    (the reference modifies its argument in place; numpy arrays given as uint8 are too)."""
    ctx = ctx or default_context()
    lo, hi = int(rng[0]), int(rng[1])
    a = np.asarray(img)
    inplace = a.dtype == np.uint8 and a.flags.c_contiguous and a.ndim == 2
    buf = a if inplace else np.array(a, np.uint8, order="C")
    h, w = buf.shape
    ctx.check(ctx.lib.me_quantise(ctx.h, ME_HOST, vptr(buf), w, w, h, lo, hi), "me_quantise")
    return buf
