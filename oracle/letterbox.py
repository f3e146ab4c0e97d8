"""CPU restatement of the reference's letterbox (utils/letterbox.py:9-62) on
uint8 HWC numpy arrays, with cv2.resize INTER_LINEAR in OpenCV's 8-bit fixed
point (11-bit coefficients; horizontal pass in integers, vertical pass as
OpenCV's VResizeLinearVec_32s8u: >>4, two >>16 products, (v+2)>>2).

TEST INFRASTRUCTURE ONLY: the checker for the device letterbox kernel
(upr_letterbox).  cv2 is not installed here and no OpenCV version is pinned by
the reference, so the resize arithmetic is "parity unpinned" (DESIGN.md §5):
it follows OpenCV 4.x's published resize.cpp and is checked against hand-derived
properties (identity, constants, convex combination) in tests/test_cpu_harness.py.
"""
import math

import numpy as np
import torch

_COEF_BITS = 11
_COEF_SCALE = 1 << _COEF_BITS


def _round(v):
    # cvRound on float: round half to even
    return int(np.rint(v))


def linear_taps(dst, src):
    """OpenCV resize INTER_LINEAR source index / fixed-point weights along one axis."""
    scale = src / dst
    idx0 = np.zeros(dst, np.int64)
    idx1 = np.zeros(dst, np.int64)
    w0 = np.zeros(dst, np.int64)
    w1 = np.zeros(dst, np.int64)
    for d in range(dst):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(math.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            f, s = np.float32(0), 0
        if s >= src - 1:
            f, s = np.float32(0), src - 1
        idx0[d] = s
        idx1[d] = min(s + 1, src - 1)
        w0[d] = _round(np.float32(np.float32(1) - f) * np.float32(_COEF_SCALE))
        w1[d] = _round(f * np.float32(_COEF_SCALE))
    return idx0, idx1, w0, w1


def resize_linear_u8(img, new_wh):
    """cv2.resize(img, (W', H'), interpolation=INTER_LINEAR) for uint8 HWC."""
    img = np.asarray(img, np.uint8)
    H, W = img.shape[:2]
    nw, nh = new_wh
    x0, x1, a0, a1 = linear_taps(nw, W)
    y0, y1, b0, b1 = linear_taps(nh, H)
    s = img.astype(np.int64)
    rows = s[:, x0] * a0[None, :, None] + s[:, x1] * a1[None, :, None]      # horizontal pass (int)
    r0, r1 = rows[y0] >> 4, rows[y1] >> 4                                    # VResizeLinearVec_32s8u
    v = ((r0 * b0[:, None, None]) >> 16) + ((r1 * b1[:, None, None]) >> 16)
    return np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)


def letterbox(img, new_shape=640, color=(114, 114, 114), auto=True, scale_fill=False, scaleup=True):
    """Reference utils/letterbox.py:9-62 on a uint8 HWC array."""
    shape = img.shape[:2]
    if isinstance(new_shape, int):
        new_shape = (new_shape, new_shape)
    r = min(new_shape[0] / shape[0], new_shape[1] / shape[1])
    if not scaleup:
        r = min(r, 1.0)
    ratio = r, r
    new_unpad = int(round(shape[1] * r)), int(round(shape[0] * r))
    dw, dh = new_shape[1] - new_unpad[0], new_shape[0] - new_unpad[1]
    if auto:
        dw, dh = np.mod(dw, 32), np.mod(dh, 32)
    elif scale_fill:
        dw, dh = 0.0, 0.0
        new_unpad = (new_shape[1], new_shape[0])
        ratio = new_shape[1] / shape[1], new_shape[0] / shape[0]
    dw /= 2
    dh /= 2
    if shape[::-1] != new_unpad:
        img = resize_linear_u8(img, new_unpad)
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    if top or bottom or left or right:
        out = np.empty((img.shape[0] + top + bottom, img.shape[1] + left + right) + img.shape[2:], np.uint8)
        out[...] = np.asarray(color, np.uint8)[: img.shape[2]] if img.ndim == 3 else color[0]
        out[top:top + img.shape[0], left:left + img.shape[1]] = img
        img = out
    return img, ratio, (dw, dh)
