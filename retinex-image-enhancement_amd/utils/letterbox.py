"""YOLO-style letterbox (drop-in for reference utils/letterbox.py:9-102).

The geometry (scale ratio, unpadded size, border split) is host scalar math as
in the reference; the pixels -- the (x*255).astype(uint8) quantisation of
letterbox_tensor, cv2.resize INTER_LINEAR in OpenCV's 8-bit fixed point
(11-bit coefficients, tables built here on the host as OpenCV builds them
and kept on the device per (size, device)),
the grey-114 border and the /255 -- are ONE device launch (upr_letterbox).
With the harness's default call (new_shape = the image's own size,
scaleup=False) it is the uint8 round trip, exact for 8-bit inputs.

Device only, like every other op of this package: a CPU tensor is moved to the
current ROCm device and the result is returned on the input's device (the
reference returns CPU tensors; the harness moves them to the device next).
cv2 is absent here, so the resize arithmetic is "parity unpinned" (DESIGN.md);
its CPU restatement is oracle/letterbox.py (test infrastructure).
"""
import math

import numpy as np
import torch

from upr import _lib as L

_COEF_SCALE = 1 << 11


def linear_taps(dst, src):
    """OpenCV resize INTER_LINEAR source indices / 11-bit weights along one axis
    -> int32 [4][dst] (index 0, index 1, weight 0, weight 1).  Vectorised, in
    OpenCV's arithmetic: fx = (float)((dx + 0.5) * scale - 0.5) in double, the
    fraction and the 2^11 weights in float32, weights rounded half to even."""
    scale = src / dst
    f = ((np.arange(dst, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo, hi = s < 0, s >= src - 1
    f[lo | hi] = np.float32(0)
    s = np.where(lo, 0, np.where(hi, src - 1, s))
    t = np.empty((4, dst), np.int32)
    t[0] = s
    t[1] = np.minimum(s + 1, src - 1)
    t[2] = np.rint((np.float32(1) - f) * np.float32(_COEF_SCALE)).astype(np.int32)
    t[3] = np.rint(f * np.float32(_COEF_SCALE)).astype(np.int32)
    return t


# device copies of the tap tables per (dst, src, device): a directory of frames
# of one size builds and uploads them once, not per call
_TAPS = {}
_TAPS_MAX = 64


def _device_taps(dst, src, dev):
    key = (dst, src, str(dev))
    t = _TAPS.get(key)
    if t is None:
        if len(_TAPS) >= _TAPS_MAX:
            _TAPS.pop(next(iter(_TAPS)))
        t = _TAPS[key] = torch.from_numpy(linear_taps(dst, src)).to(dev)
    return t


def letterbox_geometry(shape, new_shape=640, auto=True, scale_fill=False, scaleup=True):
    """Reference letterbox.py:21-52 -> (new_unpad (w, h), ratio, (dw, dh), (top, bottom, left, right))."""
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
    border = (int(round(dh - 0.1)), int(round(dh + 0.1)), int(round(dw - 0.1)), int(round(dw + 0.1)))
    return new_unpad, ratio, (dw, dh), border


def _device(t):
    if not torch.cuda.is_available():
        raise RuntimeError("letterbox runs on ROCm devices only (no CPU fallback)")
    return t.device if t.device.type == "cuda" else torch.device("cuda", torch.cuda.current_device())


def _run(src, src_kind, H, W, new_shape, color, auto, scale_fill, scaleup, out_kind):
    (nw, nh), ratio, pad, (top, bottom, left, right) = letterbox_geometry((H, W), new_shape, auto, scale_fill,
                                                                          scaleup)
    Ho, Wo = nh + top + bottom, nw + left + right
    dev = src.device
    xt = yt = None
    if (nw, nh) != (W, H):
        xt = _device_taps(nw, W, dev)
        yt = _device_taps(nh, H, dev)
    if out_kind == 0:
        out = torch.empty((3, Ho, Wo), dtype=torch.float32, device=dev)
    else:
        out = torch.empty((Ho, Wo, 3), dtype=torch.uint8, device=dev)
    col = int(color[0]) | (int(color[1]) << 8) | (int(color[2]) << 16)
    with torch.cuda.device(dev):
        rc = L.lib().upr_letterbox(src.data_ptr(), src_kind, H, W, top, left, nh, nw, Ho, Wo,
                                   xt.data_ptr() if xt is not None else None,
                                   yt.data_ptr() if yt is not None else None, col, out.data_ptr(), out_kind,
                                   torch.cuda.current_stream(dev).cuda_stream)
    L.check(rc, "upr_letterbox")
    return out, ratio, pad


def letterbox(img, new_shape=640, color=(114, 114, 114), auto=True, scale_fill=False, scaleup=True):
    """Reference letterbox.py:9-62: uint8 HWC RGB array (numpy, or a uint8
    tensor) -> (letterboxed uint8 HWC, ratio, (dw, dh)); numpy in, numpy out."""
    as_numpy = isinstance(img, np.ndarray)
    t = torch.from_numpy(np.ascontiguousarray(img)) if as_numpy else img
    if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] != 3:
        raise ValueError("letterbox expects a uint8 H x W x 3 image")
    t = t.to(_device(t)).contiguous()
    out, ratio, pad = _run(t, 0, t.shape[0], t.shape[1], new_shape, color, auto, scale_fill, scaleup, 1)
    return (out.cpu().numpy() if as_numpy else out), ratio, pad


def letterbox_tensor(img_tensor, new_shape=640, color=(114, 114, 114), auto=True, scale_fill=False, scaleup=True):
    """Reference letterbox.py:65-102: [3,H,W] float in [0,1] -> letterboxed
    [3,H',W'] float (the (x*255).astype(uint8) quantisation included)."""
    if img_tensor.dim() != 3 or img_tensor.shape[0] != 3:
        raise ValueError("letterbox_tensor expects a [3, H, W] tensor")
    dev = _device(img_tensor)
    t = img_tensor.detach().to(dev, torch.float32).contiguous()
    return _run(t, 1, t.shape[1], t.shape[2], new_shape, color, auto, scale_fill, scaleup, 0)


def letterbox_u8_image(img_u8_hwc, new_shape, color=(114, 114, 114), auto=True, scale_fill=False, scaleup=False,
                       device=None):
    """Harness fast path: a decoded uint8 HWC image goes to the device as bytes
    (3 B/pixel over PCIe, not 12) and comes back as the letterboxed [3,H',W']
    float tensor -- ToTensor + letterbox_tensor in one launch (bit-identical:
    (k/255)*255 quantises back to k)."""
    t = torch.from_numpy(np.ascontiguousarray(img_u8_hwc))
    dev = device if device is not None else _device(t)
    t = t.to(dev)
    return _run(t, 0, t.shape[0], t.shape[1], new_shape, color, auto, scale_fill, scaleup, 0)
