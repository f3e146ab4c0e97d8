"""Tensor-level wrappers over libupr.so.

PyTorch is used only for device memory and streams: every compute call goes
through the C ABI with raw device pointers and the caller's current HIP stream.
Non-ROCm tensors are rejected (no CPU fallback).
"""
import ctypes

import torch

from . import _lib as L

_DT = {torch.float32: L.UPR_F32, torch.float16: L.UPR_F16}


def dtype_code(dt):
    if dt not in _DT:
        raise TypeError(f"UP-Retinex HIP path supports float32 and float16 tensors, got {dt}")
    return _DT[dt]


def _require_device(t, name="input"):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{name} is on '{t.device}': the UP-Retinex framework executes on ROCm devices only "
            f"(MI355X HIP kernels); move the model and the tensor to a 'cuda' (ROCm) device")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


class _Workspace:
    """Grow-only scratch buffer per (device, HIP stream), torch-allocated.

    Keyed by the caller's current stream: work issued on two streams never
    shares scratch, and a buffer is allocated on (and, when it grows, released
    to torch's caching allocator from) the stream that uses it, so the
    allocator's stream ordering keeps a replaced buffer alive until the work
    queued on that stream has drained (include/upr.h: thread-safe across
    distinct handles or streams).  At most MAX_STREAMS buffers are kept (least
    recently used evicted), so code that makes a new stream per request does
    not pin a buffer per stream; an evicted buffer returns to torch's caching
    allocator, which reuses it on its own stream only (stream-ordered safe)."""

    MAX_STREAMS = 8

    def __init__(self):
        from collections import OrderedDict
        self.buf = OrderedDict()

    def get(self, dev, nbytes):
        stream = torch.cuda.current_stream(dev)
        key = (dev.type, dev.index, stream.cuda_stream)
        b = self.buf.pop(key, None)
        if b is None or b.numel() < nbytes:
            with torch.cuda.stream(stream):
                b = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
        self.buf[key] = b  # most recently used last
        while len(self.buf) > self.MAX_STREAMS:
            self.buf.popitem(last=False)
        return b


_WS = _Workspace()


class ModelHandle:
    """Owns one UprModel* (packed device weights) built from a state_dict."""

    def __init__(self, state_dict, use_preact, use_aspp, dtype, device, ienet_only=False, prefix="", head_only=False):
        lib = L.lib()
        self.dtype = dtype
        self.device = device
        self.ienet_only = ienet_only
        self.head_only = head_only
        names, descs, keep = [], [], []
        for k, v in state_dict.items():
            if not torch.is_floating_point(v):
                continue  # num_batches_tracked
            t = v.detach().to("cpu", torch.float32).contiguous()
            keep.append(t)
            nm = (prefix + k).encode()
            names.append(nm)
            d = L.UprTensorDesc()
            d.name = nm
            d.data = ctypes.cast(t.data_ptr(), ctypes.POINTER(ctypes.c_float))
            d.ndim = t.dim()
            for i, s in enumerate(t.shape):
                d.shape[i] = s
            descs.append(d)
        arr = (L.UprTensorDesc * len(descs))(*descs)
        out = ctypes.c_void_p()
        flags = (L.UPR_MODEL_IENET_ONLY if ienet_only else 0) | (L.UPR_MODEL_HEAD_ONLY if head_only else 0)
        with torch.cuda.device(device):
            rc = lib.upr_model_create(arr, len(descs), int(bool(use_preact)), int(bool(use_aspp)),
                                      dtype_code(dtype), flags, ctypes.byref(out))
        L.check(rc, "upr_model_create")
        self._h = out
        self._lib = lib

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and h.value:
            try:
                self._lib.upr_model_destroy(h)
            except Exception:
                pass
            self._h = None

    def profile(self, enable=True):
        """Record a HIP event pair around every op of later forwards."""
        L.check(self._lib.upr_model_profile(self._h, int(bool(enable))), "upr_model_profile")

    def forks(self):
        """Forwards so far that ran the two-stream (multi-scale side stream) schedule."""
        return int(self._lib.upr_model_forks(self._h))

    def profile_read(self):
        """Per-op stats (launch order): list of dicts name/kind/calls/ms/flops/bytes."""
        n = ctypes.c_int(0)
        L.check(self._lib.upr_model_profile_read(self._h, None, 0, ctypes.byref(n)), "upr_model_profile_read")
        arr = (L.UprOpStat * max(n.value, 1))()
        L.check(self._lib.upr_model_profile_read(self._h, arr, n.value, ctypes.byref(n)), "upr_model_profile_read")
        return [{"name": a.name.decode(), "kind": "conv_igemm" if a.kind == L.UPR_OP_CONV_IGEMM else "other",
                 "calls": a.calls, "ms": a.ms, "flops": a.flops, "bytes": a.bytes} for a in arr[:n.value]]

    def enhance(self, x, refl):
        """HEAD_ONLY handle: multi_scale_enhance(x, refl) -> enhanced [B,3,H,W]."""
        _require_device(x)
        _require_device(refl, "reflectance")
        if x.dim() != 4 or x.shape[1] != 3 or refl.shape != x.shape:
            raise RuntimeError(f"expected x and reflectance of one shape [B, 3, H, W], got {tuple(x.shape)} and "
                               f"{tuple(refl.shape)}")
        if x.dtype != self.dtype or refl.dtype != self.dtype:
            raise RuntimeError(f"input dtypes {x.dtype}/{refl.dtype} do not match model dtype {self.dtype}")
        x, refl = x.contiguous(), refl.contiguous()
        B, _, H, W = x.shape
        dev = x.device
        with torch.cuda.device(dev):
            enh = torch.empty_like(x)
            nbytes = self._lib.upr_model_workspace(self._h, B, H, W)
            ws = _WS.get(dev, nbytes)
            rc = self._lib.upr_model_forward(self._h, _ptr(x), B, H, W, _ptr(enh), _ptr(refl), None,
                                             _ptr(ws), ctypes.c_size_t(ws.numel()), _stream(dev))
        L.check(rc, "upr_model_forward(head only)")
        return enh

    def forward(self, x):
        _require_device(x)
        if x.dim() != 4 or x.shape[1] != 3:
            raise RuntimeError(f"expected input of shape [B, 3, H, W], got {tuple(x.shape)}")
        if x.dtype != self.dtype:
            raise RuntimeError(f"input dtype {x.dtype} does not match model dtype {self.dtype}")
        x = x.contiguous()
        B, _, H, W = x.shape
        dev = x.device
        with torch.cuda.device(dev):
            illu = torch.empty((B, 1, H, W), dtype=x.dtype, device=dev)
            if self.ienet_only:
                enh = refl = None
            else:
                enh = torch.empty((B, 3, H, W), dtype=x.dtype, device=dev)
                refl = torch.empty_like(enh)
            nbytes = self._lib.upr_model_workspace(self._h, B, H, W)
            ws = _WS.get(dev, nbytes)
            rc = self._lib.upr_model_forward(self._h, _ptr(x), B, H, W, _ptr(enh), _ptr(refl), _ptr(illu),
                                             _ptr(ws), ctypes.c_size_t(ws.numel()), _stream(dev))
        L.check(rc, "upr_model_forward")
        return enh, refl, illu


# ---------------------------------------------------------------------------
# enhancer / op wrappers
# ---------------------------------------------------------------------------
def clahe_enhance(enh, clip=2.0, tiles=(8, 8)):
    """Batched apply_clahe_enhancement: [B,3,H,W] float -> [B,3,H,W] float."""
    _require_device(enh)
    enh = enh.contiguous()
    B, C, H, W = enh.shape
    if C != 3:
        raise RuntimeError("clahe_enhance expects 3 channels")
    lib = L.lib()
    out = torch.empty_like(enh)
    with torch.cuda.device(enh.device):
        ws = _WS.get(enh.device, lib.upr_clahe_enhance_workspace(B, H, W, tiles[0], tiles[1]))
        rc = lib.upr_clahe_enhance(_ptr(enh), _ptr(out), _ptr(ws), B, H, W, float(clip), int(tiles[0]),
                                   int(tiles[1]), dtype_code(enh.dtype), _stream(enh.device))
    L.check(rc, "upr_clahe_enhance")
    return out


def gray_hist(x):
    _require_device(x)
    x = x.contiguous()
    B, C, H, W = x.shape
    hist = torch.empty((B, 256), dtype=torch.int32, device=x.device)
    with torch.cuda.device(x.device):
        rc = L.lib().upr_gray_hist(_ptr(x), _ptr(hist), B, H, W, dtype_code(x.dtype), _stream(x.device))
    L.check(rc, "upr_gray_hist")
    return hist


def multiscale(x, enh=None):
    """Returns (out or None, factor[B] float64, sums[B,3] float64)."""
    _require_device(x)
    x = x.contiguous()
    B, C, H, W = x.shape
    sums = torch.empty((B, 3), dtype=torch.float64, device=x.device)
    factor = torch.empty((B,), dtype=torch.float64, device=x.device)
    out = None
    if enh is not None:
        enh = enh.contiguous()
        if enh.shape != x.shape or enh.dtype != x.dtype:
            raise RuntimeError("multiscale: enhanced image must match the input's shape and dtype")
        out = torch.empty_like(enh)
    with torch.cuda.device(x.device):
        rc = L.lib().upr_multiscale(_ptr(x), _ptr(enh), _ptr(out), _ptr(sums), _ptr(factor), B, H, W,
                                    dtype_code(x.dtype), _stream(x.device))
    L.check(rc, "upr_multiscale")
    return out, factor, sums


def quantize_u8(x):
    _require_device(x)
    x = x.contiguous()
    out = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    with torch.cuda.device(x.device):
        rc = L.lib().upr_quantize_u8(_ptr(x), _ptr(out), x.numel(), dtype_code(x.dtype), _stream(x.device))
    L.check(rc, "upr_quantize_u8")
    return out


def to_u8_hwc(x):
    """save_image pixels: one [C,H,W] image (C 1 or 3) -> u8 [H,W,3] on the device."""
    _require_device(x)
    x = x.contiguous()
    C, H, W = x.shape
    out = torch.empty((H, W, 3), dtype=torch.uint8, device=x.device)
    with torch.cuda.device(x.device):
        rc = L.lib().upr_to_u8_hwc(_ptr(x), C, H, W, dtype_code(x.dtype), _ptr(out), _stream(x.device))
    L.check(rc, "upr_to_u8_hwc")
    return out


def rgb2lab_u8(rgb):
    """rgb: [..., 3] uint8 interleaved."""
    _require_device(rgb)
    rgb = rgb.contiguous()
    lab = torch.empty_like(rgb)
    with torch.cuda.device(rgb.device):
        rc = L.lib().upr_rgb2lab_u8(_ptr(rgb), _ptr(lab), rgb.numel() // 3, _stream(rgb.device))
    L.check(rc, "upr_rgb2lab_u8")
    return lab


def lab2rgb_u8(lab):
    _require_device(lab)
    lab = lab.contiguous()
    rgb = torch.empty_like(lab)
    with torch.cuda.device(lab.device):
        rc = L.lib().upr_lab2rgb_u8(_ptr(lab), _ptr(rgb), lab.numel() // 3, _stream(lab.device))
    L.check(rc, "upr_lab2rgb_u8")
    return rgb


def clahe_u8(src, clip=2.0, tiles=(8, 8)):
    """src: [B,H,W] or [H,W] uint8 -> same shape."""
    _require_device(src)
    squeeze = src.dim() == 2
    s = (src.unsqueeze(0) if squeeze else src).contiguous()
    B, H, W = s.shape
    dst = torch.empty_like(s)
    lut = torch.empty(B * tiles[0] * tiles[1] * 256, dtype=torch.uint8, device=s.device)
    with torch.cuda.device(s.device):
        rc = L.lib().upr_clahe_u8(_ptr(s), _ptr(dst), _ptr(lut), B, H, W, float(clip), int(tiles[0]),
                                  int(tiles[1]), _stream(s.device))
    L.check(rc, "upr_clahe_u8")
    return dst[0] if squeeze else dst


def pack_conv_weight(w):
    """torch conv weight [Cout, Cin, kh, kw] -> packed [Cout, kh*kw*Cin] (tap-major)."""
    co, ci, kh, kw = w.shape
    return w.permute(0, 2, 3, 1).reshape(co, kh * kw * ci).contiguous()


def conv2d_nhwc(x, w_packed, bias, kh, kw, stride=1, pad=0, dil=1, residual=None, relu=False):
    """x [B,H,W,Cin] -> y [B,Ho,Wo,Cout] through the implicit-GEMM MFMA kernel."""
    _require_device(x)
    x = x.contiguous()
    B, H, W, Cin = x.shape
    Cout = w_packed.shape[0]
    Ho = (H + 2 * pad - dil * (kh - 1) - 1) // stride + 1
    Wo = (W + 2 * pad - dil * (kw - 1) - 1) // stride + 1
    y = torch.empty((B, Ho, Wo, Cout), dtype=x.dtype, device=x.device)
    if residual is not None:
        residual = residual.contiguous()
    with torch.cuda.device(x.device):
        rc = L.lib().upr_conv2d_nhwc(_ptr(x), B, H, W, Cin, _ptr(w_packed.contiguous()), _ptr(bias), Cout, kh, kw,
                                     stride, pad, dil, _ptr(residual), int(bool(relu)), _ptr(y),
                                     dtype_code(x.dtype), _stream(x.device))
    L.check(rc, "upr_conv2d_nhwc")
    return y


def lab_tables():
    """Host copies of the 8-bit Lab tables (no device needed)."""
    import numpy as np
    g = np.zeros(256, np.uint16)
    c = np.zeros(3072, np.uint16)
    yf = np.zeros(512, np.uint16)
    ig = np.zeros(4096, np.uint16)
    m1 = np.zeros(9, np.int32)
    m2 = np.zeros(9, np.int32)
    L.lib().upr_lab_tables(g.ctypes.data, c.ctypes.data, yf.ctypes.data, ig.ctypes.data, m1.ctypes.data,
                           m2.ctypes.data)
    return {"gamma": g, "cbrt": c, "yf": yf, "invgamma": ig, "rgb2xyz": m1, "xyz2rgb": m2}


def multiscale_features(x, scale_idx):
    """[B,3,H,W] -> [B,7,hs,ws] feature maps of scale 0 (x1), 1 (x0.5) or 2 (x0.25)."""
    _require_device(x)
    x = x.contiguous()
    B, C, H, W = x.shape
    s = (1.0, 0.5, 0.25)[scale_idx]
    hs, ws = (H, W) if scale_idx == 0 else (int(H * s), int(W * s))
    out = torch.empty((B, 7, hs, ws), dtype=x.dtype, device=x.device)
    with torch.cuda.device(x.device):
        rc = L.lib().upr_multiscale_features(_ptr(x), _ptr(out), B, H, W, int(scale_idx), dtype_code(x.dtype),
                                             _stream(x.device))
    L.check(rc, "upr_multiscale_features")
    return out


def content_aware(x, enh=None, saliency=False, attention=False):
    """Returns (out or None, saliency [B,H,W] f32 or None, attention [B,H,W] f32 or None)."""
    _require_device(x)
    x = x.contiguous()
    B, C, H, W = x.shape
    dev = x.device
    out = None
    if enh is not None:
        enh = enh.contiguous()
        if enh.shape != x.shape or enh.dtype != x.dtype:
            raise RuntimeError("content_aware: enhanced image must match the input's shape and dtype")
        out = torch.empty_like(enh)
    sal = torch.empty((B, H, W), dtype=torch.float32, device=dev) if saliency else None
    att = torch.empty((B, H, W), dtype=torch.float32, device=dev) if attention else None
    lib = L.lib()
    with torch.cuda.device(dev):
        nbytes = lib.upr_content_aware_workspace(B, H, W)
        ws = _WS.get(dev, nbytes)
        rc = lib.upr_content_aware(_ptr(x), _ptr(enh), _ptr(out), _ptr(sal), _ptr(att), _ptr(ws),
                                   ctypes.c_size_t(ws.numel()), B, H, W, dtype_code(x.dtype), _stream(dev))
    L.check(rc, "upr_content_aware")
    return out, sal, att


class _Decompose(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, illu):
        B, C, H, W = x.shape
        refl = torch.empty_like(x)
        with torch.cuda.device(x.device):
            rc = L.lib().upr_retinex_decompose(_ptr(x), _ptr(illu), _ptr(refl), B, C, H, W, illu.shape[1],
                                               dtype_code(x.dtype), _stream(x.device))
        L.check(rc, "upr_retinex_decompose")
        ctx.save_for_backward(x, illu)
        return refl

    @staticmethod
    def backward(ctx, g):
        x, illu = ctx.saved_tensors
        B, C, H, W = x.shape
        gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        gi = torch.empty_like(illu) if ctx.needs_input_grad[1] else None
        g = g.contiguous().to(x.dtype)
        with torch.cuda.device(x.device):
            rc = L.lib().upr_retinex_decompose_bwd(_ptr(x), _ptr(illu), _ptr(g), _ptr(gx), _ptr(gi), B, C, H, W,
                                                   illu.shape[1], dtype_code(x.dtype), _stream(x.device))
        L.check(rc, "upr_retinex_decompose_bwd")
        return gx, gi


def retinex_decompose(x, illu):
    """x / (illu + 1e-6) (models/model.py:405-413) on the device, illu [B,1,H,W]
    broadcast over the channels (or [B,C,H,W]); differentiable in x and illu."""
    _require_device(x)
    _require_device(illu, "illumination")
    if x.dim() != 4 or illu.dim() != 4 or illu.shape[0] != x.shape[0] or illu.shape[2:] != x.shape[2:] or \
            illu.shape[1] not in (1, x.shape[1]):
        raise RuntimeError(f"retinex_decompose: shapes {tuple(x.shape)} and {tuple(illu.shape)} do not broadcast "
                           f"as [B,C,H,W] / [B,1 or C,H,W]")
    if x.dtype != illu.dtype:
        raise RuntimeError(f"retinex_decompose: dtype mismatch {x.dtype} vs {illu.dtype}")
    dtype_code(x.dtype)
    return _Decompose.apply(x.contiguous(), illu.contiguous())
