"""Training engine: explicit forward + backward of MultiScaleUP_Retinex on the
gfx950 kernels of include/upr_train.h (+ the inference conv kernels).

Reference: trainers/train.py:63-103 runs `model(img_low)` in train mode,
`criterion(...)` (losses/loss.py TotalLoss), `loss.backward()`,
`clip_grad_norm_(1.0)` and `Adam.step()` on PyTorch autograd.  Here the same
step is a fixed graph written out by hand: every layer object below owns the
forward kernels of one reference module and the matching backward kernels;
activations the backward needs are kept from the forward.  PyTorch only
allocates device memory (torch.empty) and supplies the stream; there is no
autograd tape and no torch compute.

Layouts: network input / outputs NCHW (the reference's tensors), every
activation NHWC fp32 (`Act`, possibly a channel slice of a concat buffer).
Parameters and their gradients live in ONE flat fp32 buffer each
(`FlatParams`), so clip_grad_norm_ and Adam are single launches.
"""
import ctypes
import os
import sys

import torch

from . import _lib as L

F32 = torch.float32


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_dev = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    """The current HIP stream of the current device (torch's), as the C ABI's
    void*.  Read through torch's raw accessors when present: the ~600 launches
    of a training step each ask, and torch.cuda.current_stream() builds a
    Stream object per call (~1 ms of host time per step)."""
    if _raw_stream is not None and _cur_dev is not None:
        return ctypes.c_void_p(_raw_stream(_cur_dev()))
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _chk(rc, what):
    L.check(rc, what)


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _fp(t, off=0):
    """Pointer to element `off` of a fp32 tensor."""
    return ctypes.c_void_p(t.data_ptr() + 4 * off) if t is not None else None


def empty(shape, dev):
    return torch.empty(shape, dtype=F32, device=dev)


# Autocast (AMP) arithmetic.  The reference runs the model forward and the
# loss under torch.cuda.amp.autocast() when use_amp (trainers/train.py:71-75),
# i.e. its convolutions in fp16.  The graph / loss engine set this flag from
# the caller's autocast state at forward time; while set, MFMA convs (and the
# input gradients of their backward) run on the fp16 kernels with fp32
# accumulation and fp32 activations in between (upr_t_conv_mfma16).  Weight
# gradients, BatchNorm, losses, FFTs and the optimiser stay fp32.
_AMP = [False]


# fp16-only activation stores (the FAM / ASPP concats, FAM branch and pool
# outputs, scale stems) where no reader needs the fp32 value; False writes the
# fp32 values too (the gradients must not change: tests/test_gpu_train.py
# test_amp_fp16_only_stores_bitwise)
_TRACE_CAST = os.environ.get("UPR_TRACE_CAST", "0") == "1"
FP16_ONLY_STORES = [True]


def autocast_active():
    """True inside torch.autocast('cuda') (any half dtype: the kernels compute fp16)."""
    try:
        return bool(torch.is_autocast_enabled("cuda"))
    except TypeError:  # older signature
        return bool(torch.is_autocast_enabled())


def set_amp(on):
    _AMP[0] = bool(on)


def _h16(n, dev):
    return torch.empty((n,), dtype=torch.float16, device=dev)


# Per-call device timing of the conv launches (bench.py's training roofline).
# While profile_begin() is active every conv call below records a HIP event
# pair on the current stream around its library call(s), tagged with its
# arithmetic ("mfma16": fp16 MFMA with fp32 accumulation, "mfma32": fp32
# MFMA, "direct": FMA kernels) and its ALGORITHMIC flops 2*B*Ho*Wo*Cout*Cin*k^2
# (forward, input gradient and weight gradient each count one such product;
# the zero-upsampled stride-2 input gradient executes 4x that and is charged 1x).
_PROF = [None]


def profile_begin():
    _PROF[0] = []


def profile_end():
    """Stops recording; returns [(kind, what, flops, ms, shape)] (synchronises);
    shape: (Cin, Cout, k, stride, H, W) of the conv's input, or None."""
    recs, _PROF[0] = _PROF[0], None
    if not recs:
        return []
    torch.cuda.synchronize()
    return [(k, w, f, e0.elapsed_time(e1), sh) for k, w, f, e0, e1, sh in recs]


class _timed:
    __slots__ = ("rec",)

    def __init__(self, kind, what, flops, shape=None):
        self.rec = None
        if _PROF[0] is not None and kind is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            self.rec = [kind, what, flops, e0, e1, shape]

    def __enter__(self):
        if self.rec is not None:
            self.rec[3].record()
        return self

    def __exit__(self, *exc):
        if self.rec is not None:
            self.rec[4].record()
            _PROF[0].append(tuple(self.rec))
        return False


class Act:
    """NHWC activation: channels [coff, coff+C) of a [B,H,W,cs] fp32 tensor.

    `fresh` marks a gradient buffer nothing has written yet: the first
    producer overwrites (or zeroes it when it scatters with atomics), later
    producers accumulate."""

    def __init__(self, t, C=None, coff=0):
        assert t.dim() == 4 and t.dtype == F32 and t.is_contiguous()
        self.t = t
        self.B, self.H, self.W, self.cs = t.shape
        self.C = self.cs if C is None else C
        self.coff = coff
        self.fresh = False
        self.t16 = None  # compact fp16 copy written by its producer (autocast conv input), or None
        self.t16_grad = False  # t16 of a gradient: written by the fused BN backward (BN.bwd), trusted by dgrad
        self.stale32 = False  # fp32 t left behind by relu_mask(only16): t16 is the gradient's only value
        # t16 is a whole concat's fp16 copy its channel slices read in place (element (m, c) of
        # a slice at t16[m * cs + coff + c]): set by the producer of a concat gradient whose
        # slices are only read afterwards (EnhancedFAM's fusion input gradient)
        self.t16_shared = False

    @staticmethod
    def new(B, H, W, C, dev, fresh=True):
        a = Act(empty((B, H, W, C), dev))
        a.fresh = fresh
        return a

    def slice(self, coff, C):
        s = Act(self.t, C, self.coff + coff)
        s.fresh = self.fresh
        if self.t16_shared and self.t16 is not None:
            s.t16, s.t16_grad, s.t16_shared, s.stale32 = self.t16, self.t16_grad, True, self.stale32
        return s

    def whole16(self):
        """t16 is this Act's own compact copy (not a slice of a shared one)."""
        return self.coff == 0 and self.cs == self.C

    @property
    def M(self):
        return self.B * self.H * self.W

    def ptr(self):
        return _fp(self.t, self.coff)

    def view(self):
        return L.UprView(self.t.data_ptr() + 4 * self.coff, self.H * self.W * self.cs, self.W * self.cs, self.cs, 1)

    def zero_if_fresh(self):
        if self.fresh:
            _chk(L.lib().upr_t_zero(_p(self.t), self.t.numel() * 4, _stream()), "zero")
            self.fresh = False

    def consume_fresh(self):
        """Returns 1 (accumulate) or 0 (overwrite) for the next producer."""
        acc = 0 if self.fresh else 1
        self.fresh = False
        self.t16 = None
        self.t16_grad = False
        self.t16_shared = False
        self.stale32 = False
        return acc


def nchw_view(t, coff=0):
    B, C, H, W = t.shape
    return L.UprView(t.data_ptr() + 4 * coff * H * W, C * H * W, W, 1, H * W)


def zero(t):
    _chk(L.lib().upr_t_zero(_p(t), t.numel() * t.element_size(), _stream()), "zero")


class FlatParams:
    """All trainable parameters of a module in one flat device buffer (and the
    gradients in another); each nn.Parameter's .data / .grad become views.
    Order = module.named_parameters() (the reference optimiser's order)."""

    def __init__(self, module):
        params = list(module.named_parameters()) if hasattr(module, "named_parameters") else \
            [(str(i), p) for i, p in enumerate(module)]
        dev = params[0][1].device
        if dev.type != "cuda":
            raise RuntimeError("HIP training needs the parameters on a ROCm device (model.to('cuda'))")
        align = 16  # 64-byte aligned tensors (the conv kernels' vector loads of bias / weights)
        n = sum((p.numel() + align - 1) // align * align for _, p in params)
        self.numel = n
        self.flat = torch.zeros((n,), dtype=F32, device=dev)
        self.grad = torch.zeros((n,), dtype=F32, device=dev)
        self.offsets = {}
        off = 0
        for name, p in params:
            k = p.numel()
            self.flat[off:off + k].view(p.shape).copy_(p.data)   # one-time device copy (plumbing)
            p.data = self.flat[off:off + k].view(p.shape)
            p._upr_flat = self
            self.offsets[name] = (off, k)
            off += (k + align - 1) // align * align
        self.params = dict(params)
        self.attach_grads()

    def attach_grads(self):
        """(Re)point every .grad at its slice of the flat gradient buffer;
        returns True if any had been detached (zero_grad(set_to_none=True))."""
        detached = False
        for name, p in self.params.items():
            off, k = self.offsets[name]
            g = p.grad
            if g is None or g.data_ptr() != self.grad.data_ptr() + 4 * off:
                detached = True
                p.grad = self.grad[off:off + k].view(p.shape)
        return detached

    def g(self, p):
        """Gradient view of parameter p."""
        return p.grad


# ---------------------------------------------------------------------------
# layers
# ---------------------------------------------------------------------------
class Conv:
    """nn.Conv2d (model.py / VGG) forward, input-gradient and weight-gradient.

    Cin, Cout multiples of 32 run on the MFMA implicit-GEMM kernels (weights
    re-packed every step: [Cout][(ky,kx,ci)] forward, flipped [Cin][(ky,kx,co)]
    for the input gradient); other shapes on the direct kernels."""

    def __init__(self, m, frozen=False):
        self.m = m
        self.Cout, self.Cin, self.kh, self.kw = m.weight.shape
        self.s = m.stride[0]
        self.p = m.padding[0]
        self.d = m.dilation[0]
        self.bias = m.bias
        self.mfma = self.Cin % 32 == 0 and self.Cout % 32 == 0
        self.frozen = frozen
        self.wp = self.wt = None
        self.wp16 = self.wt16 = None
        self.amp = False  # fp16 arithmetic of the last forward (its backward follows it)
        self.dgrad16_c3 = False
        self.only16 = False

    def out_hw(self, H, W):
        return ((H + 2 * self.p - self.d * (self.kh - 1) - 1) // self.s + 1,
                (W + 2 * self.p - self.d * (self.kw - 1) - 1) // self.s + 1)

    def _buffers(self):
        w = self.m.weight
        if self.wp is None:
            self.wp = torch.empty_like(w).view(-1)
            self.wt = torch.empty_like(w).view(-1)
            self.gp = torch.empty_like(w).view(-1)
        if _AMP[0] and self.wp16 is None:
            self.wp16, self.wt16 = _h16(w.numel(), w.device), _h16(w.numel(), w.device)

    def pack_jobs(self):
        """This conv's re-packs as UprPackJob tuples (pack_convs): the forward
        and flipped dgrad layouts, fp16 only under autocast, else fp32."""
        if not self.mfma:
            return []
        self._buffers()
        w, amp = self.m.weight, _AMP[0]
        n = w.numel()
        return [(w.data_ptr(), 0 if amp else self.wp.data_ptr(), self.wp16.data_ptr() if amp else 0, self.Cout,
                 self.Cin, self.kh, self.kw, 0, n),
                (w.data_ptr(), 0 if amp else self.wt.data_ptr(), self.wt16.data_ptr() if amp else 0, self.Cout,
                 self.Cin, self.kh, self.kw, 1, n)]

    def pack(self):
        if not self.mfma:
            return
        lib, st = L.lib(), _stream()
        w = self.m.weight
        self._buffers()
        _chk(lib.upr_t_pack_weight(_p(w), _p(self.wp), self.Cout, self.Cin, self.kh, self.kw, 0, st), "pack")
        _chk(lib.upr_t_pack_weight(_p(w), _p(self.wt), self.Cout, self.Cin, self.kh, self.kw, 1, st), "pack")
        if _AMP[0]:
            if self.wp16 is None:
                self.wp16, self.wt16 = _h16(w.numel(), w.device), _h16(w.numel(), w.device)
            _chk(lib.upr_t_cast_f16(_p(self.wp), _p(self.wp16), w.numel(), st), "cast_w")
            _chk(lib.upr_t_cast_f16(_p(self.wt), _p(self.wt16), w.numel(), st), "cast_w")

    def _mfma16(self, x, B, H, W, C, cs, coff, w16, bias, N, kh, kw, s, p, d, res, relu, out, store=0, x16=None,
                keep16=False, out16=None, only16=False, x16_strided=False):
        """fp16 MFMA conv with fp32 in / out (upr_t_conv_mfma16); res: Act or None; x16: the
        input's compact fp16 copy when its producer already wrote it; out16 = (fp16 tensor, channel
        offset, channel stride): where the (half)out copy goes when `out` is a channel slice of a
        concat whose fp16 copy the caller assembles (keep16)."""
        Ho = (H + 2 * p - d * (kh - 1) - 1) // s + 1
        Wo = (W + 2 * p - d * (kw - 1) - 1) // s + 1
        dev = out.t.device
        ready = x16 is not None
        if not ready:
            x16 = _h16(B * H * W * C, dev)
            if _TRACE_CAST:  # UPR_TRACE_CAST=1: name the convs whose fp16 operand is cast here
                import traceback
                where = " < ".join(f"{f.name}:{f.lineno}" for f in traceback.extract_stack()[-5:-1][::-1])
                print(f"upr_cast conv {C}->{N} k{kh} s{s} {H}x{W} B{B} at {where}", file=sys.stderr)
        # x16_strided: x16 is the shared fp16 copy of the concat x is a slice of (channel stride cs)
        x16p = ctypes.c_void_p(x16.data_ptr() + 2 * coff) if x16_strided else _p(x16)
        if x16_strided:
            store |= 32
        if out16 is not None:
            t16, c16, cs16 = out16
            y16p, y16cs = ctypes.c_void_p(t16.data_ptr() + 2 * c16), cs16
        else:
            y16 = _h16(B * Ho * Wo * N, dev)
            y16p, y16cs = _p(y16), 0
        _chk(L.lib().upr_t_conv_mfma16(_fp(x, 0), B, H, W, C, cs, coff, _p(w16), _p(bias), N, kh, kw, s, p, d,
                                       res.ptr() if res is not None else None, res.cs if res is not None else 0,
                                       int(relu), _fp(out.t), out.cs, out.coff,
                                       store | (2 if keep16 and res is None else 0) |
                                       (4 if only16 and keep16 and res is None else 0),
                                       x16p, int(ready), y16p, y16cs, _stream()), "conv_mfma16")
        if out16 is not None:
            out.t16 = None
            return x16
        # forward activations (keep16): without a residual y16 is (half)out exactly, and the next
        # autocast conv reading out takes it (Act.t16); forward activations are not modified in place
        whole = out.coff == 0 and out.cs == out.C == (N // 4 if store == 1 else N)
        out.t16 = y16 if keep16 and res is None and whole else None
        out.stale32 = bool(only16 and out.t16 is not None)
        return x16

    def fwd(self, x, relu=False, out=None, res=None, x_view=None, out16=None, only16=False):
        """x: Act (or x_view: (UprView, B, H, W) for an NCHW network input); out16: see _mfma16
        (autocast MFMA convs only; False is returned when the copy was not written).
        only16: under autocast every reader of the output takes its fp16 copy (the
        frozen VGG's activations): the fp32 output is not written (out.stale32)."""
        lib, st = L.lib(), _stream()
        if x_view is not None:
            xv, B, H, W = x_view
        else:
            B, H, W = x.B, x.H, x.W
        Ho, Wo = self.out_hw(H, W)
        if out is None:
            out = Act.new(B, Ho, Wo, self.Cout, x.t.device, fresh=False)
        out.fresh = False
        out.t16 = None  # any fp16 copy of an earlier content is stale now
        out.stale32 = False
        # (a channel slice of a concat qualifies when its fp16 copy goes to the concat's copy, out16)
        self.only16 = bool(only16 and _AMP[0] and res is None and
                           ((out.coff == 0 and out.cs == out.C) or out16 is not None))
        self.amp = _AMP[0] and self.mfma and x_view is None
        # autocast 3 -> 32 / 64 3x3 convs: input gradient on MFMA from an fp16 dy (upr_t_conv_dgrad_c3_16)
        self.dgrad16_c3 = _AMP[0] and self.Cin == 3 and self.Cout in (32, 64) and \
            (self.kh, self.kw, self.s, self.p, self.d) == (3, 3, 1, 1, 1)
        self.out_wo = Wo
        kind = "mfma16" if self.amp else ("mfma32" if self.mfma and x_view is None else "direct")
        with _timed(kind, "fwd", self.flops(B, Ho, Wo), (self.Cin, self.Cout, self.kh, self.s, H, W)):
            self._fwd(x, B, H, W, Ho, Wo, relu, out, res, x_view, out16 if self.amp else None)
        self.wrote16 = self.amp and out16 is not None and res is None
        return out

    def flops(self, B, Ho, Wo):
        return 2.0 * B * Ho * Wo * self.Cout * self.Cin * self.kh * self.kw

    def wgrad16_ok(self, W):
        """Under autocast, this conv's weight gradient on an input of width W runs on
        the fp16-operand GEMM (it reads the input's fp16 copy only)."""
        if not (_AMP[0] and self.mfma):
            return False
        if self.frozen:
            return True
        return ((W + 2 * self.p - self.d * (self.kw - 1) - 1) // self.s + 1) % 64 == 0

    def takes16_grad(self):
        """True when every reader of this conv's output gradient in its backward can
        take the gradient's fp16 copy alone (autocast: input gradient on the fp16
        MFMA, weight gradient on the fp16-operand GEMM, bias sum from fp16), so its
        producer (the BatchNorm backward) may skip the fp32 store."""
        if not (self.amp and self.mfma) or self.s not in (1, 2) or self.Cout % 8:
            return False
        if self.frozen:
            return True
        return getattr(self, "out_wo", 0) % 64 == 0 and getattr(self, "x16", None) is not None

    def _fwd(self, x, B, H, W, Ho, Wo, relu, out, res, x_view, out16=None):
        lib, st = L.lib(), _stream()
        if x_view is not None:
            xv = x_view[0]
        if self.amp:
            # the fp16 copy of x is the weight gradient's B operand (upr_t_conv_wgrad16)
            whole = x.coff == 0 and x.C == x.cs == self.Cin
            t16 = x.t16 if whole else None
            x16 = self._mfma16(x.t, B, H, W, self.Cin, x.cs, x.coff, self.wp16, self.bias, self.Cout, self.kh,
                               self.kw, self.s, self.p, self.d, res, relu, out, x16=t16, keep16=True, out16=out16,
                               only16=self.only16)
            if whole:
                x.t16 = x16  # the next autocast conv reading x (EnhancedFAM: three of them) reuses the copy
            self.x16 = None if self.frozen else x16
        elif self.mfma and x_view is None:
            _chk(lib.upr_t_conv_mfma(_fp(x.t), B, H, W, self.Cin, x.cs, x.coff, _p(self.wp),
                                     _p(self.bias), self.Cout, self.kh, self.kw, self.s, self.p, self.d,
                                     res.ptr() if res is not None else None, res.cs if res is not None else 0,
                                     int(relu), _fp(out.t), out.cs, out.coff, 0, st), "conv_mfma")
        else:
            assert res is None
            v = x.view() if x_view is None else xv
            if _AMP[0] and self.Cin == 3 and self.Cout in (32, 64) and out.coff == 0 and out.cs == out.C:
                # autocast: the 3-channel input convs also write their output's fp16 copy (the
                # next conv's operand) instead of a separate cast pass
                y16 = _h16(B * Ho * Wo * self.Cout, out.t.device)
                rc = lib.upr_t_conv_direct16(ctypes.byref(v), B, H, W, self.Cin, _p(self.m.weight), _p(self.bias),
                                             self.Cout, self.kh, self.kw, self.s, self.p, self.d,
                                             ctypes.byref(out.view()), Ho, Wo, int(relu), 0, _p(y16),
                                             int(self.only16), st)
                if rc == 0:
                    out.t16 = y16
                    out.stale32 = self.only16
                    return
                if rc != L.UPR_ERR_UNSUPPORTED:
                    _chk(rc, "conv_direct16")
            _chk(lib.upr_t_conv_direct(ctypes.byref(v), B, H, W, self.Cin, _p(self.m.weight), _p(self.bias),
                                       self.Cout, self.kh, self.kw, self.s, self.p, self.d,
                                       ctypes.byref(out.view()), Ho, Wo, int(relu), 0, st), "conv_direct")

    def _dgrad_s2_1x1(self, gy, src16, B, Ho, Wo, gx):
        """Input gradient of a 1x1 stride-2 conv (the projecting shortcut,
        model.py:119-122) accumulated into gx: dx(2i, 2j) += W^T dy(i, j) on the
        streaming 1x1 kernel (upr_t_conv_mfma16 store | 8), with no zero-upsampled
        operand.  False when the shape is not one that kernel takes."""
        if gy.stale32 and src16 is None:
            return False
        lib = L.lib()
        x16 = src16 if src16 is not None else _h16(B * Ho * Wo * self.Cout, gy.t.device)
        y16 = _h16(16, gy.t.device)  # not written (store has no | 2)
        rc = lib.upr_t_conv_mfma16(None if src16 is not None else _fp(gy.t, 0), B, Ho, Wo, self.Cout,
                                   gy.cs, gy.coff, _p(self.wt16), None, self.Cin, 1, 1, 1, 0, 1, gx.ptr(), gx.cs, 0,
                                   _fp(gx.t), gx.cs, gx.coff, 8, _p(x16), int(src16 is not None), _p(y16), 0,
                                   _stream())
        if rc == L.UPR_ERR_UNSUPPORTED:
            return False
        _chk(rc, "conv_dgrad_s2_1x1")
        gx.t16, gx.t16_grad = None, False  # gx changed: any fp16 copy of it is stale
        return True

    def _dgrad_s2_3x3(self, gy, src16, B, Ho, Wo, gx, acc, o16):
        """Input gradient of a 3x3 stride-2 pad-1 conv (enc1.conv1, model.py:100-178)
        straight from dy: the four output phases as small convs over dy (upr_t_conv_mfma16
        store | 16), no zero-upsampled operand.  False when the kernel does not take
        the shape (the caller then zero-upsamples)."""
        if gy.stale32 and src16 is None:
            return False
        lib, dev = L.lib(), gy.t.device
        ready = src16 is not None
        x16 = src16 if ready else _h16(B * Ho * Wo * self.Cout, dev)
        keep = bool(o16) and not acc
        y16 = _h16(B * 4 * Ho * Wo * self.Cin if keep else 16, dev)  # written only with keep
        rc = lib.upr_t_conv_mfma16(None if ready else _fp(gy.t, 0), B, Ho, Wo, self.Cout, gy.cs, gy.coff,
                                   _p(self.wt16), None, self.Cin, 3, 3, 1, 1, 1, gx.ptr() if acc else None,
                                   gx.cs if acc else 0, 0, _fp(gx.t), gx.cs, gx.coff, 16 | (6 if keep else 0),
                                   _p(x16), int(ready), _p(y16), 0, _stream())
        if rc == L.UPR_ERR_UNSUPPORTED:
            return False
        _chk(rc, "conv_dgrad_s2_3x3")
        gx.t16 = y16 if keep else None
        gx.stale32 = keep
        gx.t16_grad = keep
        return True

    def bwd_relu_stem(self, x, gy, y, x_view=None):
        """relu_mask(gy, y) then bwd(x, gy, None, x_view): the weight gradient of a
        conv whose input needs no gradient (the image stems), the ReLU backward of
        its output y fused into the small-channel weight-gradient kernel (gy is
        left unmasked: this is its only reader)."""
        # (y.stale32 -- the stem output stored fp16-only -- still takes the stem kernel,
        # whose mask reads y's fp16 copy; the generic direct kernel reads y in fp32)
        if not self.frozen and not (self.mfma and x_view is None) and not gy.stale32:
            lib, st = L.lib(), _stream()
            if x_view is not None:
                xv, B, H, W = x_view
            else:
                xv, B, H, W = x.view(), x.B, x.H, x.W
            stem = (self.Cin, self.Cout, self.kh, self.kw, self.s, self.p, self.d) == (3, 32, 3, 3, 1, 1, 1) and \
                self.bias is not None and gy.coff == 0 and gy.cs == 32 and y.t16 is not None and y.whole16() and \
                (gy.H, gy.W) == (H, W)
            if stem:  # the LDS-staged 3 -> 32 kernel, mask from y's fp16 copy
                with _timed("direct", "wgrad", self.flops(B, H, W), (3, 32, 3, 1, H, W)):
                    rc = lib.upr_t_conv_stem_wgrad_relu16(ctypes.byref(xv), gy.ptr(), _p(y.t16), B, H, W,
                                                          _p(self.m.weight.grad), _p(self.bias.grad), st)
                if rc == 0:
                    return
                if rc != L.UPR_ERR_UNSUPPORTED:
                    _chk(rc, "conv_stem_wgrad_relu16")
            if not y.stale32:
                with _timed("direct", "wgrad", self.flops(B, gy.H, gy.W),
                            (self.Cin, self.Cout, self.kh, self.s, H, W)):
                    rc = lib.upr_t_conv_direct_wgrad_relu(ctypes.byref(xv), ctypes.byref(gy.view()),
                                                          ctypes.byref(y.view()), B, H, W, self.Cin, gy.H, gy.W,
                                                          self.Cout, self.kh, self.kw, self.s, self.p, self.d,
                                                          _p(self.m.weight.grad),
                                                          _p(self.bias.grad) if self.bias is not None else None, st)
                if rc == 0:
                    return
                if rc != L.UPR_ERR_UNSUPPORTED:
                    _chk(rc, "conv_direct_wgrad_relu")
        relu_mask(gy, y)
        self.bwd(x, gy, None, x_view=x_view)

    def bwd(self, x, gy, gx=None, x_view=None, mask=None, gx_only16=False, gx_keep16=False):
        """gy: Act gradient of this conv's output (pre-activation).
        Accumulates the weight / bias gradients; gx (Act, nullable) receives
        the input gradient (overwrite when fresh, else accumulate).
        mask = (a16, cs, only16): the ReLU backward of the activation gx flows
        into, fused into the input-gradient epilogue (a16 = that activation's
        fp16 copy, channel stride cs); gx.t16 then holds the masked gradient and
        gx.t is left stale when only16.  Returns True when the mask was applied.
        gx_only16: the input gradient's reader (a BatchNorm backward) takes its fp16
        copy: under autocast gx gets gx.t16 and no fp32 store when fresh.
        gx_keep16: gx also gets its fp16 copy (fp32 kept), shared by gx's channel slices."""
        lib, st = L.lib(), _stream()
        if x_view is not None:
            xv, B, H, W = x_view
        else:
            B, H, W = x.B, x.H, x.W
        Ho, Wo = gy.H, gy.W
        F = self.flops(B, Ho, Wo)
        mf = self.mfma and x_view is None
        kw_ = ("mfma16" if self.amp and getattr(self, "x16", None) is not None else "mfma32") if mf else "direct"
        with _timed(None if self.frozen else kw_, "wgrad", F, (self.Cin, self.Cout, self.kh, self.s, H, W)):
            if not self.frozen:
                gw = self.m.weight.grad
                if self.mfma and x_view is None:
                    x16 = getattr(self, "x16", None)
                    # autocast: fp16 operands, fp32 accumulation (trainers/train.py:72); added
                    # straight into weight.grad's layout
                    # gy's fp16 copy (the fused BN backward's dx16) is the AMP A operand as is
                    # (in gy's own layout: the C ABI indexes dy16 like dy, so a slice of a shared concat
                    # copy passes the concat's base)
                    dy16 = gy.t16 if self.amp and gy.t16_grad and (gy.whole16() and gy.C == self.Cout or
                                                                   gy.t16_shared) else None
                    assert dy16 is not None or not gy.stale32, "fp16-only gradient without the fp16 weight gradient"
                    assert x16 is not None or not x.stale32, "fp16-only input without the fp16 weight gradient"
                    _chk(lib.upr_t_conv_wgrad_into(_fp(x.t), _p(x16) if self.amp else None, B, H, W, self.Cin, x.cs,
                                                   x.coff, _fp(gy.t), _p(dy16), Ho, Wo, self.Cout, gy.cs, gy.coff,
                                                   self.kh, self.kw, self.s, self.p, self.d, _p(gw), st),
                         "conv_wgrad")
                    self.x16 = None
                    if self.bias is not None:
                        if gy.stale32:
                            ws = torch.empty((L.lib().upr_t_reduce_acc_doubles(self.Cout),), dtype=torch.float64,
                                             device=gy.t.device)
                            if gy.whole16():
                                _chk(lib.upr_t_chan_sum16(_p(gy.t16), gy.M, self.Cout, _p(self.bias.grad), 1, _p(ws),
                                                          st), "dbias16")
                            else:  # a slice of a shared concat copy
                                _chk(lib.upr_t_chan_sum16s(ctypes.c_void_p(gy.t16.data_ptr() + 2 * gy.coff), gy.M,
                                                           self.Cout, gy.cs, _p(self.bias.grad), 1, _p(ws), st),
                                     "dbias16s")
                        else:
                            chan_sum(gy, self.Cout, self.bias.grad, st)
                else:
                    v = x.view() if x_view is None else xv
                    _chk(lib.upr_t_conv_direct_wgrad(ctypes.byref(v), ctypes.byref(gy.view()), B, H, W, self.Cin, Ho, Wo,
                                                     self.Cout, self.kh, self.kw, self.s, self.p, self.d, _p(gw),
                                                     _p(self.bias.grad) if self.bias is not None else None, st),
                         "conv_direct_wgrad")
        if gx is None:
            return
        with _timed("mfma16" if self.amp else ("mfma32" if self.mfma else "direct"), "dgrad", F,
                    (self.Cin, self.Cout, self.kh, self.s, H, W)):
            if self.mfma:
                acc = gx.consume_fresh()
                src, sH, sW, scs, scoff = gy.t, Ho, Wo, gy.cs, gy.coff
                src16 = gy.t16 if self.amp and gy.t16_grad and gy.coff == 0 and gy.cs == gy.C == self.Cout else None
                # a channel slice of a shared concat copy: its pixels at gy.t16[p * gy.cs + gy.coff]
                m16, m16cs = (src16, self.Cout) if src16 is not None else \
                    ((ctypes.c_void_p(gy.t16.data_ptr() + 2 * gy.coff), gy.cs)
                     if self.amp and gy.t16_grad and gy.t16_shared and gy.C == self.Cout else (None, 0))
                if mask is not None and self.amp and self.s == 1 and not acc and m16 is not None and \
                        gx.coff == 0 and gx.cs == gx.C == self.Cin:
                    a16, mcs, only16 = mask
                    y16 = _h16(B * H * W * self.Cin, gx.t.device)
                    rc = lib.upr_t_conv_mfma16_relu_bwd_cs(_p(m16) if m16 is src16 else m16, m16cs, B, Ho, Wo,
                                                           self.Cout, _p(self.wt16), self.Cin, self.kh, self.kw,
                                                           self.d * (self.kh - 1) - self.p, self.d, _fp(gx.t), gx.cs,
                                                           0, _p(y16), self.Cin, _p(a16), mcs, int(only16), st)
                    if rc == 0:
                        gx.t16, gx.t16_grad, gx.stale32 = y16, True, bool(only16)
                        return True
                    if rc != L.UPR_ERR_UNSUPPORTED:
                        _chk(rc, "conv_mfma16_relu_bwd")
                # autocast: the fp16 operand comes from gy's producer (gy.t16) or, for
                # stride 2, straight from an fp16 zero-upsample (no fp32 pass + cast)
                src16 = gy.t16 if self.amp and gy.t16_grad and gy.coff == 0 and gy.cs == gy.C == self.Cout else None
                # a channel slice of a shared concat copy (stride-1 convs read it in place)
                strided16 = src16 is None and self.amp and self.s == 1 and gy.t16_grad and gy.t16_shared
                if strided16:
                    src16 = gy.t16
                if self.s == 2 and self.amp and acc and (self.kh, self.kw, self.p, self.d) == (1, 1, 0, 1) and \
                        H == 2 * Ho and W == 2 * Wo and self._dgrad_s2_1x1(gy, src16, B, Ho, Wo, gx):
                    return
                if self.s == 2 and self.amp and (self.kh, self.kw, self.p, self.d) == (3, 3, 1, 1) and \
                        H == 2 * Ho and W == 2 * Wo and \
                        self._dgrad_s2_3x3(gy, src16, B, Ho, Wo, gx, acc,
                                           bool(gx_only16) and gx.coff == 0 and gx.cs == gx.C == self.Cin):
                    return
                if self.s != 1:
                    assert self.s == 2 and H == 2 * Ho and W == 2 * Wo, "stride-2 dgrad needs even sizes"
                    if self.amp and self.Cout % 8 == 0:
                        z16 = _h16(B * H * W * self.Cout, gy.t.device)
                        if gy.stale32:
                            _chk(lib.upr_t_zero_upsample16h(_p(gy.t16), B, Ho, Wo, self.Cout, _p(z16), st),
                                 "zero_upsample16h")
                        else:
                            _chk(lib.upr_t_zero_upsample16(_fp(gy.t), B, Ho, Wo, self.Cout, gy.cs, gy.coff, _p(z16),
                                                           st), "zero_upsample16")
                        src16, src = z16, None
                    else:
                        src16 = None
                        z = empty((B, H, W, self.Cout), gy.t.device)
                        _chk(lib.upr_t_zero_upsample(_fp(gy.t), B, Ho, Wo, self.Cout, gy.cs, gy.coff,
                                                     _p(z), st), "zero_upsample")
                        src = z
                    sH, sW, scs, scoff = H, W, self.Cout, 0
                pad_t = self.d * (self.kh - 1) - self.p
                assert src16 is not None or not gy.stale32, "fp16-only gradient without the fp16 input gradient"
                if self.amp:
                    whole_gx = not acc and gx.coff == 0 and gx.cs == gx.C == self.Cin
                    o16 = bool(gx_only16) and whole_gx
                    k16 = o16 or (bool(gx_keep16) and whole_gx)
                    self._mfma16(src, B, sH, sW, self.Cout, scs, scoff, self.wt16, None, self.Cin, self.kh, self.kw, 1,
                                 pad_t, self.d, gx if acc else None, False, gx, x16=src16, keep16=k16, only16=o16,
                                 x16_strided=strided16)
                    gx.t16_grad = gx.t16 is not None
                    gx.t16_shared = bool(gx_keep16) and gx.t16 is not None
                else:
                    _chk(lib.upr_t_conv_mfma(_fp(src), B, sH, sW, self.Cout, scs, scoff, _p(self.wt), None, self.Cin,
                                             self.kh, self.kw, 1, pad_t, self.d, gx.ptr() if acc else None,
                                             gx.cs if acc else 0, 0, _fp(gx.t), gx.cs, gx.coff, 0, st), "conv_dgrad")
            else:
                acc = gx.consume_fresh()
                if self.dgrad16_c3 and gy.t16 is not None and gy.t16_grad:
                    # autocast (VGG conv1_1): fp16 dy from the fused ReLU mask, MFMA
                    rc = lib.upr_t_conv_dgrad_c3_16(_p(gy.t16), B, H, W, _p(self.m.weight), self.Cout,
                                                    ctypes.byref(gx.view()), int(acc), st)
                    if rc == 0:
                        return
                    if rc != L.UPR_ERR_UNSUPPORTED:
                        _chk(rc, "conv_dgrad_c3_16")
                    if gy.stale32:
                        raise RuntimeError("upr: fp16-only gradient without an fp16 dgrad path")
                _chk(lib.upr_t_conv_direct_dgrad(ctypes.byref(gy.view()), Ho, Wo, _p(self.m.weight), B, H, W, self.Cin,
                                                 self.Cout, self.kh, self.kw, self.s, self.p, self.d,
                                                 ctypes.byref(gx.view()), acc, st), "conv_direct_dgrad")


class ConvT:
    """nn.ConvTranspose2d(k=2, s=2) (UpBlock.up, model.py:261): a GEMM with
    N = 4*Cout and a pixel-shuffle store; dgrad = k2 s2 conv over dy; wgrad =
    the same GEMM over pixels with dy as the 'input'."""

    def __init__(self, m):
        self.m = m
        self.Cin, self.Cout = m.weight.shape[0], m.weight.shape[1]
        self.wp = None
        self.wp16 = self.wd16 = None
        self.amp = False

    def _buffers(self):
        w = self.m.weight
        if self.wp is None:
            self.wp = torch.empty_like(w).view(-1)
            self.wd = torch.empty_like(w).view(-1)
            self.gp = torch.empty_like(w).view(-1)
            self.b4 = empty((4 * self.Cout,), w.device)
        if _AMP[0] and self.wp16 is None:
            self.wp16, self.wd16 = _h16(w.numel(), w.device), _h16(w.numel(), w.device)

    def pack_jobs(self):
        self._buffers()
        w, amp = self.m.weight, _AMP[0]
        n = w.numel()
        return [(w.data_ptr(), 0 if amp else self.wp.data_ptr(), self.wp16.data_ptr() if amp else 0, self.Cout,
                 self.Cin, 2, 2, 2, n),
                (w.data_ptr(), 0 if amp else self.wd.data_ptr(), self.wd16.data_ptr() if amp else 0, self.Cout,
                 self.Cin, 2, 2, 3, n),
                (self.m.bias.data_ptr(), self.b4.data_ptr(), 0, self.Cout, 1, 1, 1, 4, self.Cout)]

    def pack(self):
        lib, st = L.lib(), _stream()
        w = self.m.weight
        self._buffers()
        _chk(lib.upr_t_pack_weight(_p(w), _p(self.wp), self.Cout, self.Cin, 2, 2, 2, st), "pack")
        _chk(lib.upr_t_pack_weight(_p(w), _p(self.wd), self.Cout, self.Cin, 2, 2, 3, st), "pack")
        if _AMP[0]:
            if self.wp16 is None:
                self.wp16, self.wd16 = _h16(w.numel(), w.device), _h16(w.numel(), w.device)
            _chk(lib.upr_t_cast_f16(_p(self.wp), _p(self.wp16), w.numel(), st), "cast_w")
            _chk(lib.upr_t_cast_f16(_p(self.wd), _p(self.wd16), w.numel(), st), "cast_w")
        src = L.UprView(self.m.bias.data_ptr(), 0, 0, 0, 1)
        dst = L.UprView(self.b4.data_ptr(), 0, 0, self.Cout, 1)
        _chk(lib.upr_t_copy(ctypes.byref(src), ctypes.byref(dst), 1, 1, 4, self.Cout, 0, st), "bias4")

    def fwd(self, x):
        out = Act.new(x.B, 2 * x.H, 2 * x.W, self.Cout, x.t.device, fresh=False)
        self.amp = _AMP[0]
        with _timed("mfma16" if self.amp else "mfma32", "fwd", self.flops(x)):
            if self.amp:
                Conv._mfma16(self, x.t, x.B, x.H, x.W, self.Cin, x.cs, x.coff, self.wp16, self.b4, 4 * self.Cout, 1, 1,
                             1, 0, 1, None, False, out, store=1, x16=x.t16 if x.coff == 0 and x.cs == x.C == self.Cin
                             else None, keep16=True)
            else:
                _chk(L.lib().upr_t_conv_mfma(x.ptr(), x.B, x.H, x.W, self.Cin, x.cs, 0, _p(self.wp), _p(self.b4),
                                             4 * self.Cout, 1, 1, 1, 0, 1, None, 0, 0, _fp(out.t), out.cs, 0, 1,
                                             _stream()), "convT")
        return out

    def flops(self, x):
        return 2.0 * x.B * x.H * x.W * self.Cin * 4 * self.Cout

    def bwd(self, x, gy, gx):
        lib, st = L.lib(), _stream()
        F = self.flops(x)
        kind = "mfma16" if self.amp else "mfma32"
        # gy's fp16 copy from its producer (UpBlockT: the following conv's input gradient,
        # gx_keep16) is both GEMMs' fp16 operand as is -- no internal cast passes
        gy16 = gy.t16 if self.amp and gy.t16 is not None and gy.t16_grad and gy.coff == 0 and gy.cs == gy.C else None
        with _timed(kind, "wgrad", F):
            zero(self.gp)
            # dwp[ci][(a,b,co)] = sum_p x[p][ci] * gy[2y+a][2x+b][co]: a k2 s2 "conv" of gy producing x
            if self.amp:
                _chk(lib.upr_t_conv_wgrad16(gy.ptr(), _p(gy16), gy.B, gy.H, gy.W, self.Cout, gy.cs, 0, x.ptr(), x.H, x.W,
                                            self.Cin, x.cs, 0, 2, 2, 2, 0, 1, _p(self.gp), st), "convT_wgrad16")
            else:
                _chk(lib.upr_t_conv_wgrad(gy.ptr(), gy.B, gy.H, gy.W, self.Cout, gy.cs, 0, x.ptr(), x.H, x.W, self.Cin,
                                          x.cs, 0, 2, 2, 2, 0, 1, _p(self.gp), st), "convT_wgrad")
            _chk(lib.upr_t_unpack_grad(_p(self.gp), _p(self.m.weight.grad), self.Cout, self.Cin, 2, 2, 3, 1, st),
                 "unpack")
            chan_sum(gy, self.Cout, self.m.bias.grad, st)
        with _timed(kind, "dgrad", F):
            acc = gx.consume_fresh()
            if self.amp:
                Conv._mfma16(self, gy.t, gy.B, gy.H, gy.W, self.Cout, gy.cs, gy.coff, self.wd16, None, self.Cin, 2, 2, 2,
                             0, 1, gx if acc else None, False, gx, x16=gy16)
            else:
                _chk(lib.upr_t_conv_mfma(gy.ptr(), gy.B, gy.H, gy.W, self.Cout, gy.cs, 0, _p(self.wd), None, self.Cin, 2,
                                         2, 2, 0, 1, gx.ptr() if acc else None, gx.cs if acc else 0, 0, _fp(gx.t),
                                         gx.cs, gx.coff, 0, st), "convT_dgrad")


class BN:
    """nn.BatchNorm2d: training mode (batch statistics, running-stat update) or,
    when the module is in eval mode, the running statistics (a standalone
    submodule forward, upr/modules.py)."""

    def __init__(self, m):
        self.m = m
        self.C = m.num_features
        dev = m.weight.device
        self.mean = empty((self.C,), dev)
        self.invstd = empty((self.C,), dev)
        # per-channel sums + the two-stage reduction's partial slots (upr_t_reduce_acc_doubles)
        self.acc = torch.empty((L.lib().upr_t_reduce_acc_doubles(self.C),), dtype=torch.float64, device=dev)

    def fwd(self, x, relu=False, out=None, res=None, res_post=False, only16=False, out16=None):
        """only16: under autocast every reader of the output takes its fp16 copy (convs
        whose weight gradients run on the fp16-operand GEMM): the fp32 output is not
        written (out.stale32).  out16 = (fp16 tensor, channel offset, channel stride):
        `out` is a channel slice of a concat whose fp16 copy the caller assembles; the
        slice's fp16 values go there (and with only16 its fp32 values are not written);
        self.wrote16 tells whether they did."""
        self.wrote16 = False
        lib, st = L.lib(), _stream()
        m = self.m
        # under autocast x is an fp16 conv's output: its fp16 copy holds the same values
        x16 = x.t16 if _AMP[0] and x.t16 is not None and x.coff == 0 and x.cs == x.C == self.C else None
        self.x16 = x16
        if m.training:
            # fp16 input: statistics and finalise in two launches (upr_t_bn_stats16_fin)
            rc = lib.upr_t_bn_stats16_fin(_p(x16), x.M, self.C, _p(self.acc), ctypes.c_float(m.momentum),
                                          ctypes.c_float(m.eps), _p(m.running_mean), _p(m.running_var),
                                          _p(m.num_batches_tracked), _p(self.mean), _p(self.invstd), st) \
                if x16 is not None else L.UPR_ERR_UNSUPPORTED
            if rc == L.UPR_ERR_UNSUPPORTED:
                assert not x.stale32, "fp16-only BN input without an fp16 statistics path"
                _chk(lib.upr_t_bn_stats(x.ptr(), x.M, self.C, x.cs, 0, _p(self.acc), st), "bn_stats")
                _chk(lib.upr_t_bn_finalize(_p(self.acc), x.M, self.C, ctypes.c_float(m.momentum),
                                           ctypes.c_float(m.eps), _p(m.running_mean), _p(m.running_var),
                                           _p(m.num_batches_tracked), _p(self.mean), _p(self.invstd), st),
                     "bn_finalize")
            else:
                _chk(rc, "bn_stats16_fin")
        else:
            _chk(lib.upr_t_bn_eval_stats(_p(m.running_mean), _p(m.running_var), self.C, ctypes.c_float(m.eps),
                                         _p(self.mean), _p(self.invstd), st), "bn_eval_stats")
        if out is None:
            out = Act.new(x.B, x.H, x.W, self.C, x.t.device, fresh=False)
        if out16 is not None and _AMP[0] and x16 is not None and res is None:
            # a concat slice: fp16 values into the caller's copy (no fallback: the fp16
            # input path always exists here, and a half-written copy must not be claimed)
            t16, c16, cs16 = out16
            skip32 = int(bool(only16))
            _chk(lib.upr_t_bn_apply16h_cs(_p(x16), x.M, self.C, _p(self.mean), _p(self.invstd), _p(m.weight),
                                          _p(m.bias), None, 0, 0, 0, int(relu), _fp(out.t), out.cs, out.coff,
                                          ctypes.c_void_p(t16.data_ptr() + 2 * c16), cs16, skip32, st),
                 "bn_apply16h_cs")
            self.wrote16 = True
            out.t16 = None
            # (the slice object; the caller marks the concat.  An unfused backward that
            # would mask with this output refuses a stale one, below in bwd)
            out.stale32 = bool(skip32)
            self.x = x
            self.out_act = out
            self.batch_stats = bool(m.training)
            self.relu_only = bool(relu)
            self.has_res = False
            return out
        # under autocast the consumer is an fp16 conv: write its fp16 input copy here
        y16 = _h16(out.M * self.C, out.t.device) if _AMP[0] and out.coff == 0 and out.cs == self.C else None
        rc = L.UPR_ERR_UNSUPPORTED
        skip32 = int(bool(only16) and y16 is not None)
        if x16 is not None:
            rc = lib.upr_t_bn_apply16h(_p(x16), x.M, self.C, _p(self.mean), _p(self.invstd), _p(m.weight),
                                       _p(m.bias), res.ptr() if res is not None else None,
                                       res.cs if res is not None else 0, 0, int(res_post), int(relu), _fp(out.t),
                                       out.cs, out.coff, _p(y16), skip32, st)
            if rc != 0:
                skip32 = 0
        if rc == L.UPR_ERR_UNSUPPORTED:
            assert not x.stale32, "fp16-only BN input without an fp16 apply path"
            rc = lib.upr_t_bn_apply16(x.ptr(), x.M, self.C, x.cs, 0, _p(self.mean), _p(self.invstd), _p(m.weight),
                                      _p(m.bias), res.ptr() if res is not None else None,
                                      res.cs if res is not None else 0, 0, int(res_post), int(relu), _fp(out.t),
                                      out.cs, out.coff, _p(y16), st)
        _chk(rc, "bn_apply")
        out.t16 = y16
        out.stale32 = bool(skip32)
        self.x = x
        self.out_act = out
        self.batch_stats = bool(m.training)  # the backward follows the statistics this forward used
        # y = relu(bn(x)) (+ a residual added after the ReLU): the backward may fold the mask in
        self.relu_only = bool(relu) and (res is None or bool(res_post))
        self.has_res = res is not None
        return out

    def bwd(self, g, gx, relu=False, only16=False):
        """g: Act gradient of the BN output; relu=True: g is the gradient of
        relu(bn(x)) (+ a residual added after the ReLU, res_post: this
        forward's relu=True), the ReLU mask is folded into the BN backward
        (recomputed from x, no separate pass; the residual does not enter it).
        Under autocast the input gradient also gets its compact fp16 copy
        (gx.t16) for the input-gradient conv that consumes it; only16 (the
        consumer's Conv.takes16_grad()): the fp32 gx is not written at all."""
        lib, st = L.lib(), _stream()
        m, x = self.m, self.x
        assert not relu or self.relu_only, "ReLU fold needs a relu(bn(x)) forward"
        if g.coff % 4 == 0 and gx.coff % 4 == 0:
            whole = gx.coff == 0 and gx.cs == self.C
            dx16 = _h16(gx.M * self.C, gx.t.device) if _AMP[0] and whole else None
            acc = 0 if gx.fresh else 1
            rc = L.UPR_ERR_UNSUPPORTED
            skip32 = int(bool(only16) and dx16 is not None and acc == 0)
            # g's fp16 copy (the input-gradient conv's fp16 output) when it has one
            g16 = g.t16 if g.t16_grad and g.coff == 0 and g.cs == g.C == self.C else None
            if self.x16 is not None:
                rc = lib.upr_t_bn_bwd_fused16(_fp(g.t), _p(g16), g.cs, g.coff, _p(self.x16), _p(self.mean),
                                              _p(self.invstd),
                                              _p(m.weight), _p(m.bias), int(relu), x.M, self.C, _p(self.acc),
                                              _p(m.weight.grad), _p(m.bias.grad), _fp(gx.t), gx.cs, gx.coff, acc,
                                              int(self.batch_stats), _p(dx16), skip32, st)
                if rc == 0:
                    gx.consume_fresh()
                    gx.t16, gx.t16_grad, gx.stale32 = dx16, dx16 is not None, bool(skip32)
                    return
            if rc == L.UPR_ERR_UNSUPPORTED:
                assert not x.stale32 and not g.stale32, "fp16-only BN operand without an fp16 backward path"
                rc = lib.upr_t_bn_bwd_fused(_fp(g.t), g.cs, g.coff, x.ptr(), x.cs, _p(self.mean), _p(self.invstd),
                                            _p(m.weight), _p(m.bias), int(relu), x.M, self.C, _p(self.acc),
                                            _p(m.weight.grad), _p(m.bias.grad), _fp(gx.t), gx.cs, gx.coff, acc,
                                            int(self.batch_stats), _p(dx16), st)
            if rc != L.UPR_ERR_UNSUPPORTED:
                _chk(rc, "bn_bwd_fused")
                gx.consume_fresh()
                gx.t16, gx.t16_grad = dx16, dx16 is not None
                return
        if relu:
            # the mask comes from the stored output here: with a post-ReLU
            # residual that output is relu(bn(x)) + skip, not the ReLU's own
            # output, and the mask would be wrong wherever skip > 0 >= bn(x)
            if self.has_res:
                raise NotImplementedError("unfused ReLU backward of relu(bn(x)) + skip: the mask needs the "
                                          "pre-residual value (the fused BatchNorm backward takes this layer)")
            if self.out_act.stale32:
                raise NotImplementedError("unfused ReLU backward of an fp16-only BatchNorm output: the mask "
                                          "needs the fp32 value (the fused BatchNorm backward takes this layer)")
            relu_mask(g, self.out_act)
        zero(self.acc[:2 * self.C])
        _chk(lib.upr_t_bn_bwd_reduce(_fp(g.t), g.cs, g.coff, x.ptr(), x.cs, 0, _p(self.mean), _p(self.invstd), x.M,
                                     self.C, _p(self.acc), st), "bn_bwd_reduce")
        acc = gx.consume_fresh()
        _chk(lib.upr_t_bn_bwd_apply(_fp(g.t), g.cs, g.coff, x.ptr(), x.cs, 0, _p(self.mean), _p(self.invstd),
                                    _p(m.weight), _p(self.acc), x.M, self.C, _p(m.weight.grad), _p(m.bias.grad),
                                    _fp(gx.t), gx.cs, gx.coff, acc, int(self.batch_stats), st), "bn_bwd_apply")


def chan_sum(g, C, out, st):
    """out[C] += per-channel sum of the Act g (conv bias gradients; two-stage, deterministic)."""
    ws = torch.empty((L.lib().upr_t_reduce_acc_doubles(C),), dtype=torch.float64, device=g.t.device)
    _chk(L.lib().upr_t_chan_sum_ws(g.ptr(), g.M, C, g.cs, 0, _p(out), 1, _p(ws), st), "dbias")


def relu_mask(g, y, want16=False, only16=False):
    """g *= (y > 0) in place.  want16: also write the masked gradient's fp16 copy
    (g.t16, the next autocast dgrad's operand) in the same pass; only16: the fp32
    g is left unmasked (stale) -- for a gradient whose only reader is a frozen
    conv's fp16 dgrad."""
    g.t16, g.t16_grad, g.stale32 = None, False, False  # masked in place: any fp16 copy is stale
    if want16 and g.coff == 0 and g.cs == g.C:
        g16 = _h16(g.M * g.C, g.t.device)
        if y.stale32:  # y exists in fp16 only (frozen VGG activations under autocast)
            rc = L.lib().upr_t_relu_mask16h(_fp(g.t), g.cs, g.coff, _p(y.t16), y.C, g.M, g.C, _p(g16),
                                            int(not only16), _stream())
        else:
            rc = L.lib().upr_t_relu_mask16(_fp(g.t), g.cs, g.coff, _fp(y.t), y.cs, y.coff, g.M, g.C, _p(g16),
                                           int(not only16), _stream())
        if rc == 0:
            g.t16, g.t16_grad, g.stale32 = g16, True, only16
            return
        if rc != L.UPR_ERR_UNSUPPORTED:
            _chk(rc, "relu_mask16")
    assert not y.stale32, "fp16-only activation without an fp16 mask path"
    _chk(L.lib().upr_t_relu_mask(_fp(g.t), g.cs, g.coff, _fp(y.t), y.cs, y.coff, g.M, g.C, _stream()), "relu_mask")


def maxpool_into(x, y, k, s, p, code=None, only16=False):
    """nn.MaxPool2d(k, s, p) of Act x into Act y (argmax codes for the backward
    when `code`); under autocast also y's fp16 copy (y.t16) in the same pass.
    only16 (under autocast, from an fp16 input): y is written as its fp16 copy
    only (y.stale32; the max of fp16 values is an fp16 value, so nothing is
    rounded) -- the frozen VGG's pools, whose every reader takes fp16."""
    lib, st = L.lib(), _stream()
    if _AMP[0] and y.coff == 0 and y.cs == y.C:
        y16 = _h16(y.M * y.C, y.t.device)
        if x.t16 is not None and x.coff == 0 and x.cs == x.C:
            # the activation's fp16 copy (its only value when x.stale32)
            yv = y.view()
            if only16:
                yv.data = None
            rc = lib.upr_t_maxpool16_code(_p(x.t16), x.B, x.H, x.W, x.C, k, s, p, ctypes.byref(yv), y.H, y.W,
                                          _p(code), _p(y16), st)
            if rc == 0:
                y.t16 = y16
                y.stale32 = bool(only16)
                return
            if rc != L.UPR_ERR_UNSUPPORTED:
                _chk(rc, "maxpool16")
        assert not x.stale32, "fp16-only activation without an fp16 max-pool path"
        rc = lib.upr_t_maxpool_code(ctypes.byref(x.view()), x.B, x.H, x.W, x.C, k, s, p, ctypes.byref(y.view()), y.H,
                                    y.W, _p(code), _p(y16), st)
        if rc == 0:
            y.t16 = y16
            return
        if rc != L.UPR_ERR_UNSUPPORTED:
            _chk(rc, "maxpool")
    _chk(lib.upr_t_maxpool_code(ctypes.byref(x.view()), x.B, x.H, x.W, x.C, k, s, p, ctypes.byref(y.view()), y.H, y.W,
                                _p(code), None, st), "maxpool")
    y.t16 = None


def add_acts(a, b, out):
    """out = a + b (contiguous Acts of one shape); under autocast with out's fp16 copy."""
    n = out.t.numel()
    if _AMP[0]:
        o16 = _h16(n, out.t.device)
        rc = L.lib().upr_t_add16(_fp(a.t), _fp(b.t), _fp(out.t), n, _p(o16), _stream())
        if rc == 0:
            out.t16 = o16
            return
        if rc != L.UPR_ERR_UNSUPPORTED:
            _chk(rc, "add16")
    pointwise(a.t, b.t, out.t, n, 4)
    out.t16 = None


def pack_convs(convs, owner):
    """Re-pack every conv's weights for this step in ONE launch
    (upr_t_pack_weights); the device job table is rebuilt only when a pointer,
    shape or the autocast mode changed, and is kept alive on `owner`."""
    jobs = []
    for c in convs:
        jobs += c.pack_jobs()
    if not jobs:
        return
    key = tuple(jobs)
    tab = getattr(owner, "_pack_tab", None)
    if tab is None or tab[0] != key:
        arr = (L.UprPackJob * len(jobs))(*[L.UprPackJob(*j) for j in jobs])
        host = torch.frombuffer(bytearray(arr), dtype=torch.uint8)
        dev = convs[0].m.weight.device
        owner._pack_tab = (key, host.to(dev), len(jobs), max(j[-1] for j in jobs))
    _, t, nj, mx = owner._pack_tab
    _chk(L.lib().upr_t_pack_weights(_p(t), nj, mx, _stream()), "pack_weights")


def add_into(dst, src):
    """dst (+)= src (Acts of equal shape)."""
    acc = dst.consume_fresh()
    _chk(L.lib().upr_t_copy(ctypes.byref(src.view()), ctypes.byref(dst.view()), src.B, src.H, src.W, src.C, acc,
                            _stream()), "copy")


def pointwise(a, b, out, n, op, mask_in=None, mask_out=None, p=0.0, seed=0):
    _chk(L.lib().upr_t_pointwise(_p(a), _p(b), _p(out), n, op, _p(mask_in), _p(mask_out), ctypes.c_float(p),
                                 ctypes.c_uint64(seed), _stream()), "pointwise")


# ---------------------------------------------------------------------------
# reference modules
# ---------------------------------------------------------------------------
class ResBlockT:
    """ResBlock (model.py:100-135)."""

    def __init__(self, m):
        self.conv1, self.bn1 = Conv(m.conv1), BN(m.bn1)
        self.conv2, self.bn2 = Conv(m.conv2), BN(m.bn2)
        self.proj = len(m.shortcut) > 0
        if self.proj:
            self.sconv, self.sbn = Conv(m.shortcut[0]), BN(m.shortcut[1])

    def convs(self):
        return [self.conv1, self.conv2] + ([self.sconv] if self.proj else [])

    def fwd(self, x):
        self.x = x
        # a conv whose only reader is a BatchNorm keeps its output in fp16 only under
        # autocast (the BN reads the fp16 copy: the same values)
        c1 = self.conv1.fwd(x, only16=True)
        self.a1 = self.bn1.fwd(c1, relu=True, only16=self.conv2.wgrad16_ok(c1.W))
        c2 = self.conv2.fwd(self.a1, only16=True)
        sc = self.sbn.fwd(self.sconv.fwd(x, only16=True)) if self.proj else x
        self.out = self.bn2.fwd(c2, relu=True, res=sc)
        return self.out

    def bwd(self, g, gx):
        relu_mask(g, self.out)
        g_c2 = Act.new(g.B, g.H, g.W, self.conv2.Cout, g.t.device)
        self.bn2.bwd(g, g_c2, only16=self.conv2.takes16_grad())
        if self.proj:
            g_cs = Act.new(g.B, g.H, g.W, self.sconv.Cout, g.t.device)
            self.sbn.bwd(g, g_cs, only16=self.sconv.takes16_grad())
        else:
            add_into(gx, g)
        g_a1 = Act.new(self.a1.B, self.a1.H, self.a1.W, self.a1.C, g.t.device)
        self.conv2.bwd(self.a1, g_c2, g_a1, gx_only16=True)
        g_c1 = Act.new(g_a1.B, g_a1.H, g_a1.W, g_a1.C, g.t.device)
        self.bn1.bwd(g_a1, g_c1, relu=True, only16=self.conv1.takes16_grad())
        self.conv1.bwd(self.x, g_c1, gx)
        if self.proj:
            # after conv1's: the shortcut's input gradient accumulates (the 1x1
            # stride-2 one then adds at the even pixels only, _dgrad_s2_1x1);
            # fp32 addition commutes, so the sum is the same bits either order
            self.sconv.bwd(self.x, g_cs, gx)


class PreActResBlockT:
    """PreActResBlock (model.py:138-178)."""

    def __init__(self, m):
        self.bn1, self.conv1 = BN(m.bn1), Conv(m.conv1)
        self.bn2, self.conv2 = BN(m.bn2), Conv(m.conv2)
        self.proj = len(m.shortcut) > 0
        if self.proj:
            self.sconv, self.sbn = Conv(m.shortcut[0]), BN(m.shortcut[1])

    def convs(self):
        return [self.conv1, self.conv2] + ([self.sconv] if self.proj else [])

    def fwd(self, x):
        self.x = x
        self.o = self.bn1.fwd(x, relu=True)
        sc = self.sbn.fwd(self.sconv.fwd(self.o, only16=True)) if self.proj else x
        c1 = self.conv1.fwd(self.o, only16=True)
        self.a2 = self.bn2.fwd(c1, relu=True, only16=self.conv2.wgrad16_ok(c1.W))
        return self.conv2.fwd(self.a2, res=sc)

    def bwd(self, g, gx):
        dev = g.t.device
        g_a2 = Act.new(self.a2.B, self.a2.H, self.a2.W, self.a2.C, dev)
        self.conv2.bwd(self.a2, g, g_a2, gx_only16=True)
        g_c1 = Act.new(g_a2.B, g_a2.H, g_a2.W, g_a2.C, dev)
        self.bn2.bwd(g_a2, g_c1, relu=True, only16=self.conv1.takes16_grad())
        g_o = Act.new(self.o.B, self.o.H, self.o.W, self.o.C, dev)
        self.conv1.bwd(self.o, g_c1, g_o)
        if self.proj:
            g_cs = Act.new(g.B, g.H, g.W, self.sconv.Cout, dev)
            self.sbn.bwd(g, g_cs, only16=self.sconv.takes16_grad())
            self.sconv.bwd(self.o, g_cs, g_o)
        else:
            add_into(gx, g)
        self.bn1.bwd(g_o, gx, relu=True)


class ASPPT:
    """ASPPModule (model.py:181-251); Dropout(0.1) mask from a counter hash
    whose seed is drawn from torch's default generator (so, as with the
    reference's nn.Dropout, torch.manual_seed makes the masks reproducible)."""

    def __init__(self, m, dropout_mask_fn=None):
        self.c1, self.b1 = Conv(m.conv1x1[0]), BN(m.conv1x1[1])
        self.br = [(Conv(s[0]), BN(s[1])) for s in m.aspp_branches]
        self.gc, self.gb = Conv(m.global_pool[1]), BN(m.global_pool[2])
        self.fc, self.fb = Conv(m.fusion[0]), BN(m.fusion[1])
        self.p = m.fusion[3].p
        self.C = self.c1.Cout
        self.seed = 0
        self.mod = m

    @property
    def training(self):
        return self.mod.training

    def convs(self):
        return [self.c1, self.gc, self.fc] + [c for c, _ in self.br]

    def fwd(self, x):
        dev = x.t.device
        C, nb = self.C, len(self.br) + 2
        self.x = x
        cat = Act.new(x.B, x.H, x.W, C * nb, dev, fresh=False)
        self.cat = cat
        # under autocast the branch BatchNorms and the global broadcast also write the
        # concat's fp16 copy (the fusion conv's operand); only that copy when the fusion
        # conv's weight gradient reads it too (the branch BatchNorm backwards recompute
        # their ReLU masks from their inputs: nothing else reads the concat)
        cat16 = _h16(cat.M * C * nb, dev) if _AMP[0] else None
        only = FP16_ONLY_STORES[0] and cat16 is not None and self.fc.wgrad16_ok(x.W)
        o16 = (lambda k: (cat16, C * k, C * nb)) if cat16 is not None else (lambda k: None)
        ok16 = cat16 is not None
        for i, (cv, bn) in enumerate([(self.c1, self.b1)] + self.br):
            bn.fwd(cv.fwd(x, only16=True), relu=True, out=cat.slice(C * i, C), out16=o16(i), only16=only)
            ok16 = ok16 and bn.wrote16
        assert ok16 or not only, "fp16-only ASPP concat slices without the concat's fp16 copy"
        # global branch: mean -> 1x1 -> BN (over the batch) -> ReLU -> broadcast
        self.gm = Act.new(x.B, 1, 1, x.C, dev, fresh=False)
        _chk(L.lib().upr_t_pixel_sum(x.ptr(), x.B, x.H * x.W, x.C, x.cs, 0, ctypes.c_float(1.0 / (x.H * x.W)),
                                     _fp(self.gm.t), 0, _stream()), "gap")
        self.gp = self.gb.fwd(self.gc.fwd(self.gm), relu=True)
        if not only:
            _chk(L.lib().upr_t_broadcast(_fp(self.gp.t), x.B, x.H * x.W, C, ctypes.c_float(1.0), _fp(cat.t), cat.cs,
                                         C * (nb - 1), 0, _stream()), "broadcast")
        if ok16:
            _chk(L.lib().upr_t_broadcast16(_fp(self.gp.t), x.B, x.H * x.W, C, ctypes.c_float(1.0), _p(cat16),
                                           C * nb, C * (nb - 1), _stream()), "broadcast16")
        cat.t16 = cat16 if ok16 else None
        cat.stale32 = bool(only)
        self.a = self.fb.fwd(self.fc.fwd(cat, only16=True), relu=True)
        self.dropped = self.training  # the backward applies the mask only when this forward drew one
        if not self.dropped:
            self.mask = None
            return self.a  # nn.Dropout in eval mode is the identity
        out = Act.new(x.B, x.H, x.W, C, dev, fresh=False)
        self.mask = torch.empty((out.t.numel(),), dtype=torch.uint8, device=dev)
        self.seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        pointwise(self.a.t, None, out.t, out.t.numel(), 2, mask_out=self.mask, p=self.p, seed=self.seed)
        return out

    def bwd(self, g, gx):
        dev = g.t.device
        C, nb, x = self.C, len(self.br) + 2, self.x
        g_a = Act.new(g.B, g.H, g.W, C, dev)
        if self.dropped:
            pointwise(g.t, None, g_a.t, g.t.numel(), 3, mask_in=self.mask, p=self.p)
            g_a.fresh = False
        else:
            add_into(g_a, g)
        g_cf = Act.new(g.B, g.H, g.W, C, dev)
        self.fb.bwd(g_a, g_cf, relu=True)
        g_cat = Act.new(g.B, g.H, g.W, C * nb, dev)
        self.fc.bwd(self.cat, g_cf, g_cat)
        # global branch
        g_gp = Act.new(x.B, 1, 1, C, dev, fresh=False)
        _chk(L.lib().upr_t_pixel_sum(_fp(g_cat.t), x.B, x.H * x.W, C, g_cat.cs, C * (nb - 1), ctypes.c_float(1.0),
                                     _fp(g_gp.t), 0, _stream()), "gsum")
        relu_mask(g_gp, self.gp)
        g_gc = Act.new(x.B, 1, 1, C, dev)
        self.gb.bwd(g_gp, g_gc)
        g_gm = Act.new(x.B, 1, 1, x.C, dev)
        self.gc.bwd(self.gm, g_gc, g_gm)
        # conv branches (the first one initialises gx)
        for i, (cv, bn) in enumerate([(self.c1, self.b1)] + self.br):
            gs = g_cat.slice(C * i, C)
            g_c = Act.new(g.B, g.H, g.W, C, dev)
            bn.bwd(gs, g_c, relu=True)
            cv.bwd(x, g_c, gx)
        acc = gx.consume_fresh()
        _chk(L.lib().upr_t_broadcast(_fp(g_gm.t), x.B, x.H * x.W, x.C, ctypes.c_float(1.0 / (x.H * x.W)), gx.ptr(),
                                     gx.cs, 0, acc, _stream()), "broadcast_bwd")


class UpBlockT:
    """UpBlock (model.py:254-274) + the caller's skip add (model.py:346-348)."""

    def __init__(self, m):
        self.up = ConvT(m.up)
        self.c1, self.b1 = Conv(m.conv[0]), BN(m.conv[1])
        self.c2, self.b2 = Conv(m.conv[3]), BN(m.conv[4])

    def convs(self):
        return [self.up, self.c1, self.c2]

    def fwd(self, x, skip=None):
        """skip=None: UpBlock.forward alone (model.py:271-274, no skip add)."""
        self.x = x
        self.u = self.up.fwd(x)
        c1 = self.c1.fwd(self.u, only16=True)
        self.a1 = self.b1.fwd(c1, relu=True, only16=self.c2.wgrad16_ok(c1.W))
        # the skip add (model.py:346-348) in the BatchNorm apply's epilogue: relu(bn(c2)) + skip,
        # the same fp32 operations as the separate add
        return self.b2.fwd(self.c2.fwd(self.a1, only16=True), relu=True, res=skip, res_post=skip is not None)

    def bwd(self, g, gx, g_skip=None):
        dev = g.t.device
        if g_skip is not None:
            add_into(g_skip, g)
        g_c2 = Act.new(g.B, g.H, g.W, g.C, dev)
        self.b2.bwd(g, g_c2, relu=True, only16=self.c2.takes16_grad())
        g_a1 = Act.new(g.B, g.H, g.W, g.C, dev)
        self.c2.bwd(self.a1, g_c2, g_a1, gx_only16=True)
        g_c1 = Act.new(g.B, g.H, g.W, g.C, dev)
        self.b1.bwd(g_a1, g_c1, relu=True, only16=self.c1.takes16_grad())
        g_u = Act.new(g.B, g.H, g.W, g.C, dev)
        self.c1.bwd(self.u, g_c1, g_u, gx_keep16=True)  # + the fp16 copy ConvT's backward reads
        self.up.bwd(self.x, g_u, gx)


class FAMT:
    """EnhancedFAM (model.py:11-97)."""

    def __init__(self, m):
        self.b1 = Conv(m.branch1)
        self.b2 = Conv(m.branch2_conv)
        self.b3a, self.b3b = Conv(m.branch3_conv1), Conv(m.branch3_conv2)
        self.b4a, self.b4b = Conv(m.branch4_conv1), Conv(m.branch4_conv2)
        self.fu = Conv(m.fusion)
        self.ca1, self.ca2 = Conv(m.channel_attention[1]), Conv(m.channel_attention[3])
        self.sa = Conv(m.spatial_attention[0])

    def convs(self):
        return [self.b1, self.b2, self.b3a, self.b3b, self.b4a, self.b4b, self.fu, self.ca1, self.ca2, self.sa]

    def takes16_input(self, W):
        """Under autocast, every reader of this module's input x of width W takes its
        fp16 copy: branch1 / branch3 / branch4's first convs (forward on x.t16, weight
        gradients on the fp16 GEMM) and the 3x3 max-pool (fp16 path); the input may
        then be stored fp16-only."""
        return FP16_ONLY_STORES[0] and all(c.wgrad16_ok(W) for c in (self.b1, self.b3a, self.b4a))

    def fwd(self, x):
        dev = x.t.device
        lib, st = L.lib(), _stream()
        C = self.fu.Cout
        B, H, W = x.B, x.H, x.W
        HW = H * W
        self.x = x
        cat = Act.new(B, H, W, 4 * C, dev, fresh=False)
        self.cat = cat
        # under autocast the four branch convs also write the concat's fp16 copy (the fusion conv's operand)
        cat16 = _h16(B * H * W * 4 * C, dev) if _AMP[0] else None
        o16 = (lambda k: (cat16, k * C, 4 * C)) if cat16 is not None else (lambda k: None)
        # fp16-only stores: the concat's fp32 slices are read by nothing when the fusion
        # conv's weight gradient runs on the fp16 GEMM (it reads cat16), and t3 / t4 by
        # nothing when branch3 / branch4's second conv's weight gradient does (the ReLU
        # backward masks with their fp16 copies); the engine asserts on any fp32 read
        # of a stale activation
        cat16_only = FP16_ONLY_STORES[0] and cat16 is not None and self.fu.wgrad16_ok(W)
        self.b1.fwd(x, out=cat.slice(0, C), out16=o16(0), only16=cat16_only)
        ok16 = self.b1.wrote16
        self.mp = Act.new(B, H, W, x.C, dev, fresh=False)
        self.mp_code = torch.empty(B * H * W * x.C, dtype=torch.uint8, device=dev)  # argmax codes for the backward
        # mp's readers: branch2's conv (forward: its fp16 copy; weight gradient: the fp16
        # GEMM when wgrad16_ok) -- the backward of the pool itself takes the argmax codes
        maxpool_into(x, self.mp, 3, 1, 1, self.mp_code, only16=FP16_ONLY_STORES[0] and self.b2.wgrad16_ok(W))
        self.b2.fwd(self.mp, out=cat.slice(C, C), out16=o16(1), only16=cat16_only)
        ok16 = ok16 and self.b2.wrote16
        self.t3 = self.b3a.fwd(x, relu=True, only16=FP16_ONLY_STORES[0] and self.b3b.wgrad16_ok(W))
        self.b3b.fwd(self.t3, out=cat.slice(2 * C, C), out16=o16(2), only16=cat16_only)
        ok16 = ok16 and self.b3b.wrote16
        self.t4 = self.b4a.fwd(x, relu=True, only16=FP16_ONLY_STORES[0] and self.b4b.wgrad16_ok(W))
        self.b4b.fwd(self.t4, out=cat.slice(3 * C, C), out16=o16(3), only16=cat16_only)
        ok16 = ok16 and self.b4b.wrote16
        assert ok16 or not cat16_only, "fp16-only concat slices without the concat's fp16 copy"
        cat.t16 = cat16 if ok16 else None
        cat.stale32 = bool(ok16 and cat16_only)
        self.o = self.fu.fwd(cat, relu=True)
        self.pool = Act.new(B, 1, 1, C, dev, fresh=False)
        _chk(lib.upr_t_pixel_sum(_fp(self.o.t), B, HW, C, C, 0, ctypes.c_float(1.0 / HW), _fp(self.pool.t), 0, st),
             "gap")
        self.h1 = self.ca1.fwd(self.pool, relu=True)
        z = self.ca2.fwd(self.h1)
        self.ca = empty((B, C), dev)
        pointwise(z.t, None, self.ca, B * C, 0)
        self.o2 = empty((B, H, W, C), dev)
        self.m = Act.new(B, H, W, 2, dev, fresh=False)
        _chk(lib.upr_t_fam_ca_apply(_p(self.o.t), _p(self.ca), B, HW, C, _p(self.o2), _fp(self.m.t), st), "ca_apply")
        s_pre = self.sa.fwd(self.m)
        self.sav = empty((B, H, W), dev)
        out = Act.new(B, H, W, C, dev, fresh=False)
        _chk(lib.upr_t_fam_sa_apply(_p(self.o2), _fp(s_pre.t), B, HW, C, _p(self.sav), _fp(out.t), st), "sa_apply")
        return out

    def bwd(self, g, gx):
        """g: Act [B,H,W,32] (a channel slice of a wider tensor allowed); gx receives the input gradient."""
        dev = g.t.device
        lib, st = L.lib(), _stream()
        B, H, W, C = g.B, g.H, g.W, self.fu.Cout
        HW = H * W
        g_o2 = empty((B, H, W, C), dev)
        g_s = Act.new(B, H, W, 1, dev, fresh=False)
        assert not g.stale32, "FAM backward reads the fp32 gradient"
        _chk(lib.upr_t_fam_sa_bwd_cs(g.ptr(), g.cs, _p(self.o2), _p(self.sav), B, HW, C, _p(g_o2), _fp(g_s.t), st),
             "sa_bwd")
        g_m = Act.new(B, H, W, 2, dev)
        self.sa.bwd(self.m, g_s, g_m)
        g_o = Act.new(B, H, W, C, dev, fresh=False)
        g_ca = empty((B, C), dev)
        _chk(lib.upr_t_fam_ca_bwd(_p(g_o2), _fp(g_m.t), _fp(self.o.t), _p(self.o2), _p(self.ca), B, HW, C, _fp(g_o.t),
                                  _p(g_ca), st), "ca_bwd")
        g_z = Act.new(B, 1, 1, C, dev, fresh=False)
        pointwise(g_ca, self.ca, g_z.t, B * C, 1)
        g_h1 = Act.new(B, 1, 1, self.h1.C, dev)
        self.ca2.bwd(self.h1, g_z, g_h1)
        relu_mask(g_h1, self.h1)
        g_pool = Act.new(B, 1, 1, C, dev)
        self.ca1.bwd(self.pool, g_h1, g_pool)
        # under autocast the fusion conv's gradient operand (its fp16 copy) comes out of the same pass
        g16 = _h16(g_o.M * C, dev) if self.fu.amp and self.fu.mfma else None
        _chk(lib.upr_t_fam_pool_bwd16(_fp(g_o.t), _fp(g_pool.t), _fp(self.o.t), B, HW, C, _p(g16), st), "pool_bwd")
        if g16 is not None:
            g_o.t16, g_o.t16_grad = g16, True
        g_cat = Act.new(B, H, W, 4 * C, dev)
        # the four branch convs read slices of its fp16 copy; no fp32 store when every one of
        # them takes an fp16 gradient (their weight gradients on the fp16 GEMM: Wo % 64)
        only16 = all(c.takes16_grad() for c in (self.b1, self.b2, self.b3b, self.b4b))
        self.fu.bwd(self.cat, g_o, g_cat, gx_only16=only16, gx_keep16=True)
        self.b1.bwd(self.x, g_cat.slice(0, C), gx)
        g_mp = Act.new(B, H, W, self.x.C, dev)
        self.b2.bwd(self.mp, g_cat.slice(C, C), g_mp)
        gx.zero_if_fresh()
        _chk(lib.upr_t_maxpool_bwd_code(_p(self.mp_code), ctypes.byref(g_mp.view()), B, H, W, self.x.C, 3, 1, 1,
                                        H, W, ctypes.byref(gx.view()), 1, st), "maxpool_bwd")
        self.mp_code = None
        for (ca_, cb_, t) in ((self.b3a, self.b3b, self.t3), (self.b4a, self.b4b, self.t4)):
            k = 2 if cb_ is self.b3b else 3
            g_t = Act.new(B, H, W, t.C, dev)
            # the ReLU backward of t fused into this input gradient's epilogue (t's fp16 copy as
            # the mask); fp32 g_t skipped when the consuming conv takes the fp16 gradient only
            mask = (t.t16, t.C, ca_.takes16_grad()) if t.t16 is not None and t.whole16() else None
            if not cb_.bwd(t, g_cat.slice(k * C, C), g_t, mask=mask):
                relu_mask(g_t, t, want16=ca_.amp and ca_.mfma)
            ca_.bwd(self.x, g_t, gx)


class IENetT:
    """ResidualIENet (model.py:277-360)."""

    def __init__(self, m):
        Blk = PreActResBlockT if m._use_preact else ResBlockT
        self.inp = Conv(m.input_layer)
        self.enc = [Blk(m.enc1), Blk(m.enc2), Blk(m.enc3)]
        self.mid = []
        for sub in m.bottleneck:
            self.mid.append(ASPPT(sub) if type(sub).__name__ == "ASPPModule" else Blk(sub))
        self.dec = [UpBlockT(m.dec3), UpBlockT(m.dec2), UpBlockT(m.dec1)]
        self.h0, self.h2 = Conv(m.residual_head[0]), Conv(m.residual_head[2])

    def convs(self):
        out = [self.inp, self.h0, self.h2]
        for b in self.enc + self.mid + self.dec:
            out += b.convs()
        return out

    def fwd(self, x):
        B, _, H, W = x.shape
        self.x = x  # keeps the input alive: the backward reads it through the raw view below
        self.xin = (nchw_view(x), B, H, W)
        self.x1 = self.inp.fwd(None, relu=True, x_view=self.xin, out=Act.new(B, H, W, 32, x.device, fresh=False))
        self.x2 = self.enc[0].fwd(self.x1)
        self.x3 = self.enc[1].fwd(self.x2)
        self.x4 = self.enc[2].fwd(self.x3)
        t = self.x4
        self.mids = []
        for b in self.mid:
            self.mids.append(t)
            t = b.fwd(t)
        self.x5 = t
        d3 = self.dec[0].fwd(self.x5, self.x3)
        d2 = self.dec[1].fwd(d3, self.x2)
        self.d1 = self.dec[2].fwd(d2, self.x1)
        self.d3, self.d2 = d3, d2
        self.h = self.h0.fwd(self.d1, relu=True)
        r = self.h2.fwd(self.h)
        illu = empty((B, 1, H, W), x.device)
        _chk(L.lib().upr_t_head_fwd(_p(x), _fp(r.t), _p(illu), B, H, W, _stream()), "head")
        return illu

    def bwd(self, g_r):
        """g_r: Act [B,H,W,1], gradient of the residual-head output."""
        dev = g_r.t.device
        B, H, W = g_r.B, g_r.H, g_r.W

        def like(a):
            return Act.new(a.B, a.H, a.W, a.C, dev)
        g_h = like(self.h)
        self.h2.bwd(self.h, g_r, g_h)
        # under autocast the masked gradient's fp16 copy (h0's input-gradient / weight-
        # gradient operand) comes out of the mask pass, not a separate cast
        relu_mask(g_h, self.h, want16=self.h0.amp and self.h0.mfma)
        g_d1 = like(self.d1)
        self.h0.bwd(self.d1, g_h, g_d1)
        g_x1, g_x2, g_x3 = like(self.x1), like(self.x2), like(self.x3)
        g_d2, g_d3 = like(self.d2), like(self.d3)
        self.dec[2].bwd(g_d1, g_d2, g_x1)
        self.dec[1].bwd(g_d2, g_d3, g_x2)
        g_t = like(self.x5)
        self.dec[0].bwd(g_d3, g_t, g_x3)
        for b, xin in zip(reversed(self.mid), reversed(self.mids)):
            g_in = like(xin)
            b.bwd(g_t, g_in)
            g_t = g_in
        self.enc[2].bwd(g_t, g_x3)
        self.enc[1].bwd(g_x3, g_x2)
        self.enc[0].bwd(g_x2, g_x1)
        self.inp.bwd_relu_stem(None, g_x1, self.x1, x_view=self.xin)


class UPRetinexTrainGraph:
    """MultiScaleUP_Retinex.forward (model.py:415-455) in training mode and its
    backward.  Built once per model; buffers are reallocated per step by the
    caching allocator (torch.empty), weights re-packed per step."""

    def __init__(self, model, head_only=False):
        """head_only: the multi-scale enhancement head alone (multi_scale_enhance
        with a caller-given reflectance, model.py:415-443), no IENet."""
        self.model = model
        self.ie = None if head_only else IENetT(model.ie_net)
        self.s1c, self.s1f = Conv(model.scale1[0]), FAMT(model.scale1[2])
        self.s2c, self.s2f = Conv(model.scale2[1]), FAMT(model.scale2[3])
        self.s3c, self.s3f = Conv(model.scale3[1]), FAMT(model.scale3[3])
        self.fusion, self.outc = Conv(model.fusion), Conv(model.output_layer)
        self._convs = (self.ie.convs() if self.ie is not None else []) + \
            [self.s1c, self.s2c, self.s3c, self.fusion, self.outc] + \
            self.s1f.convs() + self.s2f.convs() + self.s3f.convs()

    def pack(self):
        pack_convs(self._convs, self)

    def forward(self, x):
        """x [B,3,H,W] fp32 NCHW (H, W multiples of 16) -> (enh, refl, illu)."""
        lib, st = L.lib(), _stream()
        B, _, H, W = x.shape
        dev = x.device
        self.x = x
        set_amp(autocast_active())
        self.pack()
        illu = self.ie.fwd(x)
        self.illu = illu
        o = self._head_fwd(x)
        self.e = empty((B, H, W, 3), dev)
        refl = empty((B, 3, H, W), dev)
        enh = empty((B, 3, H, W), dev)
        _chk(lib.upr_t_retinex_fwd(_p(x), _p(illu), _fp(o.t), _p(self.e), _p(refl), _p(enh), B, H, W, st),
             "retinex")
        self.refl, self.enh = refl, enh
        return enh, refl, illu

    def enhance_forward(self, x, refl):
        """Head only: x, refl [B,3,H,W] fp32 NCHW (H, W multiples of 16) -> enh."""
        lib, st = L.lib(), _stream()
        B, _, H, W = x.shape
        self.x = x
        set_amp(autocast_active())
        self.pack()
        o = self._head_fwd(x)
        self.e = empty((B, H, W, 3), x.device)
        enh = empty((B, 3, H, W), x.device)
        _chk(lib.upr_t_enhance_fwd(_p(refl), _fp(o.t), _p(self.e), _p(enh), B, H, W, st), "enhance")
        self.refl, self.enh = refl, enh
        return enh

    def enhance_backward(self, g_enh, want_refl):
        """Head only: parameter gradients into the .grad views; returns dL/drefl
        (None unless want_refl)."""
        lib, st = L.lib(), _stream()
        B, _, H, W = self.x.shape
        g_o = Act.new(B, H, W, 3, self.x.device, fresh=False)
        g_refl = empty((B, 3, H, W), self.x.device) if want_refl else None
        _chk(lib.upr_t_enhance_bwd(_p(self.e), _p(self.refl), _p(g_enh), _fp(g_o.t), _p(g_refl), B, H, W, st),
             "enhance_bwd")
        self._head_bwd(g_o)
        return g_refl

    def _head_fwd(self, x):
        """scale1/2/3 -> concat -> fusion -> output_layer (model.py:415-440): the
        pre-sigmoid output [B,H,W,3] (Act)."""
        lib, st = L.lib(), _stream()
        B, _, H, W = x.shape
        dev = x.device
        # pyramid (model.py:415-432): bilinear 0.5 / 0.25, max-pool 2 / 4
        xv = nchw_view(x)
        pyr = []
        for f, k in ((2, 2), (4, 4)):
            xs = Act.new(B, H // f, W // f, 3, dev, fresh=False)
            _chk(lib.upr_t_bilinear(ctypes.byref(xv), B, H, W, 3, ctypes.byref(xs.view()), H // f, W // f, 0, st),
                 "bilinear")
            xp = Act.new(B, H // f // k, W // f // k, 3, dev, fresh=False)
            _chk(lib.upr_t_maxpool(ctypes.byref(xs.view()), B, H // f, W // f, 3, k, k, 0, ctypes.byref(xp.view()),
                                   H // f // k, W // f // k, st), "maxpool")
            pyr.append(xp)
        self.pyr = pyr
        # the scale stems' outputs fp16-only where every reader takes fp16 (FAMT.takes16_input;
        # the stems' own ReLU backward masks with the fp16 copy)
        self.s1 = self.s1c.fwd(None, relu=True, x_view=(xv, B, H, W),
                               out=Act.new(B, H, W, 32, dev, fresh=False), only16=self.s1f.takes16_input(W))
        f1 = self.s1f.fwd(self.s1)
        self.s2 = self.s2c.fwd(pyr[0], relu=True, only16=self.s2f.takes16_input(pyr[0].W))
        f2 = self.s2f.fwd(self.s2)
        self.s3 = self.s3c.fwd(pyr[1], relu=True)
        f3 = self.s3f.fwd(self.s3)
        fused = Act.new(B, H, W, 96, dev, fresh=False)
        # under autocast the concat's fp16 copy (the fusion conv's operand) is written alongside;
        # only that copy when the fusion conv's weight gradient also reads it (wm = 2)
        f16 = _h16(B * H * W * 96, dev) if _AMP[0] else None
        ok16 = f16 is not None
        wm = 2 if ok16 and self.fusion.wgrad16_ok(W) else 0
        if ok16:
            rc = lib.upr_t_copy16(ctypes.byref(f1.view()), ctypes.byref(fused.slice(0, 32).view()), B, H, W, 32, wm,
                                  _p(f16), 96, st)
            for i, f in enumerate((f2, f3)):
                if rc != 0:
                    break
                rc = lib.upr_t_bilinear16(ctypes.byref(f.view()), B, f.H, f.W, 32,
                                          ctypes.byref(fused.slice(32 * (i + 1), 32).view()), H, W, wm,
                                          ctypes.c_void_p(f16.data_ptr() + 2 * 32 * (i + 1)), 96, st)
            if rc not in (0, L.UPR_ERR_UNSUPPORTED):
                _chk(rc, "cat16")
            ok16 = rc == 0
        if not ok16:  # every slice in fp32 (whatever the fp16 attempt left behind)
            _chk(lib.upr_t_copy(ctypes.byref(f1.view()), ctypes.byref(fused.slice(0, 32).view()), B, H, W, 32, 0, st),
                 "cat")
            for i, f in enumerate((f2, f3)):
                _chk(lib.upr_t_bilinear(ctypes.byref(f.view()), B, f.H, f.W, 32,
                                        ctypes.byref(fused.slice(32 * (i + 1), 32).view()), H, W, 0, st), "upsample")
        fused.t16 = f16 if ok16 else None
        fused.stale32 = bool(ok16 and wm == 2)
        self.fused = fused
        self.fz = self.fusion.fwd(fused)
        self.f_hw = [(f2.H, f2.W), (f3.H, f3.W)]
        return self.outc.fwd(self.fz)

    def backward(self, g_enh, g_refl=None, g_illu=None):
        """Accumulates every parameter gradient into the model's .grad views
        (zeroed first by the caller)."""
        lib, st = L.lib(), _stream()
        x = self.x
        B, _, H, W = x.shape
        dev = x.device
        g_o = Act.new(B, H, W, 3, dev, fresh=False)
        g_r = Act.new(B, H, W, 1, dev, fresh=False)
        _chk(lib.upr_t_retinex_bwd(_p(x), _p(self.illu), _p(self.e), _p(self.refl), _p(g_enh), _p(g_refl),
                                   _p(g_illu), _fp(g_o.t), _fp(g_r.t), B, H, W, st), "retinex_bwd")
        self._head_bwd(g_o)
        self.ie.bwd(g_r)

    def _head_bwd(self, g_o):
        """Backward of _head_fwd from dL/d(output_layer output) (Act [B,H,W,3])."""
        lib, st = L.lib(), _stream()
        x = self.x
        B, _, H, W = x.shape
        dev = x.device
        g_fz = Act.new(B, H, W, 32, dev)
        self.outc.bwd(self.fz, g_o, g_fz)
        g_fused = Act.new(B, H, W, 96, dev)
        self.fusion.bwd(self.fused, g_fz, g_fused)
        for (sc, sf, s_act, xin), i in zip(((self.s1c, self.s1f, self.s1, None),
                                            (self.s2c, self.s2f, self.s2, self.pyr[0]),
                                            (self.s3c, self.s3f, self.s3, self.pyr[1])), range(3)):
            if i == 0:
                g_f = g_fused.slice(0, 32)  # read in place by the FAM backward (no split copy)
            else:
                g_f = Act.new(s_act.B, s_act.H, s_act.W, 32, dev, fresh=False)
                zero(g_f.t)
                _chk(lib.upr_t_bilinear_bwd(ctypes.byref(g_fused.slice(32 * i, 32).view()), B, g_f.H, g_f.W, 32, H, W,
                                            ctypes.byref(g_f.view()), st), "upsample_bwd")
            g_s = Act.new(s_act.B, s_act.H, s_act.W, 32, dev)
            sf.bwd(g_f, g_s)
            if i == 0:
                sc.bwd_relu_stem(None, g_s, s_act, x_view=(nchw_view(x), B, H, W))
            else:
                sc.bwd_relu_stem(xin, g_s, s_act)
