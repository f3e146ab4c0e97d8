"""Standalone forward of the reference's submodules on the HIP kernels.

Reference modules (models/model.py): EnhancedFAM (:11-97), ResBlock (:100-135),
PreActResBlock (:138-178), ASPPModule (:181-251), UpBlock (:254-274).  Inside
MultiScaleUP_Retinex they run fused into the inference graph (csrc/model.hip);
called on their own they run on the per-module layer objects of upr/train.py
(fp32 NHWC activations, MFMA implicit-GEMM convs, BatchNorm kernels):

  * eval mode: BatchNorm from the running statistics (`upr_t_bn_eval_stats`),
    Dropout is the identity; the result does not record autograd history;
  * training mode: batch-statistics BatchNorm with the running-stat update,
    Dropout(0.1) masks, and an autograd node whose backward is the layer's
    explicit backward (parameter gradients accumulate into .grad, as
    autograd would).  Every recording forward gets a layer object of its own,
    held by its autograd node, so its saved activations / BatchNorm statistics /
    Dropout mask survive any later forward of the same module (reference
    autograd keeps one saved-tensor set per call); eval / no-grad forwards use
    a separate cached layer.

Input / output: NCHW tensors on a ROCm device, like the reference module's
forward, in the module's dtype.  A `.half()` module takes float16 input (a
float16 input to a float32 module, or the reverse, raises like the reference's
conv): it computes on an fp32 shadow copy of its parameters with the convs in
fp16 arithmetic (fp16 operands, fp32 accumulation: the fp16 MFMA kernels) and
BatchNorm / attention in fp32, returns float16, and in training mode writes
the running statistics back and accumulates float16 .grad like the module's
own parameters would get.  There is no CPU path.
"""
import copy
import ctypes

import torch

from . import _lib as L
from .train import (FAMT, ASPPT, Act, PreActResBlockT, ResBlockT, UpBlockT, _chk, _stream, autocast_active, empty,
                    nchw_view, set_amp)

_LAYERS = {"EnhancedFAM": FAMT, "ResBlock": ResBlockT, "PreActResBlock": PreActResBlockT, "ASPPModule": ASPPT,
           "UpBlock": UpBlockT}
_CACHE_KEYS = ("_upr_layer", "_upr_eval_layer", "_upr_shadow", "_upr_anchor")


def _to_nhwc(x):
    B, C, H, W = x.shape
    a = Act.new(B, H, W, C, x.device, fresh=False)
    _chk(L.lib().upr_t_copy(ctypes.byref(nchw_view(x)), ctypes.byref(a.view()), B, H, W, C, 0, _stream()), "to_nhwc")
    return a


def _to_nchw(a):
    out = empty((a.B, a.C, a.H, a.W), a.t.device)
    _chk(L.lib().upr_t_copy(ctypes.byref(a.view()), ctypes.byref(nchw_view(out)), a.B, a.H, a.W, a.C, 0, _stream()),
         "to_nchw")
    return out


def _compute_module(module, dev):
    """The fp32 module the layer objects read: the module itself, or for a
    .half() module an fp32 shadow copy synced from it (parameters, buffers and
    every submodule's training flag) on each call."""
    if next(module.parameters()).dtype == torch.float32:
        return module
    ent = module.__dict__.get("_upr_shadow")
    if ent is None or ent[0] != dev:
        sh = copy.deepcopy(module)
        for m in sh.modules():
            for k in _CACHE_KEYS:
                m.__dict__.pop(k, None)
        sh = sh.float()
        ent = (dev, sh)
        module.__dict__["_upr_shadow"] = ent
    sh = ent[1]
    with torch.no_grad():
        for ps, ph in zip(sh.parameters(), module.parameters()):
            ps.copy_(ph)
        for bs, bh in zip(sh.buffers(), module.buffers()):
            bs.copy_(bh)
    for ms, mh in zip(sh.modules(), module.modules()):
        ms.training = mh.training
    return sh


def _write_back_buffers(cm, module):
    """Running statistics the fp32 shadow updated -> the .half() module."""
    if cm is module:
        return
    with torch.no_grad():
        for bs, bh in zip(cm.buffers(), module.buffers()):
            bh.copy_(bs)


def _eval_layer(module, cm, dev):
    ent = module.__dict__.get("_upr_eval_layer")
    if ent is None or ent[0] != dev or ent[1] is not cm:
        ent = (dev, cm, _LAYERS[type(module).__name__](cm))
        module.__dict__["_upr_eval_layer"] = ent
    return ent[2]


def _run(layer, x, fp16):
    set_amp(fp16 or autocast_active())
    for c in layer.convs():
        c.pack()
    return layer.fwd(_to_nhwc(x))


class _SubmoduleStep(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, layer, module, cm):
        fp16 = x.dtype == torch.float16
        y = _to_nchw(_run(layer, x.float(), fp16))
        _write_back_buffers(cm, module)
        ctx.layer, ctx.module, ctx.cm = layer, module, cm
        ctx.x_shape, ctx.x_dtype = x.shape, x.dtype
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        layer, module, cm = ctx.layer, ctx.module, ctx.cm
        shadow = cm is not module
        for p in cm.parameters():
            if p.requires_grad and (p.grad is None or shadow):
                p.grad = torch.zeros_like(p)  # a shadow collects this backward's gradients alone
        B, C, H, W = ctx.x_shape
        gx = Act.new(B, H, W, C, g.device, fresh=True)
        with torch.cuda.device(g.device):
            layer.bwd(_to_nhwc(g.contiguous().to(torch.float32)), gx)
            gx.zero_if_fresh()
            out = _to_nchw(gx)
        if shadow:
            for ps, ph in zip(cm.parameters(), module.parameters()):
                if ph.requires_grad:
                    gh = ps.grad.to(ph.dtype)
                    ph.grad = gh if ph.grad is None else ph.grad + gh
        return out.to(ctx.x_dtype), None, None, None, None


def submodule_forward(module, x):
    """module(x) for one of the reference submodules (see the module docstring)."""
    name = type(module).__name__
    if not isinstance(x, torch.Tensor) or x.device.type != "cuda":
        dev = x.device if isinstance(x, torch.Tensor) else type(x)
        raise RuntimeError(f"{name}.forward: input on '{dev}'. This framework executes UP-Retinex only on ROCm "
                           f"devices (gfx950 HIP kernels, no CPU path): use module.to('cuda') and a 'cuda' tensor.")
    if x.dim() != 4:
        raise RuntimeError(f"{name}.forward: expected a [B,C,H,W] tensor, got shape {tuple(x.shape)}")
    wdt = next(module.parameters()).dtype
    if x.dtype not in (torch.float32, torch.float16) or wdt not in (torch.float32, torch.float16):
        raise TypeError(f"{name}.forward: float32 or float16 modules / inputs only (input {x.dtype}, weights {wdt})")
    if x.dtype != wdt:  # the reference's F.conv2d raises on the same mismatch
        raise RuntimeError(f"{name}.forward: Input type ({x.dtype}) and weight type ({wdt}) should be the same")
    x = x.contiguous()
    fp16 = x.dtype == torch.float16
    cm = _compute_module(module, x.device)
    if module.training and torch.is_grad_enabled():
        anchor = module.__dict__.get("_upr_anchor")
        if anchor is None or anchor.device != x.device:
            anchor = torch.empty(0, device=x.device, requires_grad=True)
            module.__dict__["_upr_anchor"] = anchor
        layer = _LAYERS[name](cm)  # this call's own saved state (held by its autograd node)
        module.__dict__["_upr_layer"] = (x.device, layer)  # the latest call's layer (tests replay its Dropout mask)
        y = _SubmoduleStep.apply(x, anchor, layer, module, cm)
    else:
        layer = _eval_layer(module, cm, x.device)
        with torch.no_grad():
            y = _to_nchw(_run(layer, x.float(), fp16)).to(x.dtype)
        _write_back_buffers(cm, module)
    if module.training:
        from .autograd import bump_weights_epoch
        bump_weights_epoch()  # BatchNorm running statistics changed in place
    return y
