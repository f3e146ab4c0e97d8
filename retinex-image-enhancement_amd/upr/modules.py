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
    autograd would).

Input / output: NCHW float32 tensors on a ROCm device, like the reference
module's forward.  There is no CPU path.
"""
import ctypes

import torch

from . import _lib as L
from .train import (FAMT, ASPPT, Act, PreActResBlockT, ResBlockT, UpBlockT, _chk, _stream, autocast_active, empty,
                    nchw_view, set_amp)

_LAYERS = {"EnhancedFAM": FAMT, "ResBlock": ResBlockT, "PreActResBlock": PreActResBlockT, "ASPPModule": ASPPT,
           "UpBlock": UpBlockT}


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


def _layer(module, dev):
    ent = module.__dict__.get("_upr_layer")
    if ent is None or ent[0] != dev:
        ent = (dev, _LAYERS[type(module).__name__](module))
        module.__dict__["_upr_layer"] = ent
    return ent[1]


def _run(layer, x):
    set_amp(autocast_active())
    for c in layer.convs():
        c.pack()
    return layer.fwd(_to_nhwc(x))


class _SubmoduleStep(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, layer, module):
        y = _to_nchw(_run(layer, x))
        ctx.layer, ctx.module = layer, module
        ctx.x_shape = x.shape
        return y

    @staticmethod
    def backward(ctx, g):
        layer, module = ctx.layer, ctx.module
        for p in module.parameters():
            if p.requires_grad and p.grad is None:
                p.grad = torch.zeros_like(p)
        B, C, H, W = ctx.x_shape
        gx = Act.new(B, H, W, C, g.device, fresh=True)
        with torch.cuda.device(g.device):
            layer.bwd(_to_nhwc(g.contiguous().to(torch.float32)), gx)
            gx.zero_if_fresh()
            out = _to_nchw(gx)
        return out, None, None, None


def submodule_forward(module, x):
    """module(x) for one of the reference submodules (see the module docstring)."""
    name = type(module).__name__
    if not isinstance(x, torch.Tensor) or x.device.type != "cuda":
        dev = x.device if isinstance(x, torch.Tensor) else type(x)
        raise RuntimeError(f"{name}.forward: input on '{dev}'. This framework executes UP-Retinex only on ROCm "
                           f"devices (gfx950 HIP kernels, no CPU path): use module.to('cuda') and a 'cuda' tensor.")
    if x.dtype != torch.float32:
        raise TypeError(f"{name}.forward: standalone submodules compute in float32 (got {x.dtype}); the fp16 "
                        f"path is the fused MultiScaleUP_Retinex forward")
    if x.dim() != 4:
        raise RuntimeError(f"{name}.forward: expected a [B,C,H,W] tensor, got shape {tuple(x.shape)}")
    x = x.contiguous()
    layer = _layer(module, x.device)
    if module.training and torch.is_grad_enabled():
        anchor = module.__dict__.get("_upr_anchor")
        if anchor is None or anchor.device != x.device:
            anchor = torch.empty(0, device=x.device, requires_grad=True)
            module.__dict__["_upr_anchor"] = anchor
        y = _SubmoduleStep.apply(x, anchor, layer, module)
    else:
        with torch.no_grad():
            y = _to_nchw(_run(layer, x))
    if module.training:
        from .autograd import bump_weights_epoch
        bump_weights_epoch()  # BatchNorm running statistics changed in place
    return y
