"""Autograd glue so the reference's training loop runs unchanged
(trainers/train.py:91-103: `model(img_low)` -> `criterion(...)` ->
`loss.backward()` -> clip -> `optimizer.step()`).

Autograd nodes, each a whole subgraph whose forward and backward are the
HIP engines of upr/train.py and upr/loss_engine.py:
  _ModelStep  MultiScaleUP_Retinex training forward; backward = the explicit
              network backward, accumulating every parameter's gradient into
              the flat gradient buffer (the .grad views);
  _HeadStep   multi_scale_enhance alone (caller-given reflectance);
  _IENetStep  ResidualIENet alone;
  _LossStep   TotalLoss forward; its gradients w.r.t. (enh, illu, refl) are
              produced with the forward and scaled on the device by the
              incoming gradient in backward (GradScaler / loss weights).
"""
import ctypes

import torch

from . import _lib as L
from .train import FlatParams, UPRetinexTrainGraph, _chk, _p, _stream, zero

_weights_epoch = [0]


def weights_epoch():
    """Bumped whenever the training kernels change parameters or BatchNorm
    buffers in place (the inference handle cache keys on it)."""
    return _weights_epoch[0]


def bump_weights_epoch():
    _weights_epoch[0] += 1


class _ModelStep(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, graph):
        enh, refl, illu = graph.forward(x)
        bump_weights_epoch()  # BatchNorm running stats were updated
        ctx.graph = graph
        return enh, refl, illu

    @staticmethod
    def backward(ctx, g_enh, g_refl, g_illu):
        graph = ctx.graph
        flat = graph.flat
        if flat.attach_grads():
            zero(flat.grad)       # zero_grad(set_to_none=True) dropped the views
        dev = graph.x.device
        if g_enh is None:
            g_enh = torch.empty_like(graph.enh)
            zero(g_enh)
        g_enh = g_enh.contiguous()
        g_refl = g_refl.contiguous() if g_refl is not None else None
        g_illu = g_illu.contiguous() if g_illu is not None else None
        with torch.cuda.device(dev):
            graph.backward(g_enh, g_refl, g_illu)
        return None, None, None


def model_train_forward(model, x):
    """Training-mode forward of MultiScaleUP_Retinex on the HIP engine."""
    st = model.__dict__.get("_upr_train")
    if st is None or st["device"] != x.device:
        ps = list(model.parameters())
        flat = getattr(ps[0], "_upr_flat", None)
        if flat is None or any(getattr(p, "_upr_flat", None) is not flat for p in ps) or \
                flat.flat.device != x.device:
            flat = FlatParams(model)
        graph = UPRetinexTrainGraph(model)
        graph.flat = flat
        anchor = torch.empty(0, device=x.device, requires_grad=True)
        st = {"device": x.device, "flat": flat, "graph": graph, "anchor": anchor}
        model.__dict__["_upr_train"] = st
    if x.dtype != torch.float32:
        raise TypeError("UP-Retinex HIP training computes in float32; pass a float32 batch")
    return _ModelStep.apply(x.contiguous(), st["anchor"], st["graph"])


class _HeadStep(torch.autograd.Function):
    """MultiScaleUP_Retinex.multi_scale_enhance (models/model.py:415-443) with a
    caller-given reflectance: forward = the head layers of the training graph
    (scale branches, FAM, fusion, output conv) and the combine; backward =
    their explicit backward from dL/d(enhanced): parameter gradients accumulate
    into the .grad views, dL/d(reflectance) is returned.  No gradient w.r.t.
    x (as the full model's node)."""

    @staticmethod
    def forward(ctx, x, refl, anchor, graph):
        enh = graph.enhance_forward(x, refl)
        ctx.graph, ctx.want_refl = graph, refl.requires_grad
        return enh

    @staticmethod
    def backward(ctx, g_enh):
        graph = ctx.graph
        flat = graph.flat
        if flat.attach_grads():
            zero(flat.grad)
        with torch.cuda.device(graph.x.device):
            g_refl = graph.enhance_backward(g_enh.contiguous().to(torch.float32), ctx.want_refl)
        return None, g_refl, None, None


def head_train_forward(model, x, refl):
    """Differentiable multi_scale_enhance on the HIP engine (fp32; H, W
    multiples of 16).  Every call gets its own head graph (saved activations)."""
    from .train import UPRetinexTrainGraph
    if x.dtype != torch.float32 or refl.dtype != torch.float32:
        raise TypeError("UP-Retinex HIP training computes in float32; pass float32 x / reflectance")
    B, C, H, W = x.shape
    if C != 3 or tuple(refl.shape) != (B, 3, H, W) or H % 16 or W % 16:
        raise ValueError(f"multi_scale_enhance (differentiable): x / reflectance [B,3,H,W] with H, W multiples "
                         f"of 16, got {tuple(x.shape)} / {tuple(refl.shape)}")
    ps = list(model.parameters())
    flat = getattr(ps[0], "_upr_flat", None)
    if flat is None or any(getattr(p, "_upr_flat", None) is not flat for p in ps) or flat.flat.device != x.device:
        flat = FlatParams(model)
    anchor = model.__dict__.get("_upr_anchor")
    if anchor is None or anchor.device != x.device:
        anchor = torch.empty(0, device=x.device, requires_grad=True)
        model.__dict__["_upr_anchor"] = anchor
    graph = UPRetinexTrainGraph(model, head_only=True)
    graph.flat = flat
    return _HeadStep.apply(x.contiguous(), refl.contiguous(), anchor, graph)


class _IENetStep(torch.autograd.Function):
    """ResidualIENet.forward (models/model.py:333-360) in training mode on its
    own: forward = the IENet layer objects of upr/train.py, backward = their
    explicit backward from dL/d(illumination) (sigmoid backward on the device,
    then the residual head and the network); parameter gradients accumulate
    into the .grad views.  No gradient w.r.t. the network input (as the full
    model's node)."""

    @staticmethod
    def forward(ctx, x, anchor, ie, flat):
        from .train import set_amp, autocast_active, pack_convs
        set_amp(autocast_active())
        pack_convs(ie.convs(), ie)
        illu = ie.fwd(x)
        bump_weights_epoch()  # BatchNorm running stats were updated
        ctx.ie, ctx.flat, ctx.illu = ie, flat, illu
        return illu

    @staticmethod
    def backward(ctx, g_illu):
        from .train import Act
        ie, flat, illu = ctx.ie, ctx.flat, ctx.illu
        if flat.attach_grads():
            zero(flat.grad)
        B, _, H, W = illu.shape
        g_r = Act.new(B, H, W, 1, illu.device, fresh=False)
        with torch.cuda.device(illu.device):
            # illu = sigmoid(mean_c(x) + r): dL/dr = g * illu * (1 - illu)  ([B,1,H,W] == NHWC with C = 1)
            _chk(L.lib().upr_t_pointwise(_p(g_illu.contiguous().to(torch.float32)), _p(illu), _p(g_r.t), illu.numel(),
                                         1, None, None, ctypes.c_float(0), ctypes.c_uint64(0), _stream()),
                 "sigmoid_bwd")
            ie.bwd(g_r)
        return None, None, None, None


def ienet_train_forward(module, x):
    """Training-mode ResidualIENet forward on the HIP engine.  Every call gets
    its own layer objects (saved activations), like reference autograd."""
    from .train import IENetT
    if x.dtype != torch.float32:
        raise TypeError("UP-Retinex HIP training computes in float32; pass a float32 batch")
    ps = list(module.parameters())
    flat = getattr(ps[0], "_upr_flat", None)
    if flat is None or any(getattr(p, "_upr_flat", None) is not flat for p in ps) or flat.flat.device != x.device:
        flat = FlatParams(module)
    anchor = module.__dict__.get("_upr_anchor")
    if anchor is None or anchor.device != x.device:
        anchor = torch.empty(0, device=x.device, requires_grad=True)
        module.__dict__["_upr_anchor"] = anchor
    return _IENetStep.apply(x.contiguous(), anchor, IENetT(module), flat)


class _LossStep(torch.autograd.Function):
    @staticmethod
    def forward(ctx, low, enh, illu, refl, engine):
        terms, grads = engine(low, enh, illu, refl, grads=True)
        ctx.grads = grads
        total = _scalar_of(terms, 7)
        ctx.mark_non_differentiable(terms)
        return total, terms

    @staticmethod
    def backward(ctx, g, _g_terms):
        lib = L.lib()
        g = g.contiguous().to(torch.float32)
        outs = []
        for t in ctx.grads:
            _chk(lib.upr_t_pointwise(_p(t), _p(g), _p(t), t.numel(), 5, None, None, ctypes.c_float(0),
                                     ctypes.c_uint64(0), _stream()), "scale_grad")
            outs.append(t)
        g_enh, g_illu, g_refl = outs
        return None, g_enh, g_illu, g_refl, None


def _scalar_of(terms, i):
    """0-dim device tensor holding terms[i] (a one-element device copy)."""
    out = torch.empty((), dtype=torch.float32, device=terms.device)
    src = L.UprView(terms.data_ptr() + 4 * i, 0, 0, 0, 1)
    dst = L.UprView(out.data_ptr(), 0, 0, 0, 1)
    _chk(L.lib().upr_t_copy(ctypes.byref(src), ctypes.byref(dst), 1, 1, 1, 1, 0, _stream()), "scalar")
    return out


def loss_forward(engine, low, enh, illu, refl):
    """TotalLoss.forward on the HIP engine -> (total 0-dim tensor, device terms[9]).
    With autograd recording (training), total carries the loss backward.

    The engine produces the gradients w.r.t. (enh, illu, refl) only: the
    reference's exposure target, smoothness edge weights and spatial /
    frequency terms also depend on img_low, so an img_low that requires grad
    is refused instead of silently getting no gradient."""
    if torch.is_grad_enabled() and low.requires_grad:
        raise NotImplementedError("UP-Retinex losses: no gradient w.r.t. img_low (the HIP loss engine "
                                  "differentiates w.r.t. enhanced / illumination / reflectance); pass "
                                  "img_low.detach() or run under torch.no_grad()")
    if torch.is_grad_enabled() and (enh.requires_grad or illu.requires_grad or refl.requires_grad):
        return _LossStep.apply(low, enh, illu, refl, engine)
    terms, _ = engine(low, enh, illu, refl, grads=False)
    return _scalar_of(terms, 7), terms
