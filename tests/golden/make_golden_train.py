#!/usr/bin/env python3
"""Training golden vectors G6/G7 (run ONCE in the build container, never on the GPU box).

Imports the reference read-only from /root/reference (losses/loss.py,
models/model.py) and records, on seeded inputs:

  G6 g6_losses.npz      every loss term of losses/loss.py + TotalLoss on
                        B=2 64x64 random maps, plus calculate_texture_complexity
                        ('tv' and 'edge_density')
  G6c3 g6_losses_c3.npz the reference self-test's shapes (loss.py:806-844):
                        3-channel illumination, smoothness / decoupling /
                        TotalLoss values and gradients
  G6nr g6_losses_norefl.npz  TotalLoss(low, enh, illu) with reflectance=None
                        (loss.py:678-682: the decoupling term is 0) on G6's
                        inputs: value, loss dict, gradients w.r.t. enh / illu
  G7 g7_train_step.npz  one train_one_epoch step body (trainers/train.py:63-103,
                        no AMP) of the plain model (seed 0) on x = rand(2,3,64,64)
                        (generator seed 2): loss dict, per-parameter gradient
                        checksums, the clip norm, params after Adam(1e-4, wd 1e-5)
                        and the updated BatchNorm running stats.

losses/loss.py imports torchvision.models at module level for the VGG19 of
PerceptualLoss (`models.vgg19(pretrained=True)`, loss.py:195).  torchvision is not
installed and pretrained weights need a download, so a minimal in-memory module
named torchvision.models is registered first whose vgg19() returns the VGG-19
"E" `features` stack with PyTorch's default Conv2d init drawn under
torch.manual_seed(VGG_SEED) — the perceptual term is pinned against that seeded
random VGG (the product/oracle rebuild it with the same seed); parity against
pretrained weights is unpinned.  No reference source or bytecode is copied.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train.py
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

REF = os.environ.get("UPR_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
VGG_SEED = 1234

VGG19_E = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]


def vgg19_features():
    layers, c = [], 3
    for v in VGG19_E:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(c, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            c = v
    return nn.Sequential(*layers)


def _install_vgg_stub():
    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")

    def vgg19(pretrained=False, **kw):
        torch.manual_seed(VGG_SEED)
        m = nn.Module()
        m.features = vgg19_features()
        return m
    tvm.vgg19 = vgg19
    tv.models = tvm
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = tvm


_install_vgg_stub()
sys.path.insert(0, REF)
from losses import loss as ref_loss  # noqa: E402  (reference losses/loss.py)
from models import model as ref_model  # noqa: E402  (reference models/model.py)


def vgg_state():
    """The first 19 layers' weights, as PerceptualLoss keeps them."""
    torch.manual_seed(VGG_SEED)
    f = vgg19_features()
    return {k: v for k, v in f.state_dict().items() if int(k.split(".")[0]) <= 18}


def g6():
    gen = torch.Generator().manual_seed(6)
    low = 0.4 * torch.rand(2, 3, 64, 64, generator=gen)
    enh = torch.rand(2, 3, 64, 64, generator=gen)
    illu = 0.2 + 0.6 * torch.rand(2, 1, 64, 64, generator=gen)
    refl = torch.rand(2, 3, 64, 64, generator=gen)
    rec = {"low": low.numpy(), "enh": enh.numpy(), "illu": illu.numpy(), "refl": refl.numpy()}
    with torch.no_grad():
        rec["exposure"] = ref_loss.AdaptiveExposureLoss()(enh, low).numpy()
        rec["smoothness"] = ref_loss.EdgeAwareSmoothnessLoss()(illu, low).numpy()
        rec["color"] = ref_loss.ColorLoss()(enh).numpy()
        rec["spatial"] = ref_loss.SpatialConsistencyLoss()(enh, low).numpy()
        rec["decouple"] = ref_loss.IlluminationReflectanceDecouplingLoss()(illu, refl).numpy()
        rec["perceptual"] = ref_loss.PerceptualLoss()(enh, low).numpy()
        rec["frequency"] = ref_loss.FrequencyLoss()(enh, low).numpy()
        rec["tex_tv"] = ref_loss.calculate_texture_complexity(low, "tv").numpy()
        rec["tex_edge"] = ref_loss.calculate_texture_complexity(low, "edge_density").numpy()
        crit = ref_loss.TotalLoss(use_freq_loss=True, adaptive_weights=False, texture_method="tv")
        total, d = crit(low, enh, illu, refl)
    rec["total"] = total.numpy()
    for k, v in d.items():
        rec["dict_" + k] = np.float64(v)
    # gradients of the total w.r.t. the three network outputs
    e = enh.clone().requires_grad_(True)
    i = illu.clone().requires_grad_(True)
    r = refl.clone().requires_grad_(True)
    t, _ = crit(low, e, i, r)
    t.backward()
    rec.update(grad_enh=e.grad.numpy(), grad_illu=i.grad.numpy(), grad_refl=r.grad.numpy())
    np.savez_compressed(os.path.join(OUT, "g6_losses.npz"), **rec)


def g6c3():
    """The reference self-test's shapes (losses/loss.py:806-844): B=2, 64x64,
    a 3-CHANNEL illumination [B,3,H,W] -> the C_illu == C_refl branches of the
    smoothness (:148, :171-172) and decoupling (:302-304, :323-324) terms and
    TotalLoss, with the gradients w.r.t. (enh, illu, refl)."""
    gen = torch.Generator().manual_seed(16)
    low = 0.4 * torch.rand(2, 3, 64, 64, generator=gen)
    enh = torch.rand(2, 3, 64, 64, generator=gen)
    illu = torch.rand(2, 3, 64, 64, generator=gen)
    refl = torch.rand(2, 3, 64, 64, generator=gen)
    rec = {"low": low.numpy(), "enh": enh.numpy(), "illu": illu.numpy(), "refl": refl.numpy()}
    with torch.no_grad():
        rec["smoothness"] = ref_loss.EdgeAwareSmoothnessLoss()(illu, low).numpy()
        rec["decouple"] = ref_loss.IlluminationReflectanceDecouplingLoss()(illu, refl).numpy()
    crit = ref_loss.TotalLoss(use_freq_loss=True, adaptive_weights=False, texture_method="tv")
    e = enh.clone().requires_grad_(True)
    i = illu.clone().requires_grad_(True)
    r = refl.clone().requires_grad_(True)
    t, d = crit(low, e, i, r)
    t.backward()
    rec["total"] = t.detach().numpy()
    for k, v in d.items():
        rec["dict_" + k] = np.float64(v)
    rec.update(grad_enh=e.grad.numpy(), grad_illu=i.grad.numpy(), grad_refl=r.grad.numpy())
    # the single terms' gradients w.r.t. the illumination (and reflectance)
    i2 = illu.clone().requires_grad_(True)
    ref_loss.EdgeAwareSmoothnessLoss()(i2, low).backward()
    rec["grad_illu_smooth"] = i2.grad.numpy()
    i3 = illu.clone().requires_grad_(True)
    r3 = refl.clone().requires_grad_(True)
    ref_loss.IlluminationReflectanceDecouplingLoss()(i3, r3).backward()
    rec["grad_illu_decouple"] = i3.grad.numpy()
    rec["grad_refl_decouple"] = r3.grad.numpy()
    np.savez_compressed(os.path.join(OUT, "g6_losses_c3.npz"), **rec)


def g6nr():
    """TotalLoss without a reflectance (losses/loss.py:678-682): decouple = 0,
    on the G6 inputs (seed 6), with the gradients w.r.t. enh and illu."""
    gen = torch.Generator().manual_seed(6)
    low = 0.4 * torch.rand(2, 3, 64, 64, generator=gen)
    enh = torch.rand(2, 3, 64, 64, generator=gen)
    illu = 0.2 + 0.6 * torch.rand(2, 1, 64, 64, generator=gen)
    rec = {"low": low.numpy(), "enh": enh.numpy(), "illu": illu.numpy()}
    crit = ref_loss.TotalLoss(use_freq_loss=True, adaptive_weights=False, texture_method="tv")
    e = enh.clone().requires_grad_(True)
    i = illu.clone().requires_grad_(True)
    t, d = crit(low, e, i)
    t.backward()
    rec["total"] = t.detach().numpy()
    for k, v in d.items():
        rec["dict_" + k] = np.float64(v)
    rec.update(grad_enh=e.grad.numpy(), grad_illu=i.grad.numpy())
    np.savez_compressed(os.path.join(OUT, "g6_losses_norefl.npz"), **rec)


def g7():
    torch.manual_seed(0)
    model = ref_model.UP_Retinex(use_preact=False, use_aspp=False)
    sd0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    crit = ref_loss.TotalLoss(use_freq_loss=True, adaptive_weights=False, texture_method="tv")
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, weight_decay=1e-5)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(2))
    model.train()
    # train.py:63-103, use_amp=False
    opt.zero_grad()
    enh, refl, illu = model(x)
    loss, d = crit(x, enh, illu, refl)
    loss.backward()
    norm = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    opt.step()
    rec = {"x": x.numpy(), "enh": enh.detach().numpy(), "refl": refl.detach().numpy(),
           "illu": illu.detach().numpy(), "loss": loss.detach().numpy(), "clip_norm": norm.numpy()}
    for k, v in d.items():
        rec["dict_" + k] = np.float64(v)
    names = [n for n, _ in model.named_parameters()]
    rec["param_names"] = np.array(names)
    # clipped gradients (what Adam consumed) and the updated parameters,
    # stored in full for the small ones, as (L2 norm, sum) for all
    rec["grad_norm"] = np.array([float(grads[n].norm()) for n in names])
    rec["grad_sum"] = np.array([float(grads[n].double().sum()) for n in names])
    new_sd = model.state_dict()
    rec["delta_norm"] = np.array([float((new_sd[n] - sd0[n]).norm()) for n in names])
    for n in names:
        if grads[n].numel() <= 4096:
            rec["grad/" + n] = grads[n].numpy()
    bufs = [k for k in new_sd if k.endswith("running_mean") or k.endswith("running_var")]
    rec["buf_names"] = np.array(bufs)
    for k in bufs:
        rec["buf/" + k] = new_sd[k].numpy()
    np.savez_compressed(os.path.join(OUT, "g7_train_step.npz"), **rec)


if __name__ == "__main__":
    torch.set_num_threads(8)
    only = sys.argv[1:]
    if not only or "g6" in only:
        g6()
    if not only or "g6c3" in only:
        g6c3()
    if not only or "g6nr" in only:
        g6nr()
    if not only or "g7" in only:
        g7()
    print("wrote", " ".join(only) if only else
          "g6_losses.npz g6_losses_c3.npz g6_losses_norefl.npz g7_train_step.npz")
