"""Functional torch-CPU fp32 restatement of the UP-Retinex training step.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the checker for the HIP
training path (upr/train.py + csrc/train.hip), never imported by the product.

Restates (paths relative to the reference root):
  * losses/loss.py:12-753   the 7 loss terms + calculate_texture_complexity +
                            TotalLoss.forward (fixed weights, dynamic smooth weight)
  * trainers/train.py:63-103 one step of train_one_epoch without AMP:
                            zero_grad -> forward -> loss -> backward ->
                            clip_grad_norm_(1.0) -> Adam(lr, weight_decay).step()
The network forward is oracle/net.py with MODE["train"] (batch-stat BatchNorm,
running-stat update, Dropout mask injectable).  The perceptual term uses a VGG19
`features` state_dict supplied by the caller (pretrained weights are not
available offline; tests use a seeded random init).
"""
import contextlib

import torch
import torch.nn.functional as F

from . import net

# VGG19 config "E" (torchvision.models.vgg19 features) up to index 18, the
# last layer PerceptualLoss keeps (loss.py:203-211): slice1 = 0..4,
# slice2 = 5..9, slice3 = 10..18.
VGG19_SLICES = (
    (("conv", 0, 3, 64), ("conv", 2, 64, 64), ("pool",)),
    (("conv", 5, 64, 128), ("conv", 7, 128, 128), ("pool",)),
    (("conv", 10, 128, 256), ("conv", 12, 256, 256), ("conv", 14, 256, 256), ("conv", 16, 256, 256), ("pool",)),
)
VGG19_E = (64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M")


def vgg19_state(seed):
    """features[0..18] of a VGG-19 "E" stack built with PyTorch's default Conv2d
    init under torch.manual_seed(seed) — the seeded stand-in for the pretrained
    weights (tests/golden/make_golden_train.py builds the same)."""
    import torch.nn as nn
    torch.manual_seed(seed)
    layers, c = [], 3
    for v in VGG19_E:
        if v == "M":
            layers.append(nn.MaxPool2d(2, 2))
        else:
            layers += [nn.Conv2d(c, v, 3, padding=1), nn.ReLU(inplace=True)]
            c = v
    sd = nn.Sequential(*layers).state_dict()
    return {k: v for k, v in sd.items() if int(k.split(".")[0]) <= 18}


VGG_MEAN = (0.485, 0.456, 0.406)
VGG_STD = (0.229, 0.224, 0.225)

WEIGHTS = {"exposure": 10.0, "smoothness": 1.0, "color": 0.5, "spatial": 1.0, "decouple": 0.1,
           "perceptual": 1.0, "frequency": 0.5}


def _grad(img):
    # loss.py:91-108 / :389-406
    return img[:, :, :, :-1] - img[:, :, :, 1:], img[:, :, :-1, :] - img[:, :, 1:, :]


def exposure_loss(enh, low, patch=16, base=0.6):
    """AdaptiveExposureLoss.forward — loss.py:29-58."""
    g_e = enh.mean(1, keepdim=True)
    g_l = low.mean(1, keepdim=True)
    target = base + (0.8 - base) * (1 - g_l.mean())
    m = F.avg_pool2d(g_e, patch, patch)
    return (m - target).abs().mean()


SOBEL_X = ((-1., 0., 1.), (-2., 0., 2.), (-1., 0., 1.))
SOBEL_Y = ((-1., -2., -1.), (0., 0., 0.), (1., 2., 1.))


def edge_map(img):
    """EdgeAwareSmoothnessLoss.compute_edge_map — loss.py:110-136."""
    gray = img.mean(1, keepdim=True) if img.shape[1] > 1 else img
    p = F.pad(gray, (1, 1, 1, 1), mode="reflect")
    kx = torch.tensor(SOBEL_X, dtype=img.dtype).view(1, 1, 3, 3)
    ky = torch.tensor(SOBEL_Y, dtype=img.dtype).view(1, 1, 3, 3)
    gx = F.conv2d(p, kx)
    gy = F.conv2d(p, ky)
    return torch.sqrt(gx ** 2 + gy ** 2)


def smoothness_loss(illu, low, lam=10.0, alpha=1.0):
    """EdgeAwareSmoothnessLoss.forward — loss.py:138-176."""
    ih, iv = _grad(illu)
    sh, sv = _grad(low)
    e = edge_map(low)
    wh = torch.exp(-lam * sh.abs().mean(1, keepdim=True))
    wv = torch.exp(-lam * sv.abs().mean(1, keepdim=True))
    efh = 1 + alpha * F.avg_pool2d(e, kernel_size=(1, wh.shape[3]), stride=1)[:, :, :, :-1]
    efv = 1 + alpha * F.avg_pool2d(e, kernel_size=(wv.shape[2], 1), stride=1)[:, :, :-1, :]
    return (wh * efh * ih.abs()).mean() + (wv * efv * iv.abs()).mean()


def color_loss(enh):
    """ColorLoss.forward — loss.py:351-371."""
    r, g, b = enh[:, 0].mean(), enh[:, 1].mean(), enh[:, 2].mean()
    return (r - g) ** 2 + (r - b) ** 2 + (g - b) ** 2


def spatial_loss(enh, low):
    """SpatialConsistencyLoss.forward — loss.py:408-427."""
    eh, ev = _grad(enh)
    lh, lv = _grad(low)
    return ((eh - lh) ** 2).mean() + ((ev - lv) ** 2).mean()


def decouple_loss(illu, refl, lam=0.1):
    """IlluminationReflectanceDecouplingLoss.forward — loss.py:275-334
    (C_illu = 1, C_refl = 3 branch: illumination expanded UNcentred, :308-312)."""
    B, ci, H, W = illu.shape
    cr = refl.shape[1]
    i_f = illu.reshape(B, ci, -1)
    r_f = refl.reshape(B, cr, -1)
    i_m = i_f.mean(2, keepdim=True)
    r_m = r_f.mean(2, keepdim=True)
    rc = r_f - r_m
    if ci == cr:
        cov = torch.bmm(i_f - i_m, rc.transpose(1, 2)) / (H * W - 1)
        md = F.mse_loss(i_m, r_m)
    else:
        cov = torch.bmm(i_f.expand(B, cr, -1), rc.transpose(1, 2)) / (H * W - 1)
        md = F.mse_loss(i_m.mean(1, keepdim=True), r_m.mean(1, keepdim=True))
    return torch.norm(cov, p="fro") ** 2 + lam * md


def vgg_features(vgg_sd, x):
    """PerceptualLoss slices 1..3 — loss.py:198-211, 239-245 (conv+ReLU, max-pool 2)."""
    feats = []
    h = x
    for sl in VGG19_SLICES:
        for layer in sl:
            if layer[0] == "conv":
                i = layer[1]
                w = vgg_sd[f"{i}.weight"]
                h = F.relu(net.amp_conv(F.conv2d, h, w, vgg_sd[f"{i}.bias"], w.shape[1], w.shape[0], padding=1))
            else:
                h = F.max_pool2d(h, 2, 2)
        feats.append(h)
    return feats


def perceptual_loss(vgg_sd, enh, low):
    """PerceptualLoss.forward — loss.py:221-255."""
    mean = torch.tensor(VGG_MEAN, dtype=enh.dtype).view(1, 3, 1, 1)
    std = torch.tensor(VGG_STD, dtype=enh.dtype).view(1, 3, 1, 1)
    fe = vgg_features(vgg_sd, (enh - mean) / std)
    fl = vgg_features(vgg_sd, (low - mean) / std)
    return sum(F.mse_loss(a, b) for a, b in zip(fe, fl))


def freq_masks(H, W):
    """FrequencyLoss._create_frequency_masks — loss.py:489-520 (no fftshift)."""
    ch, cw = H // 2, W // 2
    y, x = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    dist = torch.sqrt((x - cw).float() ** 2 + (y - ch).float() ** 2)
    r = min(H, W) // 4
    return (dist > r).float(), (dist <= r).float()


def frequency_loss(enh, low, w_high=1.0, w_low=0.5):
    """FrequencyLoss.forward — loss.py:447-487."""
    me = torch.abs(torch.fft.fft2(enh, dim=(-2, -1)))
    ml = torch.abs(torch.fft.fft2(low, dim=(-2, -1)))
    hm, lm = (m.to(enh.dtype) for m in freq_masks(enh.shape[2], enh.shape[3]))
    return w_high * F.mse_loss(me * hm, ml * hm) + w_low * F.mse_loss(me * lm, ml * lm)


def texture_complexity(img, method="tv"):
    """calculate_texture_complexity — loss.py:523-583."""
    if method == "tv":
        return (img[:, :, :, :-1] - img[:, :, :, 1:]).abs().mean((1, 2, 3)) + \
            (img[:, :, :-1, :] - img[:, :, 1:, :]).abs().mean((1, 2, 3))
    gray = img.mean(1, keepdim=True) if img.shape[1] > 1 else img
    e = edge_map(gray)
    thr = e.mean((1, 2, 3), keepdim=True) * 1.5
    return (e > thr).float().mean((1, 2, 3))


def total_loss(vgg_sd, low, enh, illu, refl, use_freq=True, texture_method="tv", weight_smooth=1.0, dynamic=True):
    """TotalLoss.forward — loss.py:656-753 (adaptive_weights=False; with
    use_dynamic_smooth_weight (dynamic) weight_smooth scales the dynamic smooth
    weight, :705-720, else it is used as is).  Returns (total, dict of python floats)."""
    terms = {
        "exposure": exposure_loss(enh, low),
        "smoothness": smoothness_loss(illu, low),
        "color": color_loss(enh),
        "spatial": spatial_loss(enh, low),
        "perceptual": perceptual_loss(vgg_sd, enh, low),
        "decouple": decouple_loss(illu, refl) if refl is not None else torch.tensor(0.0),
        "frequency": frequency_loss(enh, low) if use_freq else torch.tensor(0.0),
    }
    w = dict(WEIGHTS)
    if dynamic:
        tc = texture_complexity(low, texture_method).mean()
        w["smoothness"] = torch.clamp(weight_smooth * (1.0 - tc * 0.8), 0.1, 5.0)
    else:
        w["smoothness"] = torch.tensor(float(weight_smooth), dtype=enh.dtype)
    total = (w["exposure"] * terms["exposure"] + w["smoothness"] * terms["smoothness"] +
             w["color"] * terms["color"] + w["spatial"] * terms["spatial"] +
             w["decouple"] * terms["decouple"] + w["perceptual"] * terms["perceptual"] +
             w["frequency"] * terms["frequency"])
    d = {k: float(v.detach()) for k, v in terms.items()}
    d["total"] = float(total.detach())
    d["smooth_weight"] = float(w["smoothness"].detach())
    return total, d


@contextlib.contextmanager
def train_mode(dropout_mask=None, amp=False, eval_prefixes=()):
    """Training-mode BatchNorm / Dropout; amp: the autocast conv arithmetic
    (net.amp_conv) for the model and the VGG convs; eval_prefixes: submodules
    left in eval mode (frozen BatchNorm, identity Dropout)."""
    old = dict(net.MODE)
    net.MODE["train"] = True
    net.MODE["dropout_mask"] = dropout_mask
    net.MODE["amp"] = amp
    net.MODE["eval_prefixes"] = tuple(eval_prefixes)
    try:
        yield
    finally:
        net.MODE.update(old)


def param_names(sd):
    """Trainable parameters of the state_dict in module registration order
    (BatchNorm running stats / num_batches_tracked are buffers)."""
    return [k for k in sd if not (k.endswith("running_mean") or k.endswith("running_var")
                                   or k.endswith("num_batches_tracked"))]


def train_step(sd, vgg_sd, x, use_preact, use_aspp, lr=1e-4, weight_decay=1e-5, max_norm=1.0,
               use_freq=True, dropout_mask=None, adam_state=None, step=1):
    """One train_one_epoch step body (train.py:63-103, use_amp=False).

    sd: state_dict (float tensors; BN buffers are updated in place).  Returns
    (loss_dict, grads {name: tensor} before clipping, total_norm, new params
    {name: tensor}, adam_state)."""
    names = param_names(sd)
    params = {k: sd[k].detach().clone().requires_grad_(True) for k in names}
    work = dict(sd)
    work.update(params)
    with train_mode(dropout_mask):
        enh, refl, illu = net.forward(work, x, use_preact, use_aspp)
    for k in sd:
        if k.endswith("num_batches_tracked"):
            sd[k] += 1
    total, d = total_loss(vgg_sd, x, enh, illu, refl, use_freq)
    total.backward()
    grads = {k: params[k].grad.detach().clone() for k in names}
    # clip_grad_norm_(max_norm=1.0): total L2 norm over all grads, scale by
    # max_norm / (norm + 1e-6) clamped to 1 (torch.nn.utils.clip_grad_norm_)
    norm = torch.norm(torch.stack([torch.norm(g, 2) for g in grads.values()]), 2)
    coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    st = adam_state if adam_state is not None else {k: (torch.zeros_like(g), torch.zeros_like(g)) for k, g in
                                                      grads.items()}
    b1, b2, eps = 0.9, 0.999, 1e-8
    new = {}
    for k in names:
        g = grads[k] * coef + weight_decay * params[k].detach()   # Adam L2 weight decay
        m, v = st[k]
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        st[k] = (m, v)
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        denom = (v.sqrt() / (bc2 ** 0.5)) + eps
        new[k] = params[k].detach() - (lr / bc1) * m / denom
    return d, grads, float(norm), new, st
