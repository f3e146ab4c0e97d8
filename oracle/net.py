"""Functional torch-CPU fp32 restatement of the UP-Retinex forward (eval mode).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Operates on a plain
state_dict (name -> tensor) with the reference's key names; it does not use the
product's nn.Module classes, so a bug there cannot hide here.

Each function cites the reference code it restates (paths relative to the
reference root).
"""
import torch
import torch.nn.functional as F

BN_EPS = 1e-5  # nn.BatchNorm2d default
BN_MOMENTUM = 0.1

# Training mode (oracle/train.py switches it): BatchNorm uses batch statistics
# and updates the running buffers in place, Dropout draws its mask from
# MODE["dropout_mask"] (a callable shape -> {0,1} mask, so the checker can
# replay the product's mask) — nn.BatchNorm2d / nn.Dropout train semantics.
# MODE["eval_prefixes"]: state_dict prefixes of submodules left in eval mode
# inside a training graph (model.train() then module.eval(), nn.Module's
# per-module `training` flag): their BatchNorms use the running statistics and
# their Dropout is the identity.
MODE = {"train": False, "dropout_mask": None, "amp": False, "eval_prefixes": ()}


def _training(p):
    return MODE["train"] and not any(p.startswith(e) for e in MODE["eval_prefixes"])


def _bn(sd, p, x):
    # nn.BatchNorm2d eval: (x - rm) / sqrt(rv + eps) * w + b
    # train: batch mean / biased var normalise; running stats updated with the
    # unbiased var, momentum 0.1
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"],
                        sd[p + ".weight"], sd[p + ".bias"], _training(p), BN_MOMENTUM, BN_EPS)


def _dropout(x, p=0.1, prefix=""):
    if not _training(prefix) or p == 0.0:
        return x
    mask = MODE["dropout_mask"](x.shape)
    return x * mask / (1.0 - p)


def _r16(t):
    """fp16 rounding (autocast's cast): its backward rounds the gradient too."""
    return t.to(torch.float16).to(t.dtype)


def amp_conv(fn, x, w, b, cin, cout, **kw):
    """MODE["amp"]: the product's autocast arithmetic for MFMA-shaped convs
    (Cin, Cout multiples of 32; upr/train.py Conv / ConvT with autocast on):
    fp16 operands, wide accumulation, bias in fp32, fp16-rounded output.
    Otherwise a plain conv."""
    if MODE["amp"] and cin % 32 == 0 and cout % 32 == 0:
        return _r16(fn(_r16(x), _r16(w), b, **kw))
    return fn(x, w, b, **kw)


def _conv(sd, p, x, stride=1, padding=0, dilation=1):
    w = sd[p + ".weight"]
    return amp_conv(F.conv2d, x, w, sd.get(p + ".bias"), w.shape[1], w.shape[0], stride=stride, padding=padding,
                    dilation=dilation)


def fam(sd, p, x):
    """EnhancedFAM.forward — models/model.py:64-97."""
    b1 = _conv(sd, p + ".branch1", x)
    b2 = _conv(sd, p + ".branch2_conv", F.max_pool2d(x, 3, 1, 1))
    b3 = _conv(sd, p + ".branch3_conv2", F.relu(_conv(sd, p + ".branch3_conv1", x, padding=1)), padding=1)
    b4 = _conv(sd, p + ".branch4_conv2", F.relu(_conv(sd, p + ".branch4_conv1", x, padding=1)),
               padding=2, dilation=2)
    out = F.relu(_conv(sd, p + ".fusion", torch.cat([b1, b2, b3, b4], 1)))
    # channel attention: GAP -> 1x1 -> ReLU -> 1x1 -> sigmoid (model.py:47-53)
    g = out.mean(dim=(2, 3), keepdim=True)
    ca = torch.sigmoid(_conv(sd, p + ".channel_attention.3",
                             F.relu(_conv(sd, p + ".channel_attention.1", g))))
    out = out * ca
    # spatial attention: [mean_c, max_c] -> 7x7 conv -> sigmoid (model.py:56-59, 92-95)
    m = torch.cat([out.mean(1, keepdim=True), out.amax(1, keepdim=True)], 1)
    sa = torch.sigmoid(_conv(sd, p + ".spatial_attention.0", m, padding=3))
    return out * sa


def resblock(sd, p, x, stride):
    """ResBlock.forward — models/model.py:120-135."""
    o = F.relu(_bn(sd, p + ".bn1", _conv(sd, p + ".conv1", x, stride, 1)))
    o = _bn(sd, p + ".bn2", _conv(sd, p + ".conv2", o, 1, 1))
    if (p + ".shortcut.0.weight") in sd:
        sc = _bn(sd, p + ".shortcut.1", _conv(sd, p + ".shortcut.0", x, stride))
    else:
        sc = x
    return F.relu(o + sc)


def preact_block(sd, p, x, stride):
    """PreActResBlock.forward — models/model.py:164-178 (no trailing ReLU;
    projecting shortcut reads the pre-activated tensor, identity reads raw x)."""
    a = F.relu(_bn(sd, p + ".bn1", x))
    if (p + ".shortcut.0.weight") in sd:
        sc = _bn(sd, p + ".shortcut.1", _conv(sd, p + ".shortcut.0", a, stride))
    else:
        sc = x
    o = _conv(sd, p + ".conv1", a, stride, 1)
    o = _conv(sd, p + ".conv2", F.relu(_bn(sd, p + ".bn2", o)), 1, 1)
    return o + sc


def aspp(sd, p, x, dilations=(1, 6, 12, 18)):
    """ASPPModule.forward — models/model.py:231-251 (eval: Dropout is identity)."""
    feats = [F.relu(_bn(sd, p + ".conv1x1.1", _conv(sd, p + ".conv1x1.0", x)))]
    for i, d in enumerate(dilations[1:]):
        q = f"{p}.aspp_branches.{i}"
        feats.append(F.relu(_bn(sd, q + ".1", _conv(sd, q + ".0", x, 1, d, d))))
    g = x.mean(dim=(2, 3), keepdim=True)
    g = F.relu(_bn(sd, p + ".global_pool.2", _conv(sd, p + ".global_pool.1", g)))
    feats.append(F.interpolate(g, size=x.shape[2:], mode="bilinear", align_corners=False))
    o = _conv(sd, p + ".fusion.0", torch.cat(feats, 1))
    return _dropout(F.relu(_bn(sd, p + ".fusion.1", o)), 0.1, p + ".fusion.3")


def upblock(sd, p, x):
    """UpBlock.forward — models/model.py:271-274."""
    w = sd[p + ".up.weight"]
    u = amp_conv(F.conv_transpose2d, x, w, sd[p + ".up.bias"], w.shape[0], w.shape[1], stride=2)
    u = F.relu(_bn(sd, p + ".conv.1", _conv(sd, p + ".conv.0", u, padding=1)))
    return F.relu(_bn(sd, p + ".conv.4", _conv(sd, p + ".conv.3", u, padding=1)))


def variant_of(sd):
    """(use_preact, use_aspp) implied by the state_dict keys."""
    pre = "ie_net.enc1.bn1.running_var" in sd and "ie_net.enc1.conv1.weight" in sd and \
        sd["ie_net.enc1.bn1.running_var"].numel() == 32
    aspp_ = "ie_net.bottleneck.1.conv1x1.0.weight" in sd
    return pre, aspp_


def ienet(sd, x, use_preact, use_aspp):
    """ResidualIENet.forward — models/model.py:333-360."""
    p = "ie_net"
    blk = (lambda q, t, s: preact_block(sd, q, t, s)) if use_preact else \
        (lambda q, t, s: resblock(sd, q, t, s))
    x1 = F.relu(_conv(sd, p + ".input_layer", x, padding=1))
    x2 = blk(p + ".enc1", x1, 2)
    x3 = blk(p + ".enc2", x2, 2)
    x4 = blk(p + ".enc3", x3, 2)
    if use_aspp:
        t = blk(p + ".bottleneck.0", x4, 1)
        t = aspp(sd, p + ".bottleneck.1", t)
        x5 = blk(p + ".bottleneck.2", t, 1)
    else:
        x5 = blk(p + ".bottleneck.1", blk(p + ".bottleneck.0", x4, 1), 1)
    d3 = upblock(sd, p + ".dec3", x5) + x3
    d2 = upblock(sd, p + ".dec2", d3) + x2
    d1 = upblock(sd, p + ".dec1", d2) + x1
    r = _conv(sd, p + ".residual_head.2", F.relu(_conv(sd, p + ".residual_head.0", d1, padding=1)))
    return torch.sigmoid(x.mean(1, keepdim=True) + r)


def scale_branch(sd, p, x, pool):
    """scale1/2/3 Sequential — models/model.py:381-399."""
    if pool == 1:
        conv, famp = p + ".0", p + ".2"
    else:
        x = F.max_pool2d(x, pool)
        conv, famp = p + ".1", p + ".3"
    return fam(sd, famp, F.relu(_conv(sd, conv, x, padding=1)))


def multi_scale_enhance(sd, x, refl):
    """MultiScaleUP_Retinex.multi_scale_enhance — models/model.py:415-443."""
    x2 = F.interpolate(x, scale_factor=0.5, mode="bilinear", align_corners=False)
    x3 = F.interpolate(x, scale_factor=0.25, mode="bilinear", align_corners=False)
    f1 = scale_branch(sd, "scale1", x, 1)
    f2 = scale_branch(sd, "scale2", x2, 2)
    f3 = scale_branch(sd, "scale3", x3, 4)
    size = f1.shape[2:]
    fused = torch.cat([f1,
                       F.interpolate(f2, size=size, mode="bilinear", align_corners=False),
                       F.interpolate(f3, size=size, mode="bilinear", align_corners=False)], 1)
    e = torch.sigmoid(_conv(sd, "output_layer", _conv(sd, "fusion", fused)))
    return refl * e + (1 - refl) * (e ** 2)                            # model.py:442


def forward(sd, x, use_preact=None, use_aspp=None):
    """MultiScaleUP_Retinex.forward — models/model.py:445-455 (+405-443).

    Returns (enhanced, reflectance, illumination) in fp32 on CPU.
    """
    if use_preact is None or use_aspp is None:
        use_preact, use_aspp = variant_of(sd)
    x = x if x.dtype == torch.float64 else x.float()
    illu = ienet(sd, x, use_preact, use_aspp)
    refl = x / (illu + 1e-6)                                           # model.py:411-412
    return multi_scale_enhance(sd, x, refl), refl, illu
