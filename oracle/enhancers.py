"""CPU restatement of the enhancer pipelines — TEST INFRASTRUCTURE ONLY.

Each function cites the reference code it restates (paths relative to the
reference root).  Image tensors are NCHW float in [0, 1].
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import cv_u8, net


def clahe_enhancement(img, clip=2.0, tiles=(8, 8)):
    """AdaptiveParameterAdjuster.apply_clahe_enhancement — enhancers/adaptive_params.py:121-169,
    applied per image of a batch.  Returns float32 NCHW."""
    x = img.detach().cpu().float().numpy()
    out = np.zeros_like(x, dtype=np.float32)
    for b in range(x.shape[0]):
        rgb = cv_u8.quantize_u8(np.transpose(x[b], (1, 2, 0)))   # :142 (RGB2BGR + BGR2LAB == RGB2LAB)
        lab = cv_u8.rgb2lab_u8(rgb)                               # :145
        lab[..., 0] = cv_u8.clahe_apply(lab[..., 0], clip, tiles)  # :146-152
        rgb2 = cv_u8.lab2rgb_u8(lab)                              # :155-161
        out[b] = np.transpose(rgb2.astype(np.float32) / np.float32(255.0), (2, 0, 1))  # :164-167
    return torch.from_numpy(out)


def brightness_features(img):
    """calculate_brightness_features — adaptive_params.py:24-68 (image 0 of the batch)."""
    x = img.detach().cpu().float().numpy()
    if x.ndim == 4:
        x = x[0]
    gray = cv_u8.rgb_to_gray_u8(cv_u8.quantize_u8(np.transpose(x, (1, 2, 0))))
    return {
        "mean_brightness": np.mean(gray) / 255.0,
        "brightness_std": np.std(gray) / 255.0,
        "dark_pixel_ratio": np.sum(gray < 50) / gray.size,
        "mid_pixel_ratio": np.sum((gray >= 50) & (gray <= 200)) / gray.size,
        "bright_pixel_ratio": np.sum(gray > 200) / gray.size,
    }


def adjust_parameters(features):
    """adjust_parameters decision table — adaptive_params.py:70-119."""
    p = {"enhance_strength": 1.0, "color_balance": 1.0, "brightness_boost": 1.0, "contrast_adjust": 1.0}
    m = features["mean_brightness"]
    if m < 0.2:
        p["enhance_strength"], p["brightness_boost"] = 1.5, 1.3
    elif m < 0.4:
        p["enhance_strength"], p["brightness_boost"] = 1.3, 1.2
    elif m > 0.7:
        p["enhance_strength"], p["brightness_boost"] = 0.8, 0.9
    s = features["brightness_std"]
    p["contrast_adjust"] = 1.3 if s < 0.1 else (1.1 if s < 0.2 else 0.9)
    d = features["dark_pixel_ratio"]
    p["color_balance"] = 1.2 if d > 0.6 else (1.1 if d > 0.3 else 1.0)
    return p


def multiscale_features(img):
    """MultiScaleEnhancer.extract_multi_scale_features — enhancers/multi_scale.py:17-60 (fp32 torch CPU)."""
    img = img.detach().cpu().float()
    feats = []
    for s in (1.0, 0.5, 0.25):
        if s == 1.0:
            t = img
        else:
            h, w = img.shape[2:]
            t = F.interpolate(img, size=(int(h * s), int(w * s)), mode="bilinear", align_corners=False)
        lum = 0.299 * t[:, 0:1] + 0.587 * t[:, 1:2] + 0.114 * t[:, 2:3]
        gx = torch.gradient(t, dim=3)[0]
        gy = torch.gradient(t, dim=2)[0]
        feats.append(torch.cat([t, lum, torch.sqrt(gx ** 2 + gy ** 2)], 1))
    return feats


def multiscale_factor(img):
    """Per-image adjustment factor (multi_scale.py:87-94; the reference runs B=1
    and means over the whole batch — here image by image)."""
    out = []
    for b in range(img.shape[0]):
        f = 1.0
        for i, feat in enumerate(multiscale_features(img[b:b + 1])):
            f += [0.5, 0.3, 0.2][i] * torch.mean(feat).item() * 0.1
        out.append(f)
    return out


def multiscale_enhance(sd, x, use_preact=None, use_aspp=None):
    """apply_multi_scale_enhancement — multi_scale.py:62-100 -> (enh_adjusted, illu)."""
    enh, _, illu = net.forward(sd, x, use_preact, use_aspp)
    fac = multiscale_factor(x)
    out = torch.stack([torch.clamp(enh[b] * fac[b], 0, 1) for b in range(x.shape[0])])
    return out, illu


def adaptive_enhance(sd, x, use_preact=None, use_aspp=None):
    """apply_adaptive_enhancement — adaptive_params.py:171-200 -> (clahe(enh), illu)."""
    enh, _, illu = net.forward(sd, x, use_preact, use_aspp)
    return clahe_enhancement(enh), illu


def saliency_map(img):
    """ContentAwareEnhancer.compute_saliency_map — enhancers/content_aware.py:19-59 (image 0)."""
    x = img.detach().cpu().float().numpy()
    if x.ndim == 4:
        x = x[0]
    gray = cv_u8.rgb_to_gray_u8(cv_u8.quantize_u8(np.transpose(x, (1, 2, 0))))
    sal = np.abs(cv_u8.laplacian_k1_f64(gray))
    sal = cv_u8.gaussian_blur_f64(sal, 15, 0.0)
    sal = (sal - sal.min()) / (sal.max() - sal.min() + 1e-8)
    return torch.from_numpy(sal).float()[None, None]


def attention_map(img):
    """compute_attention_map — content_aware.py:61-91."""
    img = img.detach().cpu().float()
    lum = 0.299 * img[:, 0:1] + 0.587 * img[:, 1:2] + 0.114 * img[:, 2:3]
    att = saliency_map(img) * (1.0 / (lum + 0.1))
    return (att - torch.min(att)) / (torch.max(att) - torch.min(att) + 1e-8)
