"""TotalLoss (losses/loss.py:586-753) forward + gradient on gfx950 kernels.

One call computes every loss term AND its gradient w.r.t. the network outputs
(enhanced, illumination, reflectance) — the backward of a loss is cheap next
to the network's, so it is produced eagerly and handed to the network's
backward:

  * exposure / smoothness / colour / spatial / decoupling / texture weight:
    upr_t_loss_pixel (two reduction passes, a one-block finaliser and one
    gradient pass over the pixels);
  * perceptual (loss.py:179-255): VGG-19 features[0..18] on the MFMA conv
    kernels for both images, three MSE levels, backward through the enhanced
    branch (input gradients only: the VGG is frozen);
  * frequency (loss.py:430-520): 2-D FFTs through torch.fft (rocFFT, the
    library FFT — SURVEY.md §7), magnitude / mask / MSE and the gradient
    spectrum in upr_t_freq, inverse FFT, real part added by upr_t_add_real.
"""
import ctypes

import torch
import torch.nn as nn

from . import _lib as L
from .train import (Act, Conv, _chk, _fp, _h16, _p, _stream, autocast_active, empty, maxpool_into, pack_convs,
                    relu_mask, set_amp, zero)

WEIGHTS = dict(exposure=10.0, smoothness=1.0, color=0.5, spatial=1.0, decouple=0.1, perceptual=1.0,
               frequency=0.5)
# the loss modules' constructor arguments (reference defaults; include/upr_train.h UprLossParams)
PARAMS = dict(patch=16, base_exposure=0.6, smooth_lambda=10.0, smooth_alpha=1.0, decouple_lambda=0.1,
              freq_high=1.0, freq_low=0.5, dynamic_smooth=True)
TEXTURE = {"tv": 0, "edge_density": 1}  # calculate_texture_complexity methods (loss.py:523-583)
TERM_ORDER = ("exposure", "smoothness", "color", "spatial", "decouple", "perceptual", "frequency", "total")

VGG19_E = (64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M")


def texture_complexity(img, method):
    """img [B,C,H,W] float32 contiguous on the device -> [B] float32 (method 0 tv, 1 edge_density)."""
    B, C, H, W = img.shape
    acc = torch.empty((2 * B,), dtype=torch.float64, device=img.device)
    out = torch.empty((B,), dtype=torch.float32, device=img.device)
    with torch.cuda.device(img.device):
        _chk(L.lib().upr_t_texture_complexity(_p(img), B, C, H, W, int(method), _p(acc), _p(out), _stream()),
             "texture_complexity")
    return out


def vgg19_features(seed=None):
    """torchvision.models.vgg19().features layout (config "E"); with a seed,
    PyTorch's default Conv2d init drawn under torch.manual_seed(seed) — the
    offline stand-in for the pretrained weights (loss.py:195 downloads them)."""
    if seed is not None:
        torch.manual_seed(seed)
    layers, c = [], 3
    for v in VGG19_E:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(c, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            c = v
    return nn.Sequential(*layers)


class VGGPerceptual:
    """PerceptualLoss slices (loss.py:198-211): slice1 = features[0..4],
    slice2 = [5..9], slice3 = [10..18]; each ends with a 2x2 max-pool."""

    SLICES = ((0, 2), (5, 7), (10, 12, 14, 16))

    def __init__(self, features):
        self.convs = {i: Conv(features[i], frozen=True) for s in self.SLICES for i in s}

    def pack(self):
        pack_convs(list(self.convs.values()), self)

    def run(self, x_nhwc, keep):
        """x_nhwc: Act [B,H,W,3] (normalised).  Returns the three slice outputs;
        with keep, the intermediate activations for the backward."""
        lib, st = L.lib(), _stream()
        h = x_nhwc
        feats, trace = [], []
        for sl in self.SLICES:
            for i in sl:
                inp = h
                # autocast: the frozen VGG's activations are fp16 only (every reader takes the
                # fp16 copy: the next conv, the pool, the backward's ReLU masks), as the reference's
                h = self.convs[i].fwd(h, relu=True, only16=True) if self.convs[i].mfma else \
                    self.convs[i].fwd(None, relu=True, x_view=(h.view(), h.B, h.H, h.W),
                                      out=Act.new(h.B, h.H, h.W, self.convs[i].Cout, h.t.device, fresh=False),
                                      only16=True)
                if keep:
                    trace.append(("conv", i, inp, h))
            p = Act.new(h.B, h.H // 2, h.W // 2, h.C, h.t.device, fresh=False)
            code = torch.empty(p.B * p.H * p.W * p.C, dtype=torch.uint8, device=h.t.device) if keep else None
            maxpool_into(h, p, 2, 2, 0, code, only16=True)
            if keep:
                trace.append(("pool", code, h, p))
            h = p
            feats.append(p)
        return feats, trace

    def backward(self, trace, g_feats):
        """g_feats: gradient Acts of the three slice outputs -> gradient Act of the input."""
        lib, st = L.lib(), _stream()
        g = None
        level = 2
        entries = list(reversed(trace))
        premasked = False  # g already carries its ReLU mask (fused into the producing dgrad)
        for j, (kind, i, inp, out) in enumerate(entries):  # i: conv index, or the pool's argmax codes
            if kind == "pool":
                if g is None:
                    g = g_feats[level]
                else:
                    _chk(lib.upr_t_pointwise(_fp(g.t), _fp(g_feats[level].t), _fp(g.t), g.t.numel(), 4, None, None,
                                             ctypes.c_float(0), ctypes.c_uint64(0), st), "add")
                level -= 1
                gi = Act.new(inp.B, inp.H, inp.W, inp.C, inp.t.device, fresh=False)
                g_src, g, premasked = g, gi, False
                # the next conv's ReLU mask and fp16 operand fused into the gather when
                # that frozen conv reads the masked gradient in fp16 only (relu_mask's only16)
                nxt = entries[j + 1] if j + 1 < len(entries) else None
                if nxt is not None and nxt[0] == "conv" and inp.t16 is not None and inp.coff == 0 \
                        and inp.cs == inp.C:
                    cn = self.convs[nxt[1]]
                    if cn.frozen and ((cn.amp and cn.mfma) or cn.dgrad16_c3):
                        g16 = _h16(gi.M * gi.C, gi.t.device)
                        rc = lib.upr_t_maxpool_bwd_code16(_p(i), ctypes.byref(g_src.view()), inp.B, inp.H, inp.W,
                                                          inp.C, 2, 2, 0, out.H, out.W, _p(inp.t16), _p(g16), st)
                        if rc == 0:
                            gi.t16, gi.t16_grad, gi.stale32 = g16, True, True
                            premasked = True
                        elif rc != L.UPR_ERR_UNSUPPORTED:
                            _chk(rc, "pool_bwd16")
                if not premasked:
                    _chk(lib.upr_t_maxpool_bwd_code(_p(i), ctypes.byref(g_src.view()), inp.B, inp.H, inp.W, inp.C, 2,
                                                    2, 0, out.H, out.W, ctypes.byref(gi.view()), 0, st), "pool_bwd")
            else:
                c = self.convs[i]
                if not premasked:
                    # the frozen VGG conv's fp16 dgrad is the masked gradient's only reader
                    want16 = (c.amp and c.mfma) or c.dgrad16_c3
                    relu_mask(g, out, want16=want16, only16=c.frozen and want16)
                gi = Act.new(inp.B, inp.H, inp.W, inp.C, inp.t.device)
                # inp is the previous conv's ReLU output: its mask goes into this dgrad's epilogue
                nxt = entries[j + 1] if j + 1 < len(entries) else None
                mask = None
                if nxt is not None and nxt[0] == "conv" and inp.t16 is not None:
                    cn = self.convs[nxt[1]]
                    only16 = cn.frozen and ((cn.amp and cn.mfma) or cn.dgrad16_c3)
                    mask = (inp.t16, inp.C, only16)
                if c.mfma:
                    premasked = bool(c.bwd(inp, g, gi, mask=mask))
                else:
                    c.bwd(None, g, gi, x_view=(inp.view(), inp.B, inp.H, inp.W))
                    premasked = False
                g = gi
        return g


class TotalLossEngine:
    """losses/loss.py TotalLoss (train.py:224-234).  `w` holds the weights of
    the current step (the DWA weights when TotalLoss adapts them); `w_smooth`
    is the constructor's weight_smooth, which the dynamic smooth weight scales
    (loss.py:713) when params['dynamic_smooth'].  `params`: the loss modules'
    arguments (PARAMS).  A term whose weight is 0 still has its value computed,
    except perceptual (the VGG passes are skipped: value 0) — the single-term
    modules of losses/loss.py use that."""

    def __init__(self, vgg_features, weights=None, use_freq_loss=True, texture_method="tv", params=None):
        if texture_method not in TEXTURE:
            raise ValueError(f"不支持的纹理复杂度计算方法: {texture_method}")
        self.w = dict(WEIGHTS)
        if weights:
            self.w.update(weights)
        self.w_smooth = self.w["smoothness"]
        self.zero_decouple = False  # set per call by TotalLoss.forward(reflectance=None)
        self.texture_method = texture_method
        self.use_freq = use_freq_loss
        self.params = dict(PARAMS)
        if params:
            self.params.update(params)
        self.vgg = VGGPerceptual(vgg_features) if vgg_features is not None else None
        self.features = vgg_features

    def _cparams(self, illu_channels=1):
        p = self.params
        return L.UprLossParams(int(p["patch"]), float(p["base_exposure"]), float(p["smooth_lambda"]),
                               float(p["smooth_alpha"]), float(p["decouple_lambda"]), float(p["freq_high"]),
                               float(p["freq_low"]), int(bool(p["dynamic_smooth"])), int(illu_channels))

    def __call__(self, low, enh, illu, refl, grads=True):
        """All NCHW fp32 device tensors; illu [B,1,H,W] (the model's) or
        [B,3,H,W] (loss.py:806-844).  Returns (terms [9] device tensor in
        upr_t_loss_total order, (g_enh, g_illu, g_refl) or None)."""
        lib, st = L.lib(), _stream()
        B, C, H, W = enh.shape
        dev = enh.device
        if illu.dim() != 4 or illu.shape[1] not in (1, 3) or illu.shape[0] != B or tuple(illu.shape[2:]) != (H, W):
            raise NotImplementedError(f"loss: illumination [B,1,H,W] or [B,3,H,W] matching the images, got "
                                      f"{tuple(illu.shape)}")
        w = self.w
        terms = torch.empty(9, dtype=torch.float32, device=dev)
        zero(terms)
        prm = self._cparams(illu.shape[1])
        nws = lib.upr_t_loss_workspace_p(B, H, W, prm.patch)
        if nws == 0:
            raise ValueError(f"loss: a {H}x{W} image is smaller than the exposure patch ({prm.patch})")
        ws = torch.empty(nws, dtype=torch.uint8, device=dev)
        g_enh = g_illu = g_refl = None
        if grads:
            g_enh, g_illu, g_refl = empty(enh.shape, dev), empty(illu.shape, dev), empty(refl.shape, dev)
        _chk(lib.upr_t_loss_pixel_p(_p(low), _p(enh), _p(illu), _p(refl), B, H, W, _p(ws), _p(terms), _p(g_enh),
                                    _p(g_illu), _p(g_refl), int(grads), ctypes.c_float(w["exposure"]),
                                    ctypes.c_float(w["color"]), ctypes.c_float(w["spatial"]),
                                    ctypes.c_float(w["decouple"]), ctypes.c_float(self.w_smooth),
                                    TEXTURE[self.texture_method], ctypes.byref(prm), st), "loss_pixel")
        if self.zero_decouple:  # TotalLoss without a reflectance: that term is 0 (loss.py:678-682)
            zero(terms[TERM_ORDER.index("decouple"):TERM_ORDER.index("decouple") + 1])
        acc = torch.empty(4, dtype=torch.float64, device=dev)
        zero(acc)
        if self.vgg is not None and w["perceptual"] != 0.0:
            self._perceptual(lib, st, low, enh, B, H, W, terms, acc, grads, g_enh)
        self._frequency(lib, st, low, enh, B, C, H, W, terms, acc, grads, g_enh, prm)
        return terms, ((g_enh, g_illu, g_refl) if grads else None)

    def _perceptual(self, lib, st, low, enh, B, H, W, terms, acc, grads, g_enh):
        w = self.w
        dev = enh.device
        # ---- perceptual (VGG convs in fp16 under the caller's autocast, as the reference's) ----
        set_amp(autocast_active())
        self.vgg.pack()
        ne = Act.new(B, H, W, 3, dev, fresh=False)
        nl = Act.new(B, H, W, 3, dev, fresh=False)
        _chk(lib.upr_t_vgg_norm(_p(enh), _fp(ne.t), B, H, W, st), "vgg_norm")
        _chk(lib.upr_t_vgg_norm(_p(low), _fp(nl.t), B, H, W, st), "vgg_norm")
        fe, trace = self.vgg.run(ne, keep=grads)
        fl, _ = self.vgg.run(nl, keep=False)
        gfe = []
        for a, b in zip(fe, fl):
            n = a.t.numel()
            g = Act.new(a.B, a.H, a.W, a.C, dev, fresh=False) if grads else None
            if a.stale32 or b.stale32:  # fp16-only features (autocast): the MSE reads the fp16 copies
                rc = lib.upr_t_mse16(_p(a.t16), _p(b.t16), n, _p(acc[1:2]), _fp(g.t) if g else None,
                                     ctypes.c_float(w["perceptual"] / n), st)
            else:
                rc = lib.upr_t_mse(_fp(a.t), _fp(b.t), n, _p(acc[1:2]), _fp(g.t) if g else None,
                                   ctypes.c_float(w["perceptual"] / n), st)
            _chk(rc, "mse")
            gfe.append(g)
        _chk(lib.upr_t_scale_acc(_p(acc[1:2]), 1, ctypes.c_float(1.0), _fp(terms, 5), st), "scale")
        if grads:
            g_in = self.vgg.backward(trace, gfe)
            _chk(lib.upr_t_vgg_norm_bwd(_fp(g_in.t), _p(g_enh), B, H, W, st), "vgg_norm_bwd")

    def _frequency(self, lib, st, low, enh, B, C, H, W, terms, acc, grads, g_enh, prm):
        w = self.w
        # ---- frequency ----
        if self.use_freq:
            ze = torch.fft.fft2(enh, dim=(-2, -1))
            zl = torch.fft.fft2(low, dim=(-2, -1))
            n = enh.numel()
            G = torch.empty_like(ze) if grads else None
            _chk(lib.upr_t_freq_p(_p(ze), _p(zl), B * C, H, W, _p(acc[2:3]), _p(G),
                                  ctypes.c_float(w["frequency"] / n), ctypes.c_float(prm.freq_high),
                                  ctypes.c_float(prm.freq_low), st), "freq")
            _chk(lib.upr_t_scale_acc(_p(acc[2:3]), 1, ctypes.c_float(1.0 / n), _fp(terms, 6), st), "scale")
            if grads:
                gx = torch.fft.ifft2(G, dim=(-2, -1))
                _chk(lib.upr_t_add_real(_p(gx), _p(g_enh), n, ctypes.c_float(float(H * W)), st), "add_real")
        _chk(lib.upr_t_loss_total(_p(terms), ctypes.c_float(w["exposure"]), ctypes.c_float(w["color"]),
                                  ctypes.c_float(w["spatial"]), ctypes.c_float(w["decouple"]),
                                  ctypes.c_float(w["perceptual"]), ctypes.c_float(w["frequency"] if self.use_freq
                                                                                  else 0.0), st), "total")


class LossDict(dict):
    """The reference's loss_dict (loss.py:741-751: python floats from .item())
    plus the dynamic smooth weight, read back lazily: the 9 scalars go to a
    pinned host buffer by an asynchronous copy queued behind the loss kernels,
    and the first read of the dict waits for that copy alone.  The reference
    syncs the host in the middle of every step here (its .item()s before the
    backward); this leaves the device queue full until a caller actually reads
    a value.  Every dict access path materialises first."""

    __slots__ = ("_host", "_ev")

    def __init__(self, terms):
        super().__init__()
        self._host = torch.empty(terms.shape, dtype=terms.dtype, pin_memory=True)
        self._host.copy_(terms, non_blocking=True)
        self._ev = torch.cuda.Event()
        self._ev.record(torch.cuda.current_stream(terms.device))

    def _m(self):
        if self._ev is not None:
            self._ev.synchronize()
            v = self._host.tolist()
            for i, k in enumerate(TERM_ORDER):
                dict.__setitem__(self, k, v[i])
            dict.__setitem__(self, "smooth_weight", v[8])
            self._ev = self._host = None
        return self

    def __getitem__(self, k):
        return dict.__getitem__(self._m(), k)

    def __setitem__(self, k, v):
        dict.__setitem__(self._m(), k, v)

    def __delitem__(self, k):
        dict.__delitem__(self._m(), k)

    def __iter__(self):
        return dict.__iter__(self._m())

    def __len__(self):
        return dict.__len__(self._m())

    def __contains__(self, k):
        return dict.__contains__(self._m(), k)

    def __repr__(self):
        return dict.__repr__(self._m())

    def __eq__(self, o):
        return dict.__eq__(self._m(), o)

    def __ne__(self, o):
        return dict.__ne__(self._m(), o)

    __hash__ = None

    def __reduce__(self):
        return (dict, (dict(self.items()),))

    def get(self, k, default=None):
        return dict.get(self._m(), k, default)

    def keys(self):
        return dict.keys(self._m())

    def values(self):
        return dict.values(self._m())

    def items(self):
        return dict.items(self._m())

    def copy(self):
        return dict(self.items())

    def pop(self, *a):
        return dict.pop(self._m(), *a)

    def popitem(self):
        return dict.popitem(self._m())

    def setdefault(self, *a):
        return dict.setdefault(self._m(), *a)

    def update(self, *a, **kw):
        return dict.update(self._m(), *a, **kw)


def terms_dict(terms, lazy=False):
    """The 9 device loss scalars -> the reference's loss_dict.  lazy: a LossDict
    still waiting for its copy (the training step reads it back after its
    backward is queued); otherwise read back now, as the reference's .item()s."""
    d = LossDict(terms)
    return d if lazy else d._m()
