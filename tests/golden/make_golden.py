#!/usr/bin/env python3
"""Golden-vector generator (run ONCE in the build container, never on the GPU box).

Imports the reference implementation read-only from /root/reference and records
its outputs on seeded inputs as small .npz fixtures under tests/golden/.  The
fixtures are data (inputs + expected outputs); no reference source or bytecode
is copied.  Re-run with:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Fixture map:
  G1 state_dict checksums   -> g1_state_dict.json
  G2 forward goldens        -> g2_forward_*.npz
  G3 per-module goldens     -> g3_modules.npz
  G4 real-image crop        -> g4_real_crop.npz
  G5 multi-scale enhancer   -> g5_multiscale.npz
  G8 float->u8 cast table   -> g8_cast_u8.npz
"""
import json
import os
import sys

import numpy as np
import torch

REF = os.environ.get("UPR_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

from models import model as ref_model  # noqa: E402  (reference models/model.py)
from enhancers import multi_scale as ref_ms  # noqa: E402  (reference enhancers/multi_scale.py)

VARIANTS = [(False, False), (True, False), (False, True), (True, True)]


def vname(pre, aspp):
    return f"pre{int(pre)}_aspp{int(aspp)}"


def g1():
    out = {}
    for pre, aspp in VARIANTS:
        for seed in (0, 1):
            torch.manual_seed(seed)
            m = ref_model.UP_Retinex(use_preact=pre, use_aspp=aspp)
            sd = m.state_dict()
            rec = {}
            for k, v in sd.items():
                t = v.detach().double().reshape(-1)
                rec[k] = {
                    "shape": list(v.shape),
                    "dtype": str(v.dtype).replace("torch.", ""),
                    "sum": float(t.sum()),
                    "sumsq": float((t * t).sum()),
                    "first": [float(a) for a in t[:4]],
                }
            out[f"{vname(pre, aspp)}_seed{seed}"] = {
                "keys": list(sd.keys()),
                "n_params": int(sum(p.numel() for p in m.parameters() if p.requires_grad)),
                "tensors": rec,
            }
    with open(os.path.join(OUT, "g1_state_dict.json"), "w") as f:
        json.dump(out, f)


def g2():
    gen = torch.Generator().manual_seed(1)
    x = torch.rand(2, 3, 64, 64, generator=gen)
    x_low = 0.3 * torch.rand(2, 3, 64, 64, generator=gen)
    for pre, aspp in VARIANTS:
        torch.manual_seed(0)
        m = ref_model.UP_Retinex(use_preact=pre, use_aspp=aspp).eval()
        rec = {"x": x.numpy()}
        with torch.no_grad():
            e, r, i = m(x)
        rec.update(enh=e.numpy(), refl=r.numpy(), illu=i.numpy())
        if not pre and not aspp:
            with torch.no_grad():
                e2, r2, i2 = m(x_low)
            rec.update(x_low=x_low.numpy(), enh_low=e2.numpy(), refl_low=r2.numpy(), illu_low=i2.numpy())
        np.savez_compressed(os.path.join(OUT, f"g2_forward_{vname(pre, aspp)}.npz"), **rec)
    # non-square, non-power-of-two spatial size (H, W multiples of 16)
    torch.manual_seed(0)
    m = ref_model.UP_Retinex(use_preact=True, use_aspp=True).eval()
    gen = torch.Generator().manual_seed(3)
    x = torch.rand(1, 3, 48, 80, generator=gen)
    with torch.no_grad():
        e, r, i = m(x)
    np.savez_compressed(os.path.join(OUT, "g2_forward_rect_pre1_aspp1.npz"),
                        x=x.numpy(), enh=e.numpy(), refl=r.numpy(), illu=i.numpy())


def g3():
    rec = {}
    gen = torch.Generator().manual_seed(5)
    torch.manual_seed(10)
    fam = ref_model.EnhancedFAM(32, 32).eval()
    x = torch.randn(1, 32, 24, 24, generator=gen)
    with torch.no_grad():
        rec["fam_x"], rec["fam_y"] = x.numpy(), fam(x).numpy()
    for k, v in fam.state_dict().items():
        rec["fam_sd." + k] = v.numpy()
    torch.manual_seed(11)
    aspp = ref_model.ASPPModule(64, 64).eval()
    # give BN non-trivial running stats so the fold is exercised
    with torch.no_grad():
        for mod in aspp.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.2, 0.2, generator=gen)
                mod.running_var.uniform_(0.5, 1.5, generator=gen)
                mod.weight.uniform_(0.5, 1.5, generator=gen)
                mod.bias.uniform_(-0.2, 0.2, generator=gen)
    x = torch.randn(1, 64, 24, 24, generator=gen)
    with torch.no_grad():
        rec["aspp_x"], rec["aspp_y"] = x.numpy(), aspp(x).numpy()
    for k, v in aspp.state_dict().items():
        rec["aspp_sd." + k] = v.numpy()
    for name, cls, args in (("preact", ref_model.PreActResBlock, (32, 64, 2)),
                            ("res", ref_model.ResBlock, (32, 64, 2)),
                            ("preact_id", ref_model.PreActResBlock, (64, 64, 1)),
                            ("up", ref_model.UpBlock, (64, 32))):
        torch.manual_seed(12)
        mod = cls(*args).eval()
        with torch.no_grad():
            for sub in mod.modules():
                if isinstance(sub, torch.nn.BatchNorm2d):
                    sub.running_mean.uniform_(-0.2, 0.2, generator=gen)
                    sub.running_var.uniform_(0.5, 1.5, generator=gen)
                    sub.weight.uniform_(0.5, 1.5, generator=gen)
                    sub.bias.uniform_(-0.2, 0.2, generator=gen)
        x = torch.randn(1, args[0], 16, 16, generator=gen)
        with torch.no_grad():
            rec[f"{name}_x"], rec[f"{name}_y"] = x.numpy(), mod(x).numpy()
        for k, v in mod.state_dict().items():
            rec[f"{name}_sd." + k] = v.numpy()
    np.savez_compressed(os.path.join(OUT, "g3_modules.npz"), **rec)


def g4():
    from PIL import Image
    img = Image.open(os.path.join(REF, "data/input/102708607-003694-003694.jpg")).convert("RGB")
    a = np.asarray(img)[:128, :128].copy()  # u8 HWC crop
    x = torch.from_numpy(a.astype(np.float32) / 255.0).permute(2, 0, 1).unsqueeze(0).contiguous()
    torch.manual_seed(0)
    m = ref_model.UP_Retinex(use_preact=False, use_aspp=False).eval()
    with torch.no_grad():
        e, r, i = m(x)
    np.savez_compressed(os.path.join(OUT, "g4_real_crop.npz"), img_u8=a,
                        enh=e.numpy(), illu=i.numpy())


def g5():
    enh = ref_ms.MultiScaleEnhancer()
    gen = torch.Generator().manual_seed(7)
    rec = {}
    for tag, hw in (("a", (64, 64)), ("b", (50, 70))):
        x = torch.rand(1, 3, *hw, generator=gen)
        feats = enh.extract_multi_scale_features(x)
        rec[f"{tag}_x"] = x.numpy()
        for i, f in enumerate(feats):
            rec[f"{tag}_feat{i}"] = f.numpy()
        factor = 1.0
        for i, f in enumerate(feats):  # enhancers/multi_scale.py:87-94
            factor += [0.5, 0.3, 0.2][i] * torch.mean(f).item() * 0.1
        rec[f"{tag}_factor"] = np.array(factor, dtype=np.float64)
    # full enhancer on the plain model
    torch.manual_seed(0)
    m = ref_model.UP_Retinex(use_preact=False, use_aspp=False).eval()
    x = torch.rand(1, 3, 64, 64, generator=gen)
    y, illu = enh.enhance_with_pyramid(m, x, "cpu")
    rec.update(full_x=x.numpy(), full_y=y.numpy(), full_illu=illu.numpy())
    np.savez_compressed(os.path.join(OUT, "g5_multiscale.npz"), **rec)


def g8():
    # float32 -> uint8 conversion as written at enhancers/adaptive_params.py:142:
    # (img_np * 255).astype(np.uint8) on float32 input
    vals = np.array([0.0, 1e-9, 0.5 / 255, 0.999 / 255, 1.0 / 255, 0.5, 0.999, 1.0, 1.0001, 1.2, 2.0,
                     -1e-6, -0.1, -1.0, 255.0 / 255 * 1.00392, np.nan, np.inf, -np.inf] +
                    list(np.linspace(-1.5, 1.5, 301)), dtype=np.float32)
    with np.errstate(invalid="ignore"):
        u8 = (vals * 255).astype(np.uint8)
    np.savez_compressed(os.path.join(OUT, "g8_cast_u8.npz"), x=vals, u8=u8)


if __name__ == "__main__":
    torch.set_num_threads(8)
    g1(); print("G1 done")
    g2(); print("G2 done")
    g3(); print("G3 done")
    g4(); print("G4 done")
    g5(); print("G5 done")
    g8(); print("G8 done")
