"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py: G2, G3, G4, G5, G8)."""
import numpy as np
import pytest
import torch

from oracle import enhancers as oenh
from oracle import net as onet
from oracle import cv_u8

VARIANTS = [(False, False), (True, False), (False, True), (True, True)]


def vname(pre, aspp):
    return f"pre{int(pre)}_aspp{int(aspp)}"


def seeded_state_dict(pre, aspp, seed=0):
    from models.model import UP_Retinex
    torch.manual_seed(seed)
    return UP_Retinex(use_preact=pre, use_aspp=aspp).state_dict()


@pytest.mark.parametrize("pre,aspp", VARIANTS)
def test_forward_g2(golden, pre, aspp):
    g = golden(f"g2_forward_{vname(pre, aspp)}.npz")
    sd = seeded_state_dict(pre, aspp)
    with torch.no_grad():
        e, r, i = onet.forward(sd, torch.from_numpy(g["x"]), pre, aspp)
    np.testing.assert_allclose(e.numpy(), g["enh"], atol=2e-6, rtol=0)
    np.testing.assert_allclose(r.numpy(), g["refl"], atol=2e-6, rtol=1e-6)
    np.testing.assert_allclose(i.numpy(), g["illu"], atol=2e-6, rtol=0)
    if "x_low" in g:
        with torch.no_grad():
            e, r, i = onet.forward(sd, torch.from_numpy(g["x_low"]), pre, aspp)
        np.testing.assert_allclose(e.numpy(), g["enh_low"], atol=2e-6, rtol=0)
        np.testing.assert_allclose(i.numpy(), g["illu_low"], atol=2e-6, rtol=0)


def test_forward_rect_g2(golden):
    g = golden("g2_forward_rect_pre1_aspp1.npz")
    sd = seeded_state_dict(True, True)
    with torch.no_grad():
        e, r, i = onet.forward(sd, torch.from_numpy(g["x"]))
    np.testing.assert_allclose(e.numpy(), g["enh"], atol=2e-6, rtol=0)
    np.testing.assert_allclose(i.numpy(), g["illu"], atol=2e-6, rtol=0)


def test_variant_detection():
    for pre, aspp in VARIANTS:
        assert onet.variant_of(seeded_state_dict(pre, aspp)) == (pre, aspp)


def _sub(g, prefix):
    return {"m." + k[len(prefix):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(prefix)}


def test_modules_g3(golden):
    g = golden("g3_modules.npz")
    with torch.no_grad():
        y = onet.fam(_sub(g, "fam_sd."), "m", torch.from_numpy(g["fam_x"]))
        np.testing.assert_allclose(y.numpy(), g["fam_y"], atol=2e-6, rtol=1e-5)
        y = onet.aspp(_sub(g, "aspp_sd."), "m", torch.from_numpy(g["aspp_x"]))
        np.testing.assert_allclose(y.numpy(), g["aspp_y"], atol=1e-5, rtol=1e-5)
        y = onet.preact_block(_sub(g, "preact_sd."), "m", torch.from_numpy(g["preact_x"]), 2)
        np.testing.assert_allclose(y.numpy(), g["preact_y"], atol=1e-5, rtol=1e-5)
        y = onet.preact_block(_sub(g, "preact_id_sd."), "m", torch.from_numpy(g["preact_id_x"]), 1)
        np.testing.assert_allclose(y.numpy(), g["preact_id_y"], atol=1e-5, rtol=1e-5)
        y = onet.resblock(_sub(g, "res_sd."), "m", torch.from_numpy(g["res_x"]), 2)
        np.testing.assert_allclose(y.numpy(), g["res_y"], atol=1e-5, rtol=1e-5)
        y = onet.upblock(_sub(g, "up_sd."), "m", torch.from_numpy(g["up_x"]))
        np.testing.assert_allclose(y.numpy(), g["up_y"], atol=1e-5, rtol=1e-5)


def test_real_crop_g4(golden):
    g = golden("g4_real_crop.npz")
    x = torch.from_numpy(g["img_u8"].astype(np.float32) / 255.0).permute(2, 0, 1)[None].contiguous()
    sd = seeded_state_dict(False, False)
    with torch.no_grad():
        e, r, i = onet.forward(sd, x, False, False)
    np.testing.assert_allclose(e.numpy(), g["enh"], atol=2e-6, rtol=0)
    np.testing.assert_allclose(i.numpy(), g["illu"], atol=2e-6, rtol=0)


def test_multiscale_g5(golden):
    g = golden("g5_multiscale.npz")
    for tag in ("a", "b"):
        x = torch.from_numpy(g[f"{tag}_x"])
        feats = oenh.multiscale_features(x)
        for i, f in enumerate(feats):
            np.testing.assert_allclose(f.numpy(), g[f"{tag}_feat{i}"], atol=1e-6, rtol=0)
        assert abs(oenh.multiscale_factor(x)[0] - float(g[f"{tag}_factor"])) < 1e-12
    sd = seeded_state_dict(False, False)
    with torch.no_grad():
        y, illu = oenh.multiscale_enhance(sd, torch.from_numpy(g["full_x"]), False, False)
    np.testing.assert_allclose(y.numpy(), g["full_y"], atol=2e-6, rtol=0)
    np.testing.assert_allclose(illu.numpy(), g["full_illu"], atol=2e-6, rtol=0)


def test_cast_g8(golden):
    g = golden("g8_cast_u8.npz")
    np.testing.assert_array_equal(cv_u8.quantize_u8(g["x"]), g["u8"])
