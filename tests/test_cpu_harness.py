"""Host-side harness pieces that run without a device: the letterbox geometry
(reference utils/letterbox.py:9-62) and its CPU restatement oracle/letterbox.py
(the checker of the device kernel, tests/test_gpu_enhancers.py), image IO
helpers, CLI argument surface."""
import numpy as np
import torch
from PIL import Image

from oracle.letterbox import letterbox, linear_taps as oracle_taps, resize_linear_u8
from utils.letterbox import letterbox_geometry, linear_taps


def test_letterbox_geometry_identity():
    unpad, ratio, pad, border = letterbox_geometry((48, 80), (48, 80), auto=True, scaleup=False)
    assert unpad == (80, 48) and ratio == (1.0, 1.0) and pad == (0.0, 0.0) and border == (0, 0, 0, 0)


def test_product_taps_match_oracle_taps():
    for dst, src in ((85, 200), (128, 300), (60, 30), (13, 30), (30, 30), (640, 1920), (384, 1080), (1000, 7),
                     (7, 1000), (333, 334)):
        t = linear_taps(dst, src)
        o = oracle_taps(dst, src)
        for i in range(4):
            np.testing.assert_array_equal(t[i], o[i])


def test_letterbox_pad_geometry():
    a = np.zeros((37, 53, 3), np.uint8)
    out, ratio, (dw, dh) = letterbox(a, new_shape=64, auto=True, scaleup=False)
    # r = 1 (no upscaling); dw = (64-53) % 32 = 11 -> 5.5; dh = 27 -> 13.5
    assert out.shape == (64, 64, 3) and (dw, dh) == (5.5, 13.5)
    assert (out[:13] == 114).all() and (out[13 + 37:] == 114).all()
    assert (out[13:50, 5:58] == 0).all() and (out[13:50, :5] == 114).all()


def test_letterbox_downscale_shape():
    a = np.random.default_rng(1).integers(0, 256, (300, 200, 3)).astype(np.uint8)
    out, ratio, _ = letterbox(a, new_shape=128, auto=True, scaleup=False)
    # r = 128/300; unpad = (round(200r), round(300r)) = (85, 128); dw = 43 % 32 = 11
    assert out.shape == (128, 96, 3)
    assert abs(ratio[0] - 128 / 300) < 1e-12


def test_resize_linear_properties():
    a = np.random.default_rng(2).integers(0, 256, (20, 30, 3)).astype(np.uint8)
    assert np.array_equal(resize_linear_u8(a, (30, 20)), a)          # identity size
    c = np.full((20, 30, 3), 77, np.uint8)
    assert (resize_linear_u8(c, (13, 9)) == 77).all()                 # constants preserved
    up = resize_linear_u8(a, (60, 40))
    assert up.shape == (40, 60, 3)
    assert up.min() >= a.min() and up.max() <= a.max()                # convex combination


def test_letterbox_refuses_without_device():
    import pytest
    from utils.letterbox import letterbox_tensor
    if torch.cuda.is_available():
        pytest.skip("a ROCm device is present")
    with pytest.raises(RuntimeError, match="ROCm"):
        letterbox_tensor(torch.rand(3, 8, 8), new_shape=(8, 8))


def test_cli_surface():
    import main as cli
    ap = cli.build_parser()
    a = ap.parse_args(["--mode", "enhance", "--input_path", "x.png", "--multi_scale", "--use_preact", "--seed", "3"])
    assert a.mode == "enhance" and a.multi_scale and a.use_preact and a.seed == 3 and a.precision == "fp32"
    names = {x.dest for x in ap._actions}
    for flag in ("train_dir", "test_dir", "checkpoint", "save_dir", "num_epochs", "batch_size", "image_size", "lr",
                 "weight_decay", "resume", "weight_exp", "weight_smooth", "weight_col", "weight_spa",
                 "weight_decouple", "weight_perceptual", "weight_freq", "max_size", "no_comparison", "device",
                 "content_aware", "num_workers", "lr_decay_step", "lr_decay_gamma", "save_freq", "use_amp",
                 "patience", "use_cosine_scheduler", "use_freq_loss", "adaptive_weights", "use_aspp",
                 "advanced_augment"):
        assert flag in names, flag
