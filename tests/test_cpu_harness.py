"""Host-side harness pieces that run without a device: letterbox geometry and
uint8 round trip (reference utils/letterbox.py:9-102), image IO helpers, CLI
argument surface."""
import numpy as np
import torch
from PIL import Image

from utils.letterbox import letterbox, letterbox_tensor, resize_linear_u8


def test_letterbox_identity_roundtrip_is_exact():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (48, 80, 3)).astype(np.uint8)
    t = torch.from_numpy(a.transpose(2, 0, 1).copy()).float().div(255)
    out, ratio, pad = letterbox_tensor(t, new_shape=tuple(t.shape[1:]), auto=True, scaleup=False)
    assert ratio == (1.0, 1.0) and pad == (0.0, 0.0)
    assert torch.equal(out, t)


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


def test_save_and_compare(tmp_path):
    from enhancers.simple_enhance import save_image, create_comparison, load_image
    x = torch.rand(1, 3, 16, 24)
    save_image(x, str(tmp_path / "a.png"))
    save_image(x[:, :1], str(tmp_path / "b.png"))
    create_comparison(x, x, str(tmp_path / "c.png"))
    assert np.asarray(Image.open(tmp_path / "b.png")).shape == (16, 24, 3)
    assert np.asarray(Image.open(tmp_path / "c.png")).shape == (16, 48, 3)
    img, size = load_image(str(tmp_path / "a.png"))
    assert img.shape == (1, 3, 16, 24) and size == (24, 16)
    expect = torch.from_numpy(np.asarray(Image.open(tmp_path / "a.png")).transpose(2, 0, 1).copy()).float() / 255
    assert torch.equal(img[0], expect)


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
