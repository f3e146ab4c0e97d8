"""Host-side surface of the training path (no device calls): the drop-in
losses/ and trainers/ modules import, keep the reference's constructor
arguments, refuse CPU tensors loudly (no CPU fallback), and the seeded VGG
stand-in is the one the G6/G7 fixtures were made with."""
import inspect

import pytest
import torch

from losses import loss as L
from oracle import train as otrain
from trainers import train as T
from upr import loss_engine as E


def test_total_loss_signature_matches_reference():
    sig = inspect.signature(L.TotalLoss.__init__)
    for name, default in (("weight_exp", 10.0), ("weight_smooth", 1.0), ("weight_col", 0.5), ("weight_spa", 1.0),
                          ("weight_decouple", 0.1), ("weight_perceptual", 1.0), ("weight_freq", 0.5),
                          ("use_freq_loss", True), ("adaptive_weights", False),
                          ("use_dynamic_smooth_weight", True), ("texture_method", "tv")):
        assert sig.parameters[name].default == default, name
    fwd = inspect.signature(L.TotalLoss.forward)
    assert list(fwd.parameters)[1:] == ["img_low", "img_enhanced", "illu_map", "reflectance", "epoch"]


def test_train_one_epoch_signature():
    sig = inspect.signature(T.train_one_epoch)
    assert list(sig.parameters)[:8] == ["model", "dataloader", "criterion", "optimizer", "device", "epoch",
                                        "writer", "scaler"]


def test_losses_refuse_cpu_tensors():
    crit = L.TotalLoss()
    x = torch.rand(1, 3, 32, 32)
    with pytest.raises(RuntimeError, match="ROCm"):
        crit(x, x, x[:, :1], x)
    with pytest.raises(RuntimeError, match="ROCm"):
        L.ColorLoss()(x)


def test_unsupported_options_raise():
    L.TotalLoss(use_dynamic_smooth_weight=False)  # supported (tests/test_gpu_losses.py)
    with pytest.raises(ValueError):
        L.TotalLoss(texture_method="laplacian")


def test_model_train_forward_refuses_cpu():
    from models.model import UP_Retinex
    torch.manual_seed(0)
    m = UP_Retinex(use_preact=False, use_aspp=False).train()
    with pytest.raises(RuntimeError, match="ROCm"):
        m(torch.rand(1, 3, 32, 32))


def test_vgg_stand_in_matches_oracle():
    f = E.vgg19_features(seed=1234)
    ref = otrain.vgg19_state(1234)
    sd = f.state_dict()
    for k, v in ref.items():
        assert torch.equal(sd[k], v), k
    assert [i for s in E.VGGPerceptual.SLICES for i in s] == [0, 2, 5, 7, 10, 12, 14, 16]
