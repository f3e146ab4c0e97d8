"""Drop-in surface of models/model.py (reference models/model.py:11-464):
state_dict keys/order/values under seeded construction (G1), parameter counts,
and the no-fallback guarantees of the HIP-only forward."""
import json
import os

import pytest
import torch

from conftest import GOLDEN
from models import model as M

VARIANTS = [(False, False), (True, False), (False, True), (True, True)]


@pytest.fixture(scope="module")
def g1():
    with open(os.path.join(GOLDEN, "g1_state_dict.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("pre,aspp", VARIANTS)
@pytest.mark.parametrize("seed", [0, 1])
def test_state_dict_g1(g1, pre, aspp, seed):
    rec = g1[f"pre{int(pre)}_aspp{int(aspp)}_seed{seed}"]
    torch.manual_seed(seed)
    m = M.UP_Retinex(use_preact=pre, use_aspp=aspp)
    sd = m.state_dict()
    assert list(sd.keys()) == rec["keys"]
    assert M.count_parameters(m) == rec["n_params"]
    for k, v in sd.items():
        r = rec["tensors"][k]
        assert list(v.shape) == r["shape"], k
        assert str(v.dtype).replace("torch.", "") == r["dtype"], k
        t = v.double().reshape(-1)
        assert abs(float(t.sum()) - r["sum"]) <= 1e-9 * max(1.0, abs(r["sum"])) + 1e-9, k
        assert abs(float((t * t).sum()) - r["sumsq"]) <= 1e-9 * max(1.0, r["sumsq"]), k
        assert [float(a) for a in t[:4]] == r["first"], k


def test_defaults_and_alias():
    assert M.UP_Retinex is M.MultiScaleUP_Retinex
    m = M.UP_Retinex()  # reference default: use_preact=True, use_aspp=True (model.py:375)
    assert "ie_net.bottleneck.1.aspp_branches.2.0.weight" in m.state_dict()
    assert m.ie_net.enc1.bn1.num_features == 32  # pre-activation block
    ie = M.ResidualIENet()
    assert ie.use_aspp is False and "bottleneck.1.conv1.weight" in ie.state_dict()


def test_load_state_dict_roundtrip():
    torch.manual_seed(3)
    a = M.UP_Retinex(use_preact=False, use_aspp=True)
    b = M.UP_Retinex(use_preact=False, use_aspp=True)
    b.load_state_dict(a.state_dict(), strict=True)
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)


def test_cpu_forward_raises_no_fallback():
    m = M.UP_Retinex(use_preact=False, use_aspp=False).eval()
    with pytest.raises(RuntimeError, match="ROCm"):
        m(torch.rand(1, 3, 32, 32))
    with pytest.raises(RuntimeError, match="ROCm"):
        m.ie_net(torch.rand(1, 3, 32, 32))


def test_submodules_have_no_cpu_path():
    """Standalone submodule forwards run on the device (tests/test_gpu_modules.py);
    a CPU tensor raises like the top-level model."""
    for mod, c in ((M.EnhancedFAM(32, 32), 32), (M.ResBlock(32, 64, 2), 32), (M.PreActResBlock(32, 64, 2), 32),
                   (M.ASPPModule(64, 64), 64), (M.UpBlock(64, 32), 64)):
        with pytest.raises(RuntimeError, match="ROCm"):
            mod.eval()(torch.rand(1, c, 8, 8))
    m = M.UP_Retinex()
    with pytest.raises(RuntimeError, match="ROCm"):
        m.retinex_decompose(torch.rand(1, 3, 8, 8), torch.rand(1, 1, 8, 8))
    with pytest.raises(RuntimeError, match="ROCm"):
        m.eval().multi_scale_enhance(torch.rand(1, 3, 16, 16), torch.rand(1, 3, 16, 16), None)


def test_training_mode_cpu_input_raises():
    """Training mode is supported on the device (upr/autograd.model_train_forward /
    ienet_train_forward, tests/test_gpu_train.py, tests/test_gpu_api_surface.py);
    on a CPU tensor it raises like eval mode (no CPU path)."""
    m = M.UP_Retinex(use_preact=False, use_aspp=False)  # .train() by default
    assert m.training
    with pytest.raises(RuntimeError, match="ROCm"):
        m(torch.rand(1, 3, 32, 32))
    ie = M.ResidualIENet()
    assert ie.training
    with pytest.raises(RuntimeError, match="ROCm"):
        ie(torch.rand(1, 3, 32, 32))
