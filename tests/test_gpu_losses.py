"""The loss term modules of losses/loss.py as standalone, differentiable modules
with non-default constructor arguments (reference losses/loss.py:12-520), and
TotalLoss(use_dynamic_smooth_weight=False) (:617, :705), on the device loss
engine, against the oracle restatement (oracle/train.py, fp64 torch autograd).

The oracle's terms are pinned to the reference at the default arguments by G6
(tests/test_gpu_train.py::test_loss_terms_and_grads,
tests/test_cpu_train_oracle.py); the arguments enter the restatement exactly
where they enter the reference's formulas (exposure target and pooling,
smoothness exponent and edge factor, decoupling mean-difference weight,
frequency band weights).

Tolerances: value rel 1e-4; gradient max|d| <= 1e-4 * max|ref| + 1e-7 (fp32
device vs fp64 oracle; the reductions are fp64 on the device).
"""
import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs a ROCm device")]
DEV = "cuda"
VGG_SEED = 1234


def _inputs(H=64, W=80, seed=0):
    g = torch.Generator().manual_seed(seed)
    low = torch.rand(2, 3, H, W, generator=g) * 0.4
    enh = torch.rand(2, 3, H, W, generator=g)
    illu = torch.rand(2, 1, H, W, generator=g) * 0.8 + 0.1
    refl = enh / (illu + 1e-6)
    return low, enh, illu, refl


def _check(name, val, ref, dev_inputs, ref_inputs):
    np.testing.assert_allclose(float(val), float(ref), rtol=1e-4, atol=1e-10, err_msg=name)
    for k, (a, b) in enumerate(zip(dev_inputs, ref_inputs)):
        ga, gb = a.grad.double().cpu(), b.grad
        err = (ga - gb).abs().max().item()
        tol = 1e-4 * gb.abs().max().item() + 1e-7
        print(f"{name}: value {float(val):.6g} (oracle {float(ref):.6g}); grad[{k}] max|d| {err:.2e} tol {tol:.2e}")
        assert err <= tol, f"{name} grad[{k}]: {err:.3e} > {tol:.3e}"


def _leaf(*ts, dev=True):
    return [t.clone().to(DEV if dev else "cpu", torch.float32 if dev else torch.float64).requires_grad_(True)
            for t in ts]


CASES = [
    # name, module factory, oracle(term inputs), which inputs (indices into low, enh, illu, refl)
    ("exposure_p8_b05", lambda L: L.AdaptiveExposureLoss(patch_size=8, base_target_exposure=0.5),
     lambda o, enh, low: o.exposure_loss(enh, low, 8, 0.5), (1, 0)),
    ("exposure_p12_floor", lambda L: L.AdaptiveExposureLoss(patch_size=12),
     lambda o, enh, low: o.exposure_loss(enh, low, 12, 0.6), (1, 0)),
    ("smoothness_l5_a05", lambda L: L.EdgeAwareSmoothnessLoss(lambda_val=5.0, alpha=0.5),
     lambda o, illu, low: o.smoothness_loss(illu, low, 5.0, 0.5), (2, 0)),
    ("color", lambda L: L.ColorLoss(), lambda o, enh: o.color_loss(enh), (1,)),
    ("spatial", lambda L: L.SpatialConsistencyLoss(), lambda o, enh, low: o.spatial_loss(enh, low), (1, 0)),
    ("decouple_l03", lambda L: L.IlluminationReflectanceDecouplingLoss(lambda_val=0.3),
     lambda o, illu, refl: o.decouple_loss(illu, refl, 0.3), (2, 3)),
    ("frequency_h2_l025", lambda L: L.FrequencyLoss(weight_high=2.0, weight_low=0.25),
     lambda o, enh, low: o.frequency_loss(enh, low, 2.0, 0.25), (1, 0)),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_loss_term_module_value_and_grad(case):
    from losses import loss as Lmod
    from oracle import train as otrain
    name, make, ref_fn, idx = case
    data = _inputs()
    mod = make(Lmod).to(DEV)
    ref_in = _leaf(*[data[i] for i in idx], dev=False)
    # only the first argument is differentiable for the (x, img_low) modules:
    # img_low goes in without requires_grad (the engine has no img_low gradient
    # and refuses one that requires grad: test_loss_term_refuses_img_low_grad)
    diff = 2 if idx in ((2, 3),) or name == "color" else 1
    dev_in = _leaf(*[data[i] for i in idx[:diff]]) + [data[i].to(DEV) for i in idx[diff:]]
    val = mod(*dev_in)
    assert val.dim() == 0 and val.requires_grad
    val.backward()
    torch.cuda.synchronize()
    ref = ref_fn(otrain, *ref_in)
    ref.backward()
    _check(name, val.detach().cpu(), ref.detach(), dev_in[:diff], ref_in[:diff])


def test_loss_term_refuses_img_low_grad():
    from losses import loss as Lmod
    low, enh, _, _ = _inputs()
    mod = Lmod.AdaptiveExposureLoss().to(DEV)
    e_d, l_d = _leaf(enh, low)
    with pytest.raises(NotImplementedError):
        mod(e_d, l_d)
    with torch.no_grad():
        mod(e_d, l_d)  # no autograd recording: fine


def test_perceptual_module_value_and_grad():
    from losses import loss as Lmod
    from oracle import train as otrain
    low, enh, _, _ = _inputs(64, 64, seed=3)
    mod = Lmod.PerceptualLoss().to(DEV)
    e_d, = _leaf(enh)
    val = mod(e_d, low.to(DEV))
    val.backward()
    torch.cuda.synchronize()
    e_r, = _leaf(enh, dev=False)
    vgg = {k: v.double() for k, v in otrain.vgg19_state(VGG_SEED).items()}
    ref = otrain.perceptual_loss(vgg, e_r, low.double())
    ref.backward()
    _check("perceptual", val.detach().cpu(), ref.detach(), [e_d], [e_r])


@pytest.mark.parametrize("w_smooth", [1.0, 2.5])
def test_total_loss_without_dynamic_smooth_weight(w_smooth):
    """TotalLoss(use_dynamic_smooth_weight=False): the smoothness weight is
    weight_smooth itself (loss.py:705 branch not taken)."""
    from losses.loss import TotalLoss
    from oracle import train as otrain
    low, enh, illu, refl = _inputs(64, 64, seed=5)
    crit = TotalLoss(weight_smooth=w_smooth, use_dynamic_smooth_weight=False).to(DEV)
    e_d, i_d, r_d = _leaf(enh, illu, refl)
    total, d = crit(low.to(DEV), e_d, i_d, r_d)
    total.backward()
    torch.cuda.synchronize()
    assert d["smooth_weight"] == pytest.approx(w_smooth)
    e_r, i_r, r_r = _leaf(enh, illu, refl, dev=False)
    vgg = {k: v.double() for k, v in otrain.vgg19_state(VGG_SEED).items()}
    t_r, d_r = otrain.total_loss(vgg, low.double(), e_r, i_r, r_r, weight_smooth=w_smooth, dynamic=False)
    t_r.backward()
    for k in ("exposure", "smoothness", "color", "spatial", "decouple", "perceptual", "frequency"):
        np.testing.assert_allclose(d[k], d_r[k], rtol=1e-4, atol=1e-10, err_msg=k)
    _check("total(no dynamic)", total.detach().cpu(), t_r.detach(), [e_d, i_d, r_d], [e_r, i_r, r_r])
