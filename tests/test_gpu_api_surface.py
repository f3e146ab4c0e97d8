"""Reference methods callable on their own (VERDICT r2 Missing #5), each on the
HIP kernels and checked against the oracle:

* MultiScaleUP_Retinex.retinex_decompose (models/model.py:405-413) and its
  autograd (x and illumination gradients);
* MultiScaleUP_Retinex.multi_scale_enhance (models/model.py:415-443) with a
  caller-given reflectance (UPR_MODEL_HEAD_ONLY handle), and its gradients
  (reflectance + head parameters) against autograd through the oracle;
* calculate_texture_complexity (losses/loss.py:523-583), both methods, any C;
* ResidualIENet in training mode on its own (models/model.py:277-360);
* TotalLoss refuses an img_low that requires grad (no silent missing gradient).
"""
import numpy as np
import pytest
import torch

from oracle import net as onet
from oracle import train as otrain

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _model(pre, aspp, seed=0):
    from models.model import UP_Retinex
    torch.manual_seed(seed)
    return UP_Retinex(use_preact=pre, use_aspp=aspp)


def _maxrel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


@pytest.mark.parametrize("illu_c", [1, 3])
def test_retinex_decompose_and_grads(illu_c):
    gen = torch.Generator().manual_seed(1)
    x = torch.rand(2, 3, 24, 40, generator=gen)
    il = torch.rand(2, illu_c, 24, 40, generator=gen) * 0.9 + 0.02
    g = torch.randn(2, 3, 24, 40, generator=gen)
    m = _model(False, False).to(DEV).eval()
    xd, ild = x.to(DEV).requires_grad_(True), il.to(DEV).requires_grad_(True)
    r = m.retinex_decompose(xd, ild)
    (r * g.to(DEV)).sum().backward()
    xr, ilr = x.clone().requires_grad_(True), il.clone().requires_grad_(True)
    rr = xr / (ilr + 1e-6)  # models/model.py:411-412
    (rr * g).sum().backward()
    assert r.shape == rr.shape and r.dtype == torch.float32
    assert _maxrel(r, rr) <= 2e-7
    assert _maxrel(xd.grad, xr.grad) <= 2e-7
    assert _maxrel(ild.grad, ilr.grad) <= 2e-6
    # float16 tensors: one rounding of the fp32 quotient
    r16 = m.retinex_decompose(x.half().to(DEV), il.half().to(DEV))
    ref16 = (x.half().float() / (il.half().float() + 1e-6)).half()
    assert r16.dtype == torch.float16
    assert (r16.cpu().float() - ref16.float()).abs().max().item() <= 1e-3 * ref16.float().abs().max().item()


@pytest.mark.parametrize("pre,aspp", [(False, False), (True, True)])
def test_multi_scale_enhance_matches_forward_and_oracle(pre, aspp):
    model = _model(pre, aspp, seed=2).eval()
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(DEV)
    x = torch.rand(2, 3, 64, 48, generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        enh, refl, illu = model(x.to(DEV))
        e2 = model.multi_scale_enhance(x.to(DEV), refl, illu)
    # same head, same reflectance: the fused forward's enhanced image exactly
    assert torch.equal(e2, enh)
    # any reflectance: vs the oracle's multi_scale_enhance
    r = torch.rand(2, 3, 64, 48, generator=torch.Generator().manual_seed(4)) * 2.0
    with torch.no_grad():
        e3 = model.multi_scale_enhance(x.to(DEV), r.to(DEV), None)
        ref = onet.multi_scale_enhance(sd, x, r)
    err = (e3.cpu() - ref).abs().max().item()
    print(f"multi_scale_enhance pre={pre} aspp={aspp}: max|d| {err:.2e}")
    assert err <= 1e-4
    # an x that requires grad is refused in eval mode as in training mode (no
    # silently detached result); without grad inputs the eval result has no history
    for train in (False, True):
        with pytest.raises(NotImplementedError, match="w.r.t. x"):
            model.train(train).multi_scale_enhance(x.to(DEV).requires_grad_(True), r.to(DEV), None)
    e4 = model.eval().multi_scale_enhance(x.to(DEV), r.to(DEV), None)
    assert not e4.requires_grad and torch.equal(e4, e3)
    # float16 model
    m16 = model.half()
    with torch.no_grad():
        e16 = m16.multi_scale_enhance(x.half().to(DEV), r.half().to(DEV), None)
    assert e16.dtype == torch.float16
    assert (e16.float().cpu() - ref).abs().max().item() <= 1e-2


@pytest.mark.parametrize("train", [False, True])
def test_multi_scale_enhance_gradients(train):
    """multi_scale_enhance on its own is differentiable as the reference's
    (models/model.py:415-443): dL/d reflectance and the head parameters'
    gradients (scale1/2/3, fusion, output_layer) against autograd through the
    fp64 oracle (oracle/net.py multi_scale_enhance); fp32 engine, max|d| <=
    1e-4 * max|ref| + 1e-7 (measured: 1e-6 * max|ref| at worst)."""
    model = _model(False, True, seed=5)
    sd = {k: v.clone().double() for k, v in model.state_dict().items()}
    model = model.to(DEV).train(train)
    gen = torch.Generator().manual_seed(6)
    x = torch.rand(2, 3, 64, 48, generator=gen)
    r = torch.rand(2, 3, 64, 48, generator=gen) * 2.0
    g = torch.randn(2, 3, 64, 48, generator=gen)
    rd = r.to(DEV).requires_grad_(True)
    model.zero_grad(set_to_none=True)
    enh = model.multi_scale_enhance(x.to(DEV), rd, None)
    assert enh.requires_grad and enh.dtype == torch.float32
    (enh * g.to(DEV)).sum().backward()
    head = [k for k, _ in model.named_parameters() if not k.startswith("ie_net.")]
    for k in head:
        sd[k].requires_grad_(True)
    r64 = r.double().requires_grad_(True)
    ref = onet.multi_scale_enhance(sd, x.double(), r64)
    (ref * g.double()).sum().backward()
    assert _maxrel(enh, ref) <= 1e-5
    worst = []
    for name, a, b in [("reflectance", rd.grad, r64.grad)] + \
            [(k, dict(model.named_parameters())[k].grad, sd[k].grad) for k in head]:
        assert a is not None, name
        err = (a.detach().double().cpu() - b).abs().max().item()
        tol = 1e-4 * b.abs().max().item() + 1e-7
        worst.append((err / max(tol, 1e-30), name))
        assert err <= tol, f"{name}: max|d| {err:.3e} > {tol:.3e}"
    print("multi_scale_enhance grads: worst err/tol %.3f (%s)" % max(worst))
    # the IENet parameters get no gradient from the head alone
    for k, p in model.named_parameters():
        if k.startswith("ie_net.") and p.grad is not None:
            assert float(p.grad.abs().max()) == 0.0, k


@pytest.mark.parametrize("method", ["tv", "edge_density"])
@pytest.mark.parametrize("C", [1, 2, 3])
def test_calculate_texture_complexity(method, C):
    from losses.loss import calculate_texture_complexity
    img = torch.rand(3, C, 40, 56, generator=torch.Generator().manual_seed(5 + C))
    img[1] *= 0.1  # a darker, flatter image
    out = calculate_texture_complexity(img.to(DEV), method)
    ref = otrain.texture_complexity(img, method)
    assert out.shape == (3,) and out.dtype == torch.float32 and out.device.type == "cuda"
    d = (out.cpu() - ref).abs().max().item()
    print(f"texture {method} C={C}: {out.cpu().tolist()} vs {ref.tolist()} (max|d| {d:.2e})")
    if method == "tv":
        assert d <= 1e-6 * max(1.0, ref.abs().max().item())
    else:
        # a magnitude within rounding of the 1.5x-mean threshold may flip: at most 2 pixels per image
        assert d <= 2.0 / (40 * 56) + 1e-7
    with pytest.raises(ValueError):
        calculate_texture_complexity(img.to(DEV), "laplacian")


def test_texture_complexity_matches_reference_golden(golden):
    """G6 (reference-generated) holds tex_tv / tex_edge of its low image."""
    from losses.loss import calculate_texture_complexity
    g = golden("g6_losses.npz")
    if "low" not in g.files or "tex_tv" not in g.files:
        pytest.skip("G6 has no texture fixtures")
    low = torch.from_numpy(g["low"]).to(DEV)
    np.testing.assert_allclose(calculate_texture_complexity(low, "tv").cpu().numpy(), g["tex_tv"], rtol=1e-5)
    np.testing.assert_allclose(calculate_texture_complexity(low, "edge_density").cpu().numpy(), g["tex_edge"],
                               atol=2.0 / (low.shape[2] * low.shape[3]))


@pytest.mark.parametrize("pre,aspp", [(False, False), (True, True)])
def test_residual_ienet_standalone_training(pre, aspp):
    """ResidualIENet.train() on its own: illumination and every parameter
    gradient of a random projection vs the fp64 oracle (train-mode BatchNorm;
    the ASPP Dropout mask replayed), per tensor rel-L2 <= max(4 x the fp32
    oracle's, 2e-3); running statistics updated."""
    from models.model import ResidualIENet
    torch.manual_seed(6)
    m = ResidualIENet(use_preact=pre, use_aspp=aspp)
    sd = {"ie_net." + k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(DEV).train()
    B = 4
    x = torch.rand(B, 3, 64, 64, generator=torch.Generator().manual_seed(7))
    r = torch.randn(B, 1, 64, 64, generator=torch.Generator().manual_seed(8))
    illu = m(x.to(DEV))
    assert illu.shape == (B, 1, 64, 64) and illu.requires_grad
    (illu * r.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    mask = None
    if aspp:
        from upr.train import ASPPT
        ie = illu.grad_fn.ie
        asp = [b for b in ie.mid if isinstance(b, ASPPT)][0]
        mask = asp.mask.cpu().view(B, 8, 8, 256).permute(0, 3, 1, 2).float()
    names = [k for k in otrain.param_names(sd)]

    def oracle(dt):
        s2 = {k: (v.to(dt) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
        params = {k: s2[k].clone().requires_grad_(True) for k in names}
        work = dict(s2)
        work.update(params)
        with otrain.train_mode(dropout_mask=(lambda shape: mask.to(dt)) if aspp else None):
            i_r = onet.ienet(work, x.to(dt), pre, aspp)
        (i_r * r.to(dt)).sum().backward()
        return i_r, {k: params[k].grad.double() for k in names}, work

    i64, g64, w64 = oracle(torch.float64)
    _, g32, _ = oracle(torch.float32)
    assert (illu.detach().cpu().double() - i64).abs().max().item() <= 1e-4
    dev = dict(m.named_parameters())
    gmax = max(v.abs().max().item() for v in g64.values())
    for n in names:
        ref = g64[n]
        if ref.abs().max().item() < 1e-9 * gmax:
            continue  # BN-fed conv bias: zero true gradient
        rn = ref.norm().item()
        l2 = (dev[n[len("ie_net."):]].grad.double().cpu() - ref).norm().item() / rn
        l2c = (g32[n] - ref).norm().item() / rn
        assert l2 <= max(4.0 * l2c, 2e-3), f"grad {n}: rel-L2 {l2:.3e} (fp32 CPU {l2c:.3e})"
    for k, v in m.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            assert (v.cpu().double() - w64["ie_net." + k].double()).abs().max().item() <= 1e-5, k


def test_total_loss_refuses_img_low_requiring_grad():
    from losses.loss import TotalLoss
    model = _model(False, False).to(DEV).train()
    crit = TotalLoss(use_freq_loss=True).to(DEV)
    x = torch.rand(2, 3, 32, 32, device=DEV)
    enh, refl, illu = model(x)
    with pytest.raises(NotImplementedError):
        crit(x.clone().requires_grad_(True), enh, illu, refl)
    total, _ = crit(x, enh, illu, refl)  # a plain img_low still works
    total.backward()
