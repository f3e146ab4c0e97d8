"""Standalone submodule forwards on the device (reference models/model.py:11-274:
EnhancedFAM, ResBlock, PreActResBlock, ASPPModule, UpBlock called on their own,
upr/modules.py).

* eval mode vs the reference-generated per-module goldens G3
  (tests/golden/make_golden.py g3: non-identity BatchNorm statistics);
* training mode (batch statistics, running-stat update, Dropout mask) forward +
  backward vs the oracle restatement with torch-CPU autograd (oracle/net.py in
  train mode, the product's Dropout mask replayed).
"""
import numpy as np
import pytest
import torch

from oracle import net as onet

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)

# name, constructor, args, oracle function, extra oracle args
CASES = {
    "fam": ("EnhancedFAM", (32, 32), lambda sd, x: onet.fam(sd, "m", x)),
    "aspp": ("ASPPModule", (64, 64), lambda sd, x: onet.aspp(sd, "m", x)),
    "preact": ("PreActResBlock", (32, 64, 2), lambda sd, x: onet.preact_block(sd, "m", x, 2)),
    "preact_id": ("PreActResBlock", (64, 64, 1), lambda sd, x: onet.preact_block(sd, "m", x, 1)),
    "res": ("ResBlock", (32, 64, 2), lambda sd, x: onet.resblock(sd, "m", x, 2)),
    "up": ("UpBlock", (64, 32), lambda sd, x: onet.upblock(sd, "m", x)),
}


def build(name):
    from models import model as M
    cls, args, _ = CASES[name]
    return getattr(M, cls)(*args)


def maxdiff(a, b):
    return (a.detach().float().cpu() - b.detach().float().cpu()).abs().max().item()


@pytest.mark.parametrize("name", list(CASES))
def test_submodule_eval_matches_reference_golden(golden, name):
    g = golden("g3_modules.npz")
    pre = name + "_sd."
    sd = {k[len(pre):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(pre)}
    mod = build(name)
    mod.load_state_dict(sd)
    mod = mod.eval().to(DEV)
    x = torch.from_numpy(g[name + "_x"]).to(DEV)
    y = mod(x)
    torch.cuda.synchronize()
    ref = torch.from_numpy(g[name + "_y"])
    err = maxdiff(y, ref)
    print(f"{name}: eval vs reference golden max|d| {err:.2e}")
    assert y.shape == ref.shape and y.device == x.device and y.dtype == torch.float32
    assert not y.requires_grad
    assert err <= 1e-4


# UpBlock: conv.0 / conv.3 carry biases and feed BatchNorm2d (models/model.py:261-269)
BN_FED_BIAS = {"up": ("conv.0.bias", "conv.3.bias")}


@pytest.mark.parametrize("name", list(CASES))
def test_submodule_train_forward_backward(name):
    torch.manual_seed(3)
    mod = build(name)
    with torch.no_grad():  # non-trivial BN state
        for m in mod.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
    sd0 = {k: v.clone() for k, v in mod.state_dict().items()}
    mod = mod.train().to(DEV)
    cin = CASES[name][1][0]
    gen = torch.Generator().manual_seed(7)
    x = torch.randn(2, cin, 16, 16, generator=gen)
    xd = x.to(DEV).requires_grad_(True)
    y = mod(xd)
    r = torch.randn(y.shape, generator=gen)
    (y * r.to(DEV)).sum().backward()
    torch.cuda.synchronize()

    # oracle: same state, train mode, the product's Dropout mask (ASPP) replayed
    mask_fn = None
    if name == "aspp":
        layer = mod.__dict__["_upr_layer"][1]
        B, C, H, W = y.shape
        m = layer.mask.cpu().view(B, H, W, C).permute(0, 3, 1, 2).float()
        mask_fn = lambda shape: m  # noqa: E731
    work = {("m." + k): v.clone() for k, v in sd0.items()}
    pnames = ["m." + k for k, _ in mod.named_parameters()]
    for k in pnames:
        work[k] = work[k].requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    from oracle import train as otrain
    with otrain.train_mode(mask_fn):
        yr = CASES[name][2](work, xr)
    (yr * r).sum().backward()

    err_y = maxdiff(y, yr)
    scale_x = xr.grad.abs().max().item()
    err_x = maxdiff(xd.grad, xr.grad)
    print(f"{name}: train y max|d| {err_y:.2e}, dx max|d| {err_x:.2e} (max|dx| {scale_x:.2e})")
    assert err_y <= 1e-4
    assert err_x <= 1e-4 * max(1.0, scale_x)
    gscale = max(work[kr].grad.abs().max().item() for kr in pnames)
    for (k, p), kr in zip(mod.named_parameters(), pnames):
        gr = work[kr].grad
        if k in BN_FED_BIAS.get(name, ()):
            # a conv bias feeding a train-mode BatchNorm has a zero true gradient
            # (the batch mean absorbs it): both sides are summation noise
            noise = max(p.grad.abs().max().item(), gr.abs().max().item())
            assert noise <= 1e-4 * max(1.0, gscale), f"{name} grad {k}: {noise} (module grad scale {gscale})"
            continue
        e = maxdiff(p.grad, gr)
        assert e <= 2e-4 * max(1.0, gr.abs().max().item()), f"{name} grad {k}: {e}"
    # running statistics updated like nn.BatchNorm2d.train()
    for k, v in mod.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            assert maxdiff(v, work["m." + k]) <= 1e-5, k
        if k.endswith("num_batches_tracked"):
            assert int(v) == int(sd0[k]) + 1, k


def test_submodule_fp16_rejected():
    mod = build("fam").eval().to(DEV)
    with pytest.raises(TypeError):
        mod(torch.rand(1, 32, 8, 8, device=DEV, dtype=torch.float16))
