"""Standalone submodule forwards on the device (reference models/model.py:11-274:
EnhancedFAM, ResBlock, PreActResBlock, ASPPModule, UpBlock called on their own,
upr/modules.py).

* eval mode vs the reference-generated per-module goldens G3
  (tests/golden/make_golden.py g3: non-identity BatchNorm statistics);
* training mode (batch statistics, running-stat update, Dropout mask) forward +
  backward vs the oracle restatement with torch-CPU autograd (oracle/net.py in
  train mode, the product's Dropout mask replayed).
"""
import copy

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


def test_submodule_dtype_mismatch_raises():
    """A float16 input to a float32 module raises like the reference's conv."""
    mod = build("fam").eval().to(DEV)
    with pytest.raises(RuntimeError):
        mod(torch.rand(1, 32, 8, 8, device=DEV, dtype=torch.float16))


@pytest.mark.parametrize("name", list(CASES))
def test_submodule_half_eval_vs_oracle(name):
    """A .half() submodule on a float16 input (the reference's `.half()` module
    runs its convs in fp16): float16 output, vs the fp32 oracle on the
    fp16-rounded weights and input within 2e-2 of max(1, max|y|) (fp16 conv
    arithmetic through up to six convs; BatchNorm / attention stay fp32)."""
    torch.manual_seed(4)
    mod = build(name)
    with torch.no_grad():
        for m in mod.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
    mod = mod.half().eval().to(DEV)
    sd = {"m." + k: v.float().cpu() for k, v in mod.state_dict().items()}
    cin = CASES[name][1][0]
    x = torch.randn(2, cin, 16, 16, generator=torch.Generator().manual_seed(5)).half()
    y = mod(x.to(DEV))
    torch.cuda.synchronize()
    assert y.dtype == torch.float16 and not y.requires_grad
    with torch.no_grad():
        ref = CASES[name][2](sd, x.float())
    err = maxdiff(y, ref)
    scale = max(1.0, ref.abs().max().item())
    print(f"{name}: half eval max|d| {err:.2e} (scale {scale:.2f})")
    assert err <= 2e-2 * scale


def test_submodule_half_train_grads_follow_fp32():
    """Training mode of a .half() ResBlock: float16 .grad on the module's own
    parameters and the running statistics written back.  Yardstick: the fp64
    oracle on the fp16-rounded weights and input, plain (g64) and with the
    fp16 conv arithmetic emulated (oracle/net.py amp_conv: fp16-rounded conv
    operands and outputs, g16); per tensor the device gradient's rel-L2 from
    g64 must lie within max(2 x the emulation's, 1e-2) (+ the fp16 rounding of
    the stored gradient)."""
    from oracle import train as otrain
    torch.manual_seed(6)
    m16 = build("res").half()
    sd = {"m." + k: v.double() for k, v in m16.state_dict().items()}
    m16 = m16.train().to(DEV)
    x = torch.randn(4, 32, 16, 16, generator=torch.Generator().manual_seed(7)).half()
    r = torch.randn(4, 64, 8, 8, generator=torch.Generator().manual_seed(8))
    y16 = m16(x.to(DEV))
    assert y16.dtype == torch.float16
    (y16.float() * r.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    names = ["m." + k for k, _ in m16.named_parameters()]

    def oracle(amp):
        work = {k: v.clone() for k, v in sd.items()}
        for k in names:
            work[k].requires_grad_(True)
        with otrain.train_mode(amp=amp):
            yr = onet.resblock(work, "m", x.double(), 2)
        (yr * r.double()).sum().backward()
        return {k: work[k].grad for k in names}, work

    g64, w64 = oracle(False)
    g16, _ = oracle(True)
    for (k, p16), kr in zip(m16.named_parameters(), names):
        assert p16.grad is not None and p16.grad.dtype == torch.float16, k
        if k in ("conv1.bias", "conv2.bias"):
            continue
        ref = g64[kr]
        rn = ref.norm().item()
        dev = (p16.grad.double().cpu() - ref).norm().item() / rn
        band = (g16[kr] - ref).norm().item() / rn
        print(f"{k}: rel-L2 device {dev:.3e}, emulated fp16 convs {band:.3e}")
        assert dev <= max(2.0 * band, 1e-2), f"{k}: rel-L2 {dev:.3e} (fp16 band {band:.3e})"
    for k, b16 in m16.named_buffers():
        if k.endswith("running_mean") or k.endswith("running_var"):
            ref = w64["m." + k]
            assert (b16.double().cpu() - ref).abs().max().item() <= 5e-3 * max(1.0, ref.abs().max().item()), k


def test_submodule_two_forwards_then_backward():
    """m(x1), m(x2), then backward through both graphs: each backward uses its
    own call's saved activations / BatchNorm statistics (reference autograd
    semantics), and an eval-mode forward in between changes nothing."""
    torch.manual_seed(9)
    mod = build("preact").train().to(DEV)
    gen = torch.Generator().manual_seed(10)
    x1, x2 = torch.randn(2, 32, 16, 16, generator=gen), torch.randn(2, 32, 16, 16, generator=gen) * 2.0
    r1, r2 = torch.randn(2, 64, 8, 8, generator=gen), torch.randn(2, 64, 8, 8, generator=gen)

    def grads_of(calls):
        for p in mod.parameters():
            p.grad = None
        outs = []
        for xi in calls:
            xd = xi.to(DEV).requires_grad_(True)
            outs.append((xd, mod(xd)))
        return outs

    # reference answer: each call's backward right after its own forward
    sd0 = {k: v.clone() for k, v in mod.state_dict().items()}
    want = []
    for xi, ri in ((x1, r1), (x2, r2)):
        mod.load_state_dict(sd0)
        (xd, y), = grads_of([xi])
        (y * ri.to(DEV)).sum().backward()
        want.append((xd.grad.clone(), {k: p.grad.clone() for k, p in mod.named_parameters()}))
    # interleaved: two forwards (and an eval forward), then both backwards in reverse order
    mod.load_state_dict(sd0)
    (xa, ya), (xb, yb) = grads_of([x1, x2])
    mod.eval()
    with torch.no_grad():
        mod(x1.to(DEV))
    mod.train()
    (yb * r2.to(DEV)).sum().backward()
    gb = {k: p.grad.clone() for k, p in mod.named_parameters()}
    (ya * r1.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert maxdiff(xa.grad, want[0][0]) <= 1e-5 * max(1.0, want[0][0].abs().max().item())
    assert maxdiff(xb.grad, want[1][0]) <= 1e-5 * max(1.0, want[1][0].abs().max().item())
    for k, p in mod.named_parameters():
        tot = want[0][1][k] + want[1][1][k]
        assert maxdiff(gb[k], want[1][1][k]) <= 1e-5 * max(1.0, want[1][1][k].abs().max().item()), k
        assert maxdiff(p.grad, tot) <= 1e-5 * max(1.0, tot.abs().max().item()), k
