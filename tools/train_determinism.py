"""Diagnostic: run the device training forward+backward of one variant several
times on identical inputs and report, per parameter, the largest relative
run-to-run gradient difference (a race shows as large differences; atomic
summation order as ~1e-6)."""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "retinex-image-enhancement_amd"))
import torch
from models.model import UP_Retinex
from losses.loss import TotalLoss

pre, aspp = sys.argv[1] == "1", sys.argv[2] == "1"
torch.manual_seed(3)
model = UP_Retinex(use_preact=pre, use_aspp=aspp).to("cuda").train()
crit = TotalLoss(use_freq_loss=True).to("cuda")
x = (torch.rand(4, 3, 64, 64, generator=torch.Generator().manual_seed(5)) * 0.6).cuda()
sd0 = {k: v.clone() for k, v in model.state_dict().items()}
runs = []
for r in range(4):
    model.load_state_dict(sd0)
    for p in model.parameters():
        p.grad = None
    torch.manual_seed(7)  # same dropout mask each run if the mask draws from torch's RNG
    enh, refl, illu = model(x)
    total, d = crit(x, enh, illu, refl)
    total.backward()
    torch.cuda.synchronize()
    runs.append((enh.detach().clone(), {n: p.grad.detach().clone() for n, p in model.named_parameters()}, total.item()))
    print("run", r, "loss", total.item(), flush=True)
e0, g0, _ = runs[0]
for r in range(1, len(runs)):
    e, g, _ = runs[r]
    print(f"run {r}: enh max|d| {(e - e0).abs().max().item():.3e}")
    worst = sorted(((((g[n] - g0[n]).norm() / (g0[n].norm() + 1e-30)).item(), n) for n in g0), reverse=True)[:8]
    for v, n in worst:
        print(f"   {n}: rel-L2 run-to-run {v:.3e}")
