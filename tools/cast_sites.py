"""Which library calls of one AMP training step cast an fp32 operand to fp16
themselves (cast_act_f16_kernel) -- i.e. where the producer wrote no fp16 copy.
Wraps the ctypes entries, runs one bs-2 512^2 step, prints the call sites."""
import collections
import os
import sys
import traceback

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "retinex-image-enhancement_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))
from upr import _lib as L  # noqa: E402

lib = L.lib()
sites = collections.Counter()


def site():
    st = traceback.extract_stack()[:-2]
    fr = [f for f in st if "upr" in f.filename][-3:]
    return " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in reversed(fr))


def wrap(name, pred):
    fn = getattr(lib, name)

    class W:
        def __call__(self, *a):
            if pred(a):
                sites[(name, site())] += 1
            return fn(*a)
    setattr(lib, name, W())


wrap("upr_t_conv_mfma16", lambda a: not a[23])           # x16_ready == 0
wrap("upr_t_conv_wgrad16", lambda a: a[1] is None)       # x16 NULL
wrap("upr_t_conv_wgrad_into", lambda a: a[1] is None)
wrap("upr_t_cast_f16", lambda a: True)


def main():
    from models.model import UP_Retinex
    from losses.loss import TotalLoss
    from trainers.train import make_optimizer, train_step, GradScaler
    torch.manual_seed(0)
    m = UP_Retinex(use_preact=False, use_aspp=False).cuda().train()
    crit = TotalLoss(use_freq_loss=True).cuda()
    opt = make_optimizer(m, lr=1e-4, weight_decay=1e-5)
    x = torch.rand(2, 3, 512, 512, device="cuda")
    scaler = GradScaler()
    for _ in range(2):
        sites.clear()
        train_step(m, x, crit, opt, scaler=scaler, use_amp=True)
    torch.cuda.synchronize()
    for (n, s), c in sites.most_common():
        print(f"{c:3d} {n:24s} {s}")


if __name__ == "__main__":
    main()
