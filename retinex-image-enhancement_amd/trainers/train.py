"""UP-Retinex training step (drop-in for the reference trainers/train.py:27-131).

`train_one_epoch` keeps the reference's signature and step order
(zero_grad -> forward -> TotalLoss -> backward -> clip_grad_norm_(1.0) ->
Adam.step()); the model, loss and optimiser it is handed run on the gfx950
training kernels: `make_optimizer` builds upr.optim.Adam (flat-buffer fused
clip + Adam), and `clip_grad_norm_` is upr.optim's.  With `use_amp` and a
scaler the step follows the reference's AMP branch (train.py:71-89): scaled
backward, unscale_ (one launch over the flat gradient buffer), clip, a step
skipped on inf/nan, scale update — upr.amp.GradScaler (a torch.amp.GradScaler
handed in is mirrored by one with its settings).  As in the reference, the
forward and the loss of that branch run under torch.autocast: the engine then
computes its MFMA convolutions (and their input gradients) in fp16 with fp32
accumulation (upr/train.py, autocast_active); weight gradients, BatchNorm, the
losses and the optimiser stay fp32.  `amp_fp16=False` keeps the GradScaler
control flow with fp32 arithmetic.
"""
import time

import torch

from losses.loss import deferred_readback
from upr import amp as uamp
from upr import optim as uoptim

clip_grad_norm_ = uoptim.clip_grad_norm_
GradScaler = uamp.GradScaler
_mirrors = {}


def _as_upr_scaler(scaler):
    if scaler is None or isinstance(scaler, uamp.GradScaler):
        return scaler
    m = _mirrors.get(id(scaler))
    if m is None or m[0] is not scaler:
        m = _mirrors[id(scaler)] = (scaler, uamp.GradScaler.from_torch(scaler))
    return m[1]


def make_optimizer(model, lr=1e-4, weight_decay=1e-5):
    """optim.Adam(model.parameters(), lr, weight_decay) of train.py:241-245."""
    return uoptim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)


def train_step(model, img_low, criterion, optimizer, max_norm=1.0, scaler=None, use_amp=False, grad_hook=None,
               amp_fp16=True):
    """One step body (train.py:63-103).  Returns (loss, loss_dict).  grad_hook
    (e.g. upr.dist.allreduce_grads for data parallelism) runs between the
    backward and the unscale / clip."""
    optimizer.zero_grad()
    scaler = _as_upr_scaler(scaler) if use_amp else None
    # the loss_dict's floats are read back after the backward / optimizer work is
    # queued (returned materialised), not between forward and backward
    with torch.autocast("cuda", dtype=torch.float16, enabled=scaler is not None and amp_fp16), \
            deferred_readback():
        img_enhanced, reflectance, illu_map = model(img_low)
        loss, loss_dict = criterion(img_low, img_enhanced, illu_map, reflectance)
    if scaler is not None:
        scaler.scale(loss).backward()
        if grad_hook is not None:
            grad_hook()
        scaler.unscale_(optimizer)
        clip_grad_norm_(model.parameters(), max_norm=max_norm)
        scaler.step(optimizer)
        scaler.update()
    else:
        loss.backward()
        if grad_hook is not None:
            grad_hook()
        clip_grad_norm_(model.parameters(), max_norm=max_norm)
        optimizer.step()
    return loss, (dict(loss_dict.items()) if type(loss_dict) is not dict else loss_dict)


def train_one_epoch(model, dataloader, criterion, optimizer, device, epoch, writer=None, scaler=None, use_amp=False):
    model.train()
    keys = ('total', 'exposure', 'smoothness', 'color', 'spatial', 'decouple', 'perceptual')
    totals = {k: 0.0 for k in keys}
    n = 0
    t0 = time.time()
    for batch_idx, img_low in enumerate(dataloader):
        img_low = img_low.to(device, torch.float32)
        _, loss_dict = train_step(model, img_low, criterion, optimizer, scaler=scaler, use_amp=use_amp)
        for k in keys:
            totals[k] += loss_dict[k]
        n += 1
        if writer is not None and batch_idx % 100 == 0:
            for k, v in loss_dict.items():
                writer.add_scalar(f'Loss/{k}', v, epoch * max(1, len(dataloader)) + batch_idx)
    if n:
        totals = {k: v / n for k, v in totals.items()}
    totals["_epoch_seconds"] = time.time() - t0
    return totals
