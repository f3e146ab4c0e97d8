"""clip_grad_norm_ + Adam over the flat parameter buffer (one reduction and one
update launch per step) — the optimiser half of trainers/train.py:84-103
(`torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)` then
`optim.Adam(lr, weight_decay).step()`).

`clip_grad_norm_` launches the squared-norm reduction and records max_norm;
the following `Adam.step()` applies the clip coefficient on the device inside
the update kernel, so the step needs no host synchronisation.  The returned
norm is a device tensor (written by the step), as torch's is.
"""
import ctypes

import torch

from . import _lib as L
from .autograd import bump_weights_epoch
from .train import FlatParams, _chk, _p, _stream, zero


def _flat_of(params):
    """The FlatParams holding these parameters; flattens them on first use
    (before the first training forward, as the reference builds its optimiser)."""
    params = [p for p in params]
    f = getattr(params[0], "_upr_flat", None)
    if f is None or any(getattr(p, "_upr_flat", None) is not f for p in params):
        f = FlatParams(params)
    return f, params


class _ClipState:
    def __init__(self, dev):
        self.sq = torch.empty(1, dtype=torch.float64, device=dev)
        self.norm = torch.empty((), dtype=torch.float32, device=dev)
        self.max_norm = 0.0


_clip = {}


def clip_grad_norm_(parameters, max_norm, norm_type=2.0):
    """torch.nn.utils.clip_grad_norm_ semantics (L2 total norm, coefficient
    max_norm / (norm + 1e-6) clamped to 1), applied by the next Adam.step()."""
    if float(norm_type) != 2.0:
        raise NotImplementedError("only the L2 norm (the reference's default) is implemented")
    flat, _ = _flat_of(parameters)
    cs = _clip.get(id(flat))
    if cs is None:
        cs = _clip[id(flat)] = _ClipState(flat.grad.device)
    zero(cs.sq)
    _chk(L.lib().upr_t_sqsum(_p(flat.grad), flat.numel, _p(cs.sq), _stream()), "sqsum")
    cs.max_norm = float(max_norm)
    return cs.norm


def discard_clip(optimizer):
    """Drop the clip recorded by clip_grad_norm_ for a step that is skipped
    (GradScaler.step on a non-finite step)."""
    cs = _clip.get(id(optimizer.flat))
    if cs is not None:
        cs.max_norm = 0.0


class Adam:
    """torch.optim.Adam(params, lr, betas, eps, weight_decay) (L2 decay added to
    the gradient, bias-corrected moments) over the flat buffer."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.flat, self.params = _flat_of(params)
        self.param_groups = [{"params": self.params, "lr": lr, "betas": betas, "eps": eps,
                              "weight_decay": weight_decay}]
        dev = self.flat.grad.device
        self.m = torch.zeros(self.flat.numel, dtype=torch.float32, device=dev)
        self.v = torch.zeros(self.flat.numel, dtype=torch.float32, device=dev)
        self.step_count = 0
        self._sq = torch.empty(1, dtype=torch.float64, device=dev)

    def zero_grad(self, set_to_none=True):
        self.flat.attach_grads()
        zero(self.flat.grad)

    def step(self):
        g = self.param_groups[0]
        self.step_count += 1
        cs = _clip.get(id(self.flat))
        if cs is not None and cs.max_norm > 0:
            sq, max_norm, norm_out = cs.sq, cs.max_norm, cs.norm
            cs.max_norm = 0.0
        else:
            zero(self._sq)
            sq, max_norm, norm_out = self._sq, 0.0, None
        b1, b2 = g["betas"]
        _chk(L.lib().upr_t_adam(_p(self.flat.flat), _p(self.flat.grad), _p(self.m), _p(self.v), self.flat.numel,
                                _p(sq), ctypes.c_float(max_norm), ctypes.c_float(g["lr"]), ctypes.c_float(b1),
                                ctypes.c_float(b2), ctypes.c_float(g["eps"]), ctypes.c_float(g["weight_decay"]),
                                self.step_count, _p(norm_out), _stream()), "adam")
        bump_weights_epoch()

    def state_dict(self):
        return {"step": self.step_count, "m": self.m, "v": self.v, "param_groups": [
            {k: v for k, v in self.param_groups[0].items() if k != "params"}]}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.param_groups[0].update(sd["param_groups"][0])
