"""GradScaler for the UP-Retinex training step (trainers/train.py:71-89, the
`use_amp and scaler is not None` branch: `scaler.scale(loss).backward()`,
`scaler.unscale_(optimizer)`, `clip_grad_norm_`, `scaler.step(optimizer)`,
`scaler.update()`), over the flat gradient buffer of upr.optim.Adam.

Same constructor, methods and dynamic-scale rule as torch.amp.GradScaler
(init_scale 2**16, growth 2.0 every 2000 finite steps, backoff 0.5 on an
inf/nan step, which is skipped):

  * scale(loss)   loss * scale (the loss node's backward multiplies the loss
                  gradients by it on the device);
  * unscale_(opt) ONE launch over the flat gradient buffer: g *= 1/scale and
                  the inf/nan flag (upr_t_unscale);
  * step(opt)     one host read of the flag; opt.step() only when finite;
  * update()      the growth / backoff rule (`next_scale`), scale rewritten on
                  the device.

The forward under autocast is NOT reduced to fp16 here: the training kernels
compute in fp32 (precision >= the reference's autocast), so AMP reproduces
the reference's control flow (scaled backward, skipped non-finite steps,
scale schedule) at fp32 arithmetic.
"""
import torch

from . import _lib as L
from .train import _chk, _p, _stream, zero


def next_scale(scale, tracker, found_inf, growth_factor, backoff_factor, growth_interval):
    """torch's _amp_update_scale_ rule -> (new scale, new growth tracker)."""
    if found_inf:
        return scale * backoff_factor, 0
    tracker += 1
    if tracker == growth_interval:
        return scale * growth_factor, 0
    return scale, tracker


class GradScaler:
    def __init__(self, device="cuda", init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5,
                 growth_interval=2000, enabled=True):
        if growth_factor <= 1.0 or not 0.0 < backoff_factor < 1.0:
            raise ValueError("growth_factor must be > 1 and backoff_factor in (0, 1)")
        self._enabled = bool(enabled)
        self._scale_value = float(init_scale)
        self._growth_factor = float(growth_factor)
        self._backoff_factor = float(backoff_factor)
        self._growth_interval = int(growth_interval)
        self._tracker = 0
        self._scale = None      # device fp32 scalar
        self._found_inf = None  # device fp32 scalar
        self._stage = {}        # id(optimizer) -> "unscaled" / "stepped"
        self._inf_seen = False

    @classmethod
    def from_torch(cls, scaler):
        """A upr GradScaler with a torch.amp.GradScaler's settings and current scale."""
        return cls(init_scale=float(scaler.get_scale()) if scaler.is_enabled() else 2.0 ** 16,
                   growth_factor=scaler.get_growth_factor(), backoff_factor=scaler.get_backoff_factor(),
                   growth_interval=scaler.get_growth_interval(), enabled=scaler.is_enabled())

    def is_enabled(self):
        return self._enabled

    def get_scale(self):
        return self._scale_value if self._enabled else 1.0

    def get_growth_factor(self):
        return self._growth_factor

    def get_backoff_factor(self):
        return self._backoff_factor

    def get_growth_interval(self):
        return self._growth_interval

    def _lazy(self, dev):
        if self._scale is None or self._scale.device != dev:
            self._scale = torch.full((), self._scale_value, dtype=torch.float32, device=dev)
            self._found_inf = torch.zeros((), dtype=torch.float32, device=dev)

    def scale(self, outputs):
        if not self._enabled:
            return outputs
        self._lazy(outputs.device)
        return outputs * self._scale

    def unscale_(self, optimizer):
        if not self._enabled:
            return
        if self._stage.get(id(optimizer)) == "unscaled":
            raise RuntimeError("unscale_() has already been called on this optimizer since the last update().")
        if self._stage.get(id(optimizer)) == "stepped":
            raise RuntimeError("unscale_() is being called after step().")
        flat = optimizer.flat
        self._lazy(flat.grad.device)
        zero(self._found_inf)
        _chk(L.lib().upr_t_unscale(_p(flat.grad), flat.numel, _p(self._scale), _p(self._found_inf), _stream()),
             "unscale")
        self._stage[id(optimizer)] = "unscaled"

    def step(self, optimizer, *args, **kwargs):
        if not self._enabled:
            return optimizer.step(*args, **kwargs)
        if self._stage.get(id(optimizer)) == "stepped":
            raise RuntimeError("step() has already been called since the last update().")
        if self._stage.get(id(optimizer)) != "unscaled":
            self.unscale_(optimizer)
        found = bool(self._found_inf.item())  # the one host sync of the step (as torch's)
        self._inf_seen = self._inf_seen or found
        self._stage[id(optimizer)] = "stepped"
        if found:
            from .optim import discard_clip
            discard_clip(optimizer)  # the clip recorded for this step does not carry over
            return None
        return optimizer.step(*args, **kwargs)

    def update(self, new_scale=None):
        if not self._enabled:
            return
        if new_scale is not None:
            self._scale_value = float(new_scale)
            self._tracker = 0
        else:
            self._scale_value, self._tracker = next_scale(self._scale_value, self._tracker, self._inf_seen,
                                                          self._growth_factor, self._backoff_factor,
                                                          self._growth_interval)
        if self._scale is not None:
            self._scale.fill_(self._scale_value)
        self._stage.clear()
        self._inf_seen = False

    def state_dict(self):
        if not self._enabled:
            return {}
        return {"scale": self._scale_value, "growth_factor": self._growth_factor,
                "backoff_factor": self._backoff_factor, "growth_interval": self._growth_interval,
                "_growth_tracker": self._tracker}

    def load_state_dict(self, sd):
        self._scale_value = float(sd["scale"])
        self._growth_factor = float(sd["growth_factor"])
        self._backoff_factor = float(sd["backoff_factor"])
        self._growth_interval = int(sd["growth_interval"])
        self._tracker = int(sd["_growth_tracker"])
        if self._scale is not None:
            self._scale.fill_(self._scale_value)
