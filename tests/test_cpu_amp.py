"""GradScaler host logic (upr/amp.py) against torch's own GradScaler on CPU
(torch.amp.GradScaler("cpu") with a torch SGD over one parameter): the same
finite / non-finite step sequence must give the same scale after every
update(), and the same set of skipped steps.  Device unscale: tests/test_gpu_train.py."""
import torch

from upr.amp import GradScaler, next_scale


def test_next_scale_matches_torch_cpu_gradscaler():
    pattern = [False] * 5 + [True] + [False] * 3 + [True, True] + [False] * 9
    ref = torch.amp.GradScaler("cpu", init_scale=1024.0, growth_factor=2.0, backoff_factor=0.5,
                               growth_interval=3)
    p = torch.nn.Parameter(torch.ones(4))
    opt = torch.optim.SGD([p], lr=0.1)
    scale, tracker = 1024.0, 0
    for bad in pattern:
        opt.zero_grad()
        ref.scale(p.sum()).backward()
        if bad:
            p.grad[0] = float("inf")
        before = p.detach().clone()
        ref.step(opt)
        ref.update()
        skipped = bool(torch.equal(before, p.detach()))
        assert skipped == bad
        scale, tracker = next_scale(scale, tracker, bad, 2.0, 0.5, 3)
        assert scale == ref.get_scale()


def test_gradscaler_surface_matches_torch():
    s = GradScaler(init_scale=256.0, growth_interval=7)
    t = torch.amp.GradScaler("cpu", init_scale=256.0, growth_interval=7)
    assert s.get_scale() == t.get_scale() == 256.0
    assert s.get_growth_factor() == t.get_growth_factor()
    assert s.get_backoff_factor() == t.get_backoff_factor()
    assert s.get_growth_interval() == t.get_growth_interval()
    m = GradScaler.from_torch(t)
    assert m.get_scale() == 256.0 and m.get_growth_interval() == 7
    sd = s.state_dict()
    assert set(sd) == set(t.state_dict())
    off = GradScaler(enabled=False)
    x = torch.ones(2)
    assert off.scale(x) is x and off.get_scale() == 1.0
