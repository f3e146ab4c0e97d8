"""Host-side loss weighting of losses/loss.py: the DWA rule
(TotalLoss._compute_adaptive_weights, reference loss.py:755-798) on
hand-computed histories, and the TotalLoss argument checks.  No device calls."""
import pytest

from losses.loss import TotalLoss, dwa_weights

DEFAULTS = dict(exposure=10.0, smoothness=1.0, color=0.5, spatial=1.0, decouple=0.1, perceptual=1.0, frequency=0.5)


def test_dwa_known_answer():
    hist = {k: [] for k in DEFAULTS}
    hist["exposure"] = [2.0, 1.0]      # ratio 0.5 -> 0.25
    hist["color"] = [1.0, 3.0]         # ratio 3   -> 1.5
    hist["decouple"] = [0.0, 5.0]      # previous <= 1e-8 -> ratio 1 -> 0.5
    hist["spatial"] = [4.0]            # < 2 entries: constructor weight 1.0
    raw = dict(DEFAULTS, exposure=0.25, color=1.5, decouple=0.5)
    tot = sum(raw.values())
    want = {k: 7 * v / tot for k, v in raw.items()}
    got = dwa_weights(hist, DEFAULTS)
    assert got.keys() == want.keys()
    for k in want:
        assert got[k] == pytest.approx(want[k], rel=1e-12), k
    assert sum(got.values()) == pytest.approx(7.0)


def test_dwa_empty_history_is_normalised_defaults():
    got = dwa_weights({k: [] for k in DEFAULTS}, DEFAULTS)
    tot = sum(DEFAULTS.values())
    for k, v in DEFAULTS.items():
        assert got[k] == pytest.approx(7 * v / tot)


def test_totalloss_arguments():
    TotalLoss(texture_method="edge_density", weight_smooth=2.0, adaptive_weights=True)
    with pytest.raises(ValueError):
        TotalLoss(texture_method="sobel")
    with pytest.raises(NotImplementedError):
        TotalLoss(use_dynamic_smooth_weight=False)
