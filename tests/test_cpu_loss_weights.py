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
    t = TotalLoss(use_dynamic_smooth_weight=False, weight_smooth=3.0)
    assert t._params["dynamic_smooth"] is False and t._weights["smoothness"] == 3.0


def test_loss_term_module_arguments():
    """The term modules keep the reference's constructor arguments and pass them
    to the device engine (values vs the oracle: tests/test_gpu_losses.py)."""
    from losses import loss as L
    m = L.AdaptiveExposureLoss(patch_size=8, base_target_exposure=0.5)
    assert (m.patch_size, m.base_target_exposure) == (8, 0.5)
    assert m._params["patch"] == 8 and m._params["base_exposure"] == 0.5 and m._weights["exposure"] == 1.0
    assert sum(m._weights.values()) == 1.0 and m._params["dynamic_smooth"] is False
    s = L.EdgeAwareSmoothnessLoss(lambda_val=5.0, alpha=0.5)
    assert s._params["smooth_lambda"] == 5.0 and s._params["smooth_alpha"] == 0.5
    assert L.IlluminationReflectanceDecouplingLoss(lambda_val=0.3)._params["decouple_lambda"] == 0.3
    f = L.FrequencyLoss(weight_high=2.0, weight_low=0.25)
    assert f._params["freq_high"] == 2.0 and f._params["freq_low"] == 0.25 and f.use_freq_loss
    assert not L.ColorLoss().use_freq_loss
    with pytest.raises(ValueError):
        L.AdaptiveExposureLoss(patch_size=0)
