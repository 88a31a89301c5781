"""Host logic of the fused training step that needs no GPU: the position learning-rate schedule
(get_expon_lr_func, gaussian_utils.py:223-256) and the optimiser defaults (configs/default.py:59-90)."""
import math

import pytest


def test_expon_lr_schedule():
    from nlosgr.train import expon_lr
    assert expon_lr(0, 1e-3, 1e-5, max_steps=100) == pytest.approx(1e-3)
    assert expon_lr(100, 1e-3, 1e-5, max_steps=100) == pytest.approx(1e-5)
    assert expon_lr(250, 1e-3, 1e-5, max_steps=100) == pytest.approx(1e-5)      # clipped past max_steps
    assert expon_lr(50, 1e-3, 1e-5, max_steps=100) == pytest.approx(1e-4)
    assert expon_lr(-1, 1e-3, 1e-5) == 0.0
    assert expon_lr(3, 0.0, 0.0) == 0.0
    d = expon_lr(5, 1e-3, 1e-3, lr_delay_steps=10, lr_delay_mult=0.01, max_steps=100)
    assert d == pytest.approx(1e-3 * (0.01 + 0.99 * math.sin(0.25 * math.pi)))


def test_optimization_defaults_match_reference_config():
    from nlosgr.train import OptimizationParams
    o = OptimizationParams()
    assert (o.position_lr_init, o.position_lr_final, o.position_lr_delay_mult, o.position_lr_max_steps) == \
        (0.00016, 0.0000016, 0.01, 50_000)
    assert (o.feature_lr, o.opacity_lr, o.scaling_lr, o.rotation_lr) == (0.0025, 0.025, 0.005, 0.001)
    assert (o.regularization, o.scale_reg, o.opacity_reg) == (False, 0.01, 0.01)


def test_rendering_type_dispatch():
    """nlos_helpers dispatch (nlos_helpers.py:200-212, gaussian_model.py:297-364): occlusion off ->
    no-occlusion sum; 'netf' -> per-Gaussian self-transmittance; 'nlos-neus' crashes in the reference
    (gaussian_model.py:336 shape mismatch) and is rejected explicitly here."""
    from types import SimpleNamespace
    import pytest
    from nlosgr.nlos_helpers import _mode
    assert _mode(SimpleNamespace(occlusion=False, rendering_type="nlos-neus")) == "noocl"
    assert _mode(SimpleNamespace(occlusion=True, rendering_type="netf")) == "netf"
    assert _mode(SimpleNamespace(occlusion=True)) == "netf"
    with pytest.raises(NotImplementedError):
        _mode(SimpleNamespace(occlusion=True, rendering_type="nlos-neus"))
