"""The window-sweep forward (fwd_sweep_kernel: no-occlusion histogram at cutoff >= 5, the training
hot path) against the lane-serial TAIL drain (NLOSGR_FSWEEP=1 selects the sweep) and the dense evaluation.

Both culled drains add exact Gaussian values just outside the cutoff (the sweep up to 15 bins before
a segment's start and after its end, the lane-serial drain up to 19 after its end), so against each
other and against dense they agree to the cutoff's truncation (< 1e-7 of a Gaussian's peak per term
at 5.7 sigma) plus fp32 summation-order noise.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FWD_RTOL = 2e-5


def _close(a, b, rtol, atol=1e-7, msg=""):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = np.abs(b).max()
    err = np.abs(a - b).max()
    assert err <= rtol * scale + atol, f"{msg}: max err {err:.3e} vs scale {scale:.3e}"


def _setup(preset, ng, H, W, T, ns, seed, scale_shift=0.0):
    from nlosgr import GaussianParams, features_flat
    from nlosgr.volume import Scene
    dev = torch.device("cuda:0")
    scene = Scene(H=H, W=W, T=T, ns=ns)
    m = GaussianParams.synthetic(ng, 3, preset=preset, device=dev, seed=seed)
    if scale_shift:
        with torch.no_grad():
            m._scaling.add_(scale_shift)
    geo = scene.geometry(dev, preset)
    args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
            features_flat(m).detach().contiguous(), geo)
    return m, scene, args


def _three(args, cfg, monkeypatch):
    from dataclasses import replace
    from nlosgr.render import render_forward
    monkeypatch.setenv("NLOSGR_FSWEEP", "1")
    h_sw, _ = render_forward(*args, cfg)
    h_sw2, _ = render_forward(*args, cfg)
    monkeypatch.setenv("NLOSGR_FSWEEP", "0")
    h_ls, _ = render_forward(*args, cfg)
    monkeypatch.delenv("NLOSGR_FSWEEP", raising=False)
    h_dn, _ = render_forward(*args, replace(cfg, cutoff=0.0))
    return h_sw, h_sw2, h_ls, h_dn


@pytest.mark.parametrize("preset", ["cuda", "torch"])
def test_sweep_matches_lane_serial_and_dense(preset, monkeypatch):
    """C3-like geometry (T = 1024, 32x32 rays) with 6000 Gaussians over 3x3 wall points: every wave
    fills and sweeps its 640-record batch several times, with late takes and head passes."""
    from nlosgr.volume import make_config
    m, scene, args = _setup(preset, 6000, 3, 3, 1024, 32, seed=21)
    cfg = make_config(m, scene, preset, cutoff=5.7)
    h_sw, h_sw2, h_ls, h_dn = _three(args, cfg, monkeypatch)
    assert torch.isfinite(h_sw).all() and h_sw.abs().max() > 0
    assert torch.equal(h_sw, h_sw2), "sweep forward not bitwise repeatable"
    _close(h_sw.cpu(), h_ls.cpu(), FWD_RTOL, msg="sweep vs lane-serial")
    _close(h_sw.cpu(), h_dn.cpu(), FWD_RTOL, msg="sweep vs dense")
    # the sweep adds each window's wave-reduced sum once per bin where the lane-serial and dense
    # kernels add every term into a running fp32 total, which drops terms below half an ulp of it:
    # the sweep sits ~1e-5 above both (closer to a float64 sum, tests/test_gpu_sweep.py float64 case)
    rel = ((h_sw - h_dn).norm() / h_dn.norm()).item()
    assert rel < 4e-5, rel


def test_sweep_narrow_and_wide_gaussians(monkeypatch):
    """Gaussians from much narrower than a bin (exact per-bin path where a seed at the window start
    would underflow) to wide ones spanning several windows, ragged T (not a multiple of 16)."""
    from nlosgr.volume import make_config
    for shift, T in ((-3.0, 200), (0.8, 333)):
        m, scene, args = _setup("cuda", 1500, 2, 3, T, 12, seed=5, scale_shift=shift)
        cfg = make_config(m, scene, "cuda", cutoff=5.7)
        h_sw, h_sw2, h_ls, h_dn = _three(args, cfg, monkeypatch)
        assert torch.equal(h_sw, h_sw2)
        _close(h_sw.cpu(), h_ls.cpu(), FWD_RTOL, msg=f"sweep vs lane-serial (shift {shift})")
        _close(h_sw.cpu(), h_dn.cpu(), FWD_RTOL, msg=f"sweep vs dense (shift {shift})")


def test_sweep_empty_and_tiny(monkeypatch):
    """No Gaussian in support, and fewer Gaussians than lanes: the sweep leaves zeros / matches."""
    from nlosgr.volume import make_config
    m, scene, args = _setup("cuda", 7, 2, 2, 128, 8, seed=2)
    cfg = make_config(m, scene, "cuda", cutoff=5.7)
    h_sw, _, h_ls, h_dn = _three(args, cfg, monkeypatch)
    _close(h_sw.cpu(), h_ls.cpu(), FWD_RTOL, msg="tiny sweep vs lane-serial")
    mu = args[0].clone()
    mu[:, 1] += 100.0     # every Gaussian far outside the ToF range
    h, _, _, _ = _three((mu,) + args[1:], cfg, monkeypatch)
    assert torch.count_nonzero(h) == 0
