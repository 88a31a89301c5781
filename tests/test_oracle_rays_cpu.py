"""CPU checks of the path-C oracle restatement (oracle/torch_ref.py rays section).

Path C (CUDA) has no runnable reference here (no CUDA), so these pin the vectorised oracle to
literal restatements of the reference loops: the per-ray, per-sample marching loop with the
shared transmittance and early exit (volume_renderer.cu:66-137) and the index-order AABB filter
with its 256 cap (ray_aabb.cu:31-57).  Parity of that restatement with the .cu text itself is
unpinned."""
import math

import torch

from conftest import ROOT  # noqa: F401


def _params(ng, seed, scale_shift=0.0):
    from nlosgr.model import GaussianParams
    from oracle import torch_ref as R
    m = GaussianParams.synthetic(ng, 0, preset="cuda", device="cpu", seed=seed)
    with torch.no_grad():
        m._scaling.add_(scale_shift)
    return R.Params(m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
                    m._features_dc.detach(), m._features_rest.detach(), 0, requires_grad=False)


def _rays(nr, seed):
    g = torch.Generator().manual_seed(seed)
    o = torch.zeros(nr, 3)
    o[:, 0] = torch.rand(nr, generator=g) - 0.5
    o[:, 2] = torch.rand(nr, generator=g) - 0.5
    th = 0.3 + 1.0 * torch.rand(nr, generator=g)
    ph = 0.8 + 1.5 * torch.rand(nr, generator=g)
    d = torch.stack([torch.sin(th) * torch.cos(ph), torch.sin(th) * torch.sin(ph), torch.cos(th)], 1)
    return o, d


def test_occlusion_matches_sequential_march():
    from oracle import torch_ref as R
    P = _params(24, 3, scale_shift=1.5)
    with torch.no_grad():
        P._opacity.add_(3.0)
    o, d = _rays(6, 4)
    t = torch.linspace(0.1, 1.4, 40)
    cam = torch.zeros(3)
    c, dT = 1.0, 0.5
    bb = R.bboxes_cuda(P)
    filt = R.aabb_filter(o, d, bb)
    rho, dens, tr = R.render_rays_cuda(o, d, t, P, P._features_dc[:, :, 0], cam, 0, c, dT, 1.0, True, filt)
    # literal restatement of the marching loop
    x = (o[:, None, :] + d[:, None, :] * t[None, :, None]).reshape(-1, 3)
    pdf = R.gaussian_pdf(x, P, "cuda").view(-1, 6, 40)
    sig = torch.sigmoid(P._opacity)[:, 0]
    dn = (P._mu - cam) / (torch.sqrt(((P._mu - cam) ** 2).sum(1, keepdim=True)) + 1e-8)
    rho_g = torch.clamp_min(R.eval_sh_cuda(0, P._features_dc[:, :, 0], dn) + 0.5, 0.0)
    exits = 0
    for r in range(6):
        idx = filt[r, 1:1 + int(filt[r, 0])].long()
        T = 1.0
        for s in range(40):
            contrib = pdf[idx, r, s] * sig[idx]
            D = float(contrib.sum())
            wa = float(((1 - torch.exp(-contrib * c * dT)) * rho_g[idx]).sum())
            assert math.isclose(float(tr[r, s]), T, rel_tol=1e-5, abs_tol=1e-12)
            assert math.isclose(float(rho[r, s]), T * wa, rel_tol=1e-5, abs_tol=1e-12)
            assert math.isclose(float(dens[r, s]), D, rel_tol=1e-5, abs_tol=1e-12)
            T = T * math.exp(-D * c * dT)
            if T < 1e-4:
                assert torch.all(rho[r, s + 1:] == 0) and torch.all(dens[r, s + 1:] == 0)
                assert torch.all(tr[r, s + 1:] == 0)
                exits += 1
                break
    assert exits > 0   # the configuration exercises the early exit


def test_aabb_filter_order_and_cap():
    from oracle import torch_ref as R
    P = _params(300, 5, scale_shift=3.0)          # huge boxes: every ray hits every Gaussian
    o, d = _rays(3, 6)
    filt = R.aabb_filter(o, d, R.bboxes_cuda(P))
    assert filt.shape == (3, 257) and filt.dtype == torch.int32
    assert torch.all(filt[:, 0] == 256)
    assert torch.equal(filt[:, 1:], torch.arange(256, dtype=torch.int32).expand(3, 256))
    P = _params(50, 7)
    filt = R.aabb_filter(o, d, R.bboxes_cuda(P))
    for r in range(3):
        n = int(filt[r, 0])
        idx = filt[r, 1:1 + n]
        assert torch.all(idx[1:] > idx[:-1]) and torch.all(filt[r, 1 + n:] == -1)
