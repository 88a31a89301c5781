"""GPU parity of the path-C rays API (HIP through the C ABI) against the CPU oracle restatement
of volume_renderer.cu / ray_aabb.cu.  Tolerances (fp32):
  filter      exact (int32 rows)
  forward     max|hip - ref| <= 2e-5 * max|ref| + 1e-7 without occlusion; 2e-4 with occlusion
              (alpha = 1 - exp(-x) in the reference formula loses ~6e-8 absolute to cancellation;
              the kernel uses expm1)
  gradients   max|hip - ref| <= 2e-4 * max|ref| + 1e-6 (3e-4 with occlusion)
The reference's backward returns zeros, so gradients are pinned to torch autograd of the oracle.
"""
import numpy as np
import pytest
import torch

from conftest import ROOT  # noqa: F401

pytestmark = pytest.mark.gpu


def _close(a, b, rtol, atol=1e-7, msg=""):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, dtype=np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, dtype=np.float64)
    scale = np.abs(b).max() if b.size else 0.0
    err = np.abs(a - b).max() if b.size else 0.0
    assert err <= rtol * scale + atol, f"{msg}: max err {err:.3e} vs scale {scale:.3e}"


def _scene(ng, nrays, seed, scale_shift=1.0, opac_shift=0.0, deg=0):
    from nlosgr import GaussianParams
    dev = torch.device("cuda:0")
    m = GaussianParams.synthetic(ng, deg, preset="cuda", device=dev, seed=seed)
    with torch.no_grad():
        m._scaling.add_(scale_shift)
        m._opacity.add_(opac_shift)
    g = torch.Generator().manual_seed(seed + 1)
    o = torch.zeros(nrays, 3)
    o[:, 0] = torch.rand(nrays, generator=g) - 0.5
    o[:, 2] = torch.rand(nrays, generator=g) - 0.5
    th = 0.3 + 1.0 * torch.rand(nrays, generator=g)
    ph = 0.8 + 1.5 * torch.rand(nrays, generator=g)
    d = torch.stack([torch.sin(th) * torch.cos(ph), torch.sin(th) * torch.sin(ph), torch.cos(th)], 1)
    return m, o.to(dev), d.to(dev)


def _oracle(m, deg):
    from oracle import torch_ref as R
    cpu = lambda t: t.detach().cpu()
    feats = torch.cat([m._features_dc, m._features_rest], dim=1)[:, :, 0]
    return R.Params(cpu(m._mu), cpu(m._scaling), cpu(m._rotation), cpu(m._opacity), cpu(m._features_dc),
                    cpu(m._features_rest), deg), cpu(feats)


@pytest.mark.parametrize("ng,shift", [(200, 0.5), (400, 3.0)])
def test_filter_matches_oracle(ng, shift):
    from nlosgr.rays import gaussian_filter
    from oracle import torch_ref as R
    m, o, d = _scene(ng, 40, 11, scale_shift=shift)
    filt = gaussian_filter(o, d, m._mu, m._scaling, m._rotation)
    P, _ = _oracle(m, 0)
    ref = R.aabb_filter(o.cpu(), d.cpu(), R.bboxes_cuda(P))
    got = filt.cpu()
    # a box face within fp32 rounding of the ray can flip one hit; everything else is exact
    diff = (got != ref).any(dim=1)
    assert int(diff.sum()) <= 1, f"{int(diff.sum())} rows differ"
    if shift >= 3.0:
        assert torch.all(got[:, 0] == 256)


@pytest.mark.parametrize("occl", [False, True])
@pytest.mark.parametrize("deg", [0, 3])
def test_render_rays_fwd_bwd_vs_oracle(occl, deg):
    from nlosgr.cuda_autograd import CUDARenderFunction
    from oracle import torch_ref as R
    dev = torch.device("cuda:0")
    m, o, d = _scene(60, 24, 21, scale_shift=1.5, opac_shift=3.0 if occl else 0.0, deg=deg)
    t = torch.linspace(0.1, 1.4, 72, device=dev)
    cam = torch.tensor([0.05, 0.0, -0.02], device=dev)
    c, dT = 1.0, 0.4 if occl else 0.02
    feats = torch.cat([m._features_dc, m._features_rest], dim=1)[:, :, 0].detach().requires_grad_(True)
    outs = CUDARenderFunction.apply(o, d, t, m._mu, m._scaling, m._rotation, m._opacity, feats, cam, deg, c, dT,
                                    1.0, occl, "netf")
    P, fr = _oracle(m, deg)
    fr.requires_grad_(True)
    filt = R.aabb_filter(o.cpu(), d.cpu(), R.bboxes_cuda(P))
    refs = R.render_rays_cuda(o.cpu(), d.cpu(), t.cpu(), P, fr, cam.cpu(), deg, c, dT, 1.0, occl, filt)
    if occl:
        assert float((refs[2] == 0).float().mean()) > 0.05   # the early exit is exercised
    rt = 2e-4 if occl else 2e-5
    for name, a, b in zip(["rho", "density", "transmittance"], outs, refs):
        _close(a, b, rt, msg=f"fwd {name}")
    g = torch.Generator().manual_seed(5)
    ups = [torch.randn(refs[0].shape, generator=g) for _ in range(3)]
    sum(((a * u.to(dev)).sum() for a, u in zip(outs, ups))).backward()
    sum(((b * u).sum() for b, u in zip(refs, ups))).backward()
    grt = 3e-4 if occl else 2e-4
    pairs = [("mu", m._mu, P._mu), ("scaling", m._scaling, P._scaling), ("rotation", m._rotation, P._rotation),
             ("opacity", m._opacity, P._opacity), ("features", feats, fr)]
    for name, leaf, rleaf in pairs:
        _close(leaf.grad, rleaf.grad, grt, atol=1e-6, msg=f"grad {name}")


def test_render_module_dropin():
    """CUDARenderModule / GaussianRendererCUDA (the reference's call path, cuda_autograd.py:213-316)
    against the same computation on the oracle."""
    from nlosgr.rendering_cuda import create_cuda_renderer
    from oracle import torch_ref as R
    dev = torch.device("cuda:0")
    m, _, _ = _scene(50, 1, 31, scale_shift=1.2, deg=0)
    cam = torch.tensor([0.1, 0.0, -0.1], device=dev)
    rend = create_cuda_renderer()
    tr_, pr_ = (0.4, 1.6), (0.9, 2.3)
    nt, npp, nr, c, dT = 8, 6, 40, 1.0, 0.03
    result, hist = rend.render_transient(m, cam, tr_, pr_, (0.2, 1.4), nt, npp, nr, c, dT, 1.0, False, "netf")
    assert result.shape == (nr, nt, npp) and hist.shape == (nr,)
    P, _ = _oracle(m, 0)
    theta = torch.linspace(*tr_, nt)
    phi = torch.linspace(*pr_, npp)
    tg, pg = torch.meshgrid(theta, phi, indexing="ij")
    tf, pf = tg.reshape(-1), pg.reshape(-1)
    d = torch.stack([torch.sin(tf) * torch.cos(pf), torch.sin(tf) * torch.sin(pf), torch.cos(tf)], 1)
    o = cam.cpu().unsqueeze(0).expand(tf.shape[0], 3).contiguous()
    t = torch.linspace(0.2, 1.4, nr)
    filt = R.aabb_filter(o, d, R.bboxes_cuda(P))
    rho, _, _ = R.render_rays_cuda(o, d, t, P, P._features_dc[:, :, 0], cam.cpu(), 0, c, dT, 1.0, False, filt)
    ref = rho.T.reshape(nr, nt, npp) / (t.view(-1, 1, 1) ** 2 + 1e-8) * torch.sin(tg.unsqueeze(0))
    ref_h = ref.sum(dim=(1, 2)) * ((tr_[1] - tr_[0]) / nt) * ((pr_[1] - pr_[0]) / npp)
    _close(result, ref, 2e-5, msg="result")
    _close(hist, ref_h, 2e-5, msg="hist")
    hist.sum().backward()
    ref_h.sum().backward()
    for name, leaf, rleaf in [("mu", m._mu, P._mu), ("scaling", m._scaling, P._scaling),
                              ("rotation", m._rotation, P._rotation), ("opacity", m._opacity, P._opacity),
                              ("features_dc", m._features_dc, P._features_dc)]:
        _close(leaf.grad, rleaf.grad, 2e-4, atol=1e-6, msg=f"grad {name}")
