"""CPU checks of the analytic restatements in oracle/torch_ref.py.

Path A (the reference's analytic section renderer, volume_renderer_analytic.cu) cannot run here
(no CUDA), so `render_rays_analytic` is pinned by hand-computed cases of the reference's formulas
(analytic_integration.cuh:38-172) and by the sort / truncation / early-exit rules of the kernel
loop (volume_renderer_analytic.cu:69-170).  Parity with the .cu text itself is unpinned
(SURVEY §8c).  `bin_integrated_pdf` (C4 "analytic_exact") is pinned by its defining integral:
dense quadrature of the oracle's own point pdf over each radial bin."""
import math

import torch

from conftest import ROOT  # noqa: F401


def _single(mu, S, q, o_logit, dc=0.0):
    from oracle import torch_ref as R
    t = lambda v: torch.tensor(v, dtype=torch.float32)
    n = len(mu)
    return R.Params(t(mu), t(S), t(q), t(o_logit).reshape(n, 1), t(dc).reshape(n, 1, 1), torch.zeros(n, 0, 1),
                    0, requires_grad=False)


def _filter_all(nrays, ng):
    f = torch.full((nrays, 257), -1, dtype=torch.int32)
    f[:, 0] = ng
    f[:, 1:1 + ng] = torch.arange(ng, dtype=torch.int32)
    return f


def test_section_tau_formula_hand_case():
    """Unit isotropic Gaussian at the origin, ray along +x from (-10, 0, 0): the 3-sigma section is
    t in [7, 13] and the reference's tau = sigma sqrt(2 pi) * 1 * (erf(3) - erf(-3))."""
    from oracle import torch_ref as R
    P = _single([[0.0, 0.0, 0.0]], [[0.0, 0.0, 0.0]], [[1.0, 0.0, 0.0, 0.0]], [0.0], dc=[0.5 / R.C0])
    o = torch.tensor([[-10.0, 0.0, 0.0]])
    d = torch.tensor([[1.0, 0.0, 0.0]])
    cam = torch.tensor([0.0, -1.0, 0.0])
    out = R.render_rays_analytic(o, d, 0.0, 100.0, _filter_all(1, 1), P, P.features[:, :, 0], cam, 0)
    sig = 0.5
    tau = sig * math.sqrt(2 * math.pi) * 2 * math.erf(3.0)
    rho = 0.5 + 0.5      # SH dc: C0 * (0.5 / C0) + 0.5
    assert abs(out[0].item() - (1 - math.exp(-tau)) * rho) < 1e-6
    # clipping the ray to [0, 10] keeps only t in [7, 10]: erf((-20 + 20)/2) - erf(-3)
    out = R.render_rays_analytic(o, d, 0.0, 10.0, _filter_all(1, 1), P, P.features[:, :, 0], cam, 0)
    tau = sig * math.sqrt(2 * math.pi) * (math.erf(0.0) - math.erf(-3.0))
    assert abs(out[0].item() - (1 - math.exp(-tau)) * rho) < 1e-6


def test_sections_sorted_and_composited_front_to_back():
    """Two Gaussians on the ray, listed far-first in the filter: the near one must composite first."""
    from oracle import torch_ref as R
    P = _single([[5.0, 0.0, 0.0], [1.0, 0.0, 0.0]], [[-1.0] * 3] * 2, [[1.0, 0, 0, 0]] * 2, [2.0, 2.0],
                dc=[0.3 / R.C0, -0.2 / R.C0])
    o = torch.tensor([[-2.0, 0.0, 0.0]])
    d = torch.tensor([[1.0, 0.0, 0.0]])
    cam = torch.tensor([0.0, -3.0, 0.0])
    out = R.render_rays_analytic(o, d, 0.0, 50.0, _filter_all(1, 2), P, P.features[:, :, 0], cam, 0)
    s = math.exp(-1.0)
    sig = 1 / (1 + math.exp(-2.0))
    tau = sig * math.sqrt(2 * math.pi / (1 / s ** 2)) * s ** 3 * 2 * math.erf(3 / math.sqrt(1.0) * 1.0)
    # per section (a = b^2/4c at the symmetric 3-sigma cut): exp factor 1, erf(+-3) (the formula's
    # (b + 2ct)/(2 sqrt c) at t = peak -+ 3 s equals -+3)
    rho_near, rho_far = 0.5 - 0.2, 0.5 + 0.3
    a = 1 - math.exp(-tau)
    expect = a * rho_near + (1 - a) * a * rho_far
    assert abs(out[0].item() - expect) < 1e-5, (out[0].item(), expect)


def _chain(n, S, o_logit, ox=-1.0):
    from oracle import torch_ref as R
    mu = [[0.05 * i, 0.0, 0.0] for i in range(n)]
    P = _single(mu, [[S] * 3] * n, [[1.0, 0, 0, 0]] * n, [o_logit] * n,
                dc=[(0.1 + 0.001 * i) / R.C0 for i in range(n)])
    o = torch.tensor([[ox, 0.0, 0.0]])
    d = torch.tensor([[1.0, 0.0, 0.0]])
    cam = torch.tensor([0.0, -3.0, 0.0])
    out = R.render_rays_analytic(o, d, 0.0, 50.0, _filter_all(1, n), P, P.features[:, :, 0], cam, 0)
    s = math.exp(S)
    sig = 1 / (1 + math.exp(-o_logit))
    # symmetric +-3 sigma sections: tau = sigma sqrt(2 pi / c) s^3 (erf(3) - erf(-3)), c = 1/s^2
    return out[0].item(), 1 - math.exp(-sig * math.sqrt(2 * math.pi) * s ** 4 * 2 * math.erf(3.0))


def _composite(alpha, n_max):
    T, acc = 1.0, 0.0
    for i in range(n_max):
        acc += T * alpha * (0.6 + 0.001 * i)
        T *= 1 - alpha
        if T < 1e-4:
            break
    return acc


def test_section_cap_128():
    """200 thin Gaussians on the ray (ties broken in filter order): only the first 128 sections count."""
    out, alpha = _chain(200, -2.0, 8.0)
    assert abs(out - _composite(alpha, 128)) < 1e-5 * _composite(alpha, 128)
    assert abs(out - _composite(alpha, 200)) > 1e-4 * out


def test_early_exit_below_1e4():
    """Opaque unit Gaussians: T drops below 1e-4 after the second section and compositing stops."""
    out, alpha = _chain(40, 0.0, 8.0, ox=-10.0)
    assert (1 - alpha) ** 2 < 1e-4 < (1 - alpha)
    expect = alpha * 0.6 + (1 - alpha) * alpha * 0.601
    assert abs(out - expect) < 1e-5, (out, expect)


def test_bin_integral_matches_quadrature():
    """bin_integrated_pdf == midpoint-rule quadrature (1000 sub-samples per bin) of gaussian_pdf."""
    from nlosgr.model import GaussianParams
    from oracle import torch_ref as R
    for preset in ("cuda", "torch"):
        m = GaussianParams.synthetic(6, 0, preset=preset, device="cpu", seed=4)
        with torch.no_grad():
            if preset == "cuda":
                m._scaling.add_(1.0)
        P = R.Params(m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
                     m._features_dc.detach(), m._features_rest.detach(), 0, requires_grad=False)
        p = torch.tensor([0.1, 0.0, -0.2])
        box = R.volume_box_point((0.0, 0.5, 0.0), 0.5)
        T, ns = 24, 3
        tab = R.sample_tables(p, box, ns, T // 8, T // 8 + T, 1.0, 1.28 / T)
        exact = R.bin_integrated_pdf(P, p, tab, preset)
        r = tab["r"].double()
        dr = (r[-1] - r[0]) / (r.shape[0] - 1)
        sub = (torch.arange(1000, dtype=torch.float64) + 0.5) / 1000 - 0.5          # [-1/2, 1/2)
        acc = torch.zeros_like(exact)
        th, ph = tab["theta"].double(), tab["phi"].double()
        dirs = torch.stack([torch.sin(th)[:, None] * torch.cos(ph)[None, :],
                            torch.sin(th)[:, None] * torch.sin(ph)[None, :],
                            torch.cos(th)[:, None].expand(ns, ns)], -1).reshape(-1, 3)
        from types import SimpleNamespace
        P64 = SimpleNamespace(_mu=P._mu.double(), _scaling=P._scaling.double(), _rotation=P._rotation.double())
        for u in sub:
            rr = r + u * dr
            x = (p.double()[None, None, :] + rr[:, None, None] * dirs[None, :, :]).reshape(-1, 3)
            acc += R.gaussian_pdf(x, P64, preset)
        acc /= sub.shape[0]
        err = (exact - acc).abs().max().item() / acc.abs().max().item()
        assert err < 1e-6, (preset, err)


def test_batched_analytic_matches_loop():
    """The vectorised analytic oracle (used for the C4-size path-A check on the GPU) equals the
    line-by-line restatement on random scenes with the 128-section cap, the 256-entry filter cap,
    -1 padding and early exits."""
    from oracle import torch_ref as R
    g = torch.Generator().manual_seed(4)
    for ng, shift, opac in ((40, 0.5, 0.0), (300, 1.8, 1.5), (30, 2.5, 6.0)):
        mu = torch.rand(ng, 3, generator=g) * 0.4 + torch.tensor([-0.2, 0.3, -0.2])
        S = torch.log(torch.full((ng, 3), 0.04)) + 0.3 * torch.randn(ng, 3, generator=g) + shift
        q = torch.randn(ng, 4, generator=g)
        o = torch.randn(ng, 1, generator=g) + opac
        dc = torch.rand(ng, 1, 1, generator=g) * 0.4 - 0.2
        rest = 0.05 * torch.randn(ng, 3, 1, generator=g)
        P = R.Params(mu, S, q, o, dc, rest, 1, requires_grad=False)
        feats = torch.cat([dc, rest], dim=1)[:, :, 0]
        nr = 24
        th = 0.4 + torch.rand(nr, generator=g)
        ph = 1.0 + torch.rand(nr, generator=g)
        d = torch.stack([torch.sin(th) * torch.cos(ph), torch.sin(th) * torch.sin(ph), torch.cos(th)], 1)
        cam = torch.tensor([0.02, 0.0, -0.03])
        ray_o = cam.unsqueeze(0).expand(nr, 3).contiguous()
        filt = R.aabb_filter(ray_o, d, R.bboxes_cuda(P))
        loop = R.render_rays_analytic(ray_o, d, 0.16, 1.44, filt, P, feats, cam, 1)
        vec = R.render_rays_analytic_batched(ray_o, d, 0.16, 1.44, filt, P, feats, cam, 1, chunk=7)
        assert loop.abs().max() > 0
        assert torch.allclose(vec, loop, rtol=1e-5, atol=1e-7), (ng, (vec - loop).abs().max())
