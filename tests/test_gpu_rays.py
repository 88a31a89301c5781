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


@pytest.mark.parametrize("preset", ["cuda", "torch"])
def test_bboxes_match_oracle(preset):
    """nlosgr_bboxes vs the restated compute_gaussian_bboxes_kernel (bbox_compute.cuh:23-120, cuda)
    and GaussianModel.get_bboxes (gaussian_model.py:140-178, torch), incl. a zero quaternion (cuda:
    identity) and sigma 2.5 / modifier 0.8.  fp32 ops in a different association: 4 ulp of the box."""
    from nlosgr.render import bboxes
    from oracle import torch_ref as R
    m, _, _ = _scene(300, 1, 5, scale_shift=0.3)
    with torch.no_grad():
        if preset == "cuda":
            m._rotation[7].zero_()
    P, _ = _oracle(m, 0)
    for mod, sig in ((1.0, 3.0), (0.8, 2.5)):
        got = bboxes(m._mu, m._scaling, m._rotation, mod, sig, preset=preset).reshape(-1, 6).cpu()
        ref = (R.bboxes_cuda if preset == "cuda" else R.bboxes_torch)(P, mod, sig)
        _close(got, ref, 5e-7, 0.0, f"{preset} boxes mod {mod} sigma {sig}")
        ext = (got[:, 3:] - got[:, :3]) / 2
        assert torch.all(ext > 0)


@pytest.mark.parametrize("ng,shift", [(200, 0.5), (400, 3.0), (2000, 1.0)])
def test_filter_matches_oracle(ng, shift):
    """Index work is bit-exact: the HIP filter and the oracle's restatement of
    filter_gaussians_kernel (ray_aabb.cu:10-61, slab test cuda_utils.cuh:97-121) get the SAME boxes
    and must return identical int32 rows (count, first 256 hits by index, -1 padding)."""
    from nlosgr.rays import filter_gaussians_per_ray
    from nlosgr.render import bboxes
    from oracle import torch_ref as R
    m, o, d = _scene(ng, 40, 11, scale_shift=shift)
    bb = bboxes(m._mu, m._scaling, m._rotation, 1.0, 3.0, preset="cuda").reshape(-1, 6)
    got = filter_gaussians_per_ray(o, d, m._mu, bb).cpu()
    ref = R.aabb_filter(o.cpu(), d.cpu(), bb.cpu())
    assert got.dtype == ref.dtype == torch.int32
    assert torch.equal(got, ref)
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


@pytest.mark.parametrize("deg", [1, 3])
def test_render_module_reference_sh_reads(deg):
    """CUDARenderModule(reference_sh_reads=True) at active_sh_degree > 0 reproduces what the reference
    kernel computes with dc-only features (spherical_harmonics.cuh:64-80 with sh_dim = 1: Gaussian g
    reads the dc values of g .. g + K - 1; zero past the end): forward and the gradients (to dc
    through the gather) vs the oracle fed the same rows; the default module evaluates degree 0."""
    from nlosgr.cuda_autograd import CUDARenderModule, reference_sh_rows
    from oracle import torch_ref as R
    dev = torch.device("cuda:0")
    m, _, _ = _scene(40, 1, 33, scale_shift=1.2, deg=3)
    m.active_sh_degree = deg
    cam = torch.tensor([0.1, 0.0, -0.1], device=dev)
    tr_, pr_ = (0.4, 1.6), (0.9, 2.3)
    nt, npp, nr, c, dT = 8, 6, 40, 1.0, 0.03
    mod = CUDARenderModule(reference_sh_reads=True)
    result, hist = mod(m, cam, tr_, pr_, (0.2, 1.4), nt, npp, nr, c, dT, 1.0, False, "netf")
    P, _ = _oracle(m, deg)
    rows = reference_sh_rows(P._features_dc[:, :, 0], deg)
    K = (deg + 1) ** 2
    assert rows.shape == (40, K) and float(rows[-1, 1:].detach().abs().max()) == 0.0   # past the end: zero
    assert torch.equal(rows[0, 1:].detach(), P._features_dc[1:K, 0, 0].detach())     # neighbours' dc
    theta = torch.linspace(*tr_, nt)
    phi = torch.linspace(*pr_, npp)
    tg, pg = torch.meshgrid(theta, phi, indexing="ij")
    tf, pf = tg.reshape(-1), pg.reshape(-1)
    d = torch.stack([torch.sin(tf) * torch.cos(pf), torch.sin(tf) * torch.sin(pf), torch.cos(tf)], 1)
    o = cam.cpu().unsqueeze(0).expand(tf.shape[0], 3).contiguous()
    t = torch.linspace(0.2, 1.4, nr)
    filt = R.aabb_filter(o, d, R.bboxes_cuda(P))
    rho, _, _ = R.render_rays_cuda(o, d, t, P, rows, cam.cpu(), deg, c, dT, 1.0, False, filt)
    ref = rho.T.reshape(nr, nt, npp) / (t.view(-1, 1, 1) ** 2 + 1e-8) * torch.sin(tg.unsqueeze(0))
    ref_h = ref.sum(dim=(1, 2)) * ((tr_[1] - tr_[0]) / nt) * ((pr_[1] - pr_[0]) / npp)
    _close(hist, ref_h, 2e-5, msg=f"hist deg {deg}")
    hist.sum().backward()
    ref_h.sum().backward()
    _close(m._features_dc.grad, P._features_dc.grad, 2e-4, atol=1e-6, msg="grad features_dc")
    _close(m._mu.grad, P._mu.grad, 2e-4, atol=1e-6, msg="grad mu")
    # the default module: degree-0 evaluation, which differs once the neighbours' terms matter
    _, h0 = CUDARenderModule()(m, cam, tr_, pr_, (0.2, 1.4), nt, npp, nr, c, dT, 1.0, False, "netf")
    assert float((h0.detach() - hist.detach()).abs().max()) > 1e-6 * float(hist.abs().max())


@pytest.mark.parametrize("occl", [False, True])
def test_nlos_gaussian_renderer_dropin(occl):
    """NLOSGaussianRenderer (submodules/cuda_renderer/__init__.py:24-180): render() against the
    same computation on the oracle (boxes, filter, render_rays, attenuation, angular sum) and
    filter_gaussians() bit-exact against the oracle filter fed the same [Ng, 2, 3] boxes."""
    from nlosgr.cuda_renderer import create_renderer
    from nlosgr.render import bboxes
    from oracle import torch_ref as R
    dev = torch.device("cuda:0")
    m, _, _ = _scene(80, 1, 41, scale_shift=1.2, opac_shift=2.0 if occl else 0.0, deg=1)
    cam = torch.tensor([0.05, 0.0, -0.05], device=dev)
    rend = create_renderer(3.0)
    tr_, pr_ = (0.4, 1.6), (0.9, 2.3)
    nt, npp, nr, c, dT = 7, 9, 48, 1.0, (0.3 if occl else 0.03)
    result, hist = rend.render(m, cam, tr_, pr_, (0.2, 1.4), nt, npp, nr, c, dT, 1.0, occl, "netf")
    assert result.shape == (nr, nt, npp) and hist.shape == (nr,)
    assert not result.requires_grad
    P, _ = _oracle(m, 1)
    theta = torch.linspace(*tr_, nt)
    phi = torch.linspace(*pr_, npp)
    tg, pg = torch.meshgrid(theta, phi, indexing="ij")
    tf, pf = tg.reshape(-1), pg.reshape(-1)
    d = torch.stack([torch.sin(tf) * torch.cos(pf), torch.sin(tf) * torch.sin(pf), torch.cos(tf)], 1)
    o = cam.cpu().unsqueeze(0).expand(tf.shape[0], 3).contiguous()
    t = torch.linspace(0.2, 1.4, nr)
    with torch.no_grad():
        filt = R.aabb_filter(o, d, R.bboxes_cuda(P))
        # the reference passes features_dc only (__init__.py:112-115): degree 1 reads just the dc term
        rho, _, _ = R.render_rays_cuda(o, d, t, P, P._features_dc[:, :, 0], cam.cpu(), 0, c, dT, 1.0, occl, filt)
    ref = rho.T.reshape(nr, nt, npp) / (t.view(-1, 1, 1) ** 2 + 1e-8) * torch.sin(tg.unsqueeze(0))
    ref_h = ref.sum(dim=(1, 2)) * ((tr_[1] - tr_[0]) / nt) * ((pr_[1] - pr_[0]) / npp)
    tol = 2e-4 if occl else 2e-5
    _close(result, ref, tol, msg="result")
    _close(hist, ref_h, tol, msg="hist")
    bb = bboxes(m._mu, m._scaling, m._rotation, 1.0, 3.0, preset="cuda")
    got = rend.filter_gaussians(o.to(dev), d.to(dev), m._mu, bb).cpu()
    assert torch.equal(got, R.aabb_filter(o, d, bb.reshape(-1, 6).cpu()))


@pytest.mark.parametrize("occl", [False, True])
def test_rays_backward_deterministic(occl):
    """The rays backward has no atomics: slot-private rows (static ray schedule) summed in slot order,
    so two runs are bitwise identical (round 1 used global float atomics)."""
    from nlosgr.rays import gaussian_filter, rays_backward
    dev = torch.device("cuda:0")
    m, o, d = _scene(300, 700, 5, scale_shift=1.5, opac_shift=1.0, deg=2)
    t = torch.linspace(0.1, 1.4, 96, device=dev)
    cam = torch.tensor([0.0, 0.0, 0.0], device=dev)
    feats = torch.cat([m._features_dc, m._features_rest], dim=1)[:, :, 0].detach().contiguous()
    filt = gaussian_filter(o, d, m._mu, m._scaling, m._rotation)
    g = torch.Generator().manual_seed(1)
    g_rho = torch.randn(o.shape[0], t.shape[0], generator=g).to(dev)
    args = (o, d, t, m._mu, m._scaling, m._rotation, m._opacity, feats, cam, 2, 0.05, 1.0, occl, filt, g_rho, None, None)
    r1 = rays_backward(*args)
    r2 = rays_backward(*args)
    for a, b in zip(r1, r2):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)


@pytest.mark.parametrize("occl", [False, True])
def test_compute_loss_use_cuda_renderer(occl):
    """nlos_helpers.compute_loss with args.use_cuda_renderer=True (nlos_helpers.py:200-204) takes
    gaussian_transient_rendering_cuda (:235-278): path C via GaussianRendererCUDA with the angular
    ranges recovered from input_points, r_range = (I1, I2) c dT and x Y^2 on result AND histogram.
    Loss and all parameter gradients against the same composition on the oracle (render_rays_cuda
    over the aabb_filter rows, CUDARenderModule's attenuation and angular sum)."""
    from types import SimpleNamespace
    from nlosgr import nlos_helpers as NH
    from nlosgr.geometry import volume_box_point
    from oracle import torch_ref as R
    assert NH.CUDA_RENDERER is not None and NH.CUDA_AVAILABLE
    dev = torch.device("cuda:0")
    m, _, _ = _scene(70, 1, 51, scale_shift=1.0, opac_shift=4.0 if occl else 0.0, deg=0)
    ns, T = 6, 40
    c, deltaT = 1.0, 1.28 / T
    start = T // 8
    args = SimpleNamespace(num_sampling_points=ns, start=start, end=start + T, occlusion=occl, rendering_type="netf",
                           scaling_modifier=1.0, gt_times=100, use_cuda_renderer=True)
    walls = torch.tensor([[0.1, 0.0, -0.1], [-0.2, 0.0, 0.15]], device=dev)
    vpos = torch.tensor([0.0, 0.5, 0.0], device=dev)
    g = torch.Generator().manual_seed(3)
    data_kwargs = {"nlos_data": (torch.rand(start + T + 2, 1, 2, generator=g) * 1e-3).to(dev),
                   "camera_grid_positions": walls.t().contiguous(), "volume_position": vpos,
                   "volume_box_point": volume_box_point(vpos, 0.5).to(dev), "deltaT": deltaT, "c": c}
    crit = torch.nn.MSELoss(reduction="mean")
    total = 0.0
    P, _ = _oracle(m, 0)
    ref_total = 0.0
    for w in range(2):
        loss, eq = NH.compute_loss(args, m, data_kwargs, {"m": 0, "N": 2, "n": w, "criterion": crit}, dev)
        total = total + loss
        # oracle composition (rendering_cuda.py:208-263 -> cuda_autograd.py:213-316, x Y^2)
        cam = walls[w]
        ip, I1, I2, num_r, *_ = NH.spherical_sample_histogram(args, data_kwargs, cam)
        tr_ = (ip[:, 3].min().item(), ip[:, 3].max().item())
        pr_ = (ip[:, 4].min().item(), ip[:, 4].max().item())
        theta = torch.linspace(*tr_, ns)
        phi = torch.linspace(*pr_, ns)
        tg, pg = torch.meshgrid(theta, phi, indexing="ij")
        tf, pf = tg.reshape(-1), pg.reshape(-1)
        d = torch.stack([torch.sin(tf) * torch.cos(pf), torch.sin(tf) * torch.sin(pf), torch.cos(tf)], 1)
        o = cam.cpu().unsqueeze(0).expand(tf.shape[0], 3).contiguous()
        t = torch.linspace(I1 * c * deltaT, I2 * c * deltaT, num_r)
        filt = R.aabb_filter(o, d, R.bboxes_cuda(P))
        rho, _, _ = R.render_rays_cuda(o, d, t, P, P._features_dc[:, :, 0], cam.cpu(), 0, c, deltaT, 1.0, occl, filt)
        res = rho.T.reshape(num_r, ns, ns) / (t.view(-1, 1, 1) ** 2 + 1e-8) * torch.sin(tg.unsqueeze(0))
        hist = res.sum(dim=(1, 2)) * ((tr_[1] - tr_[0]) / ns) * ((pr_[1] - pr_[0]) / ns) * (0.5 ** 2)
        target = data_kwargs["nlos_data"][I1:I1 + num_r, 0, w].cpu() * 100
        ref_loss = crit(hist, target)
        np.testing.assert_allclose(loss.item(), ref_loss.item(), rtol=(4e-4 if occl else 4e-5))
        ref_total = ref_total + ref_loss
    total.backward()
    ref_total.backward()
    for name, leaf, rleaf in [("mu", m._mu, P._mu), ("scaling", m._scaling, P._scaling),
                              ("rotation", m._rotation, P._rotation), ("opacity", m._opacity, P._opacity),
                              ("features_dc", m._features_dc, P._features_dc)]:
        _close(leaf.grad, rleaf.grad, 3e-4 if occl else 2e-4, atol=1e-6, msg=f"grad {name}")
