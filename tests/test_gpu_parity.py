"""GPU parity: the HIP path (through the C ABI) against the reference's golden vectors and the
CPU oracle.  Tolerances (fp32):
  forward    max|hip - ref| <= 2e-5 * max|ref| + 1e-7   (dense; summation order differs)
  gradients  max|hip - ref| <= 2e-4 * max|ref| + 1e-6   per parameter tensor
"""
import numpy as np
import pytest
import torch

from conftest import CASES, load_case

pytestmark = pytest.mark.gpu

FWD_RTOL = 2e-5
GRAD_RTOL = 2e-4


def _close(a, b, rtol, atol=1e-7, msg=""):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = np.abs(b).max() if b.size else 0.0
    err = np.abs(a - b).max() if b.size else 0.0
    assert err <= rtol * scale + atol, f"{msg}: max err {err:.3e} vs scale {scale:.3e}"


def _args(m):
    from types import SimpleNamespace
    return SimpleNamespace(num_sampling_points=m["ns"], start=m["start"], end=m["end"], occlusion=m["occlusion"],
                           rendering_type="netf", scaling_modifier=1.0, gt_times=m["gt_times"])


def _model(d, dev):
    from nlosgr import GaussianParams
    t = lambda k: torch.from_numpy(d[k]).float().to(dev)
    return GaussianParams(t("mu"), t("scaling"), t("rotation"), t("opacity"), t("features_dc"),
                          t("features_rest"), d["meta"]["deg"], d["meta"]["deg"])


@pytest.mark.parametrize("name", CASES)
def test_dropin_matches_reference_golden(name):
    """nlosgr.nlos_helpers.compute_loss (HIP) vs the reference's compute_loss on the same inputs."""
    from nlosgr import nlos_helpers as NH
    dev = torch.device("cuda:0")
    d = load_case(name)
    m = d["meta"]
    model = _model(d, dev)
    args = _args(m)
    data_kwargs = {
        "nlos_data": torch.from_numpy(d["nlos_data"]).to(dev),
        "camera_grid_positions": torch.from_numpy(d["walls"]).t().contiguous().to(dev),
        "volume_position": torch.from_numpy(d["volume_position"]).to(dev),
        "volume_box_point": torch.from_numpy(d["box"]).to(dev),
        "deltaT": m["deltaT"], "c": m["c"],
    }
    crit = torch.nn.MSELoss(reduction="mean")
    total = 0.0
    for w in range(m["nwall"]):
        cam = data_kwargs["camera_grid_positions"][:, w]
        ip, I1, I2, num_r, dth, dph, *_ = NH.spherical_sample_histogram(args, data_kwargs, cam)
        assert I1 == d["I1"][w] and I2 == d["I2"][w]
        result, hist = NH.gaussian_transient_rendering(args, model, data_kwargs, ip, cam, I1, I2, num_r, dth, dph)
        _close(hist.detach().cpu(), d["hist"][w], FWD_RTOL, msg=f"{name} hist w{w}")
        _close(result.detach().cpu(), d["result"][w], FWD_RTOL, msg=f"{name} result w{w}")
        loss, eq = NH.compute_loss(args, model, data_kwargs, {"m": 0, "N": m["nwall"], "n": w, "criterion": crit}, dev)
        np.testing.assert_allclose(loss.item(), d["loss"][w], rtol=1e-4)
        total = total + loss
    total.backward()
    for pname, leaf in zip(["mu", "scaling", "rotation", "opacity", "features_dc", "features_rest"],
                           model.parameters()):
        ref = d["grad_" + pname]
        if ref.size == 0:
            continue
        _close(leaf.grad.cpu(), ref, GRAD_RTOL, atol=1e-6, msg=f"{name} grad {pname}")


def _oracle_volume(d_params, walls, box, Y, ns, start, end, c, deltaT, preset, mode, mc, deg):
    from oracle import torch_ref as R
    P = R.Params(*d_params, deg)
    hist = R.render_volume(P, walls, box, Y, ns, start, end, c, deltaT, preset=preset, mode=mode, mc=mc)
    return P, hist


@pytest.mark.parametrize("preset", ["torch", "cuda"])
@pytest.mark.parametrize("mode", ["noocl", "netf"])
@pytest.mark.parametrize("cutoff", [0.0, 3.0, 5.7])
def test_volume_vs_oracle(preset, mode, cutoff):
    """Batched volume render (several wall points in one launch) + grads vs the oracle (same
    Mahalanobis support mask when cutoff > 0; at cutoff >= 5 the no-occlusion backward also weighs
    the last round's bins past each segment's end, < 3.7e-6 of a Gaussian's peak)."""
    _volume_vs_oracle(preset, mode, cutoff, 3)


@pytest.mark.parametrize("mode", ["noocl", "netf"])
@pytest.mark.parametrize("cutoff", [0.0, 3.0])
def test_volume_vs_oracle_sh_degree4(mode, cutoff):
    """SH degree 4 (25 coefficients; sh_utils.py:102-112, torch preset): albedo, feature gradients
    and the view-direction chain into mu vs the oracle (itself pinned to the deg-4 golden cases)."""
    _volume_vs_oracle("torch", mode, cutoff, 4)


@pytest.mark.parametrize("preset", ["torch", "cuda"])
@pytest.mark.parametrize("cutoff", [0.0, 3.0, 5.7])
def test_volume_vs_oracle_netf_small_cdt(preset, cutoff):
    """netf at c dT <= 1/64 (T = 96: c dT = 0.0133; C3: 1.25e-3): the forward's transmittance factor
    and the backward's a_j take the exp-free forms (om_exp_small, constant a_c) against the oracle."""
    _volume_vs_oracle(preset, "netf", cutoff, 3, T=96)


@pytest.mark.parametrize("preset", ["torch", "cuda"])
def test_netf_long_rays_opaque_late_gaussian(preset):
    """netf over C3's radial grid (T = 1024 bins, c dT = 1.25e-3: the exp-free transmittance and the
    one-pass backward, whose per-bin suffix term a_j (E - P_j) is formed as A + E B; at cutoff >= 5 also
    the mask-free TAIL drains) with a near-opaque Gaussian (sigmoid(o) ~ 0.98) placed late on the rays,
    where the prefix P_j comes close to the ray's total E: forward and all gradients vs the oracle."""
    for cutoff in (5.7, 3.0):
        _volume_vs_oracle(preset, "netf", cutoff, 3, T=1024, opaque_late=True)


@pytest.mark.parametrize("mode", ["noocl", "netf"])
def test_tail_drains_narrow_gaussians(mode):
    """Gaussians much narrower than a bin (sigma ~ 0.05-0.3 bin along the rays) at 5.7 sigma, where the
    TAIL drains (cutoff >= 5) run: their recurrences are seeded inside the support, so no seed
    underflows and zeroes a round; forward and gradients vs the oracle (T = 96: c dT <= 1/64, so netf
    takes its TAIL drains too)."""
    _volume_vs_oracle("cuda", mode, 5.7, 3, T=96, scale_shift=-3.5)


def _volume_vs_oracle(preset, mode, cutoff, deg, T=40, opaque_late=False, scale_shift=None):
    from nlosgr import GaussianParams, features_flat
    from nlosgr.geometry import build_geometry, relay_wall_grid, volume_box_point
    from nlosgr.render import RenderConfig, render
    dev = torch.device("cuda:0")
    ng, ns = 48, 6
    c, deltaT = 1.0, 1.28 / T
    start, end = T // 8, T // 8 + T
    model = GaussianParams.synthetic(ng, deg, preset=preset, device=dev, seed=3)
    if preset == "cuda":   # make them large enough to cross several rays/bins at this coarse grid
        with torch.no_grad():
            model._scaling.add_(1.2 if scale_shift is None else scale_shift)
    walls = relay_wall_grid(2, 3, device=dev)
    if opaque_late:   # the Gaussian farthest from the wall's centre made near-opaque
        with torch.no_grad():
            far = int((model._mu - walls.mean(0)).norm(dim=1).argmax())
            model._opacity[far] = 4.0
    box = volume_box_point((0.0, 0.5, 0.0), 0.5, dev)
    geo = build_geometry(walls, box, ns, start, end, c, deltaT, 0.5, preset, mode)
    cfg = RenderConfig(preset=preset, mode=mode, sh_degree=deg, cutoff=cutoff, c_deltaT=c * deltaT)
    hist, _ = render(model._mu, model._scaling, model._rotation, model._opacity, features_flat(model), geo, cfg)
    g = torch.Generator().manual_seed(5)
    gout = torch.randn(hist.shape, generator=g)
    (hist * gout.to(dev)).sum().backward()

    cpu = lambda t: t.detach().cpu()
    params = [cpu(model._mu), cpu(model._scaling), cpu(model._rotation), cpu(model._opacity),
              cpu(model._features_dc), cpu(model._features_rest)]
    P, ref = _oracle_volume(params, cpu(walls), cpu(box), 0.5, ns, start, end, c, deltaT, preset, mode,
                            cutoff if cutoff > 0 else None, deg)
    _close(cpu(hist), ref.detach(), FWD_RTOL, msg="hist")
    (ref * gout).sum().backward()
    for pname, leaf, rleaf in zip(["mu", "scaling", "rotation", "opacity", "dc", "rest"], model.parameters(),
                                  P.leaves()):
        _close(cpu(leaf.grad), rleaf.grad, GRAD_RTOL, atol=1e-6, msg=f"grad {pname}")


def test_cutoff_converges_to_dense():
    """Support culling error shrinks with the cutoff (cuda preset, physically sized Gaussians)."""
    from nlosgr import GaussianParams
    from nlosgr.volume import Scene, make_config, render_volume
    dev = torch.device("cuda:0")
    scene = Scene(H=8, W=8, T=256, ns=32)
    model = GaussianParams.synthetic(2000, 3, preset="cuda", device=dev, seed=1)
    geo = scene.geometry(dev, "cuda")
    with torch.no_grad():
        dense = render_volume(model, geo, make_config(model, scene, cutoff=0.0))
        errs = []
        for mc in (3.0, 4.0, 5.0, 6.0):
            h = render_volume(model, geo, make_config(model, scene, cutoff=mc))
            errs.append(((h - dense).norm() / dense.norm()).item())
    # 6 sigma sits at the fp32 summation-order floor (dense and culled sum in different orders;
    # 2.0e-6 / 2.3e-6 for two candidate-box rules that enumerate identical rays and samples)
    assert errs[0] < 5e-2 and errs[1] < 3e-3 and errs[2] < 1e-4 and errs[3] < 4e-6, errs
    # monotone down to that floor (at cutoff >= 5 the drains also add the Gaussian tails of a segment's
    # last round, so 5 sigma can reach the floor as well)
    assert all(errs[i + 1] <= errs[i] or errs[i + 1] < 4e-6 for i in range(3)), errs


@pytest.mark.parametrize("preset", ["torch", "cuda"])
def test_count_support_vs_oracle(preset):
    """The kernel's work count (pairs/rays/evaluations in support) vs the oracle's count of nonzero
    masked-pdf terms; dense mode counts every sample of every live pair exactly."""
    from nlosgr import GaussianParams, features_flat
    from nlosgr.geometry import build_geometry, relay_wall_grid, volume_box_point
    from nlosgr.render import RenderConfig, count_support
    from oracle import torch_ref as R
    dev = torch.device("cuda:0")
    ng, deg, ns, T = 40, 3, 8, 48
    c, deltaT = 1.0, 1.28 / T
    start, end = T // 8, T // 8 + T
    model = GaussianParams.synthetic(ng, deg, preset=preset, device=dev, seed=7)
    if preset == "cuda":
        with torch.no_grad():
            model._scaling.add_(1.2)
    walls = relay_wall_grid(2, 2, device=dev)
    box = volume_box_point((0.0, 0.5, 0.0), 0.5, dev)
    geo = build_geometry(walls, box, ns, start, end, c, deltaT, 0.5, preset, "noocl")
    args = (model._mu, model._scaling, model._rotation, model._opacity, features_flat(model), geo)
    cpu = lambda t: t.detach().cpu()
    P = R.Params(cpu(model._mu), cpu(model._scaling), cpu(model._rotation), cpu(model._opacity),
                 cpu(model._features_dc), cpu(model._features_rest), deg)
    live = sum(int((R.albedo(P, w, preset) > 0).sum()) for w in cpu(walls))
    cfg = RenderConfig(preset=preset, mode="noocl", sh_degree=deg, cutoff=0.0, c_deltaT=c * deltaT)
    pairs, rays, evals = count_support(*args, cfg)
    assert pairs == live and rays == live * ns * ns and evals == live * ns * ns * T
    mc = 3.0
    cfg = RenderConfig(preset=preset, mode="noocl", sh_degree=deg, cutoff=mc, c_deltaT=c * deltaT)
    _, _, evals = count_support(*args, cfg)
    ref = R.count_support(P, cpu(walls), cpu(box), ns, start, end, c, deltaT, preset, mc)
    # boundary samples (m2 within fp32 rounding of mc^2) may flip
    assert abs(evals - ref) <= max(2, 1e-3 * ref), (evals, ref)


@pytest.mark.parametrize("mode", ["noocl", "netf"])
def test_ray_cache_backward_matches_uncached(mode):
    """The forward's ray record (ray_cache) changes only the order in which the backward visits
    rays: gradients equal the uncached backward within fp32 summation-order noise, and the
    forward output is unchanged."""
    from nlosgr import GaussianParams, features_flat
    from nlosgr.volume import Scene, make_config
    from nlosgr.render import render_backward, render_forward
    dev = torch.device("cuda:0")
    scene = Scene(H=6, W=5, T=256, ns=16)
    m = GaussianParams.synthetic(3000, 3, preset="cuda", device=dev, seed=4)
    with torch.no_grad():
        m._scaling.add_(0.4)       # boxes of more than 64 cells for some pairs (uncached fallback)
    geo = scene.geometry(dev, "cuda", mode)
    cfg = make_config(m, scene, mode=mode, cutoff=3.0)
    args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
            features_flat(m).detach().contiguous(), geo)
    h0, _ = render_forward(*args, cfg)
    h1, _, ws = render_forward(*args, cfg, ray_cache=True)
    assert torch.equal(h0, h1)
    g = torch.randn(h0.shape, generator=torch.Generator().manual_seed(3)).to(dev) * 1e-3
    ref = render_backward(*args, cfg, grad_hist=g)
    got = render_backward(*args, cfg, grad_hist=g, workspace=ws, ray_cache=True)
    for name, a, b in zip(["mu", "scaling", "rotation", "opacity", "features"], got, ref):
        _close(a.cpu(), b.cpu(), 1e-5, 1e-9, f"cached grad {name}")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["noocl", "netf"])
def test_bwd_shared_layout_matches_per_wave(mode):
    """The shared-row backward layout (4 waves own 256 Gaussians and share each wall point's
    staged row; chosen automatically for long rows, FLAG_BWD_SHARED forces it) gives the per-wave
    layout's gradients within fp32 summation-order noise, with and without the ray cache, for a
    ragged Gaussian count and a workspace allocated under the other layout."""
    from nlosgr import GaussianParams, features_flat
    from nlosgr.volume import Scene, make_config
    from nlosgr.render import render_backward, render_forward
    dev = torch.device("cuda:0")
    scene = Scene(H=5, W=7, T=512, ns=16)
    m = GaussianParams.synthetic(1999, 3, preset="cuda", device=dev, seed=6)
    geo = scene.geometry(dev, "cuda", mode)
    cfg = make_config(m, scene, mode=mode, cutoff=3.0)
    args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
            features_flat(m).detach().contiguous(), geo)
    g = torch.randn((scene.H * scene.W, scene.T), generator=torch.Generator().manual_seed(8)).to(dev) * 1e-3
    from dataclasses import replace
    from nlosgr import _lib
    cfg = replace(cfg, flags=_lib.FLAG_BWD_PERWAVE)
    h0, _, ws = render_forward(*args, cfg, ray_cache=True)
    ref = render_backward(*args, cfg, grad_hist=g)
    ref_c = render_backward(*args, cfg, grad_hist=g, workspace=ws, ray_cache=True)
    cfg = replace(cfg, flags=_lib.FLAG_BWD_SHARED)
    got = render_backward(*args, cfg, grad_hist=g)
    got_c = render_backward(*args, cfg, grad_hist=g, workspace=ws, ray_cache=True)   # ws from the other layout
    h1, _, ws1 = render_forward(*args, cfg, ray_cache=True)
    got_c1 = render_backward(*args, cfg, grad_hist=g, workspace=ws1, ray_cache=True)
    assert torch.equal(h0, h1)
    for name, a, b, c, d in zip(["mu", "scaling", "rotation", "opacity", "features"], got, ref, got_c, got_c1):
        _close(a.cpu(), b.cpu(), 1e-5, 1e-9, f"shared grad {name}")
        _close(c.cpu(), b.cpu(), 1e-5, 1e-9, f"shared cached grad {name}")
        _close(d.cpu(), b.cpu(), 1e-5, 1e-9, f"shared cached (own ws) grad {name}")
    for a, b in zip(ref_c, ref):
        _close(a.cpu(), b.cpu(), 1e-5, 1e-9, "per-wave cached")


@pytest.mark.parametrize("preset", ["torch", "cuda"])
@pytest.mark.parametrize("T", [40, 200])
def test_dense_register_forward_matches_lane_serial(preset, T):
    """Dense no-occlusion histograms: the lane = bin register kernel (fwd_dense_kernel, default)
    equals the lane-serial drain (FLAG_LANE_DENSE) within fp32 summation-order noise, for ragged
    bin and Gaussian counts and several Gaussian splits per wall point."""
    from nlosgr import GaussianParams, features_flat
    from nlosgr.volume import Scene, make_config
    from nlosgr.render import render_forward
    dev = torch.device("cuda:0")
    scene = Scene(H=3, W=2, T=T, ns=7)
    m = GaussianParams.synthetic(1001, 3, preset=preset, device=dev, seed=11)
    geo = scene.geometry(dev, preset)
    cfg = make_config(m, scene, preset, cutoff=0.0)
    args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
            features_flat(m).detach().contiguous(), geo)
    from dataclasses import replace
    from nlosgr import _lib
    h_reg, _ = render_forward(*args, cfg)
    h_ser, _ = render_forward(*args, replace(cfg, flags=_lib.FLAG_LANE_DENSE))
    assert torch.isfinite(h_reg).all() and h_reg.abs().max() > 0
    _close(h_reg.cpu(), h_ser.cpu(), FWD_RTOL, msg="register vs lane-serial")
