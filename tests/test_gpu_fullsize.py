"""BASELINE configurations at full size on the GPU (C1, C2, C3, C4, one C5 band).

The CPU oracle cannot render a whole C2/C3/C5 volume, so each full-size run is checked three ways:
  * the whole volume (and, where the config trains, every gradient) is finite, and the
    no-occlusion histograms are non-negative;
  * sampled wall points against the oracle (oracle/torch_ref, golden-pinned for the torch preset)
    at full geometry: C1 with all 1,000 Gaussians; C2/C3/C5 with a Gaussian subset rendered by the
    HIP path on the full-size geometry tables;
  * the parity-grade culled run (cutoff 5.7 sigma, the bench default) against the exact dense HIP
    evaluation (cutoff 0, itself pinned to the oracle in test_gpu_parity.py) on sampled wall points,
    forward and backward (gradients seeded on those points only).
Tolerances: forward max|a-b| <= 2e-5 max|b| (+1e-7 abs) vs the oracle and 1e-5 for culled vs dense;
gradients 2e-4 of each tensor's max.
"""
import numpy as np
import pytest
import torch

from conftest import ROOT  # noqa: F401

pytestmark = pytest.mark.gpu

PARITY_CUTOFF = 5.7


def _close(a, b, rtol, atol=1e-7, msg=""):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, dtype=np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, dtype=np.float64)
    scale = np.abs(b).max() if b.size else 0.0
    err = np.abs(a - b).max() if b.size else 0.0
    assert err <= rtol * scale + atol, f"{msg}: max err {err:.3e} vs scale {scale:.3e}"


def _params(m):
    from nlosgr import features_flat
    return [m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
            features_flat(m).detach().contiguous()]


def _subset(m, idx):
    from nlosgr import GaussianParams
    return GaussianParams(*(t.detach()[idx].clone() for t in (m._mu, m._scaling, m._rotation, m._opacity,
                                                               m._features_dc, m._features_rest)),
                          m.active_sh_degree, m.max_sh_degree)


def _oracle(m, scene, walls_idx, preset, mode, mc, gout=None, chunk=50):
    """oracle hist [len(walls_idx), T] of model m at the scene's full geometry, Gaussians in chunks
    (bounded memory); with gout [len(walls_idx), T] also d(sum gout*hist)/d(six raw tensors)."""
    from oracle import torch_ref as R
    cpu = [t.detach().cpu() for t in (m._mu, m._scaling, m._rotation, m._opacity, m._features_dc,
                                       m._features_rest)]
    walls = scene.walls("cpu")[walls_idx]
    box = scene.box("cpu")
    ng = cpu[0].shape[0]
    hist = None
    grads = [torch.zeros_like(t) for t in cpu]
    for g0 in range(0, ng, chunk):
        P = R.Params(*(t[g0:g0 + chunk] for t in cpu), m.active_sh_degree, requires_grad=gout is not None)
        h = R.render_volume(P, walls, box, scene.volume_position[1], scene.ns, scene.start, scene.end, scene.c,
                            scene.deltaT, preset=preset, mode=mode, mc=mc)
        if gout is not None:
            (h * gout).sum().backward()
            for gacc, leaf in zip(grads, P.leaves()):
                gacc[g0:g0 + chunk] = leaf.grad
        hist = h.detach() if hist is None else hist + h.detach()
    return hist, grads


def _hip_grads_as_ref(d):
    """HIP (d_mu, d_s, d_q, d_o, d_f[Ng,K]) -> the reference's six tensors' shapes (dc, rest split)."""
    d_mu, d_s, d_q, d_o, d_f = d
    return [d_mu, d_s, d_q, d_o.reshape(-1, 1), d_f[:, :1].reshape(-1, 1, 1), d_f[:, 1:].reshape(d_f.shape[0], -1, 1)]


def _finite_volume(hist, nonneg=True):
    assert torch.isfinite(hist).all(), "non-finite volume"
    if nonneg:
        assert float(hist.min()) >= 0.0, f"negative histogram value {float(hist.min()):.3e}"


def _culled_vs_dense(m, scene, preset, idx, hist_culled, grads_culled=None, gseed=None):
    """hist rows idx of the full culled run vs the dense HIP evaluation of those wall points;
    with grads_culled (full-volume backward seeded with gseed on rows idx only) also the gradients."""
    from nlosgr.render import render_backward, render_forward
    from nlosgr.volume import make_config
    dev = hist_culled.device
    geo = scene.geometry(dev, preset, "noocl", walls=scene.walls(dev)[idx].contiguous())
    cfg = make_config(m, scene, preset, "noocl", cutoff=0.0)
    ref, _ = render_forward(*_params(m), geo, cfg)
    _close(hist_culled[idx], ref, 1e-5, msg="culled 5.7 sigma vs dense hist")
    if grads_culled is not None:
        dref = render_backward(*_params(m), geo, cfg, grad_hist=gseed)
        for name, a, b in zip(("mu", "scaling", "rotation", "opacity", "features"), grads_culled, dref):
            _close(a, b, 2e-4, atol=1e-9, msg=f"culled vs dense grad {name}")


def test_c1_full_size():
    """C1: 1k Gaussians -> 32x32 wall x 128 bins, 32x32 angular samples, torch preset (path T, the
    golden-pinned convention), dense.  Whole volume on the GPU; 8 spread wall points (every
    Gaussian) and their gradients against the oracle."""
    from nlosgr import GaussianParams
    from nlosgr.render import render_backward, render_forward
    from nlosgr.volume import Scene, make_config
    dev = torch.device("cuda:0")
    scene = Scene(H=32, W=32, T=128, ns=32)
    m = GaussianParams.synthetic(1000, 3, preset="torch", device=dev, seed=0)
    geo = scene.geometry(dev, "torch", "noocl")
    cfg = make_config(m, scene, "torch", "noocl", cutoff=0.0)
    hist, _ = render_forward(*_params(m), geo, cfg)
    assert hist.shape == (32 * 32, 128)
    _finite_volume(hist)
    idx = torch.tensor([0, 31, 100, 333, 528, 777, 992, 1023])
    g = torch.Generator().manual_seed(7)
    gout = torch.randn(len(idx), 128, generator=g)
    gfull = torch.zeros(32 * 32, 128)
    gfull[idx] = gout
    d = render_backward(*_params(m), geo, cfg, grad_hist=gfull.to(dev))
    for t in d:
        assert torch.isfinite(t).all()
    ref, rgrads = _oracle(m, scene, idx, "torch", "noocl", None, gout=gout)
    _close(hist[idx.to(dev)], ref, 2e-5, msg="C1 hist")
    for name, a, b in zip(("mu", "scaling", "rotation", "opacity", "dc", "rest"), _hip_grads_as_ref(d), rgrads):
        _close(a, b, 2e-4, atol=1e-9, msg=f"C1 grad {name}")


def test_c2_full_size():
    """C2: 50k Gaussians -> 64x64 wall x 512 bins, forward only, cuda preset, cutoff 5.7 sigma."""
    from nlosgr import GaussianParams
    from nlosgr.render import render_forward
    from nlosgr.volume import Scene, make_config
    dev = torch.device("cuda:0")
    scene = Scene(H=64, W=64, T=512, ns=32)
    m = GaussianParams.synthetic(50_000, 3, preset="cuda", device=dev, seed=0)
    geo = scene.geometry(dev, "cuda", "noocl")
    cfg = make_config(m, scene, "cuda", "noocl", cutoff=PARITY_CUTOFF)
    hist, _ = render_forward(*_params(m), geo, cfg)
    assert hist.shape == (64 * 64, 512)
    _finite_volume(hist)
    assert float(hist.sum()) > 0
    idx = torch.tensor([0, 1000, 2080, 4095])
    _culled_vs_dense(m, scene, "cuda", idx.to(dev), hist)
    # a Gaussian subset on the full geometry against the oracle (same support rule)
    sub = _subset(m, torch.arange(0, 50_000, 250, device=dev))
    hs, _ = render_forward(*_params(sub), geo, make_config(sub, scene, "cuda", "noocl", cutoff=PARITY_CUTOFF))
    ref, _ = _oracle(sub, scene, idx, "cuda", "noocl", PARITY_CUTOFF)
    _close(hs[idx.to(dev)], ref, 2e-5, msg="C2 subset hist")


def test_c3_full_size_train_step_parity():
    """C3 (the headline): 100k Gaussians -> 128x128 wall x 1024 bins, cuda preset, cutoff 5.7 sigma,
    the forward and backward kernels TrainStep runs (ray cache per use_ray_cache), called directly in
    the given Gaussian order (TrainStep's own slab orders: test_c3_trainstep_full_ng_accuracy).  Whole
    volume finite; 2 wall points vs the dense HIP evaluation (hist and gradients seeded there); a
    Gaussian subset vs the oracle."""
    from nlosgr import GaussianParams
    from nlosgr.render import render_backward, render_forward, use_ray_cache
    from nlosgr.volume import Scene, make_config
    dev = torch.device("cuda:0")
    scene = Scene(H=128, W=128, T=1024, ns=32)
    m = GaussianParams.synthetic(100_000, 3, preset="cuda", device=dev, seed=0)
    geo = scene.geometry(dev, "cuda", "noocl")
    cfg = make_config(m, scene, "cuda", "noocl", cutoff=PARITY_CUTOFF)
    cache = use_ray_cache(cfg, geo, 100_000)          # as TrainStep decides it (off at 5.7 sigma)
    out = render_forward(*_params(m), geo, cfg, ray_cache=cache)
    hist, ws = out[0], (out[2] if cache else None)
    _finite_volume(hist)
    idx = torch.tensor([128 * 40 + 30, 128 * 100 + 90], device=dev)
    g = torch.Generator().manual_seed(3)
    gseed = torch.randn(len(idx), 1024, generator=g).to(dev)
    gfull = torch.zeros(128 * 128, 1024, device=dev)
    gfull[idx] = gseed
    d = render_backward(*_params(m), geo, cfg, grad_hist=gfull, workspace=ws, ray_cache=cache)
    del ws
    for t in d:
        assert torch.isfinite(t).all()
    _culled_vs_dense(m, scene, "cuda", idx, hist, d, gseed)
    # a 100-Gaussian subset on the full geometry vs the oracle: histogram of the 2 wall points and the
    # gradients of all six raw tensors seeded there (the culled 5.7 sigma kernels, as in the step)
    sub = _subset(m, torch.arange(0, 100_000, 1000, device=dev))
    scfg = make_config(sub, scene, "cuda", "noocl", cutoff=PARITY_CUTOFF)
    hs, _ = render_forward(*_params(sub), geo, scfg)
    ds = render_backward(*_params(sub), geo, scfg, grad_hist=gfull)
    ref, rgrads = _oracle(sub, scene, idx.cpu(), "cuda", "noocl", PARITY_CUTOFF, gout=gseed.cpu())
    _close(hs[idx], ref, 2e-5, msg="C3 subset hist")
    for name, a, b in zip(("mu", "scaling", "rotation", "opacity", "dc", "rest"), _hip_grads_as_ref(ds), rgrads):
        assert float(b.abs().max()) > 0 or name == "rest", name
        _close(a, b, 2e-4, atol=1e-9, msg=f"C3 subset grad {name}")


def test_c3_trainstep_full_ng_accuracy():
    """The headline's accuracy at full Ng through the exact path bench.py times: one C3 TrainStep
    (default slab-ordered forward and backward, 5.7 sigma) with keep_grads.
      * forward rows of 2 wall points vs the float64 sum of 400 HIP sub-histograms of 250 Gaussians each
        (float claim drain, FLAG_FLOAT_DRAIN: a few hundred terms per bin per sub-histogram), same geometry
        and cutoff: max error <= 2e-5 of the rows' max (gaussian_model.py:346-364, nlos_helpers.py:228-229
        sum over all Gaussians);
      * all six gradients vs the unordered render_backward seeded with the step's own dL/dhist, on the
        step's input parameters: fp32 summation order only, <= 2e-5 of each tensor's max (measured
        0.8e-7 - 1.6e-7; rotation 2.7e-6 since round 6's shape accumulators keep the large symmetric part of
        dL/dA out of the rotation sums, round 5: 3.6e-5)."""
    from nlosgr import GaussianParams
    from nlosgr.render import render_backward, render_forward
    from nlosgr.train import TrainStep
    from nlosgr.volume import Scene, make_config
    dev = torch.device("cuda:0")
    ng, T = 100_000, 1024
    scene = Scene(H=128, W=128, T=T, ns=32)
    m = GaussianParams.synthetic(ng, 3, preset="cuda", device=dev, seed=0)
    geo = scene.geometry(dev, "cuda", "noocl")
    cfg = make_config(m, scene, "cuda", "noocl", cutoff=PARITY_CUTOFF)
    gt = torch.Generator().manual_seed(1)
    target = (torch.rand(128 * 128, T, generator=gt) * 1e-3).to(dev)
    before = [t.detach().clone() for t in (m._mu, m._scaling, m._rotation, m._opacity, m._features_dc,
                                           m._features_rest)]
    step = TrainStep(m, geo, cfg, target, gt_times=100.0, keep_grads=True)
    assert step.fwd_order == "slab" and step.bwd_order == "slab"
    step()
    torch.cuda.synchronize()
    hist, gh, grads = step.hist, step.grad_hist, step.grads
    with torch.no_grad():      # back to the step's inputs (Adam moved them)
        for t, b in zip((m._mu, m._scaling, m._rotation, m._opacity, m._features_dc, m._features_rest), before):
            t.copy_(b)
    idx = torch.tensor([128 * 40 + 30, 128 * 100 + 90], device=dev)
    gsel = scene.geometry(dev, "cuda", "noocl", walls=geo.wall[idx].contiguous())
    from dataclasses import replace
    from nlosgr import _lib
    ref = torch.zeros(len(idx), T, dtype=torch.float64, device=dev)
    for g0 in range(0, ng, 250):
        sub = _subset(m, torch.arange(g0, min(ng, g0 + 250), device=dev))
        h, _ = render_forward(*_params(sub), gsel, replace(make_config(sub, scene, "cuda", "noocl", cutoff=PARITY_CUTOFF),
                                                           flags=_lib.FLAG_FLOAT_DRAIN))
        ref += h.double()
    a = hist[idx].double()
    err = float((a - ref).abs().max() / ref.abs().max())
    rel2 = float((a - ref).norm() / ref.norm())
    print(f"C3 TrainStep forward vs float64 sub-histogram sum: max err {err:.3e} of max, rel-L2 {rel2:.3e}")
    assert err <= 2e-5, err
    d_mu, d_s, d_q, d_o, d_f = render_backward(*_params(m), geo, cfg, grad_hist=gh)
    ref_g = [d_mu, d_f[:, :1], d_f[:, 1:], d_o, d_s, d_q]
    for name, a, b in zip(("mu", "f_dc", "f_rest", "opacity", "scaling", "rotation"), grads, ref_g):
        a, b = a.reshape(b.shape).double(), b.double()
        e = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
        print(f"C3 TrainStep ordered backward vs unordered: {name} max err {e:.3e} of max")
        assert e <= 2e-5, (name, e)


def test_c4_full_size_binint_vs_numerical():
    """C4: the bin-integrated (analytic) forward vs the numerical one on the C3 inputs, whole volume:
    the two integrate the same pdf, one per bin-average and one per bin-centre sample, so they
    agree to the curvature term (rel-L2 5e-5 measured at 3 sigma in round 1)."""
    from nlosgr import GaussianParams
    from nlosgr.render import render_forward
    from nlosgr.volume import Scene, make_config
    dev = torch.device("cuda:0")
    scene = Scene(H=128, W=128, T=1024, ns=32)
    m = GaussianParams.synthetic(100_000, 3, preset="cuda", device=dev, seed=0)
    h_num, _ = render_forward(*_params(m), scene.geometry(dev, "cuda", "noocl"),
                              make_config(m, scene, "cuda", "noocl", cutoff=PARITY_CUTOFF))
    h_int, _ = render_forward(*_params(m), scene.geometry(dev, "cuda", "binint"),
                              make_config(m, scene, "cuda", "binint", cutoff=PARITY_CUTOFF))
    _finite_volume(h_int)
    rel = float((h_int - h_num).norm() / h_num.norm())
    assert rel < 1e-3, f"binint vs numerical rel-L2 {rel:.3e}"


def test_c5_rows_shard_train_step():
    """C5 (500k Gaussians -> 256x256 wall x 2048 bins) is the 8-GPU config: one rank's shard exactly as
    bench.py --gpus 8 runs it (wall_rows(256, 256, 3, 8): whole rows 3, 11, ..., 8192 wall points),
    cutoff 5.7 sigma, through the full TrainStep (forward + MSE over the whole volume's normaliser +
    backward of all six raw tensors + Adam).  Checks: the shard's forward volume, the step's loss, all
    gradients and all updated parameters are finite; 2 sampled wall points of the shard vs the dense
    HIP evaluation, histogram and gradients seeded there (same culled kernels as the step); a Gaussian
    subset vs the oracle on one wall point of the shard."""
    from nlosgr import GaussianParams
    from nlosgr.distributed import wall_rows
    from nlosgr.render import render_backward, render_forward
    from nlosgr.train import TrainStep
    from nlosgr.volume import Scene, make_config
    dev = torch.device("cuda:0")
    H = W = 256
    T = 2048
    scene = Scene(H=H, W=W, T=T, ns=32)
    m = GaussianParams.synthetic(500_000, 3, preset="cuda", device=dev, seed=0)
    rows = wall_rows(H, W, 3, 8, device=dev)
    assert rows.numel() == 8192
    geo = scene.geometry(dev, "cuda", "noocl").rows(rows)
    cfg = make_config(m, scene, "cuda", "noocl", cutoff=PARITY_CUTOFF)
    hist, _ = render_forward(*_params(m), geo, cfg)
    assert hist.shape == (8192, T)
    _finite_volume(hist)
    idx = torch.tensor([700, 6000], device=dev)
    wsel = geo.wall[idx].contiguous()
    # culled (full shard) vs dense HIP on the sampled wall points: histogram, then gradients seeded there
    gd = scene.geometry(dev, "cuda", "noocl", walls=wsel)
    dcfg = make_config(m, scene, "cuda", "noocl", cutoff=0.0)
    ref, _ = render_forward(*_params(m), gd, dcfg)
    _close(hist[idx], ref, 1e-5, msg="C5 shard culled vs dense hist")
    g = torch.Generator().manual_seed(5)
    gseed = torch.randn(len(idx), T, generator=g).to(dev)
    gfull = torch.zeros(8192, T, device=dev)
    gfull[idx] = gseed
    d = render_backward(*_params(m), geo, cfg, grad_hist=gfull)
    dref = render_backward(*_params(m), gd, dcfg, grad_hist=gseed)
    for name, a, b in zip(("mu", "scaling", "rotation", "opacity", "features"), d, dref):
        assert torch.isfinite(a).all()
        _close(a, b, 2e-4, atol=1e-9, msg=f"C5 shard culled vs dense grad {name}")
    del d, dref, gfull
    # a Gaussian subset on the shard's geometry against the oracle (same support rule)
    sub = _subset(m, torch.arange(0, 500_000, 5000, device=dev))
    g1 = scene.geometry(dev, "cuda", "noocl", walls=wsel[:1].contiguous())
    hs, _ = render_forward(*_params(sub), g1, make_config(sub, scene, "cuda", "noocl", cutoff=PARITY_CUTOFF))
    ref, _ = _oracle(sub, scene, rows[idx[:1]].cpu(), "cuda", "noocl", PARITY_CUTOFF)
    _close(hs, ref, 2e-5, msg="C5 subset hist")
    # the step itself: TrainStep on the shard (normaliser of the whole 256x256 volume)
    gt = torch.Generator().manual_seed(1)
    target = (torch.rand(8192, T, generator=gt) * 1e-3).to(dev)
    step = TrainStep(m, geo, cfg, target, gt_times=100.0, nwall_total=H * W, keep_grads=True)
    before = [p.detach().clone() for p in m.parameters()]
    loss2 = step()
    torch.cuda.synchronize()
    assert torch.isfinite(loss2).all() and float(loss2[0]) > 0
    # the step's MSE (single process: this shard's mean; its gradient carries n_shard / n_volume)
    se = ((hist.double() - target.double() * 100.0) ** 2).mean()
    assert abs(float(loss2[0]) - float(se)) <= 1e-4 * float(se)
    for gr in step.grads:
        assert torch.isfinite(gr).all()
    assert float(step.grads[0].abs().max()) > 0
    for b, p in zip(before, m.parameters()):
        assert torch.isfinite(p).all()
    assert not torch.equal(before[0], m._mu.detach())


def test_c3_occl_full_size():
    """C3 with path C's shared-transmittance compositing (volume_renderer.cu:80-137) over the whole
    128x128 x 1024 volume (ray-tile engine, row cache off: O(tile) workspace):
      * path C's own selection (AABB: first 256 3-sigma boxes by index per ray, whole-ray pdf;
        ray_aabb.cu:10-61): forward + backward of the whole volume finite; a Gaussian subset on the
        full geometry vs oracle.render_rays_cuda with aabb_filter at 2 wall points (2e-4);
      * the parity-grade support cutoff (5.7 sigma): whole forward volume finite and non-negative;
        2 wall points vs the dense HIP evaluation (cutoff 0) of the same points (2e-5)."""
    from nlosgr import GaussianParams, features_flat
    from nlosgr.render import bboxes, render_backward, render_forward
    from nlosgr.volume import Scene, make_config
    from oracle import torch_ref as R
    dev = torch.device("cuda:0")
    scene = Scene(H=128, W=128, T=1024, ns=32)
    m = GaussianParams.synthetic(100_000, 3, preset="cuda", device=dev, seed=0)
    geo = scene.geometry(dev, "cuda", "occl")
    idx = torch.tensor([128 * 40 + 30, 128 * 100 + 90], device=dev)
    # AABB selection: full volume forward + backward
    cfg_a = make_config(m, scene, "cuda", "occl", cutoff=PARITY_CUTOFF, selection="aabb")
    hist, _ = render_forward(*_params(m), geo, cfg_a)
    assert hist.shape == (128 * 128, 1024)
    _finite_volume(hist)
    assert float(hist.sum()) > 0
    g = torch.Generator().manual_seed(3)
    d = render_backward(*_params(m), geo, cfg_a, grad_hist=(torch.randn(128 * 128, 1024, generator=g) * 1e-3).to(dev))
    for t in d:
        assert torch.isfinite(t).all()
    assert float(d[0].abs().max()) > 0
    # a Gaussian subset vs the oracle's _C.render_rays restatement (same boxes, same 256-cap filter)
    sub = _subset(m, torch.arange(0, 100_000, 1000, device=dev))
    gsel = scene.geometry(dev, "cuda", "occl", walls=geo.wall[idx].contiguous())
    hs, _ = render_forward(*_params(sub), gsel, make_config(sub, scene, "cuda", "occl", cutoff=PARITY_CUTOFF,
                                                             selection="aabb"))
    P = R.Params(*(t.detach().cpu() for t in (sub._mu, sub._scaling, sub._rotation, sub._opacity,
                                              sub._features_dc, sub._features_rest)), 3, requires_grad=False)
    bb = bboxes(sub._mu, sub._scaling, sub._rotation, 1.0, 3.0, preset="cuda").reshape(-1, 6).cpu()
    feats = P.features[:, :, 0]
    gs = torch.randn(len(idx), 1024, generator=torch.Generator().manual_seed(11))
    refs = []
    for w, p in enumerate(idx.tolist()):
        pw = scene.walls("cpu")[p]
        tab = R.sample_tables(pw, scene.box("cpu"), scene.ns, scene.start, scene.end, scene.c, scene.deltaT)
        tg, pg = torch.meshgrid(tab["theta"], tab["phi"], indexing="ij")
        tf, pf = tg.reshape(-1), pg.reshape(-1)
        dr = torch.stack([torch.sin(tf) * torch.cos(pf), torch.sin(tf) * torch.sin(pf), torch.cos(tf)], 1)
        o = pw.unsqueeze(0).expand(dr.shape[0], 3).contiguous()
        t = torch.linspace(tab["I1"] * scene.c * scene.deltaT, tab["I2"] * scene.c * scene.deltaT, tab["nr"])
        filt = R.aabb_filter(o, dr, bb)
        rho, _, _ = R.render_rays_cuda(o, dr, t, P, feats, pw, 3, scene.c, scene.deltaT, 1.0, True, filt)
        res = rho.T / (t.view(-1, 1) ** 2 + 1e-8) * torch.sin(tf).view(1, -1)
        ref = res.sum(1) * tab["dtheta"] * tab["dphi"] * scene.volume_position[1] ** 2
        assert float(ref.abs().max()) > 0
        _close(hs[w], ref, 2e-4, msg=f"C3 occl aabb subset wall point {p}")
        refs.append(ref)
    del d
    # ... and the subset's gradients seeded on those wall points vs torch autograd of the restatement
    # (path C's own backward returns zeros: cuda_autograd.py:147-156)
    P2 = R.Params(*(t.detach().cpu() for t in (sub._mu, sub._scaling, sub._rotation, sub._opacity,
                                               sub._features_dc, sub._features_rest)), 3, requires_grad=True)
    feats2 = P2.features[:, :, 0]
    loss = 0.0
    for w, p in enumerate(idx.tolist()):
        pw = scene.walls("cpu")[p]
        tab = R.sample_tables(pw, scene.box("cpu"), scene.ns, scene.start, scene.end, scene.c, scene.deltaT)
        tg, pg = torch.meshgrid(tab["theta"], tab["phi"], indexing="ij")
        tf, pf = tg.reshape(-1), pg.reshape(-1)
        dr = torch.stack([torch.sin(tf) * torch.cos(pf), torch.sin(tf) * torch.sin(pf), torch.cos(tf)], 1)
        o = pw.unsqueeze(0).expand(dr.shape[0], 3).contiguous()
        t = torch.linspace(tab["I1"] * scene.c * scene.deltaT, tab["I2"] * scene.c * scene.deltaT, tab["nr"])
        rho, _, _ = R.render_rays_cuda(o, dr, t, P2, feats2, pw, 3, scene.c, scene.deltaT, 1.0, True,
                                       R.aabb_filter(o, dr, bb))
        res = rho.T / (t.view(-1, 1) ** 2 + 1e-8) * torch.sin(tf).view(1, -1)
        loss = loss + ((res.sum(1) * tab["dtheta"] * tab["dphi"] * scene.volume_position[1] ** 2) * gs[w]).sum()
    loss.backward()
    dsub = render_backward(*_params(sub), gsel, make_config(sub, scene, "cuda", "occl", cutoff=PARITY_CUTOFF,
                                                            selection="aabb"), grad_hist=gs.to(dev))
    for name, a, b in zip(("mu", "scaling", "rotation", "opacity", "dc", "rest"), _hip_grads_as_ref(dsub),
                          P2.leaves()):
        _close(a, b.grad, 3e-4, atol=1e-9, msg=f"C3 occl aabb subset grad {name}")
    # 5.7 sigma support: whole forward volume, 2 wall points vs the dense evaluation
    cfg_s = make_config(m, scene, "cuda", "occl", cutoff=PARITY_CUTOFF)
    hist, _ = render_forward(*_params(m), geo, cfg_s)
    _finite_volume(hist)
    dcfg = make_config(m, scene, "cuda", "occl", cutoff=0.0)
    ref, _ = render_forward(*_params(m), gsel, dcfg)
    _close(hist[idx], ref, 2e-5, msg="C3 occl 5.7 sigma vs dense")
    # the 5.7 sigma occlusion backward seeded on those 2 wall points vs the dense backward there
    # (every Gaussian of the 100k in the shared-transmittance scan)
    d57 = render_backward(*_params(m), gsel, cfg_s, grad_hist=gs.to(dev) * 1e-3)
    dd = render_backward(*_params(m), gsel, dcfg, grad_hist=gs.to(dev) * 1e-3)
    for name, a, b in zip(("mu", "scaling", "rotation", "opacity", "features"), d57, dd):
        assert torch.isfinite(a).all() and float(b.abs().max()) > 0
        _close(a, b, 3e-4, atol=1e-12, msg=f"C3 occl 5.7 sigma vs dense grad {name}")
