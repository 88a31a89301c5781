"""GPU parity of the ray-tile engine (csrc/nlosgr_tiles.hip) through the C ABI:
  * NLOSGR_MODE_OCCL — path C's shared-transmittance compositing (volume_renderer.cu:80-137) over
    the batched wall-point geometry, and
  * NLOSGR_SELECT_AABB — path C's per-ray selection (ray_aabb.cu:10-61: first 256 Gaussians by index
    whose 3-sigma box the ray hits), with and without occlusion,
against the oracle's restatement of _C.render_rays (oracle.render_rays_cuda, with aabb_filter for
the AABB selection) folded into histograms exactly as CUDARenderModule does
(cuda_autograd.py:301-314: / (t^2 + 1e-8) x sin(theta), sum x dtheta dphi; x Y^2 as
nlos_helpers.py:275-276).  The reference's backward returns zeros, so gradients are pinned to torch
autograd of that oracle composition.  Tolerances (fp32):
  forward    max|hip - ref| <= 2e-5 max|ref| (no occlusion), 2e-4 with occlusion (alpha = 1 - exp(-x)
             loses ~6e-8 absolute per term to cancellation in both implementations)
  gradients  max|hip - ref| <= 3e-4 max|ref| per parameter tensor
"""
import numpy as np
import pytest
import torch

from conftest import ROOT  # noqa: F401

pytestmark = pytest.mark.gpu

C, NS, T = 1.0, 6, 40
DELTAT = 1.28 / T
START = T // 8


def _close(a, b, rtol, atol=1e-9, msg=""):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, dtype=np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, dtype=np.float64)
    scale = np.abs(b).max() if b.size else 0.0
    err = np.abs(a - b).max() if b.size else 0.0
    assert err <= rtol * scale + atol, f"{msg}: max err {err:.3e} vs scale {scale:.3e}"


def _model(ng, deg, seed, scale_shift, opac_shift):
    from nlosgr import GaussianParams
    m = GaussianParams.synthetic(ng, deg, preset="cuda", device=torch.device("cuda:0"), seed=seed)
    with torch.no_grad():
        m._scaling.add_(scale_shift)
        m._opacity.add_(opac_shift)
    return m


def _hip(m, mode, selection, cutoff, walls, box, gout=None, want_rays=False, dt=DELTAT):
    from nlosgr import features_flat
    from nlosgr.geometry import build_geometry
    from nlosgr.render import RenderConfig, render
    geo = build_geometry(walls, box, NS, START, START + T, C, dt, 0.5, "cuda", mode)
    cfg = RenderConfig(preset="cuda", mode=mode, sh_degree=m.active_sh_degree, cutoff=cutoff, c_deltaT=C * dt,
                       ray_scale=C * dt if mode == "noocl" else 1.0, selection=selection)
    hist, rays = render(m._mu, m._scaling, m._rotation, m._opacity, features_flat(m), geo, cfg,
                        want_hist=True, want_rays=want_rays)
    if gout is not None:
        (hist * gout.to(hist.device)).sum().backward()
    return hist, rays


def _oracle(m, occl, walls, box, mc=None, bb=None, gout=None, dt=DELTAT):
    from oracle import torch_ref as R
    cpu = lambda t: t.detach().cpu()
    P = R.Params(cpu(m._mu), cpu(m._scaling), cpu(m._rotation), cpu(m._opacity), cpu(m._features_dc),
                 cpu(m._features_rest), m.active_sh_degree)
    feats = P.features[:, :, 0]
    hs, rays = [], []
    for w in range(walls.shape[0]):
        p = cpu(walls[w])
        tab = R.sample_tables(p, cpu(box), NS, START, START + T, C, dt)
        tg, pg = torch.meshgrid(tab["theta"], tab["phi"], indexing="ij")
        tf, pf = tg.reshape(-1), pg.reshape(-1)
        d = torch.stack([torch.sin(tf) * torch.cos(pf), torch.sin(tf) * torch.sin(pf), torch.cos(tf)], 1)
        o = p.unsqueeze(0).expand(d.shape[0], 3).contiguous()
        t = torch.linspace(tab["I1"] * C * dt, tab["I2"] * C * dt, tab["nr"])
        filt = R.aabb_filter(o, d, bb) if bb is not None else None
        rho, _, _ = R.render_rays_cuda(o, d, t, P, feats, p, m.active_sh_degree, C, dt, 1.0, occl, filt, mc)
        rays.append(rho)
        res = rho.T / (t.view(-1, 1) ** 2 + 1e-8) * torch.sin(tf).view(1, -1)
        hs.append(res.sum(1) * tab["dtheta"] * tab["dphi"] * 0.25)
    hist = torch.stack(hs)
    if gout is not None:
        (hist * gout).sum().backward()
    return P, hist.detach(), torch.stack(rays).detach()


def _grads_close(m, P, rtol, msg):
    for name, leaf, rleaf in zip(["mu", "scaling", "rotation", "opacity", "dc", "rest"], m.parameters(), P.leaves()):
        _close(leaf.grad, rleaf.grad, rtol, atol=1e-9, msg=f"{msg} grad {name}")


def _scene():
    from nlosgr.geometry import relay_wall_grid, volume_box_point
    dev = torch.device("cuda:0")
    return relay_wall_grid(2, 2, device=dev), volume_box_point((0.0, 0.5, 0.0), 0.5, dev)


@pytest.mark.parametrize("cutoff", [0.0, 5.7, 3.0])
@pytest.mark.parametrize("deg", [0, 3])
def test_occl_volume_vs_oracle(cutoff, deg):
    """Shared-T compositing over every Gaussian (support selection, cutoff 0 = dense)."""
    walls, box = _scene()
    m = _model(40, deg, 7, 1.2, 1.5)
    g = torch.Generator().manual_seed(2)
    gout = torch.randn(walls.shape[0], T, generator=g)
    hist, rays = _hip(m, "occl", "support", cutoff, walls, box, gout, want_rays=True)
    P, ref, ref_rays = _oracle(m, True, walls, box, mc=cutoff if cutoff > 0 else None, gout=gout)
    _close(hist, ref, 2e-4, msg=f"occl hist cutoff {cutoff}")
    _close(rays.reshape(ref_rays.shape), ref_rays, 2e-4, msg="occl rays")
    _grads_close(m, P, 3e-4, f"occl cutoff {cutoff}")


def test_occl_dense_cull_round_overflows_one_block():
    """2500 Gaussians at cutoff 0: every Gaussian of a cull round (2 blocks of threads) survives, so the
    queue left after a staged window is longer than one thread per entry and moves in several passes."""
    walls, box = _scene()
    m = _model(2500, 0, 11, 0.6, -1.0)
    g = torch.Generator().manual_seed(5)
    gout = torch.randn(walls.shape[0], T, generator=g)
    hist, _ = _hip(m, "occl", "support", 0.0, walls, box, gout)
    P, ref, _ = _oracle(m, True, walls, box, gout=gout)
    _close(hist, ref, 2e-4, msg="occl dense 2500")
    _grads_close(m, P, 3e-4, "occl dense 2500")


def test_occl_early_termination():
    """Dense, opaque Gaussians: T drops below 1e-4 inside the volume, so the reference's early exit
    (volume_renderer.cu:127-137) zeroes the tails; forward and gradients still match."""
    walls, box = _scene()
    m = _model(60, 1, 9, 2.0, 6.0)
    g = torch.Generator().manual_seed(4)
    gout = torch.randn(walls.shape[0], T, generator=g)
    # a larger c dT makes the Gaussians opaque within a few bins
    hist, rays = _hip(m, "occl", "support", 0.0, walls, box, gout, want_rays=True, dt=0.2)
    P, ref, ref_rays = _oracle(m, True, walls, box, gout=gout, dt=0.2)
    assert (ref_rays == 0).float().mean() > 0.05, "scene did not reach the T < 1e-4 cut"
    _close(hist, ref, 2e-4, msg="terminated hist")
    _close(rays.reshape(ref_rays.shape), ref_rays, 2e-4, msg="terminated rays")
    _grads_close(m, P, 3e-4, "terminated")


@pytest.mark.parametrize("occl", [False, True])
@pytest.mark.parametrize("ng,shift", [(50, 1.2), (300, 2.5)])
@pytest.mark.parametrize("cutoff", [0.0, 5.7])
def test_aabb_selection_vs_oracle(occl, ng, shift, cutoff):
    """Path C's own selection: 3-sigma boxes, first 256 hits per ray by index, whole-ray pdf (the
    oracle); the engine evaluates each selected Gaussian over the whole ray (cutoff 0) or over its
    5.7-sigma samples (terms < 9e-8 of its peak dropped: the same tolerances hold).
    (300, 2.5): every box covers every ray, so the 256 cap decides which Gaussians a ray sees."""
    from nlosgr.render import bboxes
    walls, box = _scene()
    m = _model(ng, 1, 13, shift, 0.0 if not occl else 1.0)
    g = torch.Generator().manual_seed(6)
    gout = torch.randn(walls.shape[0], T, generator=g)
    mode = "occl" if occl else "noocl"
    hist, rays = _hip(m, mode, "aabb", cutoff, walls, box, gout, want_rays=True)
    bb = bboxes(m._mu, m._scaling, m._rotation, 1.0, 3.0, preset="cuda").reshape(-1, 6).cpu()
    P, ref, ref_rays = _oracle(m, occl, walls, box, bb=bb, gout=gout)
    if ng == 300:
        from oracle import torch_ref as R
        assert int(R.aabb_filter(walls[:1].cpu(), torch.tensor([[0.0, 1.0, 0.0]]), bb)[0, 0]) == 256
    tol = 2e-4 if occl else 2e-5
    _close(hist, ref, tol, msg=f"aabb {mode} hist")
    _close(rays.reshape(ref_rays.shape), ref_rays, tol, msg=f"aabb {mode} rays")
    _grads_close(m, P, 3e-4, f"aabb {mode}")


def test_tile_engine_deterministic():
    """Forward and backward are bitwise repeatable (static slot schedule, fixed-order sums)."""
    from nlosgr import features_flat
    from nlosgr.geometry import build_geometry
    from nlosgr.render import RenderConfig, render_backward, render_forward
    walls, box = _scene()
    m = _model(80, 3, 21, 1.0, 0.5)
    geo = build_geometry(walls, box, NS, START, START + T, C, DELTAT, 0.5, "cuda", "occl")
    cfg = RenderConfig(preset="cuda", mode="occl", sh_degree=3, cutoff=5.7, c_deltaT=C * DELTAT)
    args = (m._mu, m._scaling, m._rotation, m._opacity, features_flat(m).detach())
    h1, _ = render_forward(*args, geo, cfg)
    h2, _ = render_forward(*args, geo, cfg)
    assert torch.equal(h1, h2)
    gh = torch.randn_like(h1)
    d1 = render_backward(*args, geo, cfg, grad_hist=gh)
    d2 = render_backward(*args, geo, cfg, grad_hist=gh)
    for a, b in zip(d1, d2):
        assert torch.equal(a, b)


def test_train_step_occl():
    """TrainStep runs the occlusion mode end to end (forward, MSE, backward, Adam) and decreases the loss."""
    from nlosgr.geometry import build_geometry
    from nlosgr.render import RenderConfig
    from nlosgr.train import TrainStep
    walls, box = _scene()
    m = _model(40, 1, 3, 1.2, 1.0)
    geo = build_geometry(walls, box, NS, START, START + T, C, DELTAT, 0.5, "cuda", "occl")
    cfg = RenderConfig(preset="cuda", mode="occl", sh_degree=1, cutoff=5.7, c_deltaT=C * DELTAT)
    target = torch.zeros(walls.shape[0], T, device="cuda")
    step = TrainStep(m, geo, cfg, target)
    l0 = float(step()[0])
    for _ in range(5):
        l1 = float(step()[0])
    assert np.isfinite(l1) and l1 < l0


@pytest.mark.parametrize("selection,cutoff", [("support", 5.7), ("support", 0.0), ("aabb", 0.0)])
def test_occl_row_cache_backward_equals_recompute(selection, cutoff):
    """The occlusion row cache (ray_cache=True: the forward stores every tile's (D, W) rows in the
    workspace and the backward reloads them instead of re-running its forward sweep) changes nothing:
    gradients bitwise equal to the recomputing backward, forward unchanged."""
    from nlosgr import features_flat
    from nlosgr.geometry import build_geometry
    from nlosgr.render import RenderConfig, render_backward, render_forward
    walls, box = _scene()
    m = _model(90, 3, 23, 1.0, 1.0)
    geo = build_geometry(walls, box, NS, START, START + T, C, DELTAT, 0.5, "cuda", "occl")
    cfg = RenderConfig(preset="cuda", mode="occl", sh_degree=3, cutoff=cutoff, c_deltaT=C * DELTAT,
                       selection=selection)
    args = (m._mu, m._scaling, m._rotation, m._opacity, features_flat(m).detach())
    h0, _ = render_forward(*args, geo, cfg)
    h1, _, ws = render_forward(*args, geo, cfg, ray_cache=True)
    assert torch.equal(h0, h1)
    gh = torch.randn_like(h0)
    d0 = render_backward(*args, geo, cfg, grad_hist=gh)
    d1 = render_backward(*args, geo, cfg, grad_hist=gh, workspace=ws, ray_cache=True)
    assert any(bool(x.abs().max() > 0) for x in d0)
    for a, b in zip(d0, d1):
        assert torch.equal(a, b)


@pytest.mark.parametrize("selection,cutoff", [("support", 5.7), ("support", 3.0), ("support", 0.0), ("aabb", 5.7),
                                              ("aabb", 0.0)])
def test_occl_small_cdt_polynomial(selection, cutoff):
    """c dT <= 1/64 (C3: 1.25e-3) takes the polynomial 1 - exp(-x) = x (1 - x/2 + x^2/6 - x^3/24)
    (x = sigma pdf c dT <= c dT) in the forward rows and the backward pairs pass: same oracle
    comparison as above at c dT = 0.015.  At cutoffs in (0, 6] the backward walks take pdf from the exp2
    recurrence and 1 - exp(-x) as a quartic in pdf (the C3 occlusion lines' path)."""
    from nlosgr.render import bboxes
    walls, box = _scene()
    m = _model(70, 2, 31, 1.2, 3.0)
    g = torch.Generator().manual_seed(8)
    gout = torch.randn(walls.shape[0], T, generator=g)
    dt = 0.015
    assert C * dt <= 1.0 / 64
    hist, rays = _hip(m, "occl", selection, cutoff, walls, box, gout, want_rays=True, dt=dt)
    bb = bboxes(m._mu, m._scaling, m._rotation, 1.0, 3.0, preset="cuda").reshape(-1, 6).cpu() \
        if selection == "aabb" else None
    P, ref, ref_rays = _oracle(m, True, walls, box, mc=cutoff if cutoff > 0 else None, bb=bb, gout=gout, dt=dt)
    assert float(ref.abs().max()) > 0
    _close(hist, ref, 2e-4, msg=f"occl small c dT hist {selection} {cutoff}")
    _close(rays.reshape(ref_rays.shape), ref_rays, 2e-4, msg="occl small c dT rays")
    _grads_close(m, P, 3e-4, f"occl small c dT {selection} {cutoff}")


def test_aabb_early_exit_exact():
    """AABB selection stops a tile's sweep once all its rays hold 256 selections: a scene where
    every box covers every ray (the cap decides) renders identically with 600 Gaussians and with
    the first 300 + 300 Gaussians that no ray can select any more (their indices come after every
    ray's 256th hit)."""
    from nlosgr import GaussianParams, features_flat
    from nlosgr.geometry import build_geometry
    from nlosgr.render import RenderConfig, render_forward, render_backward
    walls, box = _scene()
    m = _model(600, 1, 17, 2.5, 0.5)
    geo = build_geometry(walls, box, NS, START, START + T, C, DELTAT, 0.5, "cuda", "occl")
    cfg = RenderConfig(preset="cuda", mode="occl", sh_degree=1, cutoff=0.0, c_deltaT=C * DELTAT, selection="aabb")
    full = (m._mu, m._scaling, m._rotation, m._opacity, features_flat(m).detach())
    head = tuple(t[:300].contiguous() for t in full)
    h_full, _ = render_forward(*full, geo, cfg)
    h_head, _ = render_forward(*head, geo, cfg)
    assert torch.equal(h_full, h_head)
    gh = torch.randn_like(h_full)
    d_full = render_backward(*full, geo, cfg, grad_hist=gh)
    d_head = render_backward(*head, geo, cfg, grad_hist=gh)
    for a, b in zip(d_full, d_head):
        assert torch.equal(a[:300], b)
        assert float(a[300:].abs().max()) == 0.0


@pytest.mark.parametrize("selection,cutoff", [("support", 5.7), ("aabb", 5.7)])
def test_occl_batched_train_step_matches_whole_wall(monkeypatch, selection, cutoff):
    """TrainStep's occlusion mode runs forward -> MSE -> backward per batch of wall points, the backward
    reloading the batch's (D, W) rows (a row cache bounded by the batch).  Forced to batches of two
    wall points, its gradients and loss equal the whole-wall composition without any cache: forward,
    MSE over the whole volume, recomputing backward (sums in another order: rtol 1e-5)."""
    from nlosgr import features_flat, train as T_
    from nlosgr.geometry import build_geometry
    from nlosgr.render import RenderConfig, render_backward, render_forward, tile_rows_bytes
    walls, box = _scene()
    m = _model(90, 3, 29, 1.0, 1.0)
    geo = build_geometry(walls, box, NS, START, START + T, C, DELTAT, 0.5, "cuda", "occl")
    cfg = RenderConfig(preset="cuda", mode="occl", sh_degree=3, cutoff=cutoff, c_deltaT=C * DELTAT,
                       selection=selection)
    g = torch.Generator().manual_seed(4)
    target = (torch.rand(walls.shape[0], T, generator=g) * 1e-3).cuda()
    args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
            features_flat(m).detach().contiguous())
    hist, _ = render_forward(*args, geo, cfg)
    loss4, grad = T_.mse(hist, target, 100.0, raw=True)
    ref = render_backward(*args, geo, cfg, grad_hist=grad)
    ref = [ref[0], ref[4][:, :1], ref[4][:, 1:], ref[3], ref[1], ref[2]]
    monkeypatch.setattr(T_, "OCCL_BATCH_BYTES", 2 * tile_rows_bytes(geo) // walls.shape[0])
    step = T_.TrainStep(m, geo, cfg, target, gt_times=100.0, keep_grads=True)
    assert len(step.occl_batches()) == (walls.shape[0] + 1) // 2 > 1
    loss2 = step()
    _close(loss2, loss4[:2], 1e-5, msg="loss")
    for name, a, b in zip(T_.GROUPS, step.grads, ref):
        _close(a, b.reshape(a.shape), 1e-5, atol=1e-12, msg=f"grad {name}")


@pytest.mark.parametrize("mode,selection", [("occl", "support"), ("noocl", "aabb")])
def test_tile_forward_wall_batches_bitwise(monkeypatch, mode, selection):
    """The ray-tile forward runs in wall-point batches once its tile partials would pass
    NLOSGR_TILE_HPART_MB (1 GiB: C5 with AABB selection would need 69 GB for the wall).  Batches of one
    wall point give bitwise the same histogram, per-ray output and (occlusion, row cache) gradients."""
    from nlosgr import features_flat
    from nlosgr.geometry import build_geometry
    from nlosgr.render import RenderConfig, render_backward, render_forward
    walls, box = _scene()
    m = _model(90, 3, 31, 1.0, 1.0)
    geo = build_geometry(walls, box, NS, START, START + T, C, DELTAT, 0.5, "cuda", mode)
    cfg = RenderConfig(preset="cuda", mode=mode, sh_degree=3, cutoff=5.7, c_deltaT=C * DELTAT,
                       ray_scale=1.0 if mode == "occl" else C * DELTAT, selection=selection)
    args = (m._mu, m._scaling, m._rotation, m._opacity, features_flat(m).detach())
    from nlosgr import _lib
    out = []
    for hp in (None, 0.0001):
        with _lib.batch_budgets(tile_hpart_mb=hp):
            h, r, ws = render_forward(*args, geo, cfg, want_rays=True, ray_cache=mode == "occl") \
                if mode == "occl" else (*render_forward(*args, geo, cfg, want_rays=True), None)
            gh = torch.ones_like(h)
            d = render_backward(*args, geo, cfg, grad_hist=gh, workspace=ws, ray_cache=ws is not None)
        out.append((h, r, d))
    (h0, r0, d0), (h1, r1, d1) = out
    assert torch.equal(h0, h1) and torch.equal(r0, r1)
    for a, b in zip(d0, d1):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mode,selection,cutoff,scale_shift", [
    ("occl", "aabb", 5.7, 0.0), ("noocl", "aabb", 5.7, 0.0), ("occl", "aabb", 0.0, 0.0),
    ("occl", "support", 5.7, 0.0), ("occl", "support", 3.0, 0.0), ("occl", "support", 5.7, 1.6)])
def test_tile_bins_bitwise_equal_in_kernel_cull(mode, selection, cutoff, scale_shift):
    """Tile binning (tile_bin_kernel: per wall point and tile, one bit per Gaussian whose cull sphere passes
    the tile's cone, rows in index order) feeds the ray-tile engine the same queue sequence as its in-kernel
    cull of every Gaussian against every item (FLAG_TILE_NOBIN), so forward and backward are bitwise equal.
    6000 Gaussians (about 94 words per bin row); scale_shift 1.6 makes most Gaussians pass every cone, so a
    bin round is cut at the queue's capacity (2048 entries) in the middle of the row."""
    from dataclasses import replace
    from nlosgr import _lib, features_flat
    from nlosgr.geometry import build_geometry, relay_wall_grid, volume_box_point
    from nlosgr.render import RenderConfig, render_backward, render_forward
    dev = torch.device("cuda:0")
    walls, box = relay_wall_grid(3, 3, device=dev), volume_box_point((0.0, 0.5, 0.0), 0.5, dev)
    m = _model(6000, 3, 21, scale_shift - 0.3, 1.0)
    ns, t_ = 12, 96
    dt = 1.28 / t_
    geo = build_geometry(walls, box, ns, t_ // 8, t_ // 8 + t_, C, dt, 0.5, "cuda", mode)
    cfg = RenderConfig(preset="cuda", mode=mode, sh_degree=3, cutoff=cutoff, c_deltaT=C * dt,
                       ray_scale=C * dt if mode == "noocl" else 1.0, selection=selection)
    args = (m._mu.detach(), m._scaling.detach(), m._rotation.detach(), m._opacity.detach(),
            features_flat(m).detach().contiguous(), geo)
    g = torch.randn((9, t_), generator=torch.Generator().manual_seed(4)).to(dev)
    outs = []
    for flags in (0, _lib.FLAG_TILE_NOBIN):
        c = replace(cfg, flags=flags)
        h, _ = render_forward(*args, c)
        d = render_backward(*args, c, grad_hist=g)
        outs.append((h, d))
    (h0, d0), (h1, d1) = outs
    assert float(h0.abs().max()) > 0
    assert torch.equal(h0, h1), float((h0 - h1).abs().max())
    for name, a, b in zip(("mu", "scaling", "rotation", "opacity", "features"), d0, d1):
        assert torch.equal(a, b), (name, float((a - b).abs().max()))
