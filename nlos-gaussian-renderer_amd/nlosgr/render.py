"""Autograd Function over the C ABI (nlosgr_render_fwd / nlosgr_render_bwd).

RenderFn is the single differentiable entry point everything else (the reference-API mirrors,
the batched volume renderer, the multi-GPU shard) is built on.  It returns
    hist [P, nr]              hscale[p] * att[k] * sum_{g,ij} w_g(p) sin(theta_i) pdf
    rays [P, nt*np, nr]       ray_scale * sum_g w_g(p) pdf           (optional; the reference's
                              per-(ray, sample) layout, rays in meshgrid('ij') order)
and backward yields real gradients for the five raw parameter tensors (the reference's
CUDA backward returns zeros, gaussian_model/cuda_autograd.py:147-156).
"""
import os
from dataclasses import dataclass

import torch

from . import _lib

# upper bound on the forward->backward ray cache (24 B per wall point x Gaussian pair; C3: 39 GB)
RAY_CACHE_MAX_BYTES = int(float(os.environ.get("NLOSGR_RAY_CACHE_GB", "128")) * 2 ** 30)   # of 288 GB HBM
# the cache pays at small supports and costs at large ones (C3 backward, MI355X: 3 sigma 280 ms with the
# cache vs 308 without; 5.7 sigma 1608 vs 1392 — the cached walk and the hand-off both slowed down)
RAY_CACHE_MAX_CUTOFF = float(os.environ.get("NLOSGR_RAY_CACHE_MAX_CUTOFF", "4.5"))
# occlusion engine row cache (the forward's per-ray (D, W) rows kept for the backward: 128 GiB at C3):
# off by default, so the occlusion backward stays O(tile) in memory and re-runs the tile's forward
# sweep instead; NLOSGR_OCCL_ROW_CACHE_GB > 0 allows it up to that size AND half the free device memory
OCCL_ROW_CACHE_MAX_BYTES = int(float(os.environ.get("NLOSGR_OCCL_ROW_CACHE_GB", "0")) * 2 ** 30)


@dataclass(frozen=True)
class RenderConfig:
    preset: str = "torch"        # "torch" (path T) or "cuda" (path C)
    mode: str = "noocl"          # "noocl", "netf", "binint" (bin-integrated no-occlusion, forward only) or
                                 # "occl" (path C shared-transmittance compositing, cuda preset)
    sh_degree: int = 0
    scaling_modifier: float = 1.0
    cutoff: float = 0.0          # Mahalanobis support radius; <= 0 -> dense
    c_deltaT: float = 1.0
    ray_scale: float = 1.0
    nsplit: int = 0
    flags: int = 0               # 0 in production; _lib.FLAG_* select A/B variants, bits 0-6 phase ablation
    ray_cache: bool = True       # forward records in-support rays per pair for the backward
    selection: str = "support"   # "support" (Mahalanobis cutoff) or "aabb" (path C's 3-sigma box filter,
                                 # first 256 Gaussians per ray by index; cuda preset)


def tile_rows_bytes(geo):
    """Bytes of the occlusion engine's row cache: one (D, W) float2 per (wall point, ray, bin), rays
    padded to whole tiles (tile_rays / plan in csrc/nlosgr_tiles.hip); C3: 128 GiB."""
    nr = geo.nr
    rt = 64
    while rt > 4 and 2 * rt * nr > 32768:
        rt >>= 1
    ti = 1
    while ti * ti < rt:
        ti <<= 1
    tj = rt // ti
    ntiles = (-(-geo.nt // ti)) * (-(-geo.np // tj))
    return geo.nwall * ntiles * rt * nr * 8


def use_ray_cache(cfg, geo, ng, want_rays=False):
    """The forward->backward cache: for the culled, histogram-only pair-major modes the in-support rays
    of every pair; for occlusion compositing the tiles' (D, W) rows, which spares the backward its
    re-run of the forward sweep."""
    if cfg.mode == "occl":
        need = tile_rows_bytes(geo)
        if not (bool(cfg.ray_cache) and not want_rays and 0 < need <= OCCL_ROW_CACHE_MAX_BYTES):
            return False
        free, _ = torch.cuda.mem_get_info(geo.wall.device)
        return need <= free // 2
    return (bool(cfg.ray_cache) and 0 < cfg.cutoff <= RAY_CACHE_MAX_CUTOFF and not want_rays
            and cfg.mode in ("noocl", "netf") and cfg.selection == "support"
            and geo.nwall * ng * 24 <= RAY_CACHE_MAX_BYTES)


def _as_f32(t):
    t = t.detach()
    if t.dtype != torch.float32:
        raise TypeError(f"nlosgr: expected float32 tensor, got {t.dtype}")
    if not t.is_cuda:
        raise RuntimeError("nlosgr: tensors must live on the GPU (no CPU fallback)")
    return t.contiguous()


def _structs(mu, scaling, rotation, opacity, features, geo, cfg, ray_cache=False, g_range=None):
    ng = mu.shape[0]
    k_feat = features.shape[1] if features.dim() == 2 else 0
    if mu.shape != (ng, 3) or scaling.shape != (ng, 3) or rotation.shape != (ng, 4):
        raise ValueError("nlosgr: mu/scaling must be [Ng,3] and rotation [Ng,4]")
    if opacity.numel() != ng or features.shape[0] != ng or features.dim() != 2:
        raise ValueError("nlosgr: opacity must have Ng elements and features be [Ng,K]")
    g = _lib.Gaussians(ng, k_feat, int(cfg.sh_degree), _lib.PRESETS[cfg.preset],
                       float(cfg.scaling_modifier), _lib.ptr(mu), _lib.ptr(scaling), _lib.ptr(rotation),
                       _lib.ptr(opacity), _lib.ptr(features))
    gs = _lib.Geometry(geo.nwall, geo.nt, geo.np, geo.nr, _lib.ptr(geo.wall), _lib.ptr(geo.sin_theta),
                       _lib.ptr(geo.cos_theta), _lib.ptr(geo.sin_phi), _lib.ptr(geo.cos_phi),
                       _lib.ptr(geo.grid_lin), _lib.ptr(geo.hscale), _lib.ptr(geo.r), _lib.ptr(geo.att))
    o = _lib.Options(_lib.MODES[cfg.mode], float(cfg.cutoff), float(cfg.c_deltaT), float(cfg.ray_scale),
                     int(cfg.nsplit), int(cfg.flags), int(bool(ray_cache)), _lib.SELECTIONS[cfg.selection],
                     *(g_range if g_range is not None else (0, 0)))
    return g, gs, o


def _workspace(lib, g, gs, o, device):
    nbytes = lib.nlosgr_workspace_bytes(g, gs, o)
    if nbytes == 0:
        _lib.check(1)
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


def render_forward(mu, scaling, rotation, opacity, features, geo, cfg, want_hist=True, want_rays=False,
                   workspace=None, ray_cache=False):
    """Non-differentiable forward (used by RenderFn and by inference callers).  With ray_cache the
    forward records its in-support rays in `workspace` (which must then be passed, unchanged, to
    the backward of the same inputs); returns (hist, rays) or, with ray_cache, (hist, rays, ws)."""
    lib = _lib.load()
    dev = mu.device
    mu, scaling, rotation, opacity, features = [_as_f32(t) for t in (mu, scaling, rotation, opacity, features)]
    g, gs, o = _structs(mu, scaling, rotation, opacity, features, geo, cfg, ray_cache)
    ws = _workspace(lib, g, gs, o, dev) if workspace is None else workspace
    hist = torch.empty(geo.nwall, geo.nr, device=dev) if want_hist else None
    rays = torch.zeros(geo.nwall, geo.nt * geo.np, geo.nr, device=dev) if want_rays else None
    _lib.check(lib.nlosgr_render_fwd(g, gs, o, _lib.ptr(ws), _lib.ptr(hist), _lib.ptr(rays),
                                     _lib.stream_handle(dev)))
    if ray_cache:
        return hist, rays, ws
    return hist, rays


def render_backward(mu, scaling, rotation, opacity, features, geo, cfg, grad_hist=None, grad_rays=None,
                    workspace=None, ray_cache=False, g_range=None, out=None):
    """Gradients of the five raw parameter tensors.  ray_cache: `workspace` holds the ray record of
    a forward of the same inputs (render_forward(..., ray_cache=True)).  g_range=(g0, g1) restricts
    the backward to Gaussians [g0, g1) (g0 % 256 == 0) and writes only those rows of `out`, a
    preallocated (d_mu, d_scaling, d_rotation, d_opacity, d_features) tuple (allocated if None)."""
    lib = _lib.load()
    dev = mu.device
    mu, scaling, rotation, opacity, features = [_as_f32(t) for t in (mu, scaling, rotation, opacity, features)]
    g, gs, o = _structs(mu, scaling, rotation, opacity, features, geo, cfg, ray_cache, g_range)
    if ray_cache and workspace is None:
        raise ValueError("nlosgr: ray_cache backward needs the forward's workspace")
    ws = _workspace(lib, g, gs, o, dev) if workspace is None else workspace
    gh = grad_hist.float().contiguous() if grad_hist is not None else None
    gr = grad_rays.float().contiguous() if grad_rays is not None else None
    if out is None:
        d_mu, d_s, d_q = torch.empty_like(mu), torch.empty_like(scaling), torch.empty_like(rotation)
        d_o, d_f = torch.empty(mu.shape[0], device=dev), torch.empty_like(features)
    else:
        d_mu, d_s, d_q, d_o, d_f = out
    _lib.check(lib.nlosgr_render_bwd(g, gs, o, _lib.ptr(ws), _lib.ptr(gh), _lib.ptr(gr), _lib.ptr(d_mu),
                                     _lib.ptr(d_s), _lib.ptr(d_q), _lib.ptr(d_o), _lib.ptr(d_f),
                                     _lib.stream_handle(dev)))
    return d_mu, d_s, d_q, d_o, d_f


def fx_info(mu, scaling, rotation, opacity, features, geo, cfg, workspace):
    """The fixed-point forward's state after render_forward(..., workspace=workspace) with the same inputs:
    (E, E of the largest amplitude bound, LDS flushes, bright segments); zeros when the forward did not
    take the fixed-point drain (nlosgr_fx_info)."""
    lib = _lib.load()
    dev = mu.device
    mu, scaling, rotation, opacity, features = [_as_f32(t) for t in (mu, scaling, rotation, opacity, features)]
    g, gs, o = _structs(mu, scaling, rotation, opacity, features, geo, cfg)
    out = torch.zeros(4, dtype=torch.int32, device=dev)
    _lib.check(lib.nlosgr_fx_info(g, gs, o, _lib.ptr(workspace), _lib.ptr(out), _lib.stream_handle(dev)))
    return tuple(int(v) for v in out.cpu())


def workspace_for(mu, scaling, rotation, opacity, features, geo, cfg, ray_cache=False):
    """A workspace tensor sized for these inputs (nlosgr_workspace_bytes)."""
    lib = _lib.load()
    g, gs, o = _structs(*[_as_f32(t) for t in (mu, scaling, rotation, opacity, features)], geo, cfg, ray_cache)
    return _workspace(lib, g, gs, o, mu.device)


def count_support(mu, scaling, rotation, opacity, features, geo, cfg):
    """(pairs, rays, evaluations) in support at cfg.cutoff for one forward: the work unit of the
    VALU roofline.  Dense (cutoff <= 0) counts every sample."""
    lib = _lib.load()
    dev = mu.device
    mu, scaling, rotation, opacity, features = [_as_f32(t) for t in (mu, scaling, rotation, opacity, features)]
    g, gs, o = _structs(mu, scaling, rotation, opacity, features, geo, cfg)
    ws = _workspace(lib, g, gs, o, dev)
    counts = torch.zeros(3, dtype=torch.int64, device=dev)
    _lib.check(lib.nlosgr_count_support(g, gs, o, _lib.ptr(ws), _lib.ptr(counts), _lib.stream_handle(dev)))
    return tuple(int(v) for v in counts.cpu())


class RenderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, scaling, rotation, opacity, features, geo, cfg, want_hist, want_rays):
        cache = use_ray_cache(cfg, geo, mu.shape[0], want_rays) and any(ctx.needs_input_grad[:5])
        out = render_forward(mu, scaling, rotation, opacity, features, geo, cfg, want_hist, want_rays,
                             ray_cache=cache)
        hist, rays = out[0], out[1]
        ctx.ws = out[2] if cache else None     # the ray record lives until the backward
        ctx.save_for_backward(mu, scaling, rotation, opacity, features)
        ctx.geo, ctx.cfg, ctx.oshape = geo, cfg, opacity.shape
        outs = (hist if hist is not None else torch.zeros(0, device=mu.device),
                rays if rays is not None else torch.zeros(0, device=mu.device))
        return outs

    @staticmethod
    def backward(ctx, g_hist, g_rays):
        mu, scaling, rotation, opacity, features = ctx.saved_tensors
        gh = g_hist if (g_hist is not None and g_hist.numel() > 0) else None
        gr = g_rays if (g_rays is not None and g_rays.numel() > 0) else None
        d_mu, d_s, d_q, d_o, d_f = render_backward(mu, scaling, rotation, opacity, features, ctx.geo, ctx.cfg,
                                                   gh, gr, workspace=ctx.ws, ray_cache=ctx.ws is not None)
        ctx.ws = None
        return d_mu, d_s, d_q, d_o.reshape(ctx.oshape), d_f, None, None, None, None


def render(mu, scaling, rotation, opacity, features, geo, cfg, want_hist=True, want_rays=False):
    """Differentiable render; returns (hist or None, rays or None)."""
    hist, rays = RenderFn.apply(mu, scaling, rotation, opacity, features, geo, cfg, want_hist, want_rays)
    return (hist if want_hist else None), (rays if want_rays else None)


def bboxes(mu, scaling, rotation, scaling_modifier=1.0, sigma_scale=3.0, preset="cuda"):
    """[Ng, 2, 3] axis-aligned sigma_scale boxes (GaussianModel.get_bboxes layout,
    gaussian_model.py:140-178; bbox_compute.cuh:76-120)."""
    lib = _lib.load()
    mu, scaling, rotation = [_as_f32(t) for t in (mu, scaling, rotation)]
    ng = mu.shape[0]
    dummy = torch.zeros(ng, device=mu.device)
    g = _lib.Gaussians(ng, 1, 0, _lib.PRESETS[preset], float(scaling_modifier), _lib.ptr(mu), _lib.ptr(scaling),
                       _lib.ptr(rotation), _lib.ptr(dummy), _lib.ptr(dummy))
    out = torch.empty(ng, 6, device=mu.device)
    _lib.check(lib.nlosgr_bboxes(g, float(sigma_scale), _lib.ptr(out), _lib.stream_handle(mu.device)))
    return out.view(ng, 2, 3)
