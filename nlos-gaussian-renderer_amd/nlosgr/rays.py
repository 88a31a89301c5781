"""Path C "rays" API: arbitrary rays x = o + t d through the Gaussians (HIP, through the C ABI).

Mirrors the reference's native module `nlos_gaussian_renderer._C` (bindings.cpp:26-35):
    render_rays(...)              -> (rho_density, density, transmittance) [N_rays, N_samples]
                                     (volume_renderer.cu:189-305)
    filter_gaussians_per_ray(...) -> int32 [N_rays, 257] (ray_aabb.cu:63-102)
and adds the backward the reference lacks (cuda_autograd.py:147-156 returns zeros).

Features are [Ng, K]; the kernel evaluates SH up to min(active_sh_degree, sqrt(K) - 1).  The
reference's module passes only features_dc (K = 1) with the active degree, and its kernel then
reads the NEXT Gaussians' coefficients (spherical_harmonics.cuh:64-80 with sh_dim = 1, an
out-of-bounds read at the end of the array); that undefined behaviour is not reproduced.
"""
import math

import torch

from . import _lib
from .render import _as_f32, bboxes


def _sh_degree(active_sh_degree, k_feat):
    return max(0, min(int(active_sh_degree), int(math.isqrt(max(k_feat, 1))) - 1, 3))


def _structs(ray_o, ray_d, t, cam, means, scales, rotations, opacities, features, deg, mod, preset):
    ng = means.shape[0]
    feats = features.reshape(ng, -1)
    g = _lib.Gaussians(ng, feats.shape[1], _sh_degree(deg, feats.shape[1]), _lib.PRESETS[preset], float(mod),
                       _lib.ptr(means), _lib.ptr(scales), _lib.ptr(rotations), _lib.ptr(opacities), _lib.ptr(feats))
    r = _lib.Rays(ray_o.shape[0], t.shape[0], _lib.ptr(ray_o), _lib.ptr(ray_d), _lib.ptr(t), _lib.ptr(cam))
    return g, r, feats


def filter_gaussians_per_ray(ray_origins, ray_directions, gaussian_means, gaussian_bboxes, sigma_threshold=3.0):
    """_C.filter_gaussians_per_ray: [N_rays, 257] int32 = (count, first 256 hit indices by index, -1).
    gaussian_bboxes is [Ng, 6] (or [Ng, 2, 3]); means and sigma_threshold are unused, as in the
    reference (ray_aabb.cu:63-69)."""
    lib = _lib.load()
    ro, rd = _as_f32(ray_origins), _as_f32(ray_directions)
    bb = _as_f32(gaussian_bboxes).reshape(-1, 6)
    ng = bb.shape[0]
    dummy = torch.zeros(max(ng, 1), 16, device=ro.device)
    g = _lib.Gaussians(ng, 1, 0, _lib.PRESET_CUDA, 1.0, _lib.ptr(dummy), _lib.ptr(dummy), _lib.ptr(dummy),
                       _lib.ptr(dummy), _lib.ptr(dummy))
    t = torch.zeros(1, device=ro.device)
    cam = torch.zeros(3, device=ro.device)
    r = _lib.Rays(ro.shape[0], 1, _lib.ptr(ro), _lib.ptr(rd), _lib.ptr(t), _lib.ptr(cam))
    out = torch.empty(ro.shape[0], _lib.MAX_PER_RAY + 1, dtype=torch.int32, device=ro.device)
    _lib.check(lib.nlosgr_filter_rays(g, r, _lib.ptr(bb), _lib.ptr(out), _lib.stream_handle(ro.device)))
    return out


def gaussian_filter(ray_o, ray_d, means, scales, rotations, scaling_modifier=1.0, sigma_threshold=3.0,
                    preset="cuda"):
    """3-sigma boxes (bbox_compute.cuh:76-120) + the per-ray filter, as render_rays builds them
    internally (volume_renderer.cu:220-244)."""
    bb = bboxes(means, scales, rotations, scaling_modifier, sigma_threshold, preset)
    return filter_gaussians_per_ray(ray_o, ray_d, means, bb, sigma_threshold)


def rays_forward(ray_o, ray_d, t, means, scales, rotations, opacities, features, cam, deg, c_deltaT, mod,
                 use_occlusion, filt, preset="cuda"):
    lib = _lib.load()
    dev = means.device
    ray_o, ray_d, t, cam = [_as_f32(x) for x in (ray_o, ray_d, t, cam)]
    means, scales, rotations, opacities, features = [_as_f32(x) for x in (means, scales, rotations, opacities,
                                                                           features)]
    g, r, _ = _structs(ray_o, ray_d, t, cam, means, scales, rotations, opacities, features, deg, mod, preset)
    ws = torch.empty(max(lib.nlosgr_rays_workspace_bytes(g, r), 1), dtype=torch.uint8, device=dev)
    shape = (ray_o.shape[0], t.shape[0])
    rho, dens, tr = (torch.empty(shape, device=dev) for _ in range(3))
    _lib.check(lib.nlosgr_rays_fwd(g, r, _lib.ptr(filt), float(c_deltaT), int(bool(use_occlusion)), _lib.ptr(ws),
                                   _lib.ptr(rho), _lib.ptr(dens), _lib.ptr(tr), _lib.stream_handle(dev)))
    return rho, dens, tr


def rays_backward(ray_o, ray_d, t, means, scales, rotations, opacities, features, cam, deg, c_deltaT, mod,
                  use_occlusion, filt, g_rho, g_dens, g_tr, preset="cuda"):
    lib = _lib.load()
    dev = means.device
    ray_o, ray_d, t, cam = [_as_f32(x) for x in (ray_o, ray_d, t, cam)]
    means, scales, rotations, opacities, features = [_as_f32(x) for x in (means, scales, rotations, opacities,
                                                                           features)]
    g, r, feats = _structs(ray_o, ray_d, t, cam, means, scales, rotations, opacities, features, deg, mod, preset)
    ws = torch.empty(max(lib.nlosgr_rays_workspace_bytes(g, r), 1), dtype=torch.uint8, device=dev)
    grads = [x.float().contiguous() if x is not None else None for x in (g_rho, g_dens, g_tr)]
    d_mu, d_s, d_q = torch.empty_like(means), torch.empty_like(scales), torch.empty_like(rotations)
    d_o = torch.empty(means.shape[0], device=dev)
    d_f = torch.empty_like(feats)
    _lib.check(lib.nlosgr_rays_bwd(g, r, _lib.ptr(filt), float(c_deltaT), int(bool(use_occlusion)), _lib.ptr(ws),
                                   *[_lib.ptr(x) for x in grads], _lib.ptr(d_mu), _lib.ptr(d_s), _lib.ptr(d_q),
                                   _lib.ptr(d_o), _lib.ptr(d_f), _lib.stream_handle(dev)))
    return d_mu, d_s, d_q, d_o, d_f


def render_rays(ray_origins, ray_directions, t_samples, gaussian_means, gaussian_scales, gaussian_rotations,
                gaussian_opacities, gaussian_features, camera_pos, active_sh_degree, c, deltaT, scaling_modifier,
                use_occlusion, rendering_type="netf", sigma_threshold=3.0, preset="cuda"):
    """_C.render_rays (non-differentiable; volume_renderer.cu:189-305): boxes, filter, render.
    rendering_type is accepted (any string; the reference maps it to an int it never reads,
    volume_renderer.cu:267) and does not change the result."""
    filt = gaussian_filter(ray_origins, ray_directions, gaussian_means, gaussian_scales, gaussian_rotations,
                           scaling_modifier, sigma_threshold, preset)
    return rays_forward(ray_origins, ray_directions, t_samples, gaussian_means, gaussian_scales,
                        gaussian_rotations, gaussian_opacities, gaussian_features, camera_pos, active_sh_degree,
                        c * deltaT, scaling_modifier, use_occlusion, filt, preset)


def render_rays_analytic(ray_origins, ray_directions, t_min, t_max, gaussian_filter, gaussian_means,
                         gaussian_scales, gaussian_rotations, gaussian_opacities, gaussian_features, camera_pos,
                         active_sh_degree, c, deltaT, scaling_modifier, sigma_threshold, rendering_type="netf"):
    """_C.render_rays_analytic (bindings.cpp:6-24, volume_renderer_analytic.cu:178-241): [N_rays]
    one value per ray from the sections of the filtered Gaussians.  c, deltaT and rendering_type
    are accepted and unused, as in the reference kernel.  Forward only (the reference has no
    backward for this path)."""
    lib = _lib.load()
    ro, rd, cam = [_as_f32(x) for x in (ray_origins, ray_directions, camera_pos)]
    means, scales, rotations, opacities, features = [_as_f32(x) for x in (gaussian_means, gaussian_scales,
                                                                           gaussian_rotations, gaussian_opacities,
                                                                           gaussian_features)]
    filt = gaussian_filter.detach()
    if filt.dtype != torch.int32 or filt.dim() != 2 or filt.shape != (ro.shape[0], _lib.MAX_PER_RAY + 1):
        raise ValueError("gaussian_filter must be int32 [N_rays, 257] (filter_gaussians_per_ray layout)")
    filt = filt.contiguous()
    t = torch.zeros(1, device=ro.device)
    g, r, _ = _structs(ro, rd, t, cam, means, scales, rotations, opacities, features, active_sh_degree,
                       scaling_modifier, "cuda")
    out = torch.empty(ro.shape[0], device=ro.device)
    _lib.check(lib.nlosgr_rays_analytic(g, r, _lib.ptr(filt), float(t_min), float(t_max), float(sigma_threshold),
                                        _lib.ptr(out), _lib.stream_handle(ro.device)))
    return out
