"""Drop-in for the reference's gaussian_model/cuda_autograd.py (path C autograd surface), on HIP.

Same names and signatures as the reference:
    CUDA_AVAILABLE                                              (cuda_autograd.py:10-15)
    CUDARenderFunction.apply(15 args) -> (rho_density, density, transmittance)   (:18-191)
    CUDARenderModule(sigma_threshold).forward(...) -> (result [Nr,Nθ,Nφ], hist [Nr])  (:194-316)
    create_cuda_render_module(sigma_threshold=3.0)              (:319-331)
Differences, by design: the backward returns the real gradients of the means, raw scales, raw
rotations, raw opacities and features (the reference returns zeros, :147-156), and
sigma_threshold sets the box size of the per-ray filter (the reference ignores it and uses 3.0,
volume_renderer.cu:231,242 — the default is the same).
"""
from typing import Optional, Tuple

import torch
import torch.nn as nn

from . import _lib
from .rays import gaussian_filter, rays_backward, rays_forward

CUDA_AVAILABLE = _lib.available()


class CUDARenderFunction(torch.autograd.Function):
    """Ray-based rendering (volume_renderer.cu:189-305) with a HIP backward."""

    @staticmethod
    def forward(ctx, ray_origins, ray_directions, t_samples, gaussian_means, gaussian_scales, gaussian_rotations,
                gaussian_opacities, gaussian_features, camera_pos, active_sh_degree, c, deltaT, scaling_modifier,
                use_occlusion, rendering_type, *extra):
        # optional 16th argument: sigma_threshold of the per-ray box filter (default 3.0)
        sigma_threshold = float(extra[0]) if extra else 3.0
        ctx.nextra = len(extra)
        if not CUDA_AVAILABLE:
            raise RuntimeError("CUDA renderer not available")
        # any string is accepted: the reference maps it to 0 ('netf') / 1 (anything else) and the
        # kernel never reads it (volume_renderer.cu:267)
        filt = gaussian_filter(ray_origins, ray_directions, gaussian_means, gaussian_scales, gaussian_rotations,
                               scaling_modifier, sigma_threshold)
        rho, dens, tr = rays_forward(ray_origins, ray_directions, t_samples, gaussian_means, gaussian_scales,
                                     gaussian_rotations, gaussian_opacities, gaussian_features, camera_pos,
                                     active_sh_degree, c * deltaT, scaling_modifier, use_occlusion, filt)
        ctx.save_for_backward(ray_origins, ray_directions, t_samples, gaussian_means, gaussian_scales,
                              gaussian_rotations, gaussian_opacities, gaussian_features, camera_pos, filt)
        ctx.cfg = (active_sh_degree, c * deltaT, scaling_modifier, use_occlusion)
        ctx.shapes = (gaussian_opacities.shape, gaussian_features.shape)
        return rho, dens, tr

    @staticmethod
    def backward(ctx, grad_rho_density, grad_density, grad_transmittance):
        ro, rd, t, means, scales, rots, opac, feats, cam, filt = ctx.saved_tensors
        deg, cdt, mod, occl = ctx.cfg
        d_mu, d_s, d_q, d_o, d_f = rays_backward(ro, rd, t, means, scales, rots, opac, feats, cam, deg, cdt, mod,
                                                 occl, filt, grad_rho_density, grad_density, grad_transmittance)
        need = ctx.needs_input_grad
        return (None, None, None,
                d_mu if need[3] else None,
                d_s if need[4] else None,
                d_q if need[5] else None,
                d_o.reshape(ctx.shapes[0]) if need[6] else None,
                d_f.reshape(ctx.shapes[1]) if need[7] else None,
                None, None, None, None, None, None, None) + (None,) * ctx.nextra


def reference_sh_rows(features: torch.Tensor, degree: int) -> torch.Tensor:
    """The coefficient rows the reference's path C kernel actually reads: it is handed the dc features
    only, [N, C] (cuda_autograd.py:276-280, sh_dim = C), and eval_sh reads (degree + 1)^2 consecutive
    floats from g * sh_dim (volume_renderer.cu:110,170, spherical_harmonics.cuh:64-80), i.e. for
    degree > 0 the dc values of the following Gaussians.  Row g of the result is flat[g*C : g*C + K]
    of the flattened features, K = (degree + 1)^2; reads past the last Gaussian (out of bounds in the
    reference) are zero here.  Differentiable (a gather): gradients flow back to the dc tensor."""
    n, c = features.shape
    k = (int(degree) + 1) ** 2
    flat = features.reshape(-1)
    idx = torch.arange(n, device=features.device).unsqueeze(1) * c + torch.arange(k, device=features.device)
    valid = idx < flat.numel()
    return flat[idx.clamp(max=max(flat.numel() - 1, 0))] * valid.to(features.dtype)


class CUDARenderModule(nn.Module):
    """Spherical ray grid from one relay-wall point, geometric attenuation and angular integration
    around CUDARenderFunction (cuda_autograd.py:194-316).

    reference_sh_reads=True reproduces the reference's SH evaluation at active_sh_degree > 0 as it
    actually runs (neighbouring Gaussians' dc values as higher-order coefficients, reference_sh_rows);
    the default evaluates the dc features at degree 0 (the intent of passing dc only)."""

    def __init__(self, sigma_threshold: float = 3.0, reference_sh_reads: bool = False):
        super().__init__()
        if not CUDA_AVAILABLE:
            raise RuntimeError("CUDA renderer not available")
        self.sigma_threshold = sigma_threshold
        self.reference_sh_reads = reference_sh_reads

    def forward(self, gaussian_model, camera_pos: torch.Tensor, theta_range: Tuple[float, float],
                phi_range: Tuple[float, float], r_range: Tuple[float, float], num_theta: int, num_phi: int,
                num_r: int, c: float, deltaT: float, scaling_modifier: float = 1.0, use_occlusion: bool = True,
                rendering_type: str = "netf") -> Tuple[torch.Tensor, torch.Tensor]:
        device = camera_pos.device
        theta = torch.linspace(theta_range[0], theta_range[1], num_theta, device=device)
        phi = torch.linspace(phi_range[0], phi_range[1], num_phi, device=device)
        theta_grid, phi_grid = torch.meshgrid(theta, phi, indexing="ij")
        tf, pf = theta_grid.reshape(-1), phi_grid.reshape(-1)
        ray_dirs = torch.stack([torch.sin(tf) * torch.cos(pf), torch.sin(tf) * torch.sin(pf), torch.cos(tf)], dim=1)
        ray_origins = camera_pos.unsqueeze(0).expand(tf.shape[0], 3).contiguous()
        t_samples = torch.linspace(r_range[0], r_range[1], num_r, device=device)
        # the reference passes the dc features only (cuda_autograd.py:276-280)
        features = gaussian_model.get_features_dc.squeeze(1)
        deg = int(gaussian_model.active_sh_degree)
        if self.reference_sh_reads and deg > 0:
            features = reference_sh_rows(features, min(deg, 3))
        rho, _, _ = CUDARenderFunction.apply(ray_origins, ray_dirs, t_samples, gaussian_model.get_mu,
                                             gaussian_model._scaling, gaussian_model._rotation,
                                             gaussian_model._opacity, features, camera_pos,
                                             deg, c, deltaT, scaling_modifier,
                                             use_occlusion, rendering_type, self.sigma_threshold)
        result = rho.T.reshape(num_r, num_theta, num_phi)
        distance = t_samples.view(-1, 1, 1)
        result = result / (distance ** 2 + 1e-8) * torch.sin(theta_grid.unsqueeze(0))
        dtheta = (theta_range[1] - theta_range[0]) / num_theta
        dphi = (phi_range[1] - phi_range[0]) / num_phi
        pred_histogram = torch.sum(result, dim=(1, 2)) * dtheta * dphi
        return result, pred_histogram


def create_cuda_render_module(sigma_threshold: float = 3.0,
                              reference_sh_reads: bool = False) -> Optional[CUDARenderModule]:
    """CUDARenderModule if the HIP library and a GPU are available, else None (:319-331)."""
    if not CUDA_AVAILABLE:
        return None
    return CUDARenderModule(sigma_threshold=sigma_threshold, reference_sh_reads=reference_sh_reads)
