"""Drop-in for the reference's `nlos_gaussian_renderer` package front
(submodules/cuda_renderer/__init__.py:1-187): the non-autograd ray renderer NLOSGaussianRenderer
(:24-180, `render` :43, `filter_gaussians` :154), `create_renderer` (:184) and the section
renderer re-exports (:21).  Everything runs through the C ABI (nlosgr_bboxes,
nlosgr_filter_rays, nlosgr_rays_fwd); there is no CPU path.
"""
import torch

from . import _lib
from .rays import filter_gaussians_per_ray, render_rays
from .section_renderer import SectionGaussianRendererCUDA, create_section_renderer  # noqa: F401

CUDA_AVAILABLE = _lib.available()

MAX_GAUSSIANS_PER_RAY = _lib.MAX_PER_RAY


class NLOSGaussianRenderer:
    """Ray-based renderer: per-ray AABB filtering, then volume rendering along each ray
    (__init__.py:24-41).  As in the reference, sigma_threshold changes no result: `render` uses
    the fixed 3-sigma boxes of _C.render_rays (volume_renderer.cu:226-244) and
    `filter_gaussians` passes it to a filter that ignores it (ray_aabb.cu:63-69)."""

    def __init__(self, sigma_threshold=3.0):
        if not CUDA_AVAILABLE:
            raise RuntimeError("HIP renderer library (libnlosgr.so) or GPU is not available. "
                               "Cannot use NLOSGaussianRenderer.")
        self.sigma_threshold = sigma_threshold

    def render(self, gaussian_model, camera_pos, theta_range, phi_range, r_range, num_theta, num_phi, num_r, c,
               deltaT, scaling_modifier=1.0, use_occlusion=True, rendering_type="netf"):
        """(result [num_r, num_theta, num_phi], pred_histogram [num_r]) of one relay-wall point
        (__init__.py:43-152): linspace angular grid, rays from camera_pos, linspace radii, the
        dc features only (:112-115), attenuation sin(theta)/(r^2 + 1e-8), angular sum x dtheta dphi.
        No autograd graph, as in the reference (it calls _C.render_rays directly)."""
        device = camera_pos.device
        with torch.no_grad():
            theta = torch.linspace(theta_range[0], theta_range[1], num_theta, device=device)
            phi = torch.linspace(phi_range[0], phi_range[1], num_phi, device=device)
            theta_grid, phi_grid = torch.meshgrid(theta, phi, indexing="ij")
            tf, pf = theta_grid.reshape(-1), phi_grid.reshape(-1)
            ray_dirs = torch.stack([torch.sin(tf) * torch.cos(pf), torch.sin(tf) * torch.sin(pf), torch.cos(tf)],
                                   dim=1)
            ray_origins = camera_pos.unsqueeze(0).expand(tf.shape[0], 3)
            t_samples = torch.linspace(r_range[0], r_range[1], num_r, device=device)
            sh_features = gaussian_model.get_features_dc.squeeze(1)
            rho_density, _, _ = render_rays(ray_origins.contiguous(), ray_dirs.contiguous(), t_samples,
                                            gaussian_model.get_mu, gaussian_model._scaling,
                                            gaussian_model._rotation, gaussian_model._opacity, sh_features,
                                            camera_pos, gaussian_model.active_sh_degree, c, deltaT,
                                            scaling_modifier, use_occlusion, rendering_type)
            result = rho_density.T.reshape(num_r, num_theta, num_phi)
            distance = t_samples.view(-1, 1, 1)
            result = result / (distance ** 2 + 1e-8) * torch.sin(theta_grid.unsqueeze(0))
            dtheta = (theta_range[1] - theta_range[0]) / num_theta
            dphi = (phi_range[1] - phi_range[0]) / num_phi
            pred_histogram = torch.sum(result, dim=(1, 2)) * dtheta * dphi
        return result, pred_histogram

    def filter_gaussians(self, ray_origins, ray_directions, gaussian_means, gaussian_bboxes):
        """[N_rays, 257] int32: count, then the first 256 hit Gaussian indices, -1 padding
        (__init__.py:154-180; gaussian_bboxes [Ng, 2, 3] or [Ng, 6])."""
        return filter_gaussians_per_ray(ray_origins.contiguous(), ray_directions.contiguous(),
                                        gaussian_means.contiguous(), gaussian_bboxes.contiguous().view(-1, 6),
                                        self.sigma_threshold)


def create_renderer(sigma_threshold=3.0):
    """Create an NLOSGaussianRenderer instance (__init__.py:184-186)."""
    return NLOSGaussianRenderer(sigma_threshold=sigma_threshold)
